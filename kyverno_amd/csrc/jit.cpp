// Runtime-compiled walk kernels: each ruleset's patterns are emitted as HIP source (one inlined device
// function per pattern node) and compiled for gfx950 with hipRTC once per ruleset, then loaded per device.
//
// Why: the interpreted walk (kyv_wave.h) pays for generality on every step (frame management, handler
// dispatch, 64-bit lane masks) and serialises one memory round trip per step. The generated code is the
// per-lane recursion of eval_pattern (kyv_eval.h; pkg/engine/validate/validate.go:31-247 with
// anchor/handlers.go, anchormap.go, error.go) unrolled for one pattern: keys, handlers, path templates and
// leaf ids are constants, every path-column lookup of a map is issued up front (independent loads), and the
// register footprint is what that pattern needs. The same walk-phase pieces (pair_walk, walk_chunks,
// leaf matching) are shared with the interpreted kernel, and parity tests run both against the oracle.
#include <dlfcn.h>
#include <sys/stat.h>
#include <unistd.h>
#include <hip/hip_runtime.h>
#include <hip/hiprtc.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <map>
#include <mutex>
#include <utime.h>
#include <set>
#include <sstream>
#include <unordered_map>
#include <stdexcept>
#include <string>
#include <vector>

#include "kyv_host.h"

namespace kyv {

int pattern_depth(const Ruleset& rs, uint32_t pn, int guard);

namespace {

struct Gen {
  const Ruleset& rs;
  std::ostringstream out;
  std::vector<uint8_t> emitted;  // pnode -> function emitted
  std::vector<uint32_t> emitted_log;  // pnodes in emission order (rollback of one root's functions)
  bool ok = true;                // pattern compilable (else the rule stays on the interpreter)
  // array lengths via the (count, element-0 row) columns, preloaded with the scope: on by default since round 2
  // (C3 2.83 -> 2.73 ms per evaluation; it measured slower in round 1, before the uniform-wave schedule and glob
  // masks); KYV_JIT_LEN=0 turns it off
  const bool use_len = !getenv("KYV_JIT_LEN") || atoi(getenv("KYV_JIT_LEN")) != 0;
  // array-of-maps elements whose column loads are issued together (KYV_JIT_BATCH; default 1 = one element at a
  // time: batches of 2 / 4 measured 2.1x slower on C3, 1.41 -> 2.97 ms walk, registers past the 4-wave budget)
  const size_t batch_max = getenv("KYV_JIT_BATCH") ? (size_t)std::max(1, atoi(getenv("KYV_JIT_BATCH"))) : 1;

  // Column scopes: the pattern root and every array-element pattern open a scope (one row of one row space);
  // every column lookup of the maps inside a scope (not crossing into array elements) is loaded up front by
  // the scope's caller into `pc[]`, so a scope costs one round of independent loads however deep its maps nest.
  std::vector<int> slot;                         // pentry -> index of its column in its scope's pc[], -1 none
  std::vector<int> slot_alen;                    // array pnode -> index of its length column in pc[], -1 none
  std::vector<int> slot_elen;                    // existence entry -> index of the candidates' length column
  std::vector<std::vector<uint32_t>> scope_of;   // scope-root pnode -> its column ids, in pc[] order
  std::vector<uint8_t> scoped;                   // pnode -> scope collected
  std::vector<uint32_t> node_mbase;              // pnode -> its rule's first metadata site (marked from the roots)
  std::vector<int8_t> meta_pos;                  // pnode -> static position whose metadata flags the flattener
                                                 // computed: 0 root, 1 spec.template, 2 spec.jobTemplate.spec.template

  explicit Gen(const Ruleset& r)
      : rs(r), emitted(r.pnodes.size(), 0), slot(r.pentries.size(), -1), slot_alen(r.pnodes.size(), -1),
        slot_elen(r.pentries.size(), -1), scope_of(r.pnodes.size()), scoped(r.pnodes.size(), 0),
        node_mbase(r.pnodes.size(), NONE), meta_pos(r.pnodes.size(), -1) {}

  // static key path of the pattern maps below a rule root (plain key entries only), for meta_pos
  void mark_paths(uint32_t pn, uint32_t mbase, uint32_t k0, uint32_t k1, uint32_t k2, uint32_t k3, int depth) {
    if (pn == NONE || pn >= rs.pnodes.size() || depth > 4) return;
    const PNode& P = rs.pnodes[pn];
    if (P.kind != P_MAP) return;
    node_mbase[pn] = mbase;
    const uint32_t S = SID_FIRST_FREE + K_SPEC, T = SID_FIRST_FREE + K_TEMPLATE, J = SID_FIRST_FREE + K_JOBTEMPLATE;
    if (depth == 0) meta_pos[pn] = 0;
    else if (depth == 2 && k0 == S && k1 == T) meta_pos[pn] = 1;
    else if (depth == 4 && k0 == S && k1 == J && k2 == S && k3 == T) meta_pos[pn] = 2;
    for (uint32_t e = 0; e < P.n; e++) {
      const PEntry& E = rs.pentries[P.first + e];
      if ((E.flags & EF_WILD) || E.child == NONE || E.handler == H_STAR || E.handler == H_NEGATION ||
          E.handler == H_EXISTENCE || E.handler == H_EXIST_BADPAT)
        continue;
      const uint32_t k[4] = {k0, k1, k2, k3};
      uint32_t nk[4] = {k[0], k[1], k[2], k[3]};
      if (depth < 4) nk[depth] = E.key;
      mark_paths(E.child, mbase, nk[0], nk[1], nk[2], nk[3], depth + 1);
    }
  }

  int add(std::vector<uint32_t>& list, uint32_t col) {
    list.push_back(col);
    return (int)list.size() - 1;
  }
  void collect(uint32_t pn, std::vector<uint32_t>& list, int guard) {
    if (pn == NONE || pn >= rs.pnodes.size() || guard > 4 * MAX_DEPTH) return;
    const PNode& P = rs.pnodes[pn];
    if (P.kind == P_ARR_MAPS || P.kind == P_ARR_POS || P.kind == P_ARR_SCALAR) {  // the array's own length entry
      if (rs.pn_len[pn] != NONE && use_len) {
        if (slot_alen[pn] >= 0) { ok = false; return; }
        slot_alen[pn] = add(list, rs.pn_len[pn]);
      }
      return;  // its elements open their own scopes
    }
    if (P.kind != P_MAP) return;
    for (uint32_t e = 0; e < P.n; e++) {
      const uint32_t ei = P.first + e;
      const PEntry& E = rs.pentries[ei];
      if (E.col != NONE) {
        if (slot[ei] >= 0) { ok = false; continue; }  // entry reached from two scopes: leave the rule interpreted
        slot[ei] = add(list, E.col);
      }
      if (E.handler == H_EXISTENCE && rs.pe_len[ei] != NONE && use_len) {
        if (slot_elen[ei] >= 0) { ok = false; continue; }
        slot_elen[ei] = add(list, rs.pe_len[ei]);
      }
      if (E.handler == H_STAR || E.handler == H_NEGATION || E.handler == H_EXIST_BADPAT || E.handler == H_EXISTENCE ||
          E.child == NONE)
        continue;
      collect(E.child, list, guard + 1);  // child maps share the scope; arrays open new ones
    }
  }
  void scope(uint32_t root) {
    if (root == NONE || root >= rs.pnodes.size() || scoped[root]) return;
    scoped[root] = 1;
    collect(root, scope_of[root], 0);
  }
  // open the scopes of every array-element pattern below pn
  void scopes_below(uint32_t pn, int guard) {
    if (pn == NONE || pn >= rs.pnodes.size() || guard > 4 * MAX_DEPTH) return;
    const PNode& P = rs.pnodes[pn];
    switch (P.kind) {
      case P_MAP:
        for (uint32_t e = 0; e < P.n; e++) {
          const PEntry& E = rs.pentries[P.first + e];
          if (E.handler == H_STAR || E.handler == H_NEGATION || E.handler == H_EXIST_BADPAT || E.child == NONE) continue;
          if (E.handler == H_EXISTENCE) {
            for (uint32_t j = 0; j < rs.pool[E.child]; j++) {
              scope(rs.pool[E.child + 1 + j]);
              scopes_below(rs.pool[E.child + 1 + j], guard + 1);
            }
          } else {
            scopes_below(E.child, guard + 1);
          }
        }
        break;
      case P_ARR_MAPS: scope(P.first); scopes_below(P.first, guard + 1); break;
      case P_ARR_POS:
        for (uint32_t i = 0; i < P.n; i++) { scope(rs.pool[P.first + i]); scopes_below(rs.pool[P.first + i], guard + 1); }
        break;
      default: break;
    }
  }
  // the columns of scope `root`, in pc[] order
  const std::vector<uint32_t>& scope_cols(uint32_t root) { scope(root); return scope_of[root]; }
  // preload of scope `root`'s columns at row expression `rowx` into array `name`
  // (`rd`: the column read, jself(w, ...) inside the walk, jc_col(v, ...) before the walker state exists)
  std::string preload(uint32_t root, const std::string& name, const std::string& rowx, const char* rd = "jself(w, ") {
    scope(root);
    const auto& L = scope_of[root];
    std::ostringstream o;
    o << "uint64_t " << name << "[" << std::max<size_t>(1, L.size()) << "];";
    for (size_t i = 0; i < L.size(); i++) o << " " << name << "[" << i << "] = " << rd << u(L[i]) << ", " << rowx << ");";
    return o.str();
  }

  static std::string u(uint32_t x) { return std::to_string(x) + "u"; }
  static std::string i64(int64_t x) { return "(int64_t)" + std::to_string(x) + "ll"; }

  // pattern.Validate(value, pattern) for one compiled leaf, as an expression-statement block that sets `okv`
  // (and `fb`) from Val `x`: the type matrix of leaf_match with the pattern constants folded in, and the
  // string mini-language's OR-of-AND atom groups unrolled in evaluation order.
  std::string atom_call(const Atom& a) {
    std::ostringstream o;
    o << "jatom<" << (int)a.op << ", " << (int)a.flags << ", " << (int)a.glob << ", " << (int)a.gidx << ">(w.v, x, " << u(a.pat) << ", "
      << u(a.lit) << ", " << i64(a.dur) << ", " << i64(a.qlo) << ", " << i64(a.qhi) << ", &fb)";
    return o.str();
  }
  std::string leaf_code(uint32_t lid) {
    const Leaf& L = rs.leaves[lid];
    std::ostringstream o;
    switch (L.type) {
      case L_NIL:
        o << "okv = x.t == 0xFF || x.t == N_NULL || x.t == N_FALSE || (x.t == N_INT && x.i == 0) || "
             "(x.t == N_FLOAT && x.f == 0.0) || (x.t == N_STR && x.sid == SID_EMPTY);";
        break;
      case L_BOOL: o << "okv = x.t == " << (L.bval ? "N_TRUE" : "N_FALSE") << ";"; break;
      case L_FLOAT: {
        uint64_t bits = __builtin_bit_cast(uint64_t, L.f);
        o << "{ const double pf = __builtin_bit_cast(double, (uint64_t)" << bits << "ull);\n"
          << "  okv = (x.t == N_INT && " << (L.fint ? "true" : "false") << " && " << i64(L.fi) << " == x.i) ||\n"
          << "        (x.t == N_FLOAT && x.f == pf) ||\n"
          << "        (x.t == N_STR && (gld32(w.v.str_flags + x.sid) & SF_FLOAT) && "
             "*(const KYV_AS_GLOBAL double*)(w.v.str_f64 + x.sid) == pf); }";
        break;
      }
      case L_STR: {
        o << "{ bool done = x.t == N_STR && x.sid == " << u(L.exact) << ";\n";
        for (uint32_t g = 0; g < L.ngroups; g++) {
          uint32_t a0 = rs.pool[L.groups + 2 * g], na = rs.pool[L.groups + 2 * g + 1];
          o << "  { bool all = !done;\n";
          for (uint32_t k = 0; k < na; k++) {
            const Atom& A = rs.atoms[a0 + k];
            if (A.op == A_FALSE) { o << "    all = false;\n"; continue; }
            if (A.op == A_RANGE_IN || A.op == A_RANGE_OUT) {
              const Atom &s0 = rs.atoms[A.sub], &s1 = rs.atoms[A.sub + 1];
              o << "    if (all) all = " << atom_call(s0) << (A.op == A_RANGE_IN ? " && " : " || ") << atom_call(s1) << ";\n";
            } else {
              o << "    if (all) all = " << atom_call(A) << ";\n";
            }
          }
          o << "    if (all) done = true; }\n";
        }
        o << "  okv = done; }";
        break;
      }
      case L_MAP: o << "okv = x.t == N_MAP;"; break;
      default: o << "okv = false;";
    }
    return o.str();
  }

  // emit the function of pattern node `pn` (children first)
  void node(uint32_t pn, int guard) {
    if (pn == NONE || pn >= rs.pnodes.size() || guard > 4 * MAX_DEPTH) { ok = false; return; }
    if (emitted[pn]) return;
    const PNode P = rs.pnodes[pn];
    // children first
    switch (P.kind) {
      case P_MAP:
        for (uint32_t e = 0; e < P.n; e++) {
          const PEntry& E = rs.pentries[P.first + e];
          if (E.handler == H_STAR || E.handler == H_NEGATION || E.handler == H_EXIST_BADPAT) continue;
          if (E.child == NONE) { ok = false; return; }
          if (E.handler == H_EXISTENCE) {
            uint32_t npat = rs.pool[E.child];
            for (uint32_t j = 0; j < npat; j++) node(rs.pool[E.child + 1 + j], guard + 1);
          } else {
            node(E.child, guard + 1);
          }
        }
        break;
      case P_ARR_MAPS: node(P.first, guard + 1); break;
      case P_ARR_POS:
        for (uint32_t i = 0; i < P.n; i++) node(rs.pool[P.first + i], guard + 1);
        break;
      default: break;
    }
    if (!ok) return;
    emitted[pn] = 1;
    emitted_log.push_back(pn);
    const std::string T = u(P.tmpl);
    out << "static __device__ __forceinline__ Ret p" << pn
        << "(JW& w, uint32_t rn, uint32_t rt, uint32_t ra, uint32_t row, const uint64_t* pc) {\n";
    switch (P.kind) {
      case P_MAP: map(pn, P); break;
      case P_LEAF:
        // a string / boolean / null whose type and `a` came with the column needs no row read
        out << "  const bool known = rt == N_STR || rt == N_TRUE || rt == N_FALSE || rt == N_NULL;\n"
               "  Node n{0u, 0u, 0u, 0u};\n  if (rn != NONE && !known) n = gnode(w.R + rn);\n";
        out << "  bool fb = false, okv = true;\n";
        out << "  const bool each = rn != NONE && !known && node_type(n) == N_ARR;\n"
               "  const uint32_t cnt = each ? n.b : 1u;\n"
               "  for (uint32_t i = 0; i < cnt && okv; i++) {\n"
               "    const Val x = each ? wvalue_of(w.v, w.R, n.a + i)\n"
               "                       : (rn == NONE ? wvalue_absent() : known ? jvalue(w, rn, rt, ra) : wvalue_node(w.v, n));\n"
               "    " << leaf_code(P.first) << "\n"
               "  }\n";
        out << "  if (fb) { w.ost = ST_FALLBACK; return ok_ret(); }\n";
        out << "  return okv ? ok_ret() : mkerr(EC_NONE, 0, " << T << ");\n";
        break;
      case P_ARR_EMPTY:
        out << "  return mkerr(EC_NONE, 0, " << T << ");\n";
        break;
      case P_ARR_SCALAR: {
        uint32_t leaf = rs.pnodes[P.first].first;
        array_head(pn, T);
        out << "  bool fb = false, okv = true;\n";
        const uint32_t self = rs.pn_self[pn];
        out << "  for (uint32_t i = 0; i < cnt && okv; i++) {\n";
        if (self != NONE)
          out << "    uint32_t et, ea; const uint32_t ei = jdec(jself(w, " << u(self) << ", eb == NONE ? NONE : eb + i), &et, &ea);\n"
                 "    const Val x = ei == NONE ? wvalue_of(w.v, w.R, aa + i) : jvalue(w, ei, et, ea);\n";
        else
          out << "    const Val x = wvalue_of(w.v, w.R, aa + i);\n";
        out << "    " << leaf_code(leaf) << "\n"
               "  }\n";
        out << "  if (fb) { w.ost = ST_FALLBACK; return ok_ret(); }\n";
        out << "  return okv ? ok_ret() : mkerr(EC_NONE, 0, " << T << ");\n";
        break;
      }
      case P_ARR_MAPS: case P_ARR_POS: {
        array_head(pn, T);
        if (P.kind == P_ARR_POS) out << "  if (cnt < " << u(P.n) << ") return mkerr(EC_NONE, 0, NONE);\n";
        out << "  uint32_t st = 0;\n";
        const uint32_t self = rs.pn_self[pn];
        auto elem = [&](const std::string& i, uint32_t child, bool setidx) {
          if (setidx)
            out << "    w.idx = (w.idx & ~(0xFFFFull << " << 16u * P.level << ")) | ((uint64_t)" << i << " << "
                << 16u * P.level << ");\n";
          out << "    { const uint32_t er = eb == NONE ? NONE : eb + " << i << ";\n"
              << "      " << preload(child, "pe", "er") << "\n";
          if (self != NONE)
            out << "      uint32_t et, ea; uint32_t ei = jdec(jself(w, " << u(self) << ", er), &et, &ea);\n"
                   "      if (ei == NONE) { ei = aa + " << i << "; et = T_UNK; }\n";
          else
            out << "      const uint32_t ei = aa + " << i << ", et = T_UNK, ea = 0u;\n";
          out << "      Ret r = p" << child << "(w, ei, et, ea, er, pe);\n"
              << "      if (w.ost) return r;\n"
              << "      if (r.err) { if (ret_is_skip(r)) st |= FS_SKIP | ((uint32_t)r.mask << 2); else return r; }\n"
              << "      else st |= FS_APPLY; }\n";
        };
        // elements in batches of K: the column loads of K consecutive elements (independent: rows eb + i) are
        // issued together before the first of them is walked, so an array of <= K elements costs one memory round
        // instead of one per element (K from the scope size: at most 8 preloaded 64-bit entries per batch)
        scope(P.first);
        const size_t S = scope_of[P.first].size() + (self != NONE ? 1 : 0);
        const size_t K = P.kind == P_ARR_MAPS && batch_max > 1 && S > 0 ? std::max<size_t>(1, std::min<size_t>(batch_max, 8 / S)) : 1;
        if (P.kind == P_ARR_MAPS && K > 1) {
          out << "  for (uint32_t i0 = 0; i0 < cnt; i0 += " << K << "u) {\n";
          for (size_t q = 0; q < K; q++) {
            const std::string Q = std::to_string(q);
            out << "    const uint32_t er" << Q << " = (eb == NONE || i0 + " << Q << "u >= cnt) ? NONE : eb + i0 + " << Q << "u;\n"
                << "    " << preload(P.first, "pe" + Q, "er" + Q) << "\n";
            if (self != NONE) out << "    const uint64_t sx" << Q << " = jself(w, " << u(self) << ", er" << Q << ");\n";
          }
          // one copy of the element body (the child is inlined): the batch's entries are selected by position
          const size_t NS = scope_of[P.first].size();
          out << "    #pragma nounroll\n"
                 "    for (uint32_t q = 0; q < " << K << "u && i0 + q < cnt; q++) {\n"
                 "      const uint32_t i = i0 + q;\n"
                 "      w.idx = (w.idx & ~(0xFFFFull << " << 16u * P.level << ")) | ((uint64_t)i << " << 16u * P.level << ");\n";
          auto sel = [&](const std::string& a, const std::string& b) {  // a0..a{K-1} (+ b suffix) by q
            std::string e = a + std::to_string(K - 1) + b;
            for (size_t q = K - 1; q-- > 0;) e = "(q == " + std::to_string(q) + "u ? " + a + std::to_string(q) + b + " : " + e + ")";
            return e;
          };
          out << "      const uint32_t er = " << sel("er", "") << ";\n"
              << "      uint64_t pe[" << std::max<size_t>(1, NS) << "];";
          for (size_t x = 0; x < NS; x++) out << " pe[" << x << "] = " << sel("pe", "[" + std::to_string(x) + "]") << ";";
          out << "\n";
          if (self != NONE)
            out << "      uint32_t et, ea; uint32_t ei = jdec(" << sel("sx", "") << ", &et, &ea);\n"
                   "      if (ei == NONE) { ei = aa + i; et = T_UNK; }\n";
          else
            out << "      const uint32_t ei = aa + i, et = T_UNK, ea = 0u;\n";
          out << "      Ret r = p" << P.first << "(w, ei, et, ea, er, pe);\n"
              << "      if (w.ost) return r;\n"
              << "      if (r.err) { if (ret_is_skip(r)) st |= FS_SKIP | ((uint32_t)r.mask << 2); else return r; }\n"
              << "      else st |= FS_APPLY;\n"
              << "    }\n";
          out << "  }\n";
        } else if (P.kind == P_ARR_MAPS) {
          out << "  for (uint32_t i = 0; i < cnt; i++) {\n";
          elem("i", P.first, true);
          out << "  }\n";
        } else {
          for (uint32_t i = 0; i < P.n; i++) {
            out << "  {\n";
            elem(u(i), rs.pool[P.first + i], false);
            out << "  }\n";
          }
        }
        out << "  if ((st & FS_SKIP) && !(st & FS_APPLY)) return mkerr(EC_NONE, (uint8_t)(st >> 2), " << T << ");\n";
        out << "  return ok_ret();\n";
        break;
      }
      default: ok = false;
    }
    out << "}\n";
  }

  // an array node's element count `cnt`, element-0 column row `eb` and first element row `aa`: from the
  // preloaded length column when the array came through a column (no row read), else from its row
  void array_head(uint32_t pn, const std::string& T) {
    out << "  if (rn == NONE) return mkerr(EC_NONE, 0, " << T << ");\n";
    out << "  uint32_t cnt, eb, aa = NONE;\n";
    if (slot_alen[pn] >= 0)
      out << "  if (rt == N_ARR && (uint32_t)(pc[" << slot_alen[pn] << "] >> 32) != NONE) {\n"
             "    cnt = (uint32_t)pc[" << slot_alen[pn] << "]; eb = (uint32_t)(pc[" << slot_alen[pn] << "] >> 32);\n"
             "  } else\n";
    out << "  { const Node a = gnode(w.R + rn);\n"
           "    if (node_type(a) != N_ARR) return mkerr(EC_NONE, 0, " << T << ");\n"
           "    cnt = a.b; eb = a.c; aa = a.a; }\n";
  }

  // lookup expression for entry index ei (global pentries index) into c<e>/t<e>
  void lookup(uint32_t ei, uint32_t e, const std::string& keyexpr_rowvar) {
    const PEntry& E = rs.pentries[ei];
    if (E.col != NONE) {
      if (slot[ei] < 0) { ok = false; return; }  // every column entry belongs to a collected scope
      out << "  c" << e << " = jdec(pc[" << slot[ei] << "], &t" << e << ", &a" << e << ");\n";
    } else {
      std::string key = (E.flags & EF_WILD) ? "w.keys.get(" + u(E.slot) + ")" : u(E.key);
      out << "  c" << e << " = wmap_find(w.R, " << keyexpr_rowvar << ".a, " << keyexpr_rowvar << ".b, " << key
          << "); t" << e << " = T_UNK; a" << e << " = 0u;\n";
    }
  }

  void map(uint32_t pn, const PNode& P) {
    const bool needrow = (P.flags & PF_NEEDROW) != 0;
    const std::string T = u(P.tmpl);
    out << "  Node m{0u, 0u, 0u, 0u};\n";
    out << "  if (rn != NONE && " << (needrow ? "true" : "rt == T_UNK") << ") { m = gnode(w.R + rn); rt = node_type(m); }\n";
    out << "  if (rn == NONE || rt != N_MAP) return mkerr(EC_NONE, 0, " << T << ");\n";
    // static (column) lookups up front: independent loads, issued together
    for (uint32_t e = 0; e < P.n; e++) {
      out << "  uint32_t c" << e << " = NONE, t" << e << " = T_UNK, a" << e << " = 0u;\n";
      const PEntry& E = rs.pentries[P.first + e];
      if (E.col != NONE) lookup(P.first + e, e, "m");
    }
    (void)pn;
    // AnchorMap.CheckAnchorInResource (anchormap.go:30-44); wildcard keys use the slots as they are before
    // this level's metadata expansion, exactly as the walk does
    for (uint32_t e = 0; e < P.n; e++) {
      const PEntry& E = rs.pentries[P.first + e];
      if (E.abit == 0xFF) continue;
      std::string B = "(1ull << " + std::to_string(E.abit) + ")";
      out << "  w.seen |= " << B << ";\n";
      if (E.col != NONE) {
        out << "  if (c" << e << " != NONE) w.found |= " << B << ";\n";
      } else {
        std::string key = (E.flags & EF_WILD) ? "w.keys.get(" + u(E.slot) + ")" : u(E.key);
        out << "  if (!(w.found & " << B << ") && wmap_find(w.R, m.a, m.b, " << key << ") != NONE) w.found |= " << B << ";\n";
      }
    }
    const MetaSite* site =
        (P.flags & PF_META) && node_mbase[pn] != NONE && meta_pos[pn] >= 0 ? &rs.metas[node_mbase[pn] + P.meta] : nullptr;
    if (site && site->nwild_l == 0 && site->nwild_a == 0) {
      // ExpandInMetadata without wildcard keys at the root or a pod-template position: only its type assertions,
      // decided from the header flags the flattener computed for that position (same order as expand_meta:
      // absent/null metadata, non-object, anchor-like keys, labels / annotations that are not objects of strings)
      const uint32_t sh = meta_pos[pn] == 0 ? RF_META_SHIFT : meta_pos[pn] == 1 ? RF_TMETA1_SHIFT : RF_TMETA2_SHIFT;
      out << "  { const uint32_t hf = gld32(&w.hp->flags); KYV_ACCT_ADD(0, 4);\n"
             "    if (!(hf & (1u << " << sh << "))) {\n"
             "      if (hf & (2u << " << sh << ")) { w.ost = ST_PANIC; return ok_ret(); }\n"
             "      if (hf & RF_ANCHORISH) { w.ost = ST_FALLBACK; return ok_ret(); }\n";
      if (site->has_labels) out << "      if (hf & (4u << " << sh << ")) { w.ost = ST_PANIC; return ok_ret(); }\n";
      if (site->has_ann) out << "      if (hf & (8u << " << sh << ")) { w.ost = ST_PANIC; return ok_ret(); }\n";
      out << "    } }\n";
    } else if (site && meta_pos[pn] == 0) {
      // wildcard keys at the resource root: resolved over the header's labels / annotations nodes
      out << "  { Keys kk = w.keys; uint8_t o = expand_meta_root(w.v, w.v.metas[w.mbase + " << u(P.meta)
          << "], NodeTab{w.R}, *w.hp, kk); w.keys = kk;\n"
          << "    if (o != ST_NONE) { w.ost = o; return ok_ret(); } }\n";
    } else if (P.flags & PF_META) {
      // the out-of-line call gets a copy of the key slots: taking w.keys' address would put the whole walker
      // state (JW) in scratch memory for every pattern of the kernel
      out << "  { Keys kk = w.keys; uint8_t o = expand_meta(w.v, w.v.metas[w.mbase + " << u(P.meta)
          << "], NodeTab{w.R}, rn, *w.hp, kk); w.keys = kk;\n"
          << "    if (o != ST_NONE) { w.ost = o; return ok_ret(); } }\n";
    }
    for (uint32_t e = 0; e < P.n; e++) {
      const PEntry& E = rs.pentries[P.first + e];
      const std::string ET = u(E.tmpl);
      const std::string c = "c" + std::to_string(e), t = "t" + std::to_string(e);
      if (E.col == NONE) lookup(P.first + e, e, "m");
      auto call = [&](const std::string& wrap) {
        out << "    { Ret r = p" << E.child << "(w, " << c << ", " << t << ", a" << e << ", row, pc);\n"
            << "      if (w.ost) return r;\n"
            << "      if (r.err) { " << wrap << "return r; } }\n";
      };
      switch (E.handler) {
        case H_NEGATION:
          out << "  if (" << c << " != NONE) return mkerr(EC_NEG, PH_NEG, " << ET << ");\n";
          break;
        case H_EQUALITY:
          out << "  if (" << c << " != NONE) {\n";
          call("");
          out << "  }\n";
          break;
        case H_GLOBAL:
          out << "  if (" << c << " != NONE) {\n";
          call("r.code = EC_GLOBAL; r.mask |= PH_GLOBAL; ");
          out << "  }\n";
          break;
        case H_CONDITION:
          out << "  if (" << c << " == NONE) return mkerr(EC_COND, PH_COND, " << ET << ");\n  {\n";
          call("r.code = EC_COND; r.mask |= PH_COND; ");
          out << "  }\n";
          break;
        case H_STAR:
          out << "  if (" << c << " == NONE || (" << t << " != T_UNK ? " << t << " : node_type(gnode(w.R + " << c
              << "))) == N_NULL) return mkerr(EC_NONE, 0, " << T << ");\n";
          break;
        case H_EXIST_BADPAT:
          out << "  if (" << c << " != NONE) return mkerr(EC_NONE, 0, " << ET << ");\n";
          break;
        case H_EXISTENCE: {
          uint32_t npat = rs.pool[E.child];
          out << "  if (" << c << " != NONE) {\n"
              << "    uint32_t cnt, eb, aa = NONE;\n";
          if (slot_elen[P.first + e] >= 0)
            out << "    if (" << t << " == N_ARR && (uint32_t)(pc[" << slot_elen[P.first + e] << "] >> 32) != NONE) {\n"
                << "      cnt = (uint32_t)pc[" << slot_elen[P.first + e] << "]; eb = (uint32_t)(pc[" << slot_elen[P.first + e]
                << "] >> 32);\n"
                << "    } else\n";
          out << "    { const Node a = gnode(w.R + " << c << ");\n"
              << "      if (node_type(a) != N_ARR) return mkerr(EC_NONE, 0, " << ET << ");\n"
              << "      cnt = a.b; eb = a.c; aa = a.a; }\n";
          for (uint32_t j = 0; j < npat; j++) {
            out << "    { bool hit = false;\n"
                << "      for (uint32_t i = 0; i < cnt; i++) {\n"
                << "        const uint32_t er = eb == NONE ? NONE : eb + i;\n"
                << "        " << preload(rs.pool[E.child + 1 + j], "pe", "er") << "\n"
                << "        uint32_t et = T_UNK, ea = 0u, ei = NONE;\n"
                << (rs.pe_self[P.first + e] != NONE ? "        ei = jdec(jself(w, " + u(rs.pe_self[P.first + e]) + ", er), &et, &ea);\n"
                                                      : std::string())
                << "        if (ei == NONE) { ei = aa + i; et = T_UNK; }\n"
                << "        Ret r = p" << rs.pool[E.child + 1 + j] << "(w, ei, et, ea, er, pe);\n"
                << "        if (w.ost) return r;\n"
                << "        if (!r.err) { hit = true; break; }\n"
                << "      }\n"
                << "      if (!hit) return mkerr(EC_NONE, 0, " << ET << "); }\n";
          }
          out << "  }\n";
          break;
        }
        default:  // H_DEFAULT: resourceMap[k] (absent -> nil)
          out << "  {\n";
          call("");
          out << "  }\n";
      }
    }
    out << "  return ok_ret();\n";
  }
};

// ---------------------------------------------------------------- compiled condition rules
// Deny / foreach rules (and preconditions) whose condition programs hold JMESPath-subset operands, generated as
// straight-line code over path columns (kyv_jcond.h). Semantics follow the interpreter: jmes_run / eval_prog
// (kyv_cond.h) and eval_foreach (kyv_pss.h); a program shape the generator does not cover leaves the rule on the
// interpreted kernel (match_kernel<true>).
struct CondGen {
  const Ruleset& rs;
  std::ostringstream defs;  // generated functions (operands, programs, rules), in dependency order
  std::ostringstream out;   // body of the function being generated
  bool ok = true;
  uint32_t uid = 0;
  uint32_t nslots = 1;      // LDS lists per lane the generated programs need (1 or 2)
  bool lds_used = false;    // some operand materialises its list in LDS
  uint32_t cur_etpos = NONE;  // element trie position of the program being generated (stream_cond)
  std::unordered_map<uint64_t, std::string> progs;  // (program, element trie position) -> function name

  explicit CondGen(const Ruleset& r) : rs(r) {}
  static std::string u(uint32_t x) { return std::to_string(x) + "u"; }
  std::string fresh(const char* p) { return std::string(p) + std::to_string(uid++); }

  // trie lookups along a program's static path (the compiler registered them, compiler.cpp register_jmes)
  uint32_t tchild(uint32_t t, uint32_t key) const {
    if (t == NONE) return NONE;
    for (auto& kv : rs.trie[t].kids) if (kv.first == key) return kv.second;
    return NONE;
  }
  uint32_t tstar(uint32_t t) const { return t == NONE ? NONE : rs.trie[t].star; }
  uint32_t tcol(uint32_t t) const { return t == NONE ? NONE : rs.trie[t].col; }
  uint32_t tlen(uint32_t t) const { return t == NONE || rs.trie[t].star == NONE ? NONE : rs.trie[t].lencol; }

  struct V {  // a value in generated code: variable names + static trie position
    std::string i, t, a, row;
    uint32_t tpos;
    bool key;   // a map key (JMES_KEYBIT element)
  };
  // declare a fresh value
  V decl(const std::string& i, const std::string& t, const std::string& a, const std::string& row, uint32_t tpos,
         bool key) {
    V x{fresh("vi"), fresh("vt"), fresh("va"), fresh("vr"), tpos, key};
    out << "  uint32_t " << x.i << " = " << i << ", " << x.t << " = " << t << ", " << x.a << " = " << a << ", " << x.row
        << " = " << row << ";\n";
    return x;
  }
  V field(const V& x, uint32_t key) {
    if (x.key) return decl("NONE", "T_UNK", "0u", "NONE", NONE, false);
    const uint32_t ct = tchild(x.tpos, key), col = tcol(ct);
    V y{fresh("vi"), fresh("vt"), fresh("va"), fresh("vr"), col == NONE ? NONE : ct, false};
    out << "  uint32_t " << y.i << ", " << y.t << ", " << y.a << ";\n"
        << "  jc_field(v, R, " << x.i << ", " << x.row << ", " << (col == NONE ? "NONE" : u(col)) << ", " << u(key) << ", &"
        << y.i << ", &" << y.t << ", &" << y.a << ");\n"
        << "  const uint32_t " << y.row << " = " << (col == NONE ? std::string("NONE") : x.row) << ";\n";
    return y;
  }
  // loop over the elements of array value x (when it is one): opens `if (arr) { for (j) {` and returns the element;
  // the caller emits the body, then close_loop()
  bool unroll = false;  // operand programs: element loops unrolled so that the loads of consecutive elements overlap
  V open_elems(const V& x, const std::string& notarr_then, const char* on_arr = "") {
    const std::string cnt = fresh("cn"), aa = fresh("aa"), eb = fresh("eb"), j = fresh("j");
    const uint32_t st = tstar(x.tpos);
    out << "  { uint32_t " << cnt << " = 0u, " << aa << " = 0u, " << eb << " = NONE;\n"
        << "  if (" << (x.key ? "false" : "jc_arr(v, R, " + x.i + ", " + x.t + ", " + x.a + ", " + x.row + ", " +
                                              (tlen(x.tpos) == NONE ? std::string("NONE") : u(tlen(x.tpos))) + ", &" + cnt +
                                              ", &" + aa + ", &" + eb + ")")
        << ") {\n" << on_arr << (unroll ? "  KYV_JC_UNROLL\n" : "")
        << "  for (uint32_t " << j << " = 0; " << j << " < " << cnt << "; " << j << "++) {\n";
    V e{fresh("vi"), fresh("vt"), fresh("va"), fresh("vr"), st, false};
    out << "  uint32_t " << e.i << ", " << e.t << ", " << e.a << ", " << e.row << ";\n"
        << "  jc_elem(v, R, " << aa << ", " << (st == NONE ? std::string("NONE") : eb) << ", " << j << ", "
        << (tcol(st) == NONE ? std::string("NONE") : u(tcol(st))) << ", &" << e.i << ", &" << e.t << ", &" << e.a << ", &"
        << e.row << ");\n";
    pending_else.push_back(notarr_then);
    return e;
  }
  std::vector<std::string> pending_else;
  void close_loop() {
    out << "  }\n  }";
    std::string e = pending_else.back();
    pending_else.pop_back();
    if (!e.empty()) out << " else {\n" << e << "  }";
    out << "\n  }\n";
  }

  // ---- JMESPath operand programs, materialising mode (condition operands): results into (*lst, *cur, L/*ln)
  // gen(pos, x, list, proj): ops [pos, end) applied to value x in single (list=false) or list mode
  const uint32_t* P = nullptr;
  uint32_t PN = 0, PEND = 0;
  // streaming mode (condition-set operands, stream_fn): list elements are not materialised; each element's
  // fmt.Sprint sid goes through `sacc` (the condition's per-element test) and only the count is kept
  bool streaming = false;
  std::string sacc;
  void jend(const V& x, bool list, bool proj) {
    if (!list) {
      out << "  *cur = " << (x.key ? "(" + x.i + " | JMES_KEYBIT)" : x.i) << ";\n";
      return;
    }
    if (streaming) {
      std::string sx;
      if (x.key) sx = "(gtk(R + " + x.i + ") >> 4)";
      else sx = "jc_sprint(R, " + x.i + ", " + x.t + ", " + x.a + ")";
      const std::string body = "{ const uint32_t es = " + sx + ";\n    if (++*ln > JCAP) return JS_FB;\n    " + sacc + " }";
      if (x.key) out << "  " << body << "\n";
      else if (proj) out << "  if (" << x.i << " != NONE) " << body << "\n";
      else out << "  " << body << "\n";
      return;
    }
    const std::string e = x.key ? "jc_keyent(R, " + x.i + ")" : "jc_ent(" + x.i + ", " + x.t + ", " + x.a + ")";
    if (x.key) out << "  if (!jc_push(L, ln, " << e << ")) return JS_FB;\n";
    else if (proj) out << "  if (" << x.i << " != NONE) { if (!jc_push(L, ln, " << e << ")) return JS_FB; }\n";
    else out << "  if (!jc_push(L, ln, " << x.i << " == NONE ? NONE : " << e << ")) return JS_FB;\n";
  }
  void jgen(uint32_t pos, const V& x, bool list, bool proj, int guard) {
    if (!ok || guard > 64) { ok = false; return; }
    if (pos >= PEND) { jend(x, list, proj); return; }
    const uint32_t op = P[pos];
    switch (op) {
      case JO_FIELD: {
        out << "  {\n";
        V y = field(x, P[pos + 1]);
        jgen(pos + 2, y, list, proj, guard + 1);
        out << "  }\n";
        return;
      }
      case JO_MULTI: {
        if (list) { ok = false; return; }  // the interpreter reads a stale single value here: not generated
        const uint32_t m = P[pos + 1];
        out << "  if (" << x.i << " == NONE) {\n";
        jgen(pos + 2 + m, x, false, proj, guard + 1);
        out << "  } else {\n  *lst = true;\n";
        for (uint32_t o = 0; o < m; o++) {
          out << "  {\n";
          V y = field(x, P[pos + 2 + o]);
          jgen(pos + 2 + m, y, true, proj, guard + 1);
          out << "  }\n";
        }
        out << "  }\n";
        return;
      }
      case JO_FLAT: {
        if (!list) {
          // flatten of a non-list: null single result, projection ends
          std::ostringstream save;
          save.swap(out);
          V nul{"NONE", "T_UNK", "0u", "NONE", NONE, false};
          jgen(pos + 1, nul, false, false, guard + 1);
          std::string notarr = out.str();
          out.swap(save);
          V e = open_elems(x, notarr, "  *lst = true;\n");
          jgen(pos + 1, e, true, true, guard + 1);
          close_loop();
          return;
        }
        // flatten inside a projection: nulls dropped first (when projecting), arrays spliced one level, other
        // elements kept
        out << "  if (" << (proj && !x.key ? x.i + " != NONE" : std::string("true")) << ") {\n";
        std::ostringstream save;
        save.swap(out);
        V pass{x.i, x.t, x.a, "NONE", NONE, x.key};
        jgen(pos + 1, pass, true, true, guard + 1);
        std::string notarr = out.str();
        out.swap(save);
        V e = open_elems(x, notarr);
        jgen(pos + 1, e, true, true, guard + 1);
        close_loop();
        out << "  }\n";
        return;
      }
      case JO_KEYS: {
        if (list) { ok = false; return; }
        const std::string m = fresh("mn"), j = fresh("j");
        out << "  if (" << (x.key ? std::string("true") : x.i + " == NONE || jc_type(R, " + x.i + ", " + x.t + ") != N_MAP")
            << ") return JS_FB;\n"
            << "  { const Node " << m << " = gnode(R + " << x.i << ");\n  *lst = true;\n"
            << "  for (uint32_t " << j << " = 0; " << j << " < " << m << ".b; " << j << "++) {\n";
        V k = decl(m + ".a + " + j, "T_UNK", "0u", "NONE", NONE, true);
        jgen(pos + 1, k, true, proj, guard + 1);
        out << "  }\n  }\n";
        return;
      }
      case JO_KEYS_FLAT: {
        if (!list) { jgen(pos + 1, x, false, proj, guard + 1); return; }
        const std::string m = fresh("mn"), j = fresh("j");
        out << "  if (" << (x.key ? std::string("true") : x.i + " == NONE || jc_type(R, " + x.i + ", " + x.t + ") != N_MAP")
            << ") return JS_FB;\n"
            << "  { const Node " << m << " = gnode(R + " << x.i << ");\n"
            << "  KYV_JC_UNROLL\n"
            << "  for (uint32_t " << j << " = 0; " << j << " < " << m << ".b; " << j << "++) {\n";
        V k = decl(m + ".a + " + j, "T_UNK", "0u", "NONE", NONE, true);
        jgen(pos + 1, k, true, true, guard + 1);
        out << "  }\n  }\n";
        return;
      }
      default: ok = false; return;
    }
  }
  // operand function: int joN(v, R, r, element value, L, &lst, &cur, &ln, &lit) -> JS_OK / JS_FB / JS_NOTFOUND
  std::string operand_fn(const CondOperand& o, uint32_t etpos) {
    const uint32_t* p = rs.pool.data() + o.a;
    const uint32_t n = o.nseg, root = p[0] & 0xFFu;
    const bool pure = (p[0] & JF_PURE) != 0;
    const std::string name = fresh("jo");
    const uint32_t* saveP = P;  // operand functions are generated from inside a foreach list's generation
    const uint32_t savePEND = PEND;
    std::ostringstream save;
    save.swap(out);
    out << "static __device__ __forceinline__ int " << name
        << "(const View& v, const Node* R, uint32_t r, uint32_t ei, uint32_t et, uint32_t ea, uint32_t erow, uint32_t* L, "
           "bool* lst, uint32_t* cur, uint32_t* ln, uint32_t* lit) {\n"
           "  *lst = false; *cur = NONE; *ln = 0u; *lit = NONE;\n";
    uint32_t i = 1, orlit = NONE;
    if (root == JR_OPERATION) {
      // request.operation: the literal the compiler put in the program ("CREATE" in a background scan)
      uint32_t lit = p[1];
      if (n > 2 && p[2] == JO_OR) {
        const Node& c = rs.cnodes[lit];
        bool f = node_type(c) == N_NULL || node_type(c) == N_FALSE || (node_type(c) == N_STR && c.a == SID_EMPTY) ||
                 ((node_type(c) == N_ARR || node_type(c) == N_MAP) && c.b == 0);
        if (f) lit = p[3];
      } else if (n > 2) {
        ok = false;
      }
      out << "  *lit = " << u(lit) << ";\n  return JS_OK;\n}\n";
    } else if (pure) {
      // plain field chain: a key missing from a map is a NotFoundError (the fork's rule), else as j_field
      out << "  uint32_t c = " << (root == JR_OBJECT ? "0u" : "ei") << ", f = 0u;\n";
      for (; i + 1 < n; i += 2) {
        if (p[i] != JO_FIELD) { ok = false; break; }
        out << "  if (c != NONE) {\n"
               "    const Node m = gnode(R + c);\n"
               "    if (node_type(m) != N_MAP) c = NONE;\n"
               "    else { const uint32_t x = wmap_find(R, m.a, m.b, " << u(p[i + 1]) << ");\n"
               "      if (x == NONE) { *lit = f; return JS_NOTFOUND; }\n"
               "      c = (gtk(R + x) & 0xFu) == N_NULL ? NONE : x; }\n"
               "  }\n  f++;\n";
      }
      out << "  *cur = c;\n  return JS_OK;\n}\n";
    } else {
      V x = root == JR_OBJECT ? decl("0u", "T_UNK", "0u", "r", 0u, false) : decl("ei", "et", "ea", "erow", etpos, false);
      PEND = n;
      for (uint32_t q = 1; q < n;) {  // a trailing `|| lit` ends the ops
        if (p[q] == JO_OR) { PEND = q; orlit = p[q + 1]; if (q + 2 < n) ok = false; break; }
        if (p[q] == JO_UPPER || p[q] == JO_REGEX) ok = false;
        q += jop_width(p + q);
      }
      P = p;
      const bool su = unroll;
      unroll = true;
      jgen(1, x, false, false, 0);
      unroll = su;
      if (orlit != NONE)
        out << "  if (*lst ? *ln == 0u : jc_false1(R, *cur)) { *lst = false; *cur = NONE; *lit = " << u(orlit) << "; }\n";
      out << "  return JS_OK;\n}\n";
    }
    std::string fn = out.str();
    out.swap(save);
    defs << fn;
    P = saveP;
    PEND = savePEND;
    return name;
  }
  // Streaming operand function of a condition-set condition (compiler.cpp assign_cond_sets): the same program as
  // operand_fn, but list elements only update the caller's accumulators through `acc` (shape A: *sf = 1 on an element
  // without fmt.Sprint form, else *sm counts the elements in the set; shape B: the first element that is unrenderable
  // (*sf = 2) or in the set (*sf = 1) decides, as key_exists' ordered loop does). Single (non-list) results and the
  // `|| literal` come back as operand_fn returns them.
  //   int jsN(v, R, r, element value, &lst, &cur, &ln, &lit, &sm, &sf) -> JS_OK / JS_FB / JS_NOTFOUND
  std::string stream_fn(const CondOperand& o, uint32_t etpos, const std::string& acc) {
    const uint32_t* p = rs.pool.data() + o.a;
    const uint32_t n = o.nseg, root = p[0] & 0xFFu;
    if (root == JR_OPERATION || (p[0] & JF_PURE) || jmes_chain_form(p, n)) return "";  // never a list
    const std::string name = fresh("js");
    const uint32_t* saveP = P;
    const uint32_t savePEND = PEND;
    std::ostringstream save;
    save.swap(out);
    out << "static __device__ __forceinline__ int " << name
        << "(const View& v, const Node* R, uint32_t r, uint32_t ei, uint32_t et, uint32_t ea, uint32_t erow, "
           "bool* lst, uint32_t* cur, uint32_t* ln, uint32_t* lit, uint32_t* sm, uint32_t* sf) {\n"
           "  *lst = false; *cur = NONE; *ln = 0u; *lit = NONE; (void)sm; (void)sf;\n";
    V x = root == JR_OBJECT ? decl("0u", "T_UNK", "0u", "r", 0u, false) : decl("ei", "et", "ea", "erow", etpos, false);
    uint32_t orlit = NONE;
    PEND = n;
    for (uint32_t q = 1; q < n;) {
      if (p[q] == JO_OR) { PEND = q; orlit = p[q + 1]; break; }
      q += jop_width(p + q);
    }
    P = p;
    const bool su = unroll, ss = streaming;
    const std::string sa = sacc;
    unroll = true;
    streaming = true;
    sacc = acc;
    jgen(1, x, false, false, 0);
    unroll = su;
    streaming = ss;
    sacc = sa;
    if (orlit != NONE)
      out << "  if (*lst ? *ln == 0u : jc_false1(R, *cur)) { *lst = false; *cur = NONE; *lit = " << u(orlit) << "; }\n";
    out << "  return JS_OK;\n}\n";
    std::string fn = out.str();
    out.swap(save);
    P = saveP;
    PEND = savePEND;
    if (!ok) return "";
    defs << fn;
    return name;
  }
  // the set of a condition-set condition as a device constant (the mask-less fallback of jc_inset)
  std::unordered_map<uint32_t, std::string> set_names;
  std::string set_array(uint32_t q) {
    auto it = set_names.find(q);
    if (it != set_names.end()) return it->second;
    std::string nm = "kyv_cset" + std::to_string(q);
    defs << "__device__ const uint32_t " << nm << "[" << rs.gsets[q].size() << "] = {";
    for (size_t i = 0; i < rs.gsets[q].size(); i++) defs << (i ? ", " : "") << rs.gsets[q][i] << "u";
    defs << "};\n";
    set_names[q] = nm;
    return nm;
  }
  // a single-condition program whose condition has a set (compiler.cpp assign_cond_sets): the list side streamed
  // (stream_fn), decided from the accumulators when it is a list, else by the operator on the single value / literal
  bool stream_cond(uint32_t ci, const std::string& K, const std::string& X) {
    if (ci >= rs.cond_set.size() || !rs.cond_set[ci] || getenv("KYV_JIT_NOSTREAM")) return false;
    const Cond& c = rs.conds[ci];
    const uint32_t q = rs.cond_set[ci] - 1;
    const uint32_t bit = (uint32_t)rs.gpats.size() + q;
    const bool shapeA = c.key.kind == OK_JMES && c.value.kind == OK_LIT;
    const CondOperand& lo = shapeA ? c.key : c.value;  // the resource-side (listy) operand
    const std::string S = set_array(q);
    const std::string test = "jc_inset(v, " + u(bit) + ", " + S + ", " + u((uint32_t)rs.gsets[q].size()) + ", es)";
    const std::string acc = shapeA ? "if (es == NONE) *sf = 1u; else if (" + test + ") (*sm)++;"
                                   : "if (!*sf) { if (es == NONE) *sf = 2u; else if (" + test + ") *sf = 1u; }";
    const std::string f = stream_fn(lo, cur_etpos, acc);
    if (f.empty()) return false;
    const std::string l = fresh("jl"), cc = fresh("jc"), n = fresh("jn"), t = fresh("jt"), s = fresh("js"), m = fresh("sm"),
                      fb = fresh("sf");
    out << "  bool " << l << "; uint32_t " << cc << ", " << n << ", " << t << ", " << m << " = 0u, " << fb << " = 0u;\n"
        << "  const int " << s << " = " << f << "(v, R, r, ei, et, ea, erow, &" << l << ", &" << cc << ", &" << n << ", &" << t
        << ", &" << m << ", &" << fb << ");\n"
        << "  if (" << s << " == JS_FB) return CR_FB;\n  if (" << s << " == JS_NOTFOUND) return CP_ERROR;\n"
        << "  if (" << l << ") {\n";
    if (shapeA) {
      std::string dec;
      switch (c.op) {
        case CO_ANYIN: dec = m + " > 0u"; break;
        case CO_ANYNOTIN: dec = m + " < " + n; break;
        case CO_ALLIN: dec = m + " == " + n; break;
        default: dec = m + " == 0u"; break;  // CO_ALLNOTIN
      }
      out << "    rc = " << fb << " ? CR_FB : (" << dec << ") ? CR_TRUE : CR_FALSE;\n";
    } else {
      const bool neg = c.op == CO_NOTIN || c.op == CO_ANYNOTIN || c.op == CO_ALLNOTIN;
      out << "    rc = " << fb << " == 2u ? CR_FB : ((" << fb << " == 1u) != " << (neg ? "true" : "false")
          << ") ? CR_TRUE : CR_FALSE;\n";
    }
    out << "  } else {\n";
    const std::string one = "jc_cv(v, R, false, " + cc + ", " + t + ", nullptr, 0u)";
    if (shapeA) out << "    const CV " << K << " = " << one << ";\n    const CV " << X << " = jc_lit(v, " << u(c.value.a) << ");\n";
    else out << "    const CV " << K << " = jc_lit(v, " << u(c.key.a) << ");\n    const CV " << X << " = " << one << ";\n";
    out << "    rc = " << cond_call(ci, K, X) << ";\n  }\n";
    return true;
  }

  // an operand that cannot fail (no NotFoundError, no list overflow / keys() error)
  bool infallible(const CondOperand& o) const {
    if (o.kind == OK_LIT || o.kind == OK_NIL) return true;
    if (o.kind == OK_PATH) return false;
    const uint32_t* p = rs.pool.data() + o.a;
    const uint32_t root = p[0] & 0xFFu;
    if (root == JR_OPERATION) return true;
    if (p[0] & JF_PURE) return false;
    for (uint32_t q = 1; q < o.nseg;) {
      if (p[q] == JO_OR) return q + 2 >= o.nseg;  // a function applied after the default can fail
      if (p[q] != JO_FIELD) return false;
      q += 2;
    }
    return true;
  }
  static bool listy(const Ruleset& rs, const CondOperand& o) {
    if (o.kind != OK_JMES) return false;
    const uint32_t* p = rs.pool.data() + o.a;
    for (uint32_t q = 1; q < o.nseg;) {
      if (p[q] == JO_MULTI || p[q] == JO_FLAT || p[q] == JO_KEYS || p[q] == JO_KEYS_FLAT || p[q] == JO_FILTER) return true;
      if (p[q] == JO_OR) return false;
      q += jop_width(p + q);
    }
    return false;
  }
  // code computing CV `cv` of operand o (slot: LDS list of the lane); `check`: return the program status on a
  // NotFoundError / fallback (fused single-condition programs)
  void operand_cv(const CondOperand& o, uint32_t ci, int side, uint32_t etpos, const std::string& cv, const std::string& slot,
                  bool check) {
    const std::string C = "v.conds[" + u(ci) + "]." + (side ? "value" : "key");
    switch (o.kind) {
      case OK_LIT: out << "  const CV " << cv << " = jc_lit(v, " << u(o.a) << ");\n"; return;
      case OK_PATH: {
        const std::string m = fresh("ms");
        out << "  CV " << cv << "; uint32_t " << m << ";\n"
            << "  " << (check ? "if (!" : "(void)(") << "cv_operand(v, NodeTab{R}, " << C << ", &" << cv << ", &" << m << ", r)"
            << (check ? ") return CP_ERROR;\n" : ");\n");
        return;
      }
      case OK_JMES: {
        if (jmes_chain_form(rs.pool.data() + o.a, o.nseg)) {  // the light kernels' evaluator (kyv_cond.h jmes_chain_cv)
          const std::string m = fresh("ms"), s = fresh("js");
          out << "  CV " << cv << "; uint32_t " << m << ";\n"
              << "  const int " << s << " = jmes_chain_cv(v, NodeTab{R}, " << C << ", &" << cv << ", &" << m << ", r);\n";
          if (check) out << "  if (" << s << " == JS_FB) return CR_FB;\n  if (" << s << " != JS_OK) return CP_ERROR;\n";
          else out << "  (void)" << s << ";\n";
          return;
        }
        lds_used = true;
        const std::string f = operand_fn(o, etpos);
        const std::string l = fresh("jl"), c = fresh("jc"), n = fresh("jn"), t = fresh("jt"), s = fresh("js");
        out << "  bool " << l << "; uint32_t " << c << ", " << n << ", " << t << ";\n"
            << "  const int " << s << " = " << f << "(v, R, r, ei, et, ea, erow, " << slot << ", &" << l << ", &" << c
            << ", &" << n << ", &" << t << ");\n";
        if (check) out << "  if (" << s << " == JS_FB) return CR_FB;\n  if (" << s << " == JS_NOTFOUND) return CP_ERROR;\n";
        else out << "  (void)" << s << ";\n";
        out << "  const CV " << cv << " = jc_cv(v, R, " << l << ", " << c << ", " << t << ", " << slot << ", " << n << ");\n";
        return;
      }
      default: out << "  const CV " << cv << " = cv_node(Node{N_NULL, 0, 0, 0}, false);\n"; return;
    }
  }
  // eval_cond of condition ci with the condition folded in as a constant: the operator is called directly and
  // the value operand's literal flags (SV_*) are known, so only the branches this condition can take are compiled
  static std::string opnd_init(const CondOperand& o) {
    return "{" + std::to_string(o.kind) + ", " + std::to_string(o.sv) + ", " + std::to_string(o.nseg) + ", " + u(o.a) +
           ", " + u(o.list) + ", " + u(o.nlist) + "}";
  }
  std::string cond_call(uint32_t ci, const std::string& K, const std::string& X) {
    const Cond& c = rs.conds[ci];
    const std::string C = "Cond{" + std::to_string(c.op) + ", {0, 0, 0}, " + u(c.leaf) + ", " + u(c.leaf_neg) + ", 0u, " +
                          opnd_init(c.key) + ", " + opnd_init(c.value) + "}";
    const std::string a = "v, NodeTab{R}, " + C + ", " + K + ", " + X;
    switch (c.op) {
      case CO_EQ: return "op_equal(v, NodeTab{R}, " + K + ", " + X + ", false)";
      case CO_NE: return "op_equal(v, NodeTab{R}, " + K + ", " + X + ", true)";
      case CO_IN: return "op_in(" + a + ", false)";
      case CO_NOTIN: return "op_in(" + a + ", true)";
      case CO_ANYIN: return "op_any_all(" + a + ", false, false)";
      case CO_ALLIN: return "op_any_all(" + a + ", true, false)";
      case CO_ANYNOTIN: return "op_any_all(" + a + ", false, true)";
      case CO_ALLNOTIN: return "op_any_all(" + a + ", true, true)";
      case CO_GT: case CO_GE: case CO_LT: case CO_LE:
        return "op_numeric(v, " + K + ", " + X + ", " + std::to_string(c.op) + ")";
      case CO_DGT: case CO_DGE: case CO_DLT: case CO_DLE:
        return "op_duration(v, " + K + ", " + X + ", " + std::to_string(c.op) + ")";
      default: return "CR_FALSE";
    }
  }
  // program function (eval_prog): int jpN(v, R, r, element value, L) -> CR_* / CP_ERROR
  std::string prog_fn(uint32_t prog, uint32_t etpos) {
    const uint64_t key = ((uint64_t)prog << 32) | etpos;
    auto it = progs.find(key);
    if (it != progs.end()) return it->second;
    const CondProg& p = rs.cprogs[prog];
    const uint32_t nany = p.nany == NONE ? 0u : p.nany;
    std::vector<uint32_t> cis;
    for (uint32_t i = 0; i < nany; i++) cis.push_back(p.any0 + i);
    for (uint32_t i = 0; i < p.nall; i++) cis.push_back(p.all0 + i);
    for (uint32_t ci : cis)
      if (listy(rs, rs.conds[ci].key) && listy(rs, rs.conds[ci].value)) nslots = 2;
    const std::string name = fresh("jp");
    std::ostringstream save;
    save.swap(out);  // the program body is generated into a fresh `out`; operand functions go to `defs`
    const bool fused = cis.size() == 1;
    auto cond_code = [&](uint32_t ci, bool check) {
      const Cond& c = rs.conds[ci];
      const bool two = listy(rs, c.key) && listy(rs, c.value);
      const std::string K = fresh("k"), X = fresh("x");
      if (check && !two) {
        cur_etpos = etpos;
        const std::string mark = out.str();
        if (stream_cond(ci, K, X)) return;
        out.str(""); out.clear(); out << mark;  // stream_fn bailed out: nothing of it stays in the body
      }
      operand_cv(c.key, ci, 0, etpos, K, "L", check);
      operand_cv(c.value, ci, 1, etpos, X, two ? "(L + JCAP * 64)" : "L", check);
      out << "  rc = " << cond_call(ci, K, X) << ";\n";
    };
    out << "  int rc = CR_TRUE;\n  (void)rc;\n";
    if (!fused) {
      // every reference of the document is substituted before any condition runs (vars.go:352-431)
      for (uint32_t ci : cis) {
        const Cond& c = rs.conds[ci];
        for (int side = 0; side < 2; side++) {
          const CondOperand& o = side ? c.value : c.key;
          if (infallible(o)) continue;
          out << "  {\n";
          operand_cv(o, ci, side, etpos, fresh("pc"), "L", true);
          out << "  }\n";
        }
      }
    }
    if (p.nany != NONE) {
      out << "  { bool any = false;\n  do {\n";
      for (uint32_t i = 0; i < nany; i++) {
        out << "  {\n";
        cond_code(p.any0 + i, fused);
        out << "  if (rc == CR_FB || rc == CR_PANIC) return rc;\n  if (rc == CR_TRUE) { any = true; break; }\n  }\n";
      }
      out << "  } while (0);\n  if (!any) return CR_FALSE; }\n";
    }
    for (uint32_t i = 0; i < p.nall; i++) {
      out << "  {\n";
      cond_code(p.all0 + i, fused);
      out << "  if (rc == CR_FB || rc == CR_PANIC) return rc;\n  if (rc == CR_FALSE) return CR_FALSE;\n  }\n";
    }
    out << "  return CR_TRUE;\n";
    const std::string b = out.str();
    out.swap(save);
    defs << "static __device__ __forceinline__ int " << name
         << "(const View& v, const Node* R, uint32_t r, uint32_t ei, uint32_t et, uint32_t ea, uint32_t erow, uint32_t* L) {\n"
         << "  (void)ei; (void)et; (void)ea; (void)erow;\n"
         << b << "}\n";
    progs[key] = name;
    return name;
  }

  // ---- foreach (eval_foreach, kyv_pss.h; validation.go:319-421): the entry's list streamed, each element's
  // preconditions / deny run in place. `pend`: the element just processed ended in an error (it is the rule's error
  // only when no element follows it: "an error ends the rule only on the last element").
  const ForeachEntry* FE = nullptr;
  void elem_body(const V& e) {
    out << "  do {\n";
    if (FE->scope == 2) out << "  if (jc_type(R, " << e.i << ", " << e.t << ") != N_MAP) return ST_ERROR | ST_MARK_SCOPE;\n";
    out << "  bool err = false;\n";
    const std::string args = "(v, R, r, " + e.i + ", " + e.t + ", " + e.a + ", " + e.row + ", L)";
    if (FE->pre != NONE) {
      const std::string f = prog_fn(FE->pre, e.tpos);
      out << "  { const int c = " << f << args << ";\n"
          << "    if (c == CR_FB) return ST_FALLBACK;\n    if (c == CR_PANIC) return ST_PANIC;\n"
          << "    if (c == CR_FALSE) break;\n    err = c == CP_ERROR; }\n";
    }
    const std::string f = prog_fn(FE->deny, e.tpos);
    out << "  if (!err) { const int c = " << f << args << ";\n"
        << "    if (c == CR_FB) return ST_FALLBACK;\n    if (c == CR_PANIC) return ST_PANIC;\n"
        << "    if (c == CR_TRUE) return ST_FAIL;\n    if (c != CP_ERROR) { count++; break; } }\n"
        << "  pend = true;\n  } while (0);\n";
  }
  // end of the list program: the elements
  void fend(const V& x, bool list, bool proj) {
    if (x.key) { ok = false; return; }
    if (list) {
      if (proj) {  // a projection's null results are not elements
        out << "  if (" << x.i << " != NONE) {\n  pend = false;\n";
        elem_body(x);
        out << "  }\n";
      } else {     // kept nulls are elements, skipped
        out << "  pend = false;\n  if (" << x.i << " != NONE) {\n";
        elem_body(x);
        out << "  }\n";
      }
      return;
    }
    // a single result: an array's items (null items are elements, skipped) or the value itself
    std::ostringstream save;
    save.swap(out);
    out << "  pend = false;\n  if (" << (x.i == "NONE" ? std::string("false") : x.i + " != NONE && jc_type(R, " + x.i + ", " + x.t + ") != N_NULL")
        << ") {\n";
    elem_body(x);
    out << "  }\n";
    const std::string single = out.str();
    out.swap(save);
    V e = open_elems(x, single);
    out << "  pend = false;\n  if (" << e.i << " != NONE) {\n";
    elem_body(e);
    out << "  }\n";
    close_loop();
  }
  void fgen(uint32_t pos, const V& x, bool list, bool proj, int guard) {
    if (!ok || guard > 64) { ok = false; return; }
    if (pos >= PEND) { fend(x, list, proj); return; }
    const uint32_t op = P[pos];
    switch (op) {
      case JO_FIELD: {
        out << "  {\n";
        V y = field(x, P[pos + 1]);
        fgen(pos + 2, y, list, proj, guard + 1);
        out << "  }\n";
        return;
      }
      case JO_MULTI: {
        if (list) { ok = false; return; }
        const uint32_t m = P[pos + 1];
        out << "  if (" << x.i << " == NONE) {\n";
        fgen(pos + 2 + m, x, false, proj, guard + 1);
        out << "  } else {\n";
        for (uint32_t o = 0; o < m; o++) {
          out << "  {\n";
          V y = field(x, P[pos + 2 + o]);
          fgen(pos + 2 + m, y, true, proj, guard + 1);
          out << "  }\n";
        }
        out << "  }\n";
        return;
      }
      case JO_FLAT: {
        std::ostringstream save;
        save.swap(out);
        if (!list) {
          V nul{"NONE", "T_UNK", "0u", "NONE", NONE, false};
          fgen(pos + 1, nul, false, false, guard + 1);
        } else {
          V pass{x.i, x.t, x.a, "NONE", NONE, x.key};
          fgen(pos + 1, pass, true, true, guard + 1);
        }
        const std::string notarr = out.str();
        out.swap(save);
        if (list) out << "  if (" << (proj ? x.i + " != NONE" : std::string("true")) << ") {\n";
        V e = open_elems(x, notarr);
        fgen(pos + 1, e, true, true, guard + 1);
        close_loop();
        if (list) out << "  }\n";
        return;
      }
      default: ok = false; return;  // keys() / `||` lists stay on the interpreter
    }
  }
  void foreach_entry(const ForeachEntry& fe) {
    FE = &fe;
    out << "  { uint32_t count = 0u; bool pend = false; bool skip = false; (void)skip;\n";
    const CondOperand& o = fe.list;
    const uint32_t* p = o.kind == OK_JMES ? rs.pool.data() + o.a : nullptr;
    const bool chain = o.kind == OK_PATH || (p && (p[0] & JF_PURE));
    if (chain) {
      // plain path: a key missing from a map skips the entry ("failed to evaluate list")
      const uint32_t root = p ? (p[0] & 0xFFu) : JR_OBJECT;
      if (root != JR_OBJECT) { ok = false; return; }
      const uint32_t nseg = p ? 0u : o.nseg;
      std::vector<uint32_t> keys;
      if (p) { for (uint32_t q = 1; q + 1 < o.nseg; q += 2) { if (p[q] != JO_FIELD) { ok = false; return; } keys.push_back(p[q + 1]); } }
      else for (uint32_t s = 0; s < nseg; s++) keys.push_back(rs.pool[o.a + s]);
      out << "  uint32_t lc = 0u;\n";
      for (uint32_t key : keys)
        out << "  if (lc != NONE) { const Node m = gnode(R + lc);\n"
               "    if (node_type(m) != N_MAP) lc = NONE;\n"
               "    else { const uint32_t x = wmap_find(R, m.a, m.b, " << u(key) << ");\n"
               "      if (x == NONE) { skip = true; lc = NONE; } else lc = (gtk(R + x) & 0xFu) == N_NULL ? NONE : x; } }\n";
      out << "  if (!skip) {\n";
      V x = decl("lc", "T_UNK", "0u", "NONE", NONE, false);
      fend(x, false, false);
      out << "  }\n";
    } else if (p) {
      const uint32_t root = p[0] & 0xFFu;
      if (root != JR_OBJECT) { ok = false; return; }
      PEND = o.nseg;
      for (uint32_t q = 1; q < o.nseg;) {
        if (p[q] == JO_OR || p[q] == JO_KEYS || p[q] == JO_KEYS_FLAT || p[q] == JO_FILTER) { ok = false; return; }
        q += jop_width(p + q);
      }
      P = p;
      V x = decl("0u", "T_UNK", "0u", "r", 0u, false);
      fgen(1, x, false, false, 0);
    } else {
      ok = false;
      return;
    }
    out << "  if (pend) return ST_ERROR;\n  applied += count; }\n";
  }

  // the rule's match block is decided by the resource kind alone (mark_gate_exact's conditions, compiler.cpp,
  // without the precondition clause, which only matters for the walk's direct schedule): the kernel's kind gate
  // is the whole match
  bool kind_only(const RuleDesc& rd) const {
    if (rd.empty_may_match || rd.exclude.mode != MM_NONE || rd.exc != NONE) return false;
    const MatchBlock& m = rd.match;
    if (m.mode == MM_NONE || m.nfilters == 0 || (m.mode != MM_ANY && m.nfilters != 1)) return false;
    for (uint32_t i = 0; i < m.nfilters; i++) {
      const Filter& f = rs.filters[m.filters + i];
      if (f.nkinds == 0 || f.name != NONE || f.nnames || f.nnss || f.nann ||
          (f.flags & (FF_HAS_SEL | FF_HAS_NSSEL | FF_ZERO_RD | FF_USERINFO)))
        return false;
      for (uint32_t j = 0; j < f.nkinds; j++) {
        const KindDesc& kd = rs.kinds[f.kinds + j];
        if (kd.kind != NONE && kd.gv_mode != 0) return false;
      }
    }
    return true;
  }
  // one rule: uint8_t jr<k>(v, r, L) -> the pair's status (pair_dispatch for deny / foreach rules)
  void rule_fn(uint32_t k) {
    const RuleDesc& rd = rs.rules[k];
    std::ostringstream save;
    save.swap(out);
    if (kind_only(rd)) out << "  // match block = the kind gate (checked by the kernel)\n";
    else out << "  { const int m = jc_match(v, r, " << u(k) << "); if (m >= 0) return (uint8_t)m; }\n";
    out << "#ifdef KYV_EXP_JC_EMPTY\n  return ST_PASS;\n#endif\n";
    out << "  const ResHeader& h = v.hdr[r];\n"
        << "  KYV_ACCT_ADD(0, 8);  // header: node count, root\n"
        << "  if (h.nnodes >= (1u << COL_TYPE_SHIFT)) return ST_FALLBACK;  // no path columns for this resource\n"
        << "  const Node* R = v.nodes + h.root;\n"
        << "  const uint32_t ei = NONE, et = T_UNK, ea = 0u, erow = NONE;\n";
    const std::string args = "(v, R, r, ei, et, ea, erow, L)";
    if (rd.pre != NONE) {
      const std::string f = prog_fn(rd.pre, NONE);
      out << "  { const int c = " << f << args << ";\n"
          << "    if (c == CR_FB) return ST_FALLBACK;\n    if (c == CR_PANIC) return ST_PANIC;\n"
          << "    if (c == CP_ERROR) return ST_ERROR | ST_MARK_PRE;\n    if (c == CR_FALSE) return ST_SKIP | ST_MARK_PRE; }\n";
    }
    if (rd.kind == RK_DENY) {
      const std::string f = prog_fn(rd.root, NONE);
      out << "  { const int c = " << f << args << ";\n"
          << "    if (c == CR_FB) return ST_FALLBACK;\n    if (c == CR_PANIC) return ST_PANIC;\n"
          << "    if (c == CP_ERROR) return ST_ERROR;\n    return c == CR_TRUE ? ST_FAIL : ST_PASS; }\n";
    } else if (rd.kind == RK_FOREACH) {
      const uint32_t nent = rs.pool[rd.root];
      std::vector<ForeachEntry> ents(nent);
      bool deny_only = true;
      for (uint32_t e = 0; e < nent; e++) {
        memcpy(&ents[e], rs.pool.data() + rd.root + 1 + e * (sizeof(ForeachEntry) / 4), sizeof(ForeachEntry));
        deny_only = deny_only && ents[e].kind == FE_DENY;
      }
      if (deny_only) {  // deny entries: streamed lists, conditions generated in place
        out << "  uint32_t applied = 0u;\n";
        for (uint32_t e = 0; e < nent && ok; e++) foreach_entry(ents[e]);
        out << "  return applied ? ST_PASS : ST_SKIP;\n";
      } else {  // pattern / anyPattern / nested entries: the evaluator's foreach (kyv_pss.h) inside this rule's kernel
        out << "  (void)ei; (void)et; (void)ea; (void)erow; (void)L;\n"
            << "  return eval_foreach(v, NodeTab{R}, v.rules[" << u(k) << "], r);\n";
      }
    } else {
      ok = false;
    }
    const std::string b = out.str();
    out.swap(save);
    // inlined into its rule's kernel (kyv_jit_cond_<k>): no call frame (callee-saved registers in scratch memory)
    defs << "static __device__ __forceinline__ uint8_t jr" << k << "(const View& v, uint32_t r, uint32_t* L) {\n" << b << "}\n";
  }
};

// rules the light match kernel cannot evaluate (kyv_engine.hip rule_needs_jmes): foreach, or a precondition / deny
// program with a JMESPath operand
// (chain programs -- a field chain, `|| literal`, length() / to_upper() / regex_match() -- run in the light kernels
// too: kyv_layout.h jmes_chain_form, kyv_cond.h jmes_chain_cv)
static bool heavy_jmes(const Ruleset& rs, const CondOperand& o) {
  return o.kind == OK_JMES && !jmes_chain_form(rs.pool.data() + o.a, o.nseg);
}
bool prog_has_jmes(const Ruleset& rs, uint32_t prog) {
  if (prog == NONE) return false;
  const CondProg& p = rs.cprogs[prog];
  const uint32_t nany = p.nany == NONE ? 0u : p.nany;
  for (uint32_t i = 0; i < nany; i++)
    if (heavy_jmes(rs, rs.conds[p.any0 + i].key) || heavy_jmes(rs, rs.conds[p.any0 + i].value)) return true;
  for (uint32_t i = 0; i < p.nall; i++)
    if (heavy_jmes(rs, rs.conds[p.all0 + i].key) || heavy_jmes(rs, rs.conds[p.all0 + i].value)) return true;
  return false;
}

std::string self_dir() {
  Dl_info info;
  if (dladdr((void*)&self_dir, &info) && info.dli_fname) {
    std::string p = info.dli_fname;
    size_t s = p.rfind('/');
    return s == std::string::npos ? std::string(".") : p.substr(0, s);
  }
  return ".";
}

}  // namespace

// A compiled pattern rule whose match is its kind gate (RD_GATE_EXACT: no work list, every gated lane walks) is walked by
// its group's fused kernel (kyv_jit_fused_<g>): one wave per match wave of 64 resources walks every such rule of the
// group back to back, so the wave's header / kind-gate loads and the chunk set-up are paid once per wave instead of once
// per (rule, wave) chunk. KYV_FUSED=0: every rule on the per-chunk kernels. Rulesets whose rule count exceeds the gate
// words a fused wave keeps in registers (KYV_FUSED_GW words) stay on the chunk kernels.
constexpr uint32_t kFusedGW = 8;  // = KYV_FUSED_GW of the generated source (kyv_fused.h)
bool jit_rule_fused(const Ruleset& rs, uint32_t k) {
  static const bool on = !getenv("KYV_FUSED") || atoi(getenv("KYV_FUSED")) != 0;
  if (!on || k >= rs.rules.size() || rs.rules.size() > 32u * kFusedGW) return false;
  const RuleDesc& rd = rs.rules[k];
  return (rd.kind == RK_PATTERN || rd.kind == RK_ANYPATTERN) && (rd.flags & RD_GATE_EXACT);
}

// Rules whose patterns the generator covers get a bit in `jit_rules`; the source holds their node functions,
// a root switch and the walk kernel `kyv_jit_walk`.
bool jit_shape_eligible(const Ruleset& rs, uint32_t k) {
  static const bool on = !getenv("KYV_SHAPES") || atoi(getenv("KYV_SHAPES")) != 0;
  if (!on || k >= rs.rules.size()) return false;
  const RuleDesc& rd = rs.rules[k];
  return rd.kind == RK_PATTERN && rd.pre == NONE && !(rd.flags & RD_GATE_EXACT) && !jit_rule_fused(rs, k);
}

// the content of a rule's metadata-expansion sites (what the compiled walk reads through its site base), with pool
// offsets resolved: two rules with one pattern shape and equal site contents walk identically
static std::string meta_signature(const Ruleset& rs, const RuleDesc& rd) {
  std::string o;
  if (!rd.uses_meta) return o;
  auto pool = [&](uint32_t at, uint32_t n) {
    for (uint32_t i = 0; i < 2 * n && at + i < rs.pool.size(); i++) o += std::to_string(rs.pool[at + i]) + ",";
  };
  for (uint32_t i = 0; i < rd.nmeta && rd.meta_sites + i < rs.metas.size(); i++) {
    const MetaSite& m = rs.metas[rd.meta_sites + i];
    o += "[" + std::to_string(m.has_labels) + "," + std::to_string(m.has_ann) + "," + std::to_string(m.nwild_l) + ":";
    pool(m.wild_l, m.nwild_l);
    o += std::to_string(m.nwild_a) + ":";
    pool(m.wild_a, m.nwild_a);
    o += std::to_string(m.slot_l) + "," + std::to_string(m.slot_a) + "]";
  }
  return o;
}

std::string jit_source(const Ruleset& rs, std::vector<uint8_t>* jit_rules, std::vector<uint8_t>* jit_cond,
                       std::vector<uint16_t>* jit_shape) {
  Gen g(rs);
  jit_rules->assign(rs.rules.size(), 0);
  if (jit_shape) jit_shape->assign(rs.rules.size(), 0);
  if (jit_cond) jit_cond->assign(rs.rules.size(), 0);
  // one generated function tree per pattern: rulesets with thousands of pattern rules (C4: 10k policies) would
  // give a source too large to compile in useful time; they stay on the interpreted walk kernel
  // (the cap bounds the distinct pattern shapes generated; rules beyond it stay on the interpreted walk)
  const size_t cap = getenv("KYV_JIT_MAX_RULES") ? (size_t)atol(getenv("KYV_JIT_MAX_RULES")) : 1024;
  // compiled condition rules: deny / foreach rules with JMESPath operands (the rest of the interpreted
  // match_kernel<true>'s rules); KYV_JIT_COND=0 leaves them all on the interpreter
  CondGen cg(rs);
  std::vector<uint32_t> crules;
  const bool cond_on = !getenv("KYV_JIT_COND") || atoi(getenv("KYV_JIT_COND")) != 0;
  for (size_t k = 0; k < rs.rules.size() && cond_on && crules.size() < cap; k++) {
    const RuleDesc& rd = rs.rules[k];
    if (rd.kind != RK_DENY && rd.kind != RK_FOREACH) continue;
    if (rd.kind == RK_DENY && !prog_has_jmes(rs, rd.pre) && !prog_has_jmes(rs, rd.root)) continue;
    const std::string mark = cg.defs.str();
    const auto progs = cg.progs;
    cg.ok = true;
    cg.rule_fn((uint32_t)k);
    if (!cg.ok) {  // roll back this rule's functions: it stays on the interpreted kernel
      cg.defs.str("");
      cg.defs.clear();
      cg.defs << mark;
      cg.progs = progs;
      continue;
    }
    crules.push_back((uint32_t)k);
  }
  std::vector<std::pair<uint32_t, std::vector<uint32_t>>> rule_roots;  // covered rule -> its pattern roots
  // Structurally identical patterns (same keys, handlers, leaves, path templates and columns; C4's 10k generated
  // policies use a handful) generate identical code up to pnode numbering: each root's functions are generated
  // alone, canonicalised (function names numbered by first appearance) and kept only for the first root of that
  // shape; later roots alias its root function
  std::ostringstream body;
  std::unordered_map<std::string, uint32_t> shapes;  // canonical code -> representative root
  std::unordered_map<uint32_t, uint32_t> rep_of;     // root -> representative root
  auto canon = [](const std::string& t) {
    std::unordered_map<std::string, size_t> ids;
    std::string o;
    o.reserve(t.size());
    for (size_t i = 0; i < t.size();) {
      if (t[i] == 'p' && (i == 0 || !(isalnum((unsigned char)t[i - 1]) || t[i - 1] == '_')) && i + 1 < t.size() &&
          isdigit((unsigned char)t[i + 1])) {
        size_t j = i + 1;
        while (j < t.size() && isdigit((unsigned char)t[j])) j++;
        if (j < t.size() && t[j] == '(') {
          auto it = ids.emplace(t.substr(i, j - i), ids.size()).first;
          o += "p#" + std::to_string(it->second);
          i = j;
          continue;
        }
      }
      o += t[i++];
    }
    return o;
  };
  size_t nshapes = 0;
  const bool only_cond = getenv("KYV_JIT_ONLY_COND") && atoi(getenv("KYV_JIT_ONLY_COND")) != 0;  // experiments only
  for (size_t k = 0; k < rs.rules.size() && !only_cond; k++) {
    const RuleDesc& rd = rs.rules[k];
    if (rd.kind != RK_PATTERN && rd.kind != RK_ANYPATTERN) continue;
    std::vector<uint32_t> rr;
    if (rd.kind == RK_PATTERN) rr.push_back(rd.root);
    else for (uint32_t a = 0; a < rd.nalts; a++) rr.push_back(rs.pool[rd.root + a]);
    bool ok = true;
    for (uint32_t r : rr) if (pattern_depth(rs, r, 0) > MAX_DEPTH) ok = false;  // the walk would fall back
    if (!ok) continue;
    g.ok = true;
    for (uint32_t r : rr) g.mark_paths(r, rd.meta_sites, NONE, NONE, NONE, NONE, 0);
    for (uint32_t r : rr) { g.scope(r); g.scopes_below(r, 0); }
    std::vector<std::pair<uint32_t, std::string>> texts;  // root -> its functions (new shapes only)
    std::vector<std::pair<uint32_t, uint32_t>> alias;
    const size_t log0 = g.emitted_log.size();
    for (uint32_t r : rr) {
      std::ostringstream t;
      t.swap(g.out);
      g.node(r, 0);
      t.swap(g.out);
      if (!g.ok) break;
      std::string c = canon(t.str());
      auto it = shapes.find(c);
      if (it != shapes.end()) alias.push_back({r, it->second});
      else texts.push_back({r, t.str()});
    }
    if (!g.ok || nshapes + texts.size() > cap) {  // roll back this rule: it stays on the interpreted walk
      for (size_t i = log0; i < g.emitted_log.size(); i++) g.emitted[g.emitted_log[i]] = 0;
      g.emitted_log.resize(log0);
      continue;
    }
    for (auto& tx : texts) {
      shapes.emplace(canon(tx.second), tx.first);
      rep_of[tx.first] = tx.first;
      body << tx.second;
      nshapes++;
    }
    for (auto& al : alias) rep_of[al.first] = al.second;
    (*jit_rules)[k] = 1;
    rule_roots.push_back({(uint32_t)k, rr});
  }
  std::ostringstream src;
  // KYV_JC_UNROLL: the condition programs' element loops, not unrolled. Unrolled 4x (rounds 2-5, so that consecutive
  // elements' loads overlap) the C3 condition kernels held ~136k instructions each (every unrolled body inlines the
  // operand conversions and glob calls) with 7k SGPR / 74 VGPR spills at 8 waves/SIMD; round 6 A/B, C3 10M condition
  // phase: unroll 4 2.82 ms, 2 2.76, 1 2.53 (2.6k SGPR / 10 VGPR spills, half the code).
  // KYV_JIT_DEFS='-DKYV_JC_UNROLL=_Pragma("unroll 4")' for experiments
  src << "// generated by kyverno_amd/csrc/jit.cpp for one ruleset\n"
         "#ifndef KYV_JC_UNROLL\n#define KYV_JC_UNROLL _Pragma(\"unroll 1\")\n#endif\n"
         "#define KYV_FUSED_GW " << kFusedGW
      << "\n#include \"kyv_jcond.h\"\n#include \"kyv_fused.h\"\nnamespace kyv {\n";
  // KYV_RULE_VIEW: the View reference each rule of a multi-rule kernel (fused part, condition group) walks with. The
  // View's tables (column offsets, entry columns) are read-only uniform loads the compiler hoists to the kernel entry
  // and keeps live in SGPRs for the whole kernel (C3: 1.4-7k SGPR spills per kernel into VGPR lanes). Experiment
  // (round 6): KYV_JIT_DEFS='-DKYV_RULE_VIEW(x)=(*::kyv::kyv_launder(&(x)))' passes it through an empty asm at each
  // rule's start, so each rule reads the few it uses itself: 20-30 % fewer SGPR spills, but each rule then waits for a
  // chain of three dependent scalar loads before its first column read and VGPR spills grow (condition kernel 10 ->
  // 368): C3 walk 6.86 -> 10.67 ms, conditions 2.53 -> 3.95 ms. Default: the plain reference.
  src << "__device__ __forceinline__ const View* kyv_launder(const View* p) { asm volatile(\"\" : \"+s\"(p)); return p; }\n"
         "#ifndef KYV_RULE_VIEW\n#define KYV_RULE_VIEW(x) (x)\n#endif\n";
  src << body.str();
  if (!crules.empty()) {
    // the match part of pair_dispatch, out of line (one copy for every rule that needs more than the kind gate):
    // -1 matched, else the pair's status
    src << "static __device__ __attribute__((noinline)) int jc_match(const View& v, uint32_t r, uint32_t k) {\n"
           "  uint8_t st;\n  return pair_match(v, r, v.rules[k], &st) ? -1 : (int)st;\n}\n";
    src << cg.defs.str();
  }
  // Rules are split into groups of a few, one kernel per group (kyv_jit_walk_<g>): the compiler allocates
  // registers per group instead of for the worst pattern of the whole ruleset, and a group's code stays in
  // the instruction cache. jit_rules[k] = group + 1.
  // Default: two groups by register need. Rules whose patterns expand wildcard metadata keys (expand_meta: C3's
  // apparmor rules need ~100 VGPRs alone) go to a kernel at 4 waves/SIMD; every other rule (<= ~64 VGPRs alone) to
  // one at KYV_JIT_WPE_LIGHT (8) waves/SIMD, so the register hogs do not set the occupancy of the whole walk.
  // KYV_JIT_GROUP=n: consecutive groups of n rules (experiments); KYV_JIT_SPLIT=0: one group.
  std::vector<std::vector<size_t>> groups;
  std::vector<int> gwpe;
  std::function<bool(uint32_t, uint32_t, int)> wild_meta = [&](uint32_t pn, uint32_t mbase, int guard) -> bool {
    if (pn == NONE || pn >= rs.pnodes.size() || guard > 4 * MAX_DEPTH) return false;
    const PNode& P = rs.pnodes[pn];
    switch (P.kind) {
      case P_MAP: {
        if (P.flags & PF_META) {
          const MetaSite& ms = rs.metas[mbase + P.meta];
          if (ms.nwild_l + ms.nwild_a) return true;
        }
        for (uint32_t e = 0; e < P.n; e++) {
          const PEntry& E = rs.pentries[P.first + e];
          if (E.child == NONE || E.handler == H_STAR || E.handler == H_NEGATION || E.handler == H_EXIST_BADPAT) continue;
          if (E.handler == H_EXISTENCE) {
            for (uint32_t j = 0; j < rs.pool[E.child]; j++) if (wild_meta(rs.pool[E.child + 1 + j], mbase, guard + 1)) return true;
          } else if (wild_meta(E.child, mbase, guard + 1)) {
            return true;
          }
        }
        return false;
      }
      case P_ARR_MAPS: return wild_meta(P.first, mbase, guard + 1);
      case P_ARR_POS:
        for (uint32_t i = 0; i < P.n; i++) if (wild_meta(rs.pool[P.first + i], mbase, guard + 1)) return true;
        return false;
      default: return false;
    }
  };
  if (getenv("KYV_JIT_GROUP")) {
    const size_t per = (size_t)std::max(1, atoi(getenv("KYV_JIT_GROUP")));
    const size_t ng = std::min<size_t>(250, (rule_roots.size() + per - 1) / per);
    for (size_t gi = 0; gi < ng; gi++) {
      groups.emplace_back();
      gwpe.push_back(-1);
      for (size_t i = rule_roots.size() * gi / ng; i < rule_roots.size() * (gi + 1) / ng; i++) groups.back().push_back(i);
    }
  } else {
    const bool split = !getenv("KYV_JIT_SPLIT") || atoi(getenv("KYV_JIT_SPLIT")) != 0;
    std::vector<size_t> light, heavy;
    for (size_t i = 0; i < rule_roots.size(); i++) {
      bool h = false;
      const RuleDesc& rd = rs.rules[rule_roots[i].first];
      for (uint32_t r : rule_roots[i].second) h = h || wild_meta(r, rd.meta_sites, 0);
      (split && h ? heavy : light).push_back(i);
    }
    if (!light.empty()) { groups.push_back(light); gwpe.push_back(split ? -2 : -1); }
    if (!heavy.empty()) { groups.push_back(heavy); gwpe.push_back(-1); }
  }
  const size_t ngroups = groups.size();
  // Compiled condition rules folded into the fused walk (round 6): a fused wave runs them for its 64 resources after the
  // pattern rules of its part, so the kind-gate words and headers it already holds serve them too and the container
  // rows the pattern rules just read are cache hits; no separate condition kernel re-streams its kind's waves
  // (kyv_jit_condg_<k> at C3: 3.06 ms, wait 0.80, and no overlap with the walk on the second stream: every wave slot is
  // taken by the fused kernels). KYV_FOLD_COND=0 (default): the condition kernels; 1: round-robin over the light
  // group's parts; 2: all in its last part. jit_cond[k] = 2 + group for a folded rule.
  // Measured (r6 A/B, C3 10M): folded walk 11.16 ms against walk 6.99 + conditions 3.07 ms separate (evaluation 12.32
  // vs 11.24 ms): the condition code in the 64-VGPR fused parts costs more than the shared loads save, and the parts'
  // hipRTC compile grows from ~3 to ~27 min. Kept as an experiment, off.
  static const int fold_mode = getenv("KYV_FOLD_COND") ? atoi(getenv("KYV_FOLD_COND")) : 0;
  size_t fold_group = SIZE_MAX;
  std::vector<uint32_t> folded;
  if (fold_mode && !crules.empty() && rs.rules.size() <= 32u * kFusedGW) {
    for (int pass = 0; pass < 2 && fold_group == SIZE_MAX; pass++)  // the light group first, else any with fused rules
      for (size_t gi = 0; gi < ngroups && fold_group == SIZE_MAX; gi++) {
        if (pass == 0 && gwpe[gi] != -2) continue;
        for (size_t i : groups[gi])
          if (jit_rule_fused(rs, rule_roots[i].first)) { fold_group = gi; break; }
      }
    if (fold_group != SIZE_MAX) folded = crules;
  }
  const std::string jc_lds = std::to_string(cg.lds_used ? cg.nslots : 0u) + "u * kyv::JCAP * 64u + 64u";
  std::vector<std::pair<size_t, size_t>> fused_kernels;  // (group, part): kyv_jit_fused_<g>[p<part>]
  std::vector<size_t> merged_groups;                      // groups with a kyv_jit_fusedm_<g> (KYV_FUSED_MERGE)
  for (size_t gi = 0; gi < ngroups; gi++) {
    std::vector<uint32_t> roots, chunk_roots;  // every root of the group; those of its per-chunk (non-fused) rules
    std::vector<size_t> fused;                 // rule_roots indices of the group's fused rules
    for (size_t i : groups[gi]) {
      (*jit_rules)[rule_roots[i].first] = (uint8_t)(gi + 1);
      const bool f = jit_rule_fused(rs, rule_roots[i].first);
      if (f) fused.push_back(i);
      for (uint32_t r : rule_roots[i].second) { roots.push_back(r); if (!f) chunk_roots.push_back(r); }
    }
    // KYV_FUSED_ORDER (experiment): the group's fused rules reordered before they are cut into parts -- 1: by (kind
    // gate, root-scope columns), 2: by (root-scope columns, kind gate) -- so that rules reading the same columns run in
    // one part, back to back. The order of a wave's rules is free: each writes only its own verdicts and staging chunk.
    // Measured slower (round 6, C3 10M walk ms): policy order 6.56, order 1 8.79, order 2 7.97, order 1 in 4 parts 7.83,
    // order 3 8.14 (policy order 6.70 in that run)
    // -- a part then holds one kind family's rules, so a wave finds all its work in one kernel and none in the others,
    // and the column cache's slots cover fewer of that kernel's columns.
    static const int forder = getenv("KYV_FUSED_ORDER") ? atoi(getenv("KYV_FUSED_ORDER")) : 0;
    if (forder) {
      std::map<size_t, std::pair<std::vector<uint32_t>, std::vector<uint32_t>>> key;
      for (size_t i : fused) {
        KindGate kg = rule_gate(rs, rs.rules[rule_roots[i].first]);
        std::sort(kg.kinds.begin(), kg.kinds.end());
        if (kg.any) kg.kinds.clear();
        std::set<uint32_t> cols;
        for (uint32_t r : rule_roots[i].second) {
          g.scope(rep_of[r]);
          for (uint32_t c : g.scope_of[rep_of[r]]) cols.insert(c);
        }
        std::vector<uint32_t> cv(cols.begin(), cols.end());
        key[i] = forder == 2 ? std::make_pair(cv, kg.kinds) : std::make_pair(kg.kinds, cv);
      }
      std::stable_sort(fused.begin(), fused.end(), [&](size_t a, size_t b) { return key[a] < key[b]; });
      if (forder == 3) {  // 3: the mode-1 order dealt round-robin over the parts (each part an equal share of every kind)
        const size_t np = std::max<size_t>(1, std::min<size_t>(fused.size(), getenv("KYV_FUSED_SPLIT") ? (size_t)atoi(getenv("KYV_FUSED_SPLIT")) : 3));
        std::vector<size_t> dealt;
        for (size_t p = 0; p < np; p++)
          for (size_t j = p; j < fused.size(); j += np) dealt.push_back(fused[j]);
        fused.swap(dealt);
      }
    }
    // the root scope's column preload is issued before the lane's walk predicate is known: it depends on the
    // resource row only, so its loads overlap the header loads the predicate waits for (one memory round, not two)
    for (uint32_t r : roots)
      if (rep_of[r] == r)  // one root function per pattern shape
      src << "static __device__ __forceinline__ void root" << r
          << "(const View& v, const Node* R, const ResHeader* hp, uint32_t row, uint32_t mbase, bool rootmap, bool walk,\n"
             "    PatOut& out) {\n"
             "  " << g.preload(r, "pc", "row", "jc_col(v, ") << "\n"
             "  if (!walk) return;\n"
             "#ifdef KYV_EXP_JIT_PRELOAD\n  { uint64_t x = 0; for (auto q : pc) x ^= q; out.status = x == 0x123456789ull ? ST_FAIL : ST_PASS; return; }\n#endif\n"
             "  JW w{v, R, hp, 0ull, 0ull, Keys{NONE, NONE}, 0ull, mbase, (uint8_t)ST_NONE};\n"
             "  Ret r = p" << r << "(w, 0u, rootmap ? (uint32_t)N_MAP : T_UNK, 0u, row, pc);\n"
             "  jfinish(w, r, out);\n"
             "}\n";
    // Root-column cache of the fused parts (round 6). The rules of a part preload their root-scope path columns one
    // rule after another, and most of those entries are the same few columns (C3 pod rules: spec and the three
    // container lists' entry and length columns; 141 root-column loads per pod over the light group's three parts,
    // 45 distinct): each reload is a 512-B wave read that, with ~1,000 waves per XCD streaming through its 4 MB L2,
    // has usually left the cache again (measured: root-column preloads are 13.5 of the walk's 25.6 GB per C3
    // evaluation, accounting build with KYV_ACCT_SEL). A fused wave now loads each column that two or more of the
    // group's rules read once per part into an LDS slot (8 B per lane, the lane's own entry: no sharing between
    // lanes, so no barrier), and the rules' root functions (rootc<r>_<g>) read it from there. Columns whose rules'
    // kind gates are disjoint share a slot (a lane's kind admits at most one of them: the pod rules' container
    // columns and the workload rules' template columns). KYV_COLCACHE = slots per wave (default 4: 2 KB of LDS per
    // wave); 0: off. C3 10M walk ms by slots (round 6 A/B): 0 6.94, 2 6.79, 3 6.71, 4 6.66, 5 6.69, 8 6.81, 12 (at 6
    // waves/SIMD) 7.12 -- the slots beyond the most shared columns cost more in registers (the slot reads' addresses
    // and the fill) than the reloads they save.
    static const uint32_t cc_max = getenv("KYV_COLCACHE") ? (uint32_t)std::max(0, atoi(getenv("KYV_COLCACHE"))) : 4u;
    std::map<uint32_t, uint32_t> cslot;                 // cached root column -> its LDS slot
    std::map<size_t, std::vector<uint32_t>> rule_cols;  // rule_roots index -> its roots' preload columns
    uint32_t ncslots = 0;
    if (cc_max && !fused.empty()) {
      std::map<uint32_t, size_t> cnt;
      std::map<uint32_t, std::set<uint32_t>> ckinds;  // column -> kinds of the rules reading it
      std::set<uint32_t> call;                        // columns a kind-unrestricted rule reads (share no slot)
      for (size_t i : fused) {
        std::set<uint32_t> cols;
        for (uint32_t r : rule_roots[i].second) {
          g.scope(rep_of[r]);
          for (uint32_t c : g.scope_of[rep_of[r]]) cols.insert(c);
        }
        rule_cols[i].assign(cols.begin(), cols.end());
        const KindGate kg = rule_gate(rs, rs.rules[rule_roots[i].first]);
        for (uint32_t c : cols) {
          cnt[c]++;
          if (kg.any || kg.kinds.empty()) call.insert(c);
          else ckinds[c].insert(kg.kinds.begin(), kg.kinds.end());
        }
      }
      std::vector<uint32_t> cand;
      for (const auto& e : cnt) if (e.second >= 2) cand.push_back(e.first);
      std::stable_sort(cand.begin(), cand.end(), [&](uint32_t a, uint32_t b) { return cnt[a] > cnt[b]; });
      std::vector<std::vector<uint32_t>> slots;
      for (uint32_t c : cand) {
        for (uint32_t s = 0; s < cc_max; s++) {
          if (s == slots.size()) slots.emplace_back();
          bool ok = true;
          for (uint32_t c2 : slots[s]) {
            if (call.count(c) || call.count(c2)) ok = false;
            else for (uint32_t kk : ckinds[c]) if (ckinds[c2].count(kk)) { ok = false; break; }
            if (!ok) break;
          }
          if (ok) { slots[s].push_back(c); cslot[c] = s; break; }
        }
      }
      ncslots = (uint32_t)slots.size();
      if (cslot.empty()) ncslots = 0;
    }
    if (ncslots) {
      std::set<uint32_t> reps;
      for (size_t i : fused) for (uint32_t r : rule_roots[i].second) reps.insert(rep_of[r]);
      for (uint32_t r : reps) {
        const auto& L = g.scope_of[r];
        src << "static __device__ __forceinline__ void rootc" << r << "_" << gi
            << "(const View& v, const Node* R, const ResHeader* hp, uint32_t row, uint32_t mbase, bool rootmap, bool walk,\n"
               "    PatOut& out, const uint64_t* jcc) {\n"
               "  const uint32_t lane = threadIdx.x & 63u;\n"
               "  (void)lane;\n"
               "  uint64_t pc[" << std::max<size_t>(1, L.size()) << "];";
        for (size_t i = 0; i < L.size(); i++) {
          auto it = cslot.find(L[i]);
          if (it != cslot.end()) src << " pc[" << i << "] = jcc[" << it->second * 64u << "u + lane];";
          else src << " pc[" << i << "] = jc_col(v, " << Gen::u(L[i]) << ", row);";
        }
        src << "\n"
               "  if (!walk) return;\n"
               "  JW w{v, R, hp, 0ull, 0ull, Keys{NONE, NONE}, 0ull, mbase, (uint8_t)ST_NONE};\n"
               "  Ret r = p" << r << "(w, 0u, rootmap ? (uint32_t)N_MAP : T_UNK, 0u, row, pc);\n"
               "  jfinish(w, r, out);\n"
               "}\n";
      }
    }
    if (roots.size() > 256) {
      std::map<uint32_t, std::vector<uint32_t>> br2;
      for (uint32_t r : roots) br2[rep_of[r]].push_back(r);
      std::vector<uint16_t> tab(rs.pnodes.size(), 0xFFFF);
      uint16_t si = 0;
      for (auto& b : br2) { for (uint32_t r : b.second) tab[r] = si; si++; }
      src << "__device__ const unsigned short kyv_shape" << gi << "[" << std::max<size_t>(1, tab.size()) << "] = {";
      for (size_t i = 0; i < tab.size(); i++) src << (i ? "," : "") << tab[i];
      src << "};\n";
    }
    src << "struct JitWalker" << gi << " {\n"
           "  bool rootmap;\n"
           "  __device__ __forceinline__ void run(const View& v, uint32_t root, bool walk, const Node* R, const ResHeader* hp,\n"
           "                                     uint32_t row, const RuleDesc& rd, PatOut& out) {\n"
           "    out.status = ST_NONE; out.idx = 0; out.tmpl = NONE; out.key0 = NONE; out.key1 = NONE;\n"
           "#ifdef KYV_EXP_JIT_EMPTY\n    if (walk) out.status = ST_PASS; return;\n#endif\n"
           << (roots.size() <= 256 ? std::string("    switch (root) {\n") : "    switch (root < " + std::to_string(rs.pnodes.size()) +
                                                                "u ? (uint32_t)kyv_shape" + std::to_string(gi) +
                                                                "[root] : 0xFFFFu) {\n");
    // roots of one shape share a case (and its root function); with many roots (C4: 10k rules over 15 shapes) the
    // switch goes over a root -> shape table instead of one label per root (a 10k-label switch took the compiler
    // minutes)
    std::map<uint32_t, std::vector<uint32_t>> by_rep;
    for (uint32_t r : chunk_roots) by_rep[rep_of[r]].push_back(r);
    if (roots.size() <= 256) {
      for (auto& br : by_rep) {
        for (uint32_t r : br.second) src << "      case " << r << "u:";
        src << " root" << br.first << "(v, R, hp, row, rd.meta_sites, rootmap, walk, out); break;\n";
      }
    } else {
      uint32_t si = 0;
      for (auto& br : by_rep) {
        src << "      case " << si++ << "u: root" << br.first << "(v, R, hp, row, rd.meta_sites, rootmap, walk, out); break;\n";
      }
    }
    src << "      default: if (walk) out.status = ST_FALLBACK;\n"
           "    }\n"
           "  }\n"
           "};\n";
    if (fused.empty()) continue;
    // the group's fused rules, back to back for one wave (walk_fused, kyv_wave.h): per rule the slice / kind-gate test
    // (uniform), the alternative loop of validatePatterns with the rule's roots as constants, the verdict bytes and the
    // staged failing-path records of chunk (rule, wave). KYV_FUSED_SPLIT=n splits the group's fused rules into n
    // kernels (contiguous runs; part p > 0 is kyv_jit_fused_<g>p<p>), each with the register need of its own rules.
    // (Tried and removed, round 4: prefetching the next rule's root-scope columns into registers before the current
    // rule's walk -- 110 VGPR spills at 5 waves/EU, 896 at 6; C3 walk 8.1 -> 9.1 / 10.2 ms.)
    // C3 (r4 A/B, evaluation / walk ms): one kernel at 6 waves/EU 12.04 / 7.74; 2 parts at 8 waves 11.35 / 7.43; 3 at 8
    // 11.25 / 7.34; 4 at 8 11.33 / 7.26 (smaller kernels: fewer spills at 8 waves, and they interleave with the
    // condition kernels on the other stream)
    // KYV_FUSED_SPLIT_HEAVY: the parts of the wildcard-metadata group, whose kernels run at the heavy target. Default 1:
    // its few rules (C3: app-armor for pods, workloads, CronJobs) have disjoint kind gates, so as parts every kernel
    // but one passed over the whole batch for nothing (round 6, C3 walk 6.56-6.67 -> 6.39 ms as one kernel)
    const bool heavy_grp = gwpe[gi] == -1 && std::count(gwpe.begin(), gwpe.end(), -2);
    const char* split_env = heavy_grp ? getenv("KYV_FUSED_SPLIT_HEAVY") : getenv("KYV_FUSED_SPLIT");
    const size_t nparts = std::max<size_t>(1, std::min<size_t>(fused.size(), split_env ? (size_t)atoi(split_env) : heavy_grp ? 1 : 3));
    for (size_t pi = 0; pi < nparts; pi++) {
      const std::vector<size_t> part(fused.begin() + fused.size() * pi / nparts, fused.begin() + fused.size() * (pi + 1) / nparts);
      const std::string sname = "JitFused" + std::to_string(gi) + (pi ? "p" + std::to_string(pi) : std::string());
      std::vector<uint32_t> conds;  // the folded condition rules this part runs after its pattern rules
      if (gi == fold_group)
        for (size_t j = 0; j < folded.size(); j++)
          if (fold_mode == 2 ? pi + 1 == nparts : j % nparts == pi) conds.push_back(folded[j]);
      src << "struct " << sname << " {\n"
             "  __device__ __forceinline__ void run(const View& v, const DevOut& o, uint32_t nwaves, uint32_t w, uint32_t r,\n"
             "                                     bool active, uint32_t hflags, uint32_t hroot, const uint32_t* gw) {\n"
             "    const uint32_t lane = threadIdx.x & 63u;\n"
             "    const Node* R = v.nodes + hroot;\n"
             "    const ResHeader* hp = v.hdr + r;\n"
             "    const uint32_t row = r < v.nres ? r : NONE;\n"
             "    const bool rootmap = (hflags & RF_ROOT_MAP) != 0;\n"
             "    (void)lane; (void)hp; (void)rootmap;\n";
      if (!conds.empty()) src << "    __shared__ uint32_t jl[" << jc_lds << "];\n";
      if (ncslots) {
        // the part's cached root columns, each loaded by the lanes some rule of this part (in this rule slice) walks
        std::map<uint32_t, std::vector<uint32_t>> users;  // column -> rules of this part reading it
        for (size_t i : part)
          for (uint32_t c : rule_cols[i]) if (cslot.count(c)) users[c].push_back(rule_roots[i].first);
        // (a lane needs a column when a rule reading it is in the rule slice and its kind gate admits the lane: one
        // mask test per gate word over the slice's rule bits, not the rules' own gate expressions, which the compiler
        // would otherwise evaluate once here for every rule and keep live through the part)
        src << "    __shared__ uint64_t jcc[" << ncslots * 64u << "u];\n"
               "    uint32_t jsl[KYV_FUSED_GW];\n"
               "#pragma unroll\n"
               "    for (uint32_t i = 0; i < KYV_FUSED_GW; i++) {\n"
               "      const uint32_t b0 = 32u * i, lo = o.rule_lo > b0 ? o.rule_lo - b0 : 0u, hi = o.rule_hi > b0 ? o.rule_hi - b0 : 0u;\n"
               "      const uint32_t mlo = lo >= 32u ? 0u : (0xFFFFFFFFu << lo), mhi = hi >= 32u ? 0xFFFFFFFFu : ((1u << hi) - 1u);\n"
               "      jsl[i] = active ? (gw[i] & mlo & mhi) : 0u;\n"
               "    }\n";
        for (const auto& cu : users) {
          std::map<uint32_t, uint32_t> wm;  // gate word -> bits of the column's rules
          for (uint32_t k : cu.second) wm[k / 32] |= 1u << (k % 32);
          src << "    if (";
          size_t j = 0;
          for (const auto& e : wm) src << (j++ ? " | " : "") << "(jsl[" << e.first << "] & " << e.second << "u)";
          src << ") jcc[" << cslot[cu.first] * 64u << "u + lane] = jc_col(v, " << Gen::u(cu.first) << ", row);\n";
        }
      }
      for (size_t j = 0; j < part.size(); j++) {
      const size_t i = part[j];
      const uint32_t k = rule_roots[i].first;
      const RuleDesc& rd = rs.rules[k];
      const bool pat = rd.kind == RK_PATTERN;
      const uint32_t nalts = pat ? 1u : rd.nalts, alts = pat ? 1u : std::min<uint32_t>(rd.nalts, MAX_ALTS);
      const std::string K = Gen::u(k);
      src << "    if (" << K << " >= o.rule_lo && " << K << " < o.rule_hi) {\n"
             "      const bool gated = active && ((gw[" << k / 32 << "] >> " << k % 32 << "u) & 1u);\n"
             "      if (__ballot(gated)) {\n"
             "        const View& vl = KYV_RULE_VIEW(v);\n";
      src << "        const bool magic = gated && (hflags & RF_MAGIC);\n"
             "        WaveSink sink{o.stage + sld32(o.rbase + (" << K << " - o.rule_lo)) + (size_t)w * 64u * " << alts
          << "u, 0u, " << (rd.uses_meta ? "true" : "false") << "};\n"
             "        uint8_t st = pair_walk_alts(" << (pat ? "true" : "false") << ", " << nalts << "u, gated && !magic, r, " << K
          << ", sink, [&](uint32_t a, bool wk, PatOut& po) {\n"
             "          po.status = ST_NONE; po.idx = 0; po.tmpl = NONE; po.key0 = NONE; po.key1 = NONE;\n"
             "          switch (a) {\n";
      for (uint32_t a = 0; a < nalts; a++) {
        const uint32_t root = rule_roots[i].second[a];
        if (ncslots)
          src << "            case " << a << "u: rootc" << rep_of[root] << "_" << gi << "(vl, R, hp, row, " << Gen::u(rd.meta_sites)
              << ", rootmap, wk, po, jcc); break;\n";
        else
          src << "            case " << a << "u: root" << rep_of[root] << "(vl, R, hp, row, " << Gen::u(rd.meta_sites)
              << ", rootmap, wk, po); break;\n";
      }
      src << "            default: break;\n"
             "          }\n"
             "        });\n"
             "        if (magic) st = ST_FALLBACK;\n"
             "        if (gated) { o.status[(size_t)" << K << " * v.nres + r] = st; KYV_ACCT_ADD(1, 1); }\n"
             "        if (sink.n && lane == 0) {\n"
             "          o.rcnt[(size_t)(" << K << " - o.rule_lo) * nwaves + w] = (uint16_t)sink.n; KYV_ACCT_ADD(1, 2);\n"
             "        }\n"
             "      }\n"
             "    }\n";
    }
      // folded condition rules: the kyv_jit_condg_<k> member body for this wave's lanes (same gate, same verdict store)
      for (uint32_t k : conds) {
        const std::string K = Gen::u(k);
        src << "    if (" << K << " >= o.rule_lo && " << K << " < o.rule_hi) {\n"
               "      const bool gated = active && ((gw[" << k / 32 << "] >> " << k % 32 << "u) & 1u);\n"
               "      if (__ballot(gated)) {\n"
               "        uint8_t st = ST_NONE;\n"
               "        if (gated) st = jr" << k << "(KYV_RULE_VIEW(v), r, jl + lane);\n"
               "        if (gated && st != ST_NONE) { o.status[(size_t)" << K << " * v.nres + r] = st; KYV_ACCT_ADD(1, 1); }\n"
               "      }\n"
               "    }\n";
      }
      src << "  }\n"
             "};\n";
      fused_kernels.push_back(std::make_pair(gi, pi));
    }
    // KYV_FUSED_MERGE=1 (experiment): the parts once more as ONE kernel, kyv_jit_fusedm_<g>, run back to back for the
    // same wave, each part's resource index and root laundered through an empty asm so its loads are its own (no value
    // kept live from one part's rules into the next: the register need stays that of one part). The resource rows and
    // columns a later part reads again were just read by this wave: L2 hits instead of a second pass over HBM.
    if (nparts > 1 && getenv("KYV_FUSED_MERGE") && atoi(getenv("KYV_FUSED_MERGE")) != 0) {
      src << "struct JitFusedM" << gi << " {\n"
             "  __device__ __forceinline__ void run(const View& v, const DevOut& o, uint32_t nwaves, uint32_t w, uint32_t r,\n"
             "                                     bool active, uint32_t hflags, uint32_t hroot, const uint32_t* gw) {\n";
      for (size_t pi = 0; pi < nparts; pi++) {
        const std::string sname = "JitFused" + std::to_string(gi) + (pi ? "p" + std::to_string(pi) : std::string());
        src << "    {\n"
               "      uint32_t r2 = r, h2 = hroot;\n"
               "      asm volatile(\"\" : \"+v\"(r2), \"+v\"(h2));\n"
               "      " << sname << " f;\n"
               "      f.run(v, o, nwaves, w, r2, active, hflags, h2, gw);\n"
               "    }\n";
      }
      src << "  }\n"
             "};\n";
      merged_groups.push_back(gi);
    }
  }
  // Pattern shapes shared by match-record rules (round 5): each distinct (shape, metadata-site base) of the eligible
  // rules is walked once per resource its users' kind gates admit (kyv_jit_shapes), and the match phase decides every
  // matched pair of those rules from that verdict and record (kyv_kernels.h mrec_shape_out): the walk of a compiled
  // pattern is a function of the resource alone (no rule input but the metadata-site base), so rules with one shape
  // share one walk per resource instead of one per matched pair (C4: 10,440 rules, 15 shapes, 1.03 G matched pairs).
  // (representative root, metadata-site base of the shape's first rule); shapes are keyed by the root's code and the
  // content of the rule's metadata-expansion sites, so rules with equal sites at other pool offsets share a shape
  std::vector<std::pair<uint32_t, uint32_t>> shape_list;
  {
    std::map<std::pair<uint32_t, std::string>, uint32_t> sid;
    for (const auto& rr : rule_roots) {
      const uint32_t k = rr.first;
      if (!jit_shape_eligible(rs, k) || rr.second.size() != 1) continue;
      const auto key = std::make_pair(rep_of[rr.second[0]], meta_signature(rs, rs.rules[k]));
      auto it = sid.find(key);
      if (it == sid.end()) {
        if (shape_list.size() >= JIT_MAX_SHAPES) continue;
        it = sid.emplace(key, (uint32_t)shape_list.size()).first;
        shape_list.push_back(std::make_pair(rep_of[rr.second[0]], rs.rules[k].meta_sites));
      }
      if (jit_shape) (*jit_shape)[k] = (uint16_t)(it->second + 1);
    }
  }
  if (!shape_list.empty()) {
    // every root function a shape needs is already in the source (its users are covered rules of some group)
    src << "struct JitShapes {\n"
           "  __device__ __forceinline__ void run(const View& v, const ShapeOut& so, uint32_t r, bool active, uint32_t hflags,\n"
           "                                     uint32_t hroot, uint32_t cls) {\n"
           "    const Node* R = v.nodes + hroot;\n"
           "    const ResHeader* hp = v.hdr + r;\n"
           "    const uint32_t row = r < v.nres ? r : NONE;\n"
           "    const bool rootmap = (hflags & RF_ROOT_MAP) != 0;\n"
           "    (void)hp; (void)rootmap;\n";
    for (size_t si = 0; si < shape_list.size(); si++) {
      const std::string S = Gen::u((uint32_t)si);
      src << "    {\n"
             "      const bool gated = active && ((so.gate[(size_t)cls * so.words + " << si / 32 << "u] >> " << si % 32 << "u) & 1u);\n"
             "      if (__ballot(gated)) {\n"
             "        const bool magic = gated && (hflags & RF_MAGIC);\n"
             "        ShapeSink sink{so.rec + (size_t)" << S << " * v.nres + r};\n"
             "        uint8_t st = pair_walk_alts(true, 1u, gated && !magic, r, 0u, sink, [&](uint32_t, bool wk, PatOut& po) {\n"
             "          po.status = ST_NONE; po.idx = 0; po.tmpl = NONE; po.key0 = NONE; po.key1 = NONE;\n"
             "          root" << shape_list[si].first << "(v, R, hp, row, " << Gen::u(shape_list[si].second) << ", rootmap, wk, po);\n"
             "        });\n"
             "        if (magic) st = ST_FALLBACK;\n"
             "        if (gated) { so.st[(size_t)" << S << " * v.nres + r] = st; KYV_ACCT_ADD(1, 1); }\n"
             "      }\n"
             "    }\n";
    }
    src << "  }\n"
           "};\n";
  }
  src << "}  // namespace kyv\n"
         "#ifndef KYV_JIT_WPE\n#define KYV_JIT_WPE 4\n#endif\n";
  if (!shape_list.empty())
    // one workgroup (one wave) per match wave, grid-stride; every shape its kind class needs, back to back
    src << "extern \"C\" __global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(KYV_JIT_WPE)))\n"
           "kyv_jit_shapes(const kyv::View* __restrict__ vp, kyv::ShapeOut so) {\n"
           "  kyv::JitShapes f;\n"
           "  kyv::walk_shapes(*vp, so, f);\n"
           "}\n";
  if (!crules.empty()) {
    // compiled condition rules, inlined (one big kernel with a switch over the rules needs an out-of-line call per
    // rule, whose callee-saved registers go through scratch memory, or, inlined, compiles for tens of minutes); one
    // lane per resource, launched over the match waves [w0, w0 + grid) that hold resources of the rule's kind gate
    // (kind-major batch). Rules with the same kind gate share one kernel (kyv_jit_condg_<first rule>, jit_cond_groups;
    // `mask`: the members the launch runs, those of the current rule slice): a wave loads its resources' header once
    // for all of them and the later rules find the lists the first one read (C3: the three capability rules of a pod
    // kind read the same container lists) in the caches. KYV_JC_GROUP=0: one kernel per rule (kyv_jit_cond_<k>)
    // 5 waves/SIMD: measured 1.30 -> 1.05 ms on C3 with the round-2 kernel (4: 1.11, 6: 1.08); round 6 (12 rules in 3
    // kernels, C3 10M, condition phase ms): 5 (77 VGPRs) 3.05, 6 3.07, 7 2.88, 8 (64 VGPRs, 74 spills) 2.82
    src << "#ifndef KYV_JC_WPE\n#define KYV_JC_WPE 8\n#endif\n";
    const bool grouped = !getenv("KYV_JC_GROUP") || atoi(getenv("KYV_JC_GROUP")) != 0;
    const std::string& lds = jc_lds;
    std::vector<uint32_t> kept;  // the rules the fused walk does not run
    for (uint32_t k : crules) if (std::find(folded.begin(), folded.end(), k) == folded.end()) kept.push_back(k);
    auto member = [&](uint32_t k, const std::string& on) {
      src << "  {\n"
             "    const bool gated = " << on << "((gw[" << k / 32 << "u] >> " << k % 32 << "u) & 1u);\n"
             "    if (__ballot(gated)) {\n"
             "      uint8_t st = kyv::ST_NONE;\n"
             "      if (gated) st = kyv::jr" << k << "(KYV_RULE_VIEW(v), r, jl + lane);\n"
             "      if (gated && st != kyv::ST_NONE) { o.status[(size_t)" << k << "u * v.nres + r] = st; KYV_ACCT_ADD(1, 1); }\n"
             "    }\n"
             "  }\n";
    };
    if (grouped) {
      for (const auto& grp : jit_cond_groups(rs, kept)) {
        src << "extern \"C\" __global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(KYV_JC_WPE)))\n"
               "kyv_jit_condg_" << grp[0] << "(const kyv::View* __restrict__ vp, kyv::DevOut o, uint32_t w0, uint32_t mask) {\n"
               "  __shared__ uint32_t jl[" << lds << "];\n"
               "  const kyv::View& v = *vp;\n"
               "  const uint32_t lane = threadIdx.x, r = (w0 + blockIdx.x) * 64u + lane;\n"
               "  const uint32_t* gw = r < v.nres ? v.gate + (size_t)v.hdr[r].kclass * v.gate_words : nullptr;\n"
               "  if (r < v.nres) KYV_ACCT_ADD(0, 4);  // header: kind class\n";
        for (size_t i = 0; i < grp.size(); i++) member(grp[i], "gw && (mask & " + std::to_string(1u << i) + "u) && ");
        src << "}\n";
      }
    } else {
      for (uint32_t k : kept) {
        src << "extern \"C\" __global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(KYV_JC_WPE)))\n"
               "kyv_jit_cond_" << k << "(const kyv::View* __restrict__ vp, kyv::DevOut o, uint32_t w0) {\n"
               "  __shared__ uint32_t jl[" << lds << "];\n"
               "  const kyv::View& v = *vp;\n"
               "  const uint32_t lane = threadIdx.x, r = (w0 + blockIdx.x) * 64u + lane;\n"
               "  const uint32_t* gw = r < v.nres ? v.gate + (size_t)v.hdr[r].kclass * v.gate_words : nullptr;\n"
               "  if (r < v.nres) KYV_ACCT_ADD(0, 4);  // header: kind class\n";
        member(k, "gw && ");
        src << "}\n";
      }
    }
    for (uint32_t k : crules) if (jit_cond) (*jit_cond)[k] = 1;
    for (uint32_t k : folded) if (jit_cond) (*jit_cond)[k] = (uint8_t)(2 + fold_group);
  }
  src << "#ifndef KYV_JIT_WPE_LIGHT\n#define KYV_JIT_WPE_LIGHT 8\n#endif\n";
  for (size_t gi = 0; gi < ngroups; gi++)
    src << "extern \"C\" __global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu("
        << (gwpe[gi] == -2 ? "KYV_JIT_WPE_LIGHT" : "KYV_JIT_WPE") << ")))\n"
           "kyv_jit_walk_" << gi << "(const kyv::View* __restrict__ vp, kyv::DevOut o, kyv::WorkLists wl, kyv::ChunkMap cm) {\n"
           "  kyv::JitWalker" << gi << " wk{false};\n"
           "  kyv::walk_chunks(*vp, o, wl, cm, wk);\n"
           "}\n";
  // fused kernels: one workgroup (one wave) per match wave of the batch. A fused kernel holds every direct rule of its
  // group inline: as one kernel at the light group's 8-waves target (64 VGPRs) it spills (round-4 C3 profile: 94-128
  // VGPR spills, 5 GB of scratch writes per evaluation; one kernel, C3 walk ms: 8 waves 9.44, 7: 8.14, 6: 8.11,
  // 5: 8.46, 4: 9.53); split in parts (KYV_FUSED_SPLIT, above) each part fits 8 waves with a few spills
  // (the group of wildcard-metadata rules keeps the walk's heavy target, KYV_JIT_WPE_FUSED_HEAVY = 4)
  src << "#ifndef KYV_JIT_WPE_FUSED\n#define KYV_JIT_WPE_FUSED 8\n#endif\n"
         "#ifndef KYV_JIT_WPE_FUSED_HEAVY\n#define KYV_JIT_WPE_FUSED_HEAVY 4\n#endif\n";
  for (const auto& gp : fused_kernels) {
    const std::string sfx = std::to_string(gp.first) + (gp.second ? "p" + std::to_string(gp.second) : std::string());
    src << "extern \"C\" __global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu("
        << (gwpe[gp.first] == -1 && std::count(gwpe.begin(), gwpe.end(), -2) ? "KYV_JIT_WPE_FUSED_HEAVY" : "KYV_JIT_WPE_FUSED")
        << ")))\n"
           "kyv_jit_fused_" << sfx << "(const kyv::View* __restrict__ vp, kyv::DevOut o, uint32_t nwaves) {\n"
           "  kyv::JitFused" << sfx << " f;\n"
           "  kyv::walk_fused(*vp, o, nwaves, f);\n"
           "}\n";
  }
  for (size_t gi : merged_groups) {
    src << "extern \"C\" __global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu("
        << (gwpe[gi] == -1 && std::count(gwpe.begin(), gwpe.end(), -2) ? "KYV_JIT_WPE_FUSED_HEAVY" : "KYV_JIT_WPE_FUSED")
        << ")))\n"
           "kyv_jit_fusedm_" << gi << "(const kyv::View* __restrict__ vp, kyv::DevOut o, uint32_t nwaves) {\n"
           "  kyv::JitFusedM" << gi << " f;\n"
           "  kyv::walk_fused(*vp, o, nwaves, f);\n"
           "}\n";
  }
  return src.str();
}

std::vector<std::vector<uint32_t>> jit_cond_groups(const Ruleset& rs, const std::vector<uint32_t>& crules) {
  std::vector<std::vector<uint32_t>> out;
  std::map<std::pair<bool, std::vector<uint32_t>>, size_t> open;  // kind gate -> its group still taking members
  for (uint32_t k : crules) {
    KindGate g = rule_gate(rs, rs.rules[k]);
    std::sort(g.kinds.begin(), g.kinds.end());
    g.kinds.erase(std::unique(g.kinds.begin(), g.kinds.end()), g.kinds.end());
    if (g.any) g.kinds.clear();
    const auto key = std::make_pair(g.any, g.kinds);
    auto it = open.find(key);
    if (it == open.end() || out[it->second].size() >= 8) {
      open[key] = out.size();
      out.push_back({});
      it = open.find(key);
    }
    out[it->second].push_back(k);
  }
  return out;
}

std::vector<char> jit_compile_uncached(const std::string& src, double* seconds, bool acct);

namespace {
uint64_t fnv1a(const std::string& s, uint64_t h = 1469598103934665603ull) {
  for (unsigned char c : s) { h ^= c; h *= 1099511628211ull; }
  return h;
}
std::string read_file(const std::string& path) {
  FILE* f = fopen(path.c_str(), "rb");
  if (!f) return "";
  std::string out;
  char buf[65536];
  size_t n;
  while ((n = fread(buf, 1, sizeof buf, f)) > 0) out.append(buf, n);
  fclose(f);
  return out;
}
// On-disk code-object cache: a ruleset's walk kernel is compiled once per (generated source, device headers,
// compile options) and reused by every later process (first evaluation seconds instead of a ~20 s hipRTC compile).
// KYV_JIT_CACHE overrides the directory (default <library dir>/jitcache); "0" disables it.
std::string cache_path(const std::string& src, bool acct) {
  const char* env = getenv("KYV_JIT_CACHE");
  if (env && std::string(env) == "0") return "";
  std::string dir = env ? std::string(env) : self_dir() + "/jitcache";
  const char* cs = getenv("KYV_CSRC");
  std::string csrc = cs ? std::string(cs) : self_dir() + "/csrc";
  // name = walk-<toolchain hash>-<source hash>.co: the first part covers the device headers, compile options and
  // the hipRTC version, so a cache prune can drop exactly the entries older sources produced
  uint64_t h = fnv1a("");
  for (const char* hdr : {"kyv_layout.h", "kyv_eval.h", "kyv_cond.h", "kyv_pss.h", "kyv_wave.h", "kyv_walk.h", "kyv_jcond.h",
                          "kyv_fused.h"})
    h = fnv1a(read_file(csrc + "/" + hdr), h);
  h = fnv1a(std::string(acct ? "acct|" : "") + "gfx950|O3|c++17|wpe=" + (getenv("KYV_JIT_WPE") ? getenv("KYV_JIT_WPE") : "4") + "|" +
                (getenv("KYV_JIT_DEFS") ? getenv("KYV_JIT_DEFS") : "-DKYV_JIT_NOEXTRA"), h);
  int maj = 0, min = 0;
  hiprtcVersion(&maj, &min);
  h = fnv1a(std::to_string(maj) + "." + std::to_string(min), h);
  char name[80];
  snprintf(name, sizeof name, "/%s-%08llx-%016llx.co", acct ? "acct" : "walk", (unsigned long long)(h >> 32),
           (unsigned long long)fnv1a(src));
  return dir + name;
}
}  // namespace

// hipRTC compile of the generated source for gfx950 -> code object (acct: the byte-accounting build, -DKYV_ACCT)
std::vector<char> jit_compile(const std::string& src, double* seconds, bool acct) {
  // process-wide cache: identical rulesets (same generated source) compile once
  static std::mutex mu;
  static std::unordered_map<std::string, std::vector<char>> cache;
  const std::string ckey = (acct ? "A" : "P") + src;
  {
    std::lock_guard<std::mutex> lk(mu);
    auto it = cache.find(ckey);
    if (it != cache.end()) { if (seconds) *seconds = 0; return it->second; }
  }
  const std::string path = cache_path(src, acct);
  std::vector<char> code;
  if (!path.empty()) {
    std::string blob = read_file(path);
    if (blob.size() > 64) {  // written whole (temp file + rename)
      code.assign(blob.begin(), blob.end());
      if (seconds) *seconds = 0;
      utime(path.c_str(), nullptr);  // last use (build() keeps the newest entry's toolchain generation)
    }
  }
  if (code.empty()) {
    code = jit_compile_uncached(src, seconds, acct);
    if (!path.empty()) {  // best effort: a read-only tree just recompiles next time
      std::string dir = path.substr(0, path.rfind('/'));
      mkdir(dir.c_str(), 0755);
      std::string tmp = path + ".tmp" + std::to_string((unsigned long long)getpid());
      if (FILE* f = fopen(tmp.c_str(), "wb")) {
        bool ok = fwrite(code.data(), 1, code.size(), f) == code.size();
        ok = fclose(f) == 0 && ok;
        if (!ok || rename(tmp.c_str(), path.c_str()) != 0) remove(tmp.c_str());
      }
    }
  }
  std::lock_guard<std::mutex> lk(mu);
  cache.emplace(ckey, code);
  return code;
}

std::vector<char> jit_compile_uncached(const std::string& src, double* seconds, bool acct) {
  auto t0 = std::chrono::steady_clock::now();
  std::string dir = self_dir();
  const char* env = getenv("KYV_CSRC");
  std::string inc = "-I" + (env ? std::string(env) : dir + "/csrc");
  std::string inc2 = "-I" + dir + "/../include";
  std::string wpe = std::string("-DKYV_JIT_WPE=") + (getenv("KYV_JIT_WPE") ? getenv("KYV_JIT_WPE") : "4");
  std::string extra = getenv("KYV_JIT_DEFS") ? getenv("KYV_JIT_DEFS") : "-DKYV_JIT_NOEXTRA";  // experiments only
  const char* opts[] = {"--offload-arch=gfx950", "-O3", "-std=c++17", inc.c_str(), inc2.c_str(), wpe.c_str(), extra.c_str(),
                        "-DKYV_ACCT=1"};
  hiprtcProgram prog;
  if (hiprtcCreateProgram(&prog, src.c_str(), "kyv_jit_walk.hip", 0, nullptr, nullptr) != HIPRTC_SUCCESS)
    throw std::runtime_error("hiprtcCreateProgram failed");
  hiprtcResult r = hiprtcCompileProgram(prog, acct ? 8 : 7, opts);
  if (r != HIPRTC_SUCCESS) {
    size_t ls = 0;
    hiprtcGetProgramLogSize(prog, &ls);
    std::string log(ls + 1, '\0');
    hiprtcGetProgramLog(prog, &log[0]);
    hiprtcDestroyProgram(&prog);
    throw std::runtime_error("hipRTC compile of the ruleset walk kernel failed: " + log.substr(0, 4000));
  }
  size_t cs = 0;
  hiprtcGetCodeSize(prog, &cs);
  std::vector<char> code(cs);
  hiprtcGetCode(prog, code.data());
  hiprtcDestroyProgram(&prog);
  if (seconds) *seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  return code;
}

}  // namespace kyv
