// Wave-uniform pattern walker (device only): the MI355X execution of validate.MatchPattern.
//
// Same semantics as eval_pattern (kyv_eval.h, the per-lane restatement of pkg/engine/validate/validate.go:31-247
// with anchor/handlers.go, anchormap.go, error.go), organised for a 64-wide wavefront whose lanes hold 64
// different resources walking ONE compiled pattern:
//
//  * the program position (pattern node, map entry, array element, existence candidate) is wave-uniform, so
//    control flow is scalar branches and the program is read with scalar loads (s_load through the
//    constant address space) instead of per-lane vector loads;
//  * which lanes take part in a step is a uniform 64-bit mask (ballot); a lane that leaves a frame early
//    (its error ends validateMap / validateArray for that resource) just drops out of the frame's `alive`
//    mask and keeps its per-lane return value until the frame pops;
//  * the top frame lives in registers; deeper frames are spilled to LDS only on push/pop: the uniform part
//    once per wave, the per-lane part (child range + array state) lane-strided and conflict-free;
//  * map lookups of static key paths read the batch's path columns (kyv_layout.h): one coalesced 4-byte
//    load per lane that also carries the child's type, so most maps are entered without touching their row;
//    dynamic keys (metadata wildcards) binary-search the key-sorted children; rows use global (not flat) loads.
//
// Every per-lane side effect (return value, anchor map, array indices, metadata keys) happens only for lanes
// inside the step's mask, so each lane sees exactly the sequence of operations the per-lane walk performs.
#pragma once
#include "kyv_eval.h"
#include "kyv_walk.h"

namespace kyv {

#define KYV_AS_CONST __attribute__((address_space(4)))
#define KYV_AS_GLOBAL __attribute__((address_space(1)))

// word-wise loads so that uniform addresses become s_load (constant AS) and per-lane ones global_load
template <class T>
__device__ __forceinline__ T sld(const T* p) {
  static_assert(sizeof(T) % 4 == 0, "sld: 4-byte multiple");
  uint32_t w[sizeof(T) / 4];
  const KYV_AS_CONST uint32_t* q = (const KYV_AS_CONST uint32_t*)p;
#pragma unroll
  for (int i = 0; i < (int)(sizeof(T) / 4); i++) w[i] = q[i];
  T out;
  __builtin_memcpy(&out, w, sizeof(T));  // no type punning through uint32_t* (strict aliasing)
  return out;
}
__device__ __forceinline__ uint32_t sld32(const uint32_t* p) { return *(const KYV_AS_CONST uint32_t*)p; }
typedef uint32_t kyv_u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ Node gnode(const Node* p) {
  KYV_ACCT_ADDK(1u, 0, 16);
  const KYV_AS_GLOBAL kyv_u32x4* q = (const KYV_AS_GLOBAL kyv_u32x4*)p;
  kyv_u32x4 x = *q;
  Node n;
  n.tk = x.x; n.a = x.y; n.b = x.z; n.c = x.w;
  return n;
}
__device__ __forceinline__ uint32_t gtk(const Node* p) {
  KYV_ACCT_ADDK(1u, 0, 4);
  return *(const KYV_AS_GLOBAL uint32_t*)p;
}
__device__ __forceinline__ uint32_t uni(uint32_t x) { return __builtin_amdgcn_readfirstlane(x); }
__device__ __forceinline__ uint64_t uni64(uint64_t x) {
  return ((uint64_t)uni((uint32_t)(x >> 32)) << 32) | uni((uint32_t)x);
}
__device__ __forceinline__ uint64_t wballot(bool p) { return __ballot(p); }

// binary search over the key-sorted children [a, a+n) of a map (rows relative to the resource root)
__device__ __forceinline__ uint32_t wmap_find(const Node* R, uint32_t a, uint32_t n, uint32_t key) {
  uint32_t lo = a, hi = a + n;
  while (lo < hi) {
    uint32_t mid = (lo + hi) >> 1;
    uint32_t k = gtk(R + mid) >> 4;
    if (k == key) return mid;
    if (k < key) lo = mid + 1; else hi = mid;
  }
  return NONE;
}

constexpr uint32_t T_UNK = 0xE;  // node type not known yet (row not loaded)

__device__ __forceinline__ uint32_t gld32(const uint32_t* p) { return *(const KYV_AS_GLOBAL uint32_t*)p; }

// Column entry of one map-entry lookup (the device entry table holds absolute column offsets in `col`)
__device__ __forceinline__ uint32_t wcol(const View& v, const PEntry& E, bool al, uint32_t row) {
  if (al) KYV_ACCT_ADDK(2u, 0, 4);
  return al ? gld32((const uint32_t*)(v.colv + (size_t)E.col + row)) : NONE;
}
__device__ __forceinline__ uint32_t col_decode(uint32_t enc, uint32_t* ctype) {
  if (enc == NONE) { *ctype = T_UNK; return NONE; }
  *ctype = enc >> COL_TYPE_SHIFT;
  return enc & COL_INDEX_MASK;
}
// resourceMap[key] for one map entry: a path-column read (one coalesced 4-B load per lane, node type included)
// when the compiler gave the entry a column, else a binary search over the map's key-sorted children
__device__ __forceinline__ uint32_t wlookup(const View& v, const PEntry& E, bool al, const Node* R, uint32_t a, uint32_t b,
                                            uint32_t row, const Keys& keys, uint32_t* ctype) {
  *ctype = T_UNK;
  if (!al) return NONE;
  if (E.col != NONE) return col_decode(wcol(v, E, al, row), ctype);
  uint32_t key = (E.flags & EF_WILD) ? keys.get(E.slot) : E.key;
  return wmap_find(R, a, b, key);
}

__device__ __forceinline__ Val wvalue_node(const View& v, Node n) {
  Val x;
  x.wsid = NONE; x.nsid = NONE; x.sid = NONE; x.i = 0; x.f = 0;
  x.t = node_type(n);
  switch (x.t) {
    case N_NULL: x.nsid = SID_ZERO; break;
    case N_FALSE: x.wsid = SID_FALSE; break;
    case N_TRUE: x.wsid = SID_TRUE; break;
    case N_INT: x.i = (int64_t)(((uint64_t)n.b << 32) | n.a); x.wsid = n.c; x.nsid = n.c; break;
    case N_FLOAT: {
      uint64_t bits = ((uint64_t)n.b << 32) | n.a;
      x.f = __builtin_bit_cast(double, bits);
      x.wsid = gld32(&v.faux[n.c].sid_E);
      x.nsid = gld32(&v.faux[n.c].sid_F);
      break;
    }
    case N_STR: x.sid = n.a; x.wsid = n.a; x.nsid = n.a; break;
    default: break;
  }
  return x;
}
__device__ __forceinline__ Val wvalue_absent() {
  Val x;
  x.t = 0xFF; x.wsid = NONE; x.nsid = SID_ZERO; x.sid = NONE; x.i = 0; x.f = 0;
  return x;
}
__device__ __forceinline__ Val wvalue_of(const View& v, const Node* R, uint32_t rn) {
  return rn == NONE ? wvalue_absent() : wvalue_node(v, gnode(R + rn));
}

// ---------------------------------------------------------------- leaves (pattern.go:26-321), wave form
// The leaf / atom program is wave-uniform (scalar loads); only the value side is per lane. Same evaluation
// order as leaf_match / atom_eval (kyv_eval.h): a lane evaluates atom k of group g exactly when no earlier
// group matched and every earlier atom of group g matched, so the fallback flag is raised identically.
__device__ __forceinline__ uint8_t gld8(const uint8_t* p) { return *(const KYV_AS_GLOBAL uint8_t*)p; }
__device__ __forceinline__ bool wbytes_eq(const uint8_t* a, const uint8_t* b, uint32_t n) {
  for (uint32_t i = 0; i < n; i++) if (gld8(a + i) != gld8(b + i)) return false;
  return true;
}
__device__ __forceinline__ bool wglob(const View& v, uint8_t kind, uint32_t pat, uint32_t lit, uint32_t s,
                                      uint32_t gi1 = 0) {
  if (gi1 && v.str_gmask) return gmask_bit(v, gi1, s);  // precomputed per batch (prefix/suffix/contains/general)
  switch (kind) {
    case G_ANY: return true;
    case G_EMPTY: return s == SID_EMPTY;
    case G_EXACT: return s == pat;
    case G_NONEMPTY: return gld32(v.str_len + s) > 0;
    case G_PREFIX: case G_SUFFIX: case G_CONTAINS: {
      const uint32_t ln = gld32(v.str_len + lit), sn = gld32(v.str_len + s);
      if (ln > sn) return false;
      const uint8_t* a = v.heap + gld32(v.str_off + s);
      const uint8_t* b = v.heap + gld32(v.str_off + lit);
      if (kind == G_PREFIX) return wbytes_eq(a, b, ln);
      if (kind == G_SUFFIX) return wbytes_eq(a + (sn - ln), b, ln);
      for (uint32_t i = 0; i + ln <= sn; i++) if (wbytes_eq(a + i, b, ln)) return true;
      return false;
    }
    default: return glob_runes(sbytes(v, pat), v.str_len[pat], sbytes(v, s), v.str_len[s]);
  }
}
__device__ __forceinline__ bool watom_simple(const View& v, const Atom& a, const Val& x, bool* fb) {
  if ((a.flags & AF_DUR) && x.nsid != NONE && (gld32(v.str_flags + x.nsid) & SF_DUR)) {
    int64_t d = *(const KYV_AS_GLOBAL int64_t*)(v.str_dur + x.nsid);
    if (cmp_op(a.op, d < a.dur ? -1 : (d > a.dur ? 1 : 0))) return true;
  }
  if ((a.flags & AF_QTY) && x.nsid != NONE) {
    uint32_t f = gld32(v.str_flags + x.nsid);
    if (f & SF_QTY_BIG) { *fb = true; return false; }
    if (f & SF_QTY) {
      const KYV_AS_GLOBAL int64_t* q = (const KYV_AS_GLOBAL int64_t*)(v.str_qty + 2 * (size_t)x.nsid);
      int c = cmp128(q[1], (uint64_t)q[0], a.qhi, (uint64_t)a.qlo);
      if (cmp_op(a.op, c)) return true;
    }
  }
  if ((a.op == A_EQ || a.op == A_NE) && x.wsid != NONE) {
    bool r = wglob(v, a.glob, a.pat, a.lit, x.wsid, a.gidx);
    return a.op == A_NE ? !r : r;
  }
  return false;
}
// pattern.Validate(value, pattern) for the lanes with `go`
__device__ __forceinline__ bool wleaf_match(const View& v, const Leaf& L, bool go, const Val& x, bool* fb) {
  switch (L.type) {
    case L_NIL:
      switch (x.t) {
        case 0xFF: case N_NULL: case N_FALSE: return true;
        case N_INT: return x.i == 0;
        case N_FLOAT: return x.f == 0.0;
        case N_STR: return x.sid == SID_EMPTY;
        default: return false;
      }
    case L_BOOL: return (x.t == N_TRUE && L.bval) || (x.t == N_FALSE && !L.bval);
    case L_FLOAT:
      switch (x.t) {
        case N_INT: return L.fint && L.fi == x.i;
        case N_FLOAT: return x.f == L.f;
        case N_STR: return go && (gld32(v.str_flags + x.sid) & SF_FLOAT) &&
                           *(const KYV_AS_GLOBAL double*)(v.str_f64 + x.sid) == L.f;
        default: return false;
      }
    case L_STR: {
      bool done = x.t == N_STR && x.sid == L.exact;
      for (uint32_t g = 0; g < L.ngroups; g++) {
        const uint32_t a0 = sld32(v.pool + L.groups + 2 * g), na = sld32(v.pool + L.groups + 2 * g + 1);
        bool all = go && !done;
        for (uint32_t k = 0; k < na; k++) {
          const Atom A = sld(v.atoms + a0 + k);
          if (A.op == A_RANGE_IN || A.op == A_RANGE_OUT) {
            const Atom s0 = sld(v.atoms + A.sub), s1 = sld(v.atoms + A.sub + 1);
            if (all) {
              bool r0 = watom_simple(v, s0, x, fb);
              all = A.op == A_RANGE_IN ? (r0 && watom_simple(v, s1, x, fb)) : (r0 || watom_simple(v, s1, x, fb));
            }
          } else if (A.op == A_FALSE) {
            all = false;
          } else if (all) {
            all = watom_simple(v, A, x, fb);
          }
        }
        if (all) done = true;
      }
      return done;
    }
    case L_MAP: return x.t == N_MAP;
    default: return false;
  }
}

// per-lane part of a spilled frame: child range of the map / array node + array-frame state + column row
struct LaneFrame {
  uint32_t a;     // first child row
  uint32_t bst;   // child count (low 16) | FrameSt bits << 16
  uint32_t row;   // map: its row in the path-column row space; array: row of element 0
  uint32_t pad;
};
// uniform part of a spilled frame
struct UFrame {
  uint32_t kind, pn, i, j;
  uint64_t alive, cmask, search;
  uint64_t pad;
};
static_assert(sizeof(UFrame) == 48, "UFrame");

#ifdef KYV_EXP_STEPS
__device__ unsigned long long kyv_exp_steps;
#endif
struct WaveWalker {
  LaneFrame* lf;   // LDS, [cap][64]
  UFrame* uf;      // LDS, [cap]
  int cap;
  bool rootmap;    // per lane (unused by the interpreter)

  __device__ void run(const View& v, uint32_t root, bool walk, const Node* R, const ResHeader* hp, uint32_t row,
                      const RuleDesc& rd, PatOut& out) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t lbit = 1ull << lane;
    uint64_t seen = 0, found = 0;
    Keys keys{NONE, NONE};
    out.idx = 0;
    out.tmpl = NONE;
    out.key0 = NONE;
    out.key1 = NONE;
    Ret ret = ok_ret();
    uint8_t ost = ST_NONE;
    uint64_t dead = 0;
    uint64_t emask = wballot(walk);
    if (!emask) { out.status = ST_NONE; return; }
#ifdef KYV_EXP_NOWALK
    out.status = walk ? ST_PASS : ST_NONE;
    return;
#endif
    const uint32_t meta_base = rd.meta_sites;

    int sp = 0;
    // top frame (uniform)
    uint32_t t_kind = 0, t_pn = 0, t_i = 0, t_j = 0;
    uint64_t t_alive = 0, t_cmask = 0, t_search = 0;
    // top frame (per lane)
    uint32_t t_a = 0, t_b = 0, t_st = 0, t_row = 0;

    int action = 0;
    uint32_t epn = root, ern = 0;
    uint32_t etype = T_UNK;        // per lane: type of the node being entered, when a column supplied it
    uint32_t erow = row == NONE ? 0u : row;  // per lane: column row of the node being entered (root: the resource)

#define KYV_PUSH(KIND, PN, ALIVE, A, B, ROW)                                                   \
  do {                                                                                      \
    if (sp > 0) {                                                                           \
      if (lane == 0) {                                                                      \
        UFrame& u = uf[sp - 1];                                                             \
        u.kind = t_kind; u.pn = t_pn; u.i = t_i; u.j = t_j;                                 \
        u.alive = t_alive; u.cmask = t_cmask; u.search = t_search;                          \
      }                                                                                     \
      LaneFrame& l = lf[(uint32_t)(sp - 1) * 64u + lane];                                   \
      l.a = t_a; l.bst = (t_b & 0xFFFFu) | (t_st << 16); l.row = t_row;                  \
    }                                                                                       \
    t_kind = (KIND); t_pn = (PN); t_i = 0; t_j = 0;                                         \
    t_alive = (ALIVE); t_cmask = 0; t_search = (ALIVE);                                     \
    t_a = (A); t_b = (B); t_st = 0; t_row = (ROW);                                          \
    sp++;                                                                                   \
  } while (0)

#define KYV_POP()                                                                           \
  do {                                                                                      \
    sp--;                                                                                   \
    if (sp > 0) {                                                                           \
      const UFrame& u = uf[sp - 1];                                                         \
      t_kind = uni(u.kind); t_pn = uni(u.pn); t_i = uni(u.i); t_j = uni(u.j);               \
      t_alive = uni64(u.alive); t_cmask = uni64(u.cmask); t_search = uni64(u.search);       \
      LaneFrame l = lf[(uint32_t)(sp - 1) * 64u + lane];                                    \
      t_a = l.a; t_b = l.bst & 0xFFFFu; t_st = l.bst >> 16; t_row = l.row;                  \
    }                                                                                       \
  } while (0)

#ifdef KYV_EXP_STEPS
    uint32_t nsteps = 0;
#endif
    for (;;) {
#ifdef KYV_EXP_STEPS
      nsteps++;
#endif
      if (action == 0) {
        // ---------------------------------------------------------------- enter epn for lanes in emask
        const PNode P = sld(v.pn + epn);
        const bool in = (emask & lbit) != 0;
        uint32_t rt = 0xFF;
        Node rnode{0, 0, 0, 0};
        // maps whose entries all have path columns never need their own row (type came with the column)
        const bool needrow = P.kind != P_MAP || (P.flags & PF_NEEDROW);
        if (in && ern != NONE) {
          if (needrow || etype == T_UNK) { rnode = gnode(R + ern); rt = node_type(rnode); }
          else rt = etype;
        }
        if (P.kind == P_MAP) {
          uint64_t bad = wballot(in && rt != N_MAP);
          if (bad & lbit) ret = mkerr(EC_NONE, 0, P.tmpl);
          uint64_t go = emask & ~bad;
          if (go) {
            // AnchorMap.CheckAnchorInResource (anchormap.go:30-44)
            for (uint32_t e = 0; e < P.n; e++) {
              const PEntry E = sld(v.pe + P.first + e);
              if (E.abit != 0xFF) {
                const uint64_t b = 1ull << E.abit;
                const bool chk = (go & lbit) && !(found & b);
                uint32_t ct, c;
                if (go & lbit) seen |= b;
                c = wlookup(v, E, chk, R, rnode.a, rnode.b, erow, keys, &ct);
                if (c != NONE) found |= b;
              }
            }
            if (P.flags & PF_META) {
              uint8_t o = ST_NONE;
              if (go & lbit) o = expand_meta(v, v.metas[meta_base + P.meta], NodeTab{R}, ern, *hp, keys);
              uint64_t d = wballot(o != ST_NONE);
              if (d & lbit) ost = o;
              dead |= d;
              go &= ~d;
            }
            if (go && sp >= cap) {
              if (go & lbit) ost = ST_FALLBACK;
              dead |= go;
              go = 0;
            }
          }
          if (go) {
            KYV_PUSH(F_MAP, epn, go, rnode.a, rnode.b, erow);
            action = 1;
          } else {
            action = 2;
          }
          continue;
        }
        if (P.kind == P_LEAF || P.kind == P_ARR_SCALAR) {
          // pattern.Validate on the value, or on each element (scalar pattern vs resource array,
          // validate.go:96-102; scalar-element pattern array, validate.go:163-214): one leaf_match site
          uint64_t bad = 0;
          uint32_t leaf = P.first;
          if (P.kind == P_ARR_SCALAR) {
            bad = wballot(in && rt != N_ARR);
            if (bad & lbit) ret = mkerr(EC_NONE, 0, P.tmpl);
            leaf = sld(v.pn + P.first).first;
          }
          const Leaf L = sld(v.leaves + leaf);
          const bool go = in && !(bad & lbit);
          const bool each = rt == N_ARR;
          const uint32_t cnt = go ? (each ? rnode.b : 1u) : 0u;
          bool fb = false, okv = true;
          for (uint32_t i = 0; i < cnt && okv; i++) okv = wleaf_match(v, L, true, wvalue_of(v, R, each ? rnode.a + i : ern), &fb);
          uint64_t d = wballot(go && fb);
          if (d & lbit) ost = ST_FALLBACK;
          dead |= d;
          if (go && !fb) ret = okv ? ok_ret() : mkerr(EC_NONE, 0, P.tmpl);
          action = 2;
          continue;
        }
        // arrays
        uint64_t bad = wballot(in && (rt != N_ARR || P.kind == P_ARR_EMPTY));
        if (bad & lbit) ret = mkerr(EC_NONE, 0, P.tmpl);
        uint64_t go = emask & ~bad;
        if (P.kind == P_ARR_POS) {
          uint64_t shortl = wballot((go & lbit) && rnode.b < P.n);
          if (shortl & lbit) ret = mkerr(EC_NONE, 0, NONE);
          go &= ~shortl;
        }
        if (go && sp >= cap) {
          if (go & lbit) ost = ST_FALLBACK;
          dead |= go;
          go = 0;
        }
        if (go) {
          KYV_PUSH(P.kind == P_ARR_MAPS ? F_AOM : F_POS, epn, go, rnode.a, rnode.b, rnode.c);
          action = 1;
        } else {
          action = 2;
        }
        continue;
      }

      if (action == 1) {
        // ---------------------------------------------------------------- next step of the top frame
        if (t_kind == F_MAP) {
          const PNode P = sld(v.pn + t_pn);
          const uint64_t alive = t_alive & ~dead;
          if (t_i == P.n || !alive) {
            if (alive & lbit) ret = ok_ret();
            KYV_POP();
            action = 2;
            continue;
          }
          const PEntry E = sld(v.pe + P.first + t_i);
          t_i++;
          const bool al = (alive & lbit) != 0;
          uint32_t ct, c;
          c = wlookup(v, E, al, R, t_a, t_b, t_row, keys, &ct);
          t_alive = alive;
          switch (E.handler) {
            case H_NEGATION: {
              uint64_t hit = wballot(al && c != NONE);
              if (hit & lbit) ret = mkerr(EC_NEG, PH_NEG, E.tmpl);
              t_alive &= ~hit;
              continue;
            }
            case H_EQUALITY: case H_GLOBAL: {
              uint64_t ent = wballot(al && c != NONE);
              if (ent) { t_cmask = ent; emask = ent; epn = E.child; ern = c; etype = ct; erow = t_row; action = 0; }
              continue;
            }
            case H_CONDITION: {
              uint64_t pres = wballot(al && c != NONE);
              uint64_t absent = alive & ~pres;
              if (absent & lbit) ret = mkerr(EC_COND, PH_COND, E.tmpl);
              t_alive &= ~absent;
              if (pres) { t_cmask = pres; emask = pres; epn = E.child; ern = c; etype = ct; erow = t_row; action = 0; }
              continue;
            }
            case H_STAR: {
              bool isnull = false;
              if (al && c != NONE) isnull = (ct != T_UNK ? ct : node_type(gnode(R + c))) == N_NULL;
              uint64_t badl = wballot(al && (c == NONE || isnull));
              if (badl & lbit) ret = mkerr(EC_NONE, 0, P.tmpl);  // dh.path: the parent path
              t_alive &= ~badl;
              continue;
            }
            case H_EXISTENCE: case H_EXIST_BADPAT: {
              Node cn{0, 0, 0, 0};
              const bool pres = al && c != NONE;
              if (pres) cn = gnode(R + c);
              const bool arr = pres && node_type(cn) == N_ARR && E.handler == H_EXISTENCE;
              uint64_t badl = wballot(pres && !arr);
              if (badl & lbit) ret = mkerr(EC_NONE, 0, E.tmpl);
              t_alive &= ~badl;
              uint64_t ex = wballot(arr);
              if (ex) {
                if (sp >= cap) {
                  if (ex & lbit) ost = ST_FALLBACK;
                  dead |= ex;
                  continue;
                }
                t_cmask = ex;
                KYV_PUSH(F_EXIST, P.first + t_i - 1, ex, cn.a, cn.b, cn.c);
              }
              continue;
            }
            default: {  // H_DEFAULT: recurse on resourceMap[k] (absent -> nil)
              t_cmask = alive; emask = alive; epn = E.child; ern = c; etype = ct; erow = t_row; action = 0;
              continue;
            }
          }
        }
        if (t_kind == F_AOM || t_kind == F_POS) {
          const PNode P = sld(v.pn + t_pn);
          const uint64_t alive = t_alive & ~dead;
          const uint32_t n = t_kind == F_AOM ? t_b : P.n;
          const uint64_t part = wballot((alive & lbit) && t_i < n);
          if (!part) {
            if (alive & lbit) {
              if ((t_st & FS_SKIP) && !(t_st & FS_APPLY)) ret = mkerr(EC_NONE, (uint8_t)(t_st >> 2), P.tmpl);
              else ret = ok_ret();
            }
            KYV_POP();
            action = 2;
            continue;
          }
          if (part & lbit) {
            if (t_kind == F_AOM) {
              uint32_t sh = 16u * P.level;
              out.idx = (out.idx & ~(0xFFFFull << sh)) | ((uint64_t)t_i << sh);
            }
            ern = t_a + t_i;
            erow = t_row == NONE ? NONE : t_row + t_i;
            etype = T_UNK;
          }
          epn = t_kind == F_AOM ? P.first : sld32(v.pool + P.first + t_i);
          t_i++;
          t_alive = alive;
          t_cmask = part;
          emask = part;
          action = 0;
          continue;
        }
        // F_EXIST: entry index in t_pn; candidate pattern maps in pool[E.child + 1 ..]
        {
          const PEntry E = sld(v.pe + t_pn);
          const uint32_t npat = sld32(v.pool + E.child);
          uint64_t alive = t_alive & ~dead;
          uint64_t search = t_search & alive;
          if (t_j == npat || !alive) {
            if (alive & lbit) ret = ok_ret();
            KYV_POP();
            action = 2;
            continue;
          }
          uint64_t exh = wballot((search & lbit) && t_i >= t_b);
          if (exh & lbit) ret = mkerr(EC_NONE, 0, E.tmpl);
          alive &= ~exh;
          search &= ~exh;
          t_alive = alive;
          if (!search) {  // every lane still alive found a match for pattern j
            t_j++;
            t_i = 0;
            t_search = alive;
            continue;
          }
          epn = sld32(v.pool + E.child + 1 + t_j);
          if (search & lbit) {
            ern = t_a + t_i;
            erow = t_row == NONE ? NONE : t_row + t_i;
            etype = T_UNK;
          }
          t_i++;
          t_search = search;
          t_cmask = search;
          emask = search;
          action = 0;
          continue;
        }
      }

      // ---------------------------------------------------------------- action 2: deliver ret to the top frame
      if (sp == 0) break;
      {
        const uint64_t cm = t_cmask & ~dead;
        const bool cin = (cm & lbit) != 0;
        if (t_kind == F_MAP) {
          uint64_t errl = wballot(cin && ret.err);
          if (errl) {
            const PNode P = sld(v.pn + t_pn);
            const PEntry E = sld(v.pe + P.first + t_i - 1);
            if (errl & lbit) {
              if (E.handler == H_CONDITION) { ret.code = EC_COND; ret.mask |= PH_COND; }
              else if (E.handler == H_GLOBAL) { ret.code = EC_GLOBAL; ret.mask |= PH_GLOBAL; }
            }
            t_alive &= ~errl;
          }
        } else if (t_kind == F_AOM || t_kind == F_POS) {
          const bool e = cin && ret.err;
          const bool sk = e && ret_is_skip(ret);
          if (sk) t_st |= FS_SKIP | ((uint32_t)ret.mask << 2);
          if (cin && !ret.err) t_st |= FS_APPLY;
          t_alive &= ~wballot(e && !sk);
        } else {  // F_EXIST: lanes whose candidate matched stop searching for pattern j
          t_search &= ~wballot(cin && !ret.err);
        }
        action = 1;
      }
    }
#undef KYV_PUSH
#undef KYV_POP
#ifdef KYV_EXP_STEPS
    if (lane == 0) atomicAdd(&kyv_exp_steps, (unsigned long long)nsteps);
#endif

    out.key0 = keys.k0;
    out.key1 = keys.k1;
    if (!walk) { out.status = ST_NONE; return; }
    if (dead & lbit) { out.status = ost; return; }
    if (!ret.err) { out.status = ST_PASS; out.tmpl = NONE; return; }
    if (ret_is_skip(ret)) { out.status = ST_SKIP; out.tmpl = NONE; return; }
    if (ret_is_neg(ret)) { out.status = ST_FAIL; out.tmpl = ret.tmpl; return; }
    if (seen & ~found) { out.status = ST_ERROR; out.tmpl = NONE; return; }
    out.tmpl = ret.tmpl;
    out.status = ret.tmpl == NONE ? ST_ERROR : ST_FAIL;
  }
};

// ---------------------------------------------------------------- runtime-compiled walkers (jit.cpp)
// Per-lane state of one compiled pattern walk. The generated code is the per-lane recursion of eval_pattern
// (kyv_eval.h) unrolled over one pattern: one inlined function per pattern node, arrays as loops, errors as
// return values; `ost` != ST_NONE ends the walk with that status (fallback / panic / nondeterministic).
struct JW {
  const View& v;
  const Node* R;
  const ResHeader* hp;
  uint64_t seen, found;  // AnchorMap (anchormap.go)
  Keys keys;             // resolved metadata wildcard keys (wildcards.go)
  uint64_t idx;          // array indices of the failing path
  uint32_t mbase;        // rule's first metadata-expansion site
  uint8_t ost;
};
// one simple comparison with the atom's operator, flags and glob class as template constants (the generated
// leaf code instantiates exactly the branches watom_simple would take for that atom)
template <uint8_t OP, uint8_t FLAGS, uint8_t GLOB, uint32_t GI1 = 0>
__device__ __forceinline__ bool jatom(const View& v, const Val& x, uint32_t pat, uint32_t lit, int64_t dur, int64_t qlo,
                                      int64_t qhi, bool* fb) {
  if ((FLAGS & AF_DUR) && x.nsid != NONE && (gld32(v.str_flags + x.nsid) & SF_DUR)) {
    int64_t d = *(const KYV_AS_GLOBAL int64_t*)(v.str_dur + x.nsid);
    if (cmp_op(OP, d < dur ? -1 : (d > dur ? 1 : 0))) return true;
  }
  if ((FLAGS & AF_QTY) && x.nsid != NONE) {
    uint32_t f = gld32(v.str_flags + x.nsid);
    if (f & SF_QTY_BIG) { *fb = true; return false; }
    if (f & SF_QTY) {
      const KYV_AS_GLOBAL int64_t* q = (const KYV_AS_GLOBAL int64_t*)(v.str_qty + 2 * (size_t)x.nsid);
      if (cmp_op(OP, cmp128(q[1], (uint64_t)q[0], qhi, (uint64_t)qlo))) return true;
    }
  }
  if ((OP == A_EQ || OP == A_NE) && x.wsid != NONE) {
    bool r = wglob(v, GLOB, pat, lit, x.wsid, GI1);
    return OP == A_NE ? !r : r;
  }
  return false;
}
constexpr uint64_t COL_NONE = 0xFFFFFFFFull;
// raw 8-byte column entry of a lookup (speculative preload of a column scope; NONE rows give COL_NONE); the
// device entry table holds the column's absolute offset in `col`
__device__ __forceinline__ uint64_t jraw(const JW& w, uint32_t e, uint32_t row) {
  const uint32_t off = sld32(&w.v.pe[e].col);
  if (row != NONE) KYV_ACCT_ADDK(4u, 0, 8);
  return row == NONE ? COL_NONE : *(const KYV_AS_GLOBAL uint64_t*)(w.v.colv + (size_t)off + row);
}
// self column (array elements) by column id
__device__ __forceinline__ uint64_t jself(const JW& w, uint32_t col, uint32_t row) {
  const uint32_t off = sld32(w.v.col_off + col);
  if (row != NONE) KYV_ACCT_ADDK(8u, 0, 8);
  return row == NONE ? COL_NONE : *(const KYV_AS_GLOBAL uint64_t*)(w.v.colv + (size_t)off + row);
}
// entry -> node index (NONE absent), type (T_UNK absent) and the node's `a`
__device__ __forceinline__ uint32_t jdec(uint64_t x, uint32_t* t, uint32_t* a) {
  const uint32_t lo = (uint32_t)x;
  *a = (uint32_t)(x >> 32);
  if (lo == NONE) { *t = T_UNK; return NONE; }
  *t = lo >> COL_TYPE_SHIFT;
  return lo & COL_INDEX_MASK;
}
// value of a node known by (index, type, a): strings, booleans and null need no row read
__device__ __forceinline__ Val jvalue(const JW& w, uint32_t idx, uint32_t t, uint32_t a) {
  if (idx == NONE) return wvalue_absent();
  Val x;
  x.wsid = NONE; x.nsid = NONE; x.sid = NONE; x.i = 0; x.f = 0;
  switch (t) {
    case N_STR: x.t = N_STR; x.sid = a; x.wsid = a; x.nsid = a; return x;
    case N_TRUE: x.t = N_TRUE; x.wsid = SID_TRUE; return x;
    case N_FALSE: x.t = N_FALSE; x.wsid = SID_FALSE; return x;
    case N_NULL: x.t = N_NULL; x.nsid = SID_ZERO; return x;
    default: return wvalue_node(w.v, gnode(w.R + idx));
  }
}
// MatchPattern's classification (validate.go:31-56), as at the end of eval_pattern
__device__ __forceinline__ void jfinish(const JW& w, const Ret& ret, PatOut& out) {
  out.key0 = w.keys.k0;
  out.key1 = w.keys.k1;
  out.idx = w.idx;
  out.tmpl = NONE;
  if (w.ost != ST_NONE) { out.status = w.ost; return; }
  if (!ret.err) { out.status = ST_PASS; return; }
  if (ret_is_skip(ret)) { out.status = ST_SKIP; return; }
  if (ret_is_neg(ret)) { out.status = ST_FAIL; out.tmpl = ret.tmpl; return; }
  if (w.seen & ~w.found) { out.status = ST_ERROR; return; }
  out.tmpl = ret.tmpl;
  out.status = ret.tmpl == NONE ? ST_ERROR : ST_FAIL;
}

// ---------------------------------------------------------------- walk-phase kernel pieces (shared by the
// interpreted walk_kernel and the runtime-compiled per-ruleset kernels of jit.cpp)
constexpr int WAVE = 64;
struct DevOut {
  uint8_t* status;         // [rule][res]
  uint32_t* pss_fails;     // [pss rule slot][res]
  const uint32_t* pss_slot;// rule -> pss slot or NONE
  FailRec* stage;          // failing-path records, staged per walk chunk: chunk (k, w) owns 64 * alts(k) slots
  const uint32_t* rbase;   // [nrules] first staging slot of rule k (its chunks follow, wave-major)
  uint16_t* rcnt;          // [nrules][nwaves] records staged by chunk (k, w)
  uint32_t rule_lo, rule_hi;   // rule slice of this launch: work lists, rbase and rcnt are indexed by k - rule_lo
};

// Shape tables (round 5, jit.cpp kyv_jit_shapes): the walk verdict of each deduplicated pattern shape for every resource
// its users' kind gates admit, and the shape's failing-path record where that verdict is FAIL; read by match_rec_kernel
// (ShapeTab), written by the runtime-compiled kyv_jit_shapes (ShapeOut: per kind class, the shapes to compute)
struct ShapeTab {
  const uint8_t* st;      // [shape][res] verdict byte
  const FailRec* rec;     // [shape][res] failing-path record (valid where the verdict is ST_FAIL; rule field unset)
  uint32_t nwaves;        // match waves of the batch (rcnt row length)
  uint32_t nshapes;
};
struct ShapeOut {
  uint8_t* st;
  FailRec* rec;
  const uint32_t* gate;   // [kind class][words]: bit s = some user of shape s admits the class
  uint32_t words;
  uint32_t nwaves;
};

// Failing-path records of one walk chunk, packed with wave ballots into the chunk's own staging slots (no
// atomics, no waiting); compact_kernel gathers the chunks' records afterwards.
struct WaveSink {
  FailRec* recs;
  uint32_t n;  // wave-uniform
  bool wide;   // wave-uniform: the rule has metadata-expansion sites, records carry keys (whole FailRecs)
  __device__ __forceinline__ void emit(bool has, const FailRec& f) {
#ifdef KYV_EXP_NOSINK
    return;
#endif
    unsigned long long m = __ballot(has);
    if (!m) return;
    const uint32_t lane = threadIdx.x & (WAVE - 1);
    if (has) {
      KYV_ACCT_ADD(2, wide ? sizeof(FailRec) : sizeof(StageRec));  // staged failing-path record
      const uint32_t at = n + (uint32_t)__popcll(m & ((1ull << lane) - 1));
      if (wide) {
        recs[at] = f;
      } else {  // 16-byte StageRec: a wave's records are one contiguous run of 16-byte stores
        StageRec s;
        s.tmpl = f.tmpl;
        s.lane_alt = (f.res & (WAVE - 1)) | ((uint32_t)f.alt << 8);
        for (int i = 0; i < MAX_IDX; i++) s.idx[i] = f.idx[i];
        reinterpret_cast<StageRec*>(recs)[at] = s;
      }
    }
    n += (uint32_t)__popcll(m);
  }
};

// Walk work lists, written by match_kernel without atomics: for rule k and match wave w (64 consecutive
// resources of the kind-major batch), cnt[k][w] pairs need the walk and items[k][w][0..cnt) are their resource
// positions (compacted with a ballot prefix).
constexpr uint32_t ITEM_ROOT_MAP = 1u << 31;  // items[].x: resource position | root-is-a-map flag
struct WorkLists {
  uint2* items;      // [nrules][nwaves][64]: (resource position | ITEM_ROOT_MAP, node offset of its root)
  uint8_t* cnt;      // [nrules][nwaves]
  uint32_t nwaves;
};
__device__ __forceinline__ uint32_t sld8(const uint8_t* p) {  // scalar load of one byte (uniform address)
  const size_t a = (size_t)p;
  return (sld32((const uint32_t*)(a & ~(size_t)3)) >> (8 * (a & 3))) & 0xFFu;
}

// Chunk schedule of a walk kernel, laid out on the host as one (rule, match wave) pair per slot: runs of match
// waves with the same gated rule set, each run wave-major with its rules in windows of a few rules. Slots whose
// work list is empty (no pair matched) are skipped.
struct ChunkMap {
  const uint2* slots;  // [total] (rule, match wave | SLOT_UNIFORM)
  uint32_t total;
};
// slot flag: every resource of the match wave has the same kind class, so a direct-walk (RD_GATE_EXACT) rule the
// schedule lists for the wave gates all of its lanes: the chunk skips the per-lane kind-class -> gate-word loads
constexpr uint32_t SLOT_UNIFORM = 1u << 31;

// Grid-stride over the schedule; every wave walks ONE rule over the (up to 64) resources of one work list;
// verdict bytes and records as in match_kernel (the status counts are one histogram pass afterwards).
template <class Walker>
__device__ __forceinline__ void walk_chunks(const View& v, DevOut o, WorkLists wl, ChunkMap cm, Walker& wk) {
  const uint32_t lane = threadIdx.x & (WAVE - 1);
  // (prefetching the next chunk's slot measured slower: C3 10M walk 9.19 -> 9.52 ms; so did 16-byte slots carrying the
  // rule fields, 9.18 -> 9.43 ms)
  for (uint32_t c = blockIdx.x; c < cm.total; c += gridDim.x) {
    const uint2 kw = sld(cm.slots + c);
    const uint32_t k = kw.x, w = kw.y & ~SLOT_UNIFORM;
    const bool uniform = (kw.y & SLOT_UNIFORM) != 0;
    const size_t list = (size_t)(k - o.rule_lo) * wl.nwaves + w;
    const RuleDesc rd = sld(v.rules + k);
    bool active;
    uint32_t r;
    uint2 it = make_uint2(0u, 0u);
    bool magic = false;
    if (rd.flags & RD_GATE_EXACT) {
      // match == kind gate: the chunk's pairs are the gated lanes of match wave w, read straight from the headers
      r = w * WAVE + lane;
      bool gated = false;
      if (r < v.nres) {
        const ResHeader* h = v.hdr + r;
        const uint32_t fl = gld32(&h->flags);
        if (uniform) {
          gated = true;  // the host checked the wave's (single) kind class against the rule
        } else {
          const uint32_t cls = gld32(&h->kclass);
          gated = (gld32(v.gate + (size_t)cls * v.gate_words + (k >> 5)) >> (k & 31)) & 1u;
        }
        magic = gated && (fl & RF_MAGIC);  // pattern pairs on such resources go to the CPU engine (pair_dispatch)
        if (gated) KYV_ACCT_ADD(0, uniform ? 8 : 12);  // header: flags, root (+ kind class)
        it = make_uint2(r | ((fl & RF_ROOT_MAP) ? ITEM_ROOT_MAP : 0u), gld32(&h->root));
      }
      active = gated && !magic;
      if (!uniform && !__ballot(gated)) continue;
    } else {
      const uint32_t n = sld8(wl.cnt + list);
      if (lane == 0) KYV_ACCT_ADD(0, 1);  // work-list count
      if (!n) continue;
      active = lane < n;
      if (active) { it = wl.items[list * WAVE + lane]; KYV_ACCT_ADD(0, 8); }  // work-list item
      r = it.x & ~ITEM_ROOT_MAP;
    }
    wk.rootmap = (it.x & ITEM_ROOT_MAP) != 0;
    const uint32_t alts = rd.kind == RK_PATTERN ? 1u : min(rd.nalts, (uint32_t)MAX_ALTS);
    WaveSink sink{o.stage + sld32(o.rbase + (k - o.rule_lo)) + (size_t)w * WAVE * alts, 0u, rd.uses_meta != 0};
    uint8_t st = pair_walk(v, rd, active, r, k, v.nodes + it.y, wk, sink);
    if (magic) st = ST_FALLBACK;
    if (active || magic) { o.status[(size_t)k * v.nres + r] = st; KYV_ACCT_ADD(1, 1); }
    if (sink.n && lane == 0) { o.rcnt[list] = (uint16_t)sink.n; KYV_ACCT_ADD(1, 2); }
  }
}

}  // namespace kyv
