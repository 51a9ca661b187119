// Pair evaluator: one (resource, compiled rule) -> verdict, written once as __host__ __device__ code.
// The HIP kernel (kyv_engine.hip) runs it with one lane per resource and the rule uniform across the
// wavefront; the host instantiation exists for the explicit CPU backend (debug / message formatting) only.
//
// Semantics follow the reference exactly (paths relative to /root/reference):
//   match/exclude            pkg/engine/utils.go:37-289, pkg/utils/match/*.go, pkg/utils/kube/kind.go
//   OldResource retry        pkg/engine/validation.go:600-615
//   pattern walk             pkg/engine/validate/validate.go:31-247 (+ anchor/handlers.go, anchormap.go, error.go)
//   leaf comparison          pkg/engine/pattern/pattern.go:26-321, pkg/engine/operator/operator.go
//   metadata wildcard keys   pkg/engine/wildcards/wildcards.go:62-151
//   PodSecurity              pkg/pss/evaluate.go:16-146 (+ pod-security-admission v0.26.1 checks)
#pragma once
#ifndef __HIPCC_RTC__  // hipRTC (runtime-compiled walk kernels, jit.cpp) provides the HIP runtime itself
#include <hip/hip_runtime.h>
#endif

#include "kyv_layout.h"

namespace kyv {

#define KYV_HD __host__ __device__ inline
#define KYV_BIG __host__ __device__ inline __attribute__((noinline))  // inline: one definition across translation units
// Inlining policy of the large evaluator stages (overridable for experiments)
// (everything on the pattern path inlines into the kernel; the PodSecurity checks stay out of line)
#ifndef KYV_FN_MATCH
#define KYV_FN_MATCH KYV_HD
#endif
#ifndef KYV_FN_PATTERN
#define KYV_FN_PATTERN KYV_HD
#endif
#ifndef KYV_FN_PSS
#define KYV_FN_PSS KYV_BIG
#endif

// Algorithmic-byte accounting (bench roofline): on the host backend with accounting on,
// every node-table row a pair reads is marked once; the device build compiles the hook away.
struct TouchAcct {
  uint8_t* seen;   // one flag per node row of the current resource
  uint32_t n;      // rows of the current resource
  uint64_t rows;   // distinct rows touched by the current pair
};
inline thread_local TouchAcct* g_touch = nullptr;

// Device byte accounting (bench roofline), compiled in only with KYV_ACCT: the accounting build of the
// kernels (kyv_acct.hip; the runtime-compiled kernels with -DKYV_ACCT) adds the bytes of every per-resource load and
// result store to spread 64-bit counters, class 0 = reads of resource data (node rows, path-column entries, header
// fields, walk work lists), class 1 = writes (verdict bytes, PSS masks, work lists), class 2 = staged failing-path
// records (written by the walk, read back by the compaction). Dictionary columns and rule programs are amortised and
// not counted. The product build compiles every KYV_ACCT_ADD away.
#define KYV_ACCT_SLOTS 4096u
#if defined(KYV_ACCT)
extern "C" {
__device__ unsigned long long kyv_acct_bytes[3 * KYV_ACCT_SLOTS];
}
#endif
#if defined(KYV_ACCT) && defined(__HIP_DEVICE_COMPILE__)
#define KYV_ACCT_ADD(cls, b)                                                                                      \
  atomicAdd(&::kyv::kyv_acct_bytes[(cls) * KYV_ACCT_SLOTS + ((blockIdx.x * blockDim.x + threadIdx.x) & (KYV_ACCT_SLOTS - 1))], \
            (unsigned long long)(b))
#else
#define KYV_ACCT_ADD(cls, b) ((void)0)
#endif
// accounting experiments (KYV_JIT_DEFS=-DKYV_ACCT_SEL=<bits>, runtime-compiled kernels): count only the selected kinds of
// resource-data loads -- 1 node rows, 2 path-column entries by column id (jc_col, wcol), 4 pattern-entry columns (jraw),
// 8 element self columns (jself) -- besides every other counted access; default: all
#ifndef KYV_ACCT_SEL
#define KYV_ACCT_SEL 15u
#endif
#define KYV_ACCT_ADDK(kind, cls, b) \
  do {                              \
    if ((KYV_ACCT_SEL) & (kind)) KYV_ACCT_ADD(cls, b); \
  } while (0)

#if defined(__HIP_DEVICE_COMPILE__)
KYV_HD void touch_row(uint32_t) { KYV_ACCT_ADDK(1u, 0, 16); }
#else
KYV_HD void touch_row(uint32_t i) {
  TouchAcct* t = g_touch;
  if (t && i < t->n && !t->seen[i]) { t->seen[i] = 1; t->rows++; }
}
#endif

// Why a pair was handed to the CPU engine (kyv_results_fallback_reason): the host instantiation records the site
// of the last ST_FALLBACK it produced; the device build compiles the hook away (the reason is recomputed on the host
// for the pairs a caller asks about).
enum FallbackWhy : int { FBW_NONE = 0, FBW_MATCH = 1, FBW_PHRASE = 2, FBW_COND = 3, FBW_DEPTH = 4, FBW_VALUE = 5,
                         FBW_META = 6 };
inline thread_local int g_fb_why = FBW_NONE;
#if defined(__HIP_DEVICE_COMPILE__)
#define KYV_WHY(c) ((void)0)
#else
#define KYV_WHY(c) (::kyv::g_fb_why = (c))
#endif

// node table of one resource (rows relative to its root)
struct NodeTab {
  const Node* p;
  KYV_HD const Node& operator[](uint32_t i) const { touch_row(i); return p[i]; }
  KYV_HD explicit operator bool() const { return p != nullptr; }
};

struct View {
  // batch
  const Node* nodes;
  const ResHeader* hdr;
  uint32_t nres;
  const FloatAux* faux;
  const uint32_t* str_off;
  const uint32_t* str_len;
  const uint32_t* str_flags;
  const int64_t* str_dur;
  const int64_t* str_qty;   // 2 per string (lo, hi)
  const double* str_f64;
  const uint8_t* heap;
  const uint32_t* nsl_off;  // namespace label sets: pairs (key sid, value sid)
  const uint32_t* nsl_kv;
  const uint32_t* gate;     // [kind class][gate_words] rule bits (batch.cpp order_by_kind)
  uint32_t gate_words;
  const uint32_t* str_gmask;  // [string][gmask_words] glob-mask bits (device only; nullptr: match bytes)
  uint32_t gmask_words;
  const uint32_t* str_upper;  // [string] id of strings.ToUpper(s) (NONE: not ASCII), or nullptr (no to_upper rule)
  const uint32_t* str_rx;     // [string] regex_match bits of the ruleset's regexes (RX_FB: outside printable ASCII)
  const uint64_t* colv;     // path columns (kyv_layout.h): colv[col_off[c] + row]
  const uint32_t* col_off;  // (device View: pe[].col already holds col_off[col])
  // ruleset
  const RuleDesc* rules;
  uint32_t nrules;
  const Filter* filters;
  const KindDesc* kinds;
  const SelDesc* sels;
  const SelReq* reqs;
  const PNode* pn;
  const PEntry* pe;
  const Leaf* leaves;
  const Atom* atoms;
  const MetaSite* metas;
  const PssDesc* pss;
  const uint32_t* pool;
  const Node* cnodes;       // condition literals
  const Cond* conds;
  const CondProg* cprogs;
};

// ---------------------------------------------------------------- strings
KYV_HD int utf8_decode(const uint8_t* s, uint32_t n, uint32_t i, uint32_t* r) {  // unicode/utf8 semantics
  uint8_t b0 = s[i];
  if (b0 < 0x80) { *r = b0; return 1; }
  uint32_t rem = n - i;
  auto c = [&](uint32_t k, uint32_t lo, uint32_t hi) { return k < rem && s[i + k] >= lo && s[i + k] <= hi; };
  if (b0 >= 0xC2 && b0 <= 0xDF) {
    if (c(1, 0x80, 0xBF)) { *r = ((b0 & 0x1Fu) << 6) | (s[i + 1] & 0x3Fu); return 2; }
  } else if (b0 >= 0xE0 && b0 <= 0xEF) {
    uint32_t lo = b0 == 0xE0 ? 0xA0 : 0x80, hi = b0 == 0xED ? 0x9F : 0xBF;
    if (c(1, lo, hi) && c(2, 0x80, 0xBF)) {
      *r = ((b0 & 0x0Fu) << 12) | ((s[i + 1] & 0x3Fu) << 6) | (s[i + 2] & 0x3Fu);
      return 3;
    }
  } else if (b0 >= 0xF0 && b0 <= 0xF4) {
    uint32_t lo = b0 == 0xF0 ? 0x90 : 0x80, hi = b0 == 0xF4 ? 0x8F : 0xBF;
    if (c(1, lo, hi) && c(2, 0x80, 0xBF) && c(3, 0x80, 0xBF)) {
      *r = ((b0 & 0x07u) << 18) | ((s[i + 1] & 0x3Fu) << 12) | ((s[i + 2] & 0x3Fu) << 6) | (s[i + 3] & 0x3Fu);
      return 4;
    }
  }
  *r = 0xFFFD;
  return 1;
}

// go-wildcard v1.0.3 glob over runes ('*' any run, '?' one rune); iterative star-backtracking decides
// the same language as the library's recursion.
KYV_BIG bool glob_runes(const uint8_t* p, uint32_t pl, const uint8_t* s, uint32_t sl) {
  uint32_t pi = 0, si = 0, star = NONE, mark = 0;
  while (si < sl) {
    uint32_t pr = 0, sr;
    int pw = 0;
    if (pi < pl) pw = utf8_decode(p, pl, pi, &pr);
    int sw = utf8_decode(s, sl, si, &sr);
    if (pi < pl && pr != '*' && (pr == '?' || pr == sr)) { pi += pw; si += sw; continue; }
    if (pi < pl && pr == '*') { star = pi; pi += pw; mark = si; continue; }
    if (star != NONE) {
      pi = star + 1;
      uint32_t mr;
      mark += utf8_decode(s, sl, mark, &mr);
      si = mark;
      continue;
    }
    return false;
  }
  while (pi < pl && p[pi] == '*') pi++;
  return pi == pl;
}

KYV_HD const uint8_t* sbytes(const View& v, uint32_t sid) { return v.heap + v.str_off[sid]; }

KYV_HD bool bytes_eq(const uint8_t* a, const uint8_t* b, uint32_t n) {
  for (uint32_t i = 0; i < n; i++) if (a[i] != b[i]) return false;
  return true;
}

// wildcard.Match(pattern, s) with the pattern pre-classified at compile time
KYV_HD bool glob(const View& v, uint8_t kind, uint32_t pat, uint32_t lit, uint32_t s) {
  switch (kind) {
    case G_ANY: return true;
    case G_EMPTY: return s == SID_EMPTY;
    case G_EXACT: return s == pat;
    case G_NONEMPTY: return v.str_len[s] > 0;
    case G_PREFIX: {
      uint32_t ln = v.str_len[lit], sn = v.str_len[s];
      return sn >= ln && bytes_eq(sbytes(v, s), sbytes(v, lit), ln);
    }
    case G_SUFFIX: {
      uint32_t ln = v.str_len[lit], sn = v.str_len[s];
      return sn >= ln && bytes_eq(sbytes(v, s) + (sn - ln), sbytes(v, lit), ln);
    }
    case G_CONTAINS: {
      uint32_t ln = v.str_len[lit], sn = v.str_len[s];
      if (ln > sn) return false;
      const uint8_t* a = sbytes(v, s);
      const uint8_t* b = sbytes(v, lit);
      for (uint32_t i = 0; i + ln <= sn; i++) if (bytes_eq(a + i, b, ln)) return true;
      return false;
    }
    default: return glob_runes(sbytes(v, pat), v.str_len[pat], sbytes(v, s), v.str_len[s]);
  }
}

// generic wildcard.Match for match-program globs (pattern sid; classification by content)
KYV_HD bool glob_sid_raw(const View& v, uint32_t pat, uint32_t s) {
  if (pat == s) return true;
  // an ASCII pattern without '*' / '?' matches exactly its own runes: an interned string, so only itself (a
  // non-ASCII subject decodes to runes no ASCII pattern rune equals)
  if (!(v.str_flags[pat] & SF_GLOBBY)) return false;
  uint32_t pl = v.str_len[pat];
  if (pl == 0) return s == SID_EMPTY || v.str_len[s] == 0;
  return glob_runes(sbytes(v, pat), pl, sbytes(v, s), v.str_len[s]);
}
// glob-mask bit of (pattern index gi + 1, string s)
KYV_HD bool gmask_bit(const View& v, uint32_t gi1, uint32_t s) {
  const uint32_t g = gi1 - 1;
  return (v.str_gmask[(size_t)s * v.gmask_words + g / 32] >> (g % 32)) & 1u;
}
KYV_HD bool glob_sid(const View& v, uint32_t pat, uint32_t s) {
  if (pat == s) return true;
  const uint32_t f = v.str_flags[pat];
  if (!(f & SF_GLOBBY)) return false;
  const uint32_t gi1 = (f >> SF_GIDX_SHIFT) & 0xFFu;
  if (gi1 && v.str_gmask) return gmask_bit(v, gi1, s);
  return glob_sid_raw(v, pat, s);
}

// ---------------------------------------------------------------- resource values
struct Val {
  uint32_t t;     // NodeType, or 0xFF for absent (nil)
  uint32_t wsid;  // string form for compareString (NONE when ok=false: nil/map/array)
  uint32_t nsid;  // convertNumberToString form (NONE on error: bool/map/array)
  uint32_t sid;   // string value sid (N_STR)
  int64_t i;
  double f;
};

KYV_HD Val value_of(const View& v, NodeTab R, uint32_t rn) {
  Val x;
  x.wsid = NONE; x.nsid = NONE; x.sid = NONE; x.i = 0; x.f = 0;
  if (rn == NONE) { x.t = 0xFF; x.nsid = SID_ZERO; return x; }
  const Node& n = R[rn];
  x.t = node_type(n);
  switch (x.t) {
    case N_NULL: x.nsid = SID_ZERO; break;
    case N_FALSE: x.wsid = SID_FALSE; break;
    case N_TRUE: x.wsid = SID_TRUE; break;
    case N_INT: x.i = (int64_t)(((uint64_t)n.b << 32) | n.a); x.wsid = n.c; x.nsid = n.c; break;
    case N_FLOAT: {
      uint64_t bits = ((uint64_t)n.b << 32) | n.a;
      x.f = __builtin_bit_cast(double, bits);
      x.wsid = v.faux[n.c].sid_E;
      x.nsid = v.faux[n.c].sid_F;
      break;
    }
    case N_STR: x.sid = n.a; x.wsid = n.a; x.nsid = n.a; break;
    default: break;
  }
  return x;
}

KYV_HD bool is_nil(uint32_t t) { return t == 0xFF || t == N_NULL; }

KYV_HD bool cmp_op(uint8_t op, int c) {
  switch (op) {
    case A_EQ: return c == 0;
    case A_NE: return c != 0;
    case A_GT: return c > 0;
    case A_LT: return c < 0;
    case A_GE: return c >= 0;
    case A_LE: return c <= 0;
    default: return false;
  }
}

KYV_HD int cmp128(int64_t ahi, uint64_t alo, int64_t bhi, uint64_t blo) {
  if (ahi != bhi) return ahi < bhi ? -1 : 1;
  if (alo != blo) return alo < blo ? -1 : 1;
  return 0;
}

// one simple comparison: compareDuration || compareQuantity || compareString (pattern.go:207-301)
KYV_HD bool atom_simple(const View& v, const Atom& a, const Val& x, bool* fb) {
  if ((a.flags & AF_DUR) && x.nsid != NONE && (v.str_flags[x.nsid] & SF_DUR)) {
    int64_t d = v.str_dur[x.nsid];
    if (cmp_op(a.op, d < a.dur ? -1 : (d > a.dur ? 1 : 0))) return true;
  }
  if ((a.flags & AF_QTY) && x.nsid != NONE) {
    uint32_t f = v.str_flags[x.nsid];
    if (f & SF_QTY_BIG) { *fb = true; return false; }
    if (f & SF_QTY) {
      int c = cmp128(v.str_qty[2 * x.nsid + 1], (uint64_t)v.str_qty[2 * x.nsid], a.qhi, (uint64_t)a.qlo);
      if (cmp_op(a.op, c)) return true;
    }
  }
  if ((a.op == A_EQ || a.op == A_NE) && x.wsid != NONE) {
    bool r = glob(v, a.glob, a.pat, a.lit, x.wsid);
    return a.op == A_NE ? !r : r;
  }
  return false;
}

KYV_HD bool atom_eval(const View& v, const Atom& a, const Val& x, bool* fb) {
  if (a.op == A_RANGE_IN) return atom_simple(v, v.atoms[a.sub], x, fb) && atom_simple(v, v.atoms[a.sub + 1], x, fb);
  if (a.op == A_RANGE_OUT) return atom_simple(v, v.atoms[a.sub], x, fb) || atom_simple(v, v.atoms[a.sub + 1], x, fb);
  if (a.op == A_FALSE) return false;
  return atom_simple(v, a, x, fb);
}

// pattern.Validate(value, pattern) (pattern.go:26-49)
KYV_HD bool leaf_match(const View& v, const Leaf& L, const Val& x, bool* fb) {
#ifdef KYV_EXP_LEAFTRUE
  return true;
#endif
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
        case N_STR: return (v.str_flags[x.sid] & SF_FLOAT) && v.str_f64[x.sid] == L.f;
        default: return false;
      }
    case L_STR: {
      if (x.t == N_STR && x.sid == L.exact) return true;
      for (uint32_t g = 0; g < L.ngroups; g++) {
        uint32_t a0 = v.pool[L.groups + 2 * g], na = v.pool[L.groups + 2 * g + 1];
        bool all = true;
        for (uint32_t k = 0; k < na; k++)
          if (!atom_eval(v, v.atoms[a0 + k], x, fb)) { all = false; break; }
        if (all) return true;
      }
      return false;
    }
    case L_MAP: return x.t == N_MAP;
    default: return false;
  }
}

// pattern.Validate(value, p) for a leaf substituted from an element variable (L_DYN): p is the variable's value as the
// JSON context holds it (numbers float64, so an integer element field is a float64 pattern); *fb for a pattern the
// device does not decide (a string that is not SF_PLAIN, a map or array value)
KYV_HD bool leaf_match_dyn(const View& v, const Val& p, const Val& x, bool* fb) {
  switch (p.t) {
    case N_NULL:  // validateNilPattern
      switch (x.t) {
        case 0xFF: case N_NULL: case N_FALSE: return true;
        case N_INT: return x.i == 0;
        case N_FLOAT: return x.f == 0.0;
        case N_STR: return x.sid == SID_EMPTY;
        default: return false;
      }
    case N_TRUE: case N_FALSE: return x.t == p.t;  // validateBoolPattern
    case N_INT: case N_FLOAT: {  // validateFloatPattern (pattern.go:87-116)
      const double pf = p.t == N_INT ? (double)p.i : p.f;
      switch (x.t) {
        case N_INT: {
          if (pf != __builtin_trunc(pf)) return false;
          if (!(pf > -9.223372036854775808e18 && pf < 9.223372036854775807e18)) return false;
          return (int64_t)pf == x.i;
        }
        case N_FLOAT: return x.f == pf;
        case N_STR: return (v.str_flags[x.sid] & SF_FLOAT) && v.str_f64[x.sid] == pf;
        default: return false;
      }
    }
    case N_STR:
      if (!(v.str_flags[p.sid] & SF_PLAIN)) { *fb = true; return false; }
      return (x.t == N_STR && x.sid == p.sid) || ((x.t == N_TRUE || x.t == N_FALSE) && x.wsid == p.sid);
    default: *fb = true; return false;
  }
}

// ---------------------------------------------------------------- resource helpers
KYV_HD uint32_t map_find(NodeTab R, uint32_t m, uint32_t key) {
  const Node& mn = R[m];
  uint32_t lo = mn.a, hi = mn.a + mn.b;
  while (lo < hi) {  // entries sorted by key sid
    uint32_t mid = (lo + hi) >> 1;
    uint32_t k = node_key(R[mid]);
    if (k == key) return mid;
    if (k < key) lo = mid + 1; else hi = mid;
  }
  return NONE;
}

// ---------------------------------------------------------------- match programs
// label lookup in a string map node (labels/annotations) or a namespace label set
struct LabelSet {
  NodeTab R;   // node-map form (R != nullptr)
  uint32_t map;
  const uint32_t* kv;  // pair form
  uint32_t n;
};

KYV_HD uint32_t ls_count(const LabelSet& s) { return s.R ? (s.map == NONE ? 0 : s.R[s.map].b) : s.n; }
KYV_HD uint32_t ls_key(const LabelSet& s, uint32_t i) { return s.R ? node_key(s.R[s.R[s.map].a + i]) : s.kv[2 * i]; }
KYV_HD uint32_t ls_val(const LabelSet& s, uint32_t i) { return s.R ? s.R[s.R[s.map].a + i].a : s.kv[2 * i + 1]; }
KYV_HD uint32_t ls_find(const LabelSet& s, uint32_t key) {
  uint32_t n = ls_count(s);
  for (uint32_t i = 0; i < n; i++) if (ls_key(s, i) == key) return i;
  return NONE;
}

// CheckSelector incl. ReplaceInSelector (pkg/utils/match/labels.go:10-24, wildcards.go:13-50): 1 match, 0 no, -1 error
#ifdef KYV_SEL_INLINE
KYV_HD __attribute__((always_inline))
#else
KYV_BIG
#endif
int check_selector(const View& v, const SelDesc& sd, const LabelSet& ls, bool* nd) {
  if (sd.invalid) return -1;
  int res = 1;
  for (uint32_t q = 0; q < sd.nreqs; q++) {
    const SelReq& r = v.reqs[sd.reqs + q];
    if (r.op == RQ_WILD) {
      uint32_t n = ls_count(ls), hit = NONE, nhit = 0;
      bool valid_hit = false, invalid_hit = false;
      for (uint32_t i = 0; i < n; i++) {
        uint32_t k = ls_key(ls, i), val = ls_val(ls, i);
        if (glob_sid(v, r.key, k) && glob_sid(v, r.vals, val)) {
          if (hit == NONE) hit = i;
          nhit++;
          bool ok = (v.str_flags[k] & SF_LKEY) && (v.str_flags[val] & SF_LVAL);
          if (ok) valid_hit = true; else invalid_hit = true;
        }
      }
      if (nhit > 1 && valid_hit && invalid_hit) *nd = true;
      if (nhit == 0) {
        if (r.rkey == NONE) return -1;           // replacement key/value invalid -> selector error
        if (ls_find(ls, r.rkey) != NONE && ls_val(ls, ls_find(ls, r.rkey)) == r.rval) {} else res = 0;
      } else if (invalid_hit && !valid_hit) {
        return -1;
      }
      continue;
    }
    uint32_t i = ls_find(ls, r.key);
    bool has = i != NONE;
    bool inset = false;
    if (has) {
      uint32_t val = ls_val(ls, i);
      for (uint32_t k = 0; k < r.nvals; k++) if (v.pool[r.vals + k] == val) { inset = true; break; }
    }
    bool ok;
    switch (r.op) {
      case RQ_EQ: case RQ_IN: ok = inset; break;
      case RQ_NOTIN: ok = !has || !inset; break;
      case RQ_EXISTS: ok = has; break;
      default: ok = !has; break;
    }
    if (!ok) res = 0;
  }
  return res;
}

struct ResView {   // unstructured accessors of one resource (or of the empty OldResource)
  NodeTab R;
  const ResHeader* h;  // nullptr for the empty resource
};

KYV_HD bool kinds_match(const View& v, const Filter& f, const ResHeader* h) {
  uint32_t gk = h ? h->gvk_kind : SID_EMPTY;
  for (uint32_t i = 0; i < f.nkinds; i++) {
    const KindDesc& k = v.kinds[f.kinds + i];
    if (k.kind == NONE) return true;  // "*"
    bool r = k.kind == gk;
    if (r && k.gv_mode != 0) {
      uint32_t g = h ? h->group : SID_EMPTY, ver = h ? h->version : SID_EMPTY, gv = h ? h->gv : SID_EMPTY;
      if (k.gv_mode == 1) r = k.g == g && k.v == ver;
      else if (k.gv_mode == 2) {
        uint32_t ln = v.str_len[k.g], sn = v.str_len[gv];
        r = sn >= ln && bytes_eq(sbytes(v, gv), sbytes(v, k.g), ln);
      } else r = false;
    }
    if (r) return true;
  }
  return false;
}

// doesResourceMatchConditionBlock (utils.go:71-160); true when the block produces no errors
KYV_HD bool condition_block(const View& v, const Filter& f, const ResView& rv, const LabelSet& nsl, bool userinfo_checked,
                            bool* nd) {
  const ResHeader* h = rv.h;
  if (f.nkinds && !kinds_match(v, f, h)) return false;
  uint32_t name = h ? h->name : SID_EMPTY;
  uint32_t rname = (h && name == SID_EMPTY) ? h->gen_name : name;
  if (f.name != NONE && !glob_sid(v, f.name, rname)) return false;
  if (f.nnames) {
    bool any = false;
    for (uint32_t i = 0; i < f.nnames && !any; i++) any = glob_sid(v, v.pool[f.names + i], rname);
    if (!any) return false;
  }
  uint32_t kind = h ? h->kind : SID_EMPTY;
  bool isNamespaceKind = h && (v.str_len[kind] == 9 && bytes_eq(sbytes(v, kind), (const uint8_t*)"Namespace", 9));
  if (f.nnss) {
    uint32_t rns = isNamespaceKind ? name : (h ? h->ns : SID_EMPTY);
    bool any = false;
    for (uint32_t i = 0; i < f.nnss && !any; i++) any = glob_sid(v, v.pool[f.nss + i], rns);
    if (!any) return false;
  }
  if (f.nann) {
    LabelSet as{rv.R, h ? h->ann : NONE, nullptr, 0};
    uint32_t n = ls_count(as);
    for (uint32_t q = 0; q < f.nann; q++) {
      uint32_t kp = v.pool[f.ann + 2 * q], vp = v.pool[f.ann + 2 * q + 1];
      bool m = false;
      for (uint32_t i = 0; i < n && !m; i++) m = glob_sid(v, kp, ls_key(as, i)) && glob_sid(v, vp, ls_val(as, i));
      if (!m) return false;
    }
  }
  if (f.flags & FF_HAS_SEL) {
    LabelSet ls{rv.R, h ? h->labels : NONE, nullptr, 0};
    if (check_selector(v, v.sels[f.sel], ls, nd) != 1) return false;
  }
  if ((f.flags & FF_HAS_NSSEL) && !isNamespaceKind && (kind != SID_EMPTY || (f.flags & FF_KINDS_STAR))) {
    if (check_selector(v, v.sels[f.sel + 1], nsl, nd) != 1) return false;
  }
  if (userinfo_checked && (f.flags & FF_USERINFO)) return false;
  return true;
}

// MatchesResourceDescription (utils.go:185-256) with empty admission info
KYV_FN_MATCH bool match_rule(const View& v, const RuleDesc& rd, const ResView& rv, const LabelSet& nsl, bool* nd) {
  bool failed = false;
  const MatchBlock& m = rd.match;
  if (m.mode == MM_ANY) {
    bool one = false;
    for (uint32_t i = 0; i < m.nfilters && !one; i++) {
      const Filter& f = v.filters[m.filters + i];
      if (!(f.flags & FF_ZERO_RD) && condition_block(v, f, rv, nsl, false, nd)) one = true;
    }
    if (!one) failed = true;
  } else if (m.mode == MM_ALL || m.mode == MM_PLAIN) {
    for (uint32_t i = 0; i < m.nfilters && !failed; i++) {
      const Filter& f = v.filters[m.filters + i];
      if ((f.flags & FF_ZERO_RD) || !condition_block(v, f, rv, nsl, false, nd)) failed = true;
    }
  } else {
    failed = true;  // MM_NONE never produced by the compiler
  }
  if (failed) return false;
  const MatchBlock& e = rd.exclude;
  if (e.mode == MM_ANY || e.mode == MM_PLAIN) {
    for (uint32_t i = 0; i < e.nfilters; i++) {
      const Filter& f = v.filters[e.filters + i];
      if ((f.flags & FF_ZERO_RD) && !(f.flags & FF_USERINFO)) continue;
      if (condition_block(v, f, rv, nsl, true, nd)) return false;
    }
  } else if (e.mode == MM_ALL) {
    bool byAll = true;
    for (uint32_t i = 0; i < e.nfilters && byAll; i++) {
      const Filter& f = v.filters[e.filters + i];
      bool excl = !((f.flags & FF_ZERO_RD) && !(f.flags & FF_USERINFO)) && condition_block(v, f, rv, nsl, true, nd);
      if (!excl) byAll = false;
    }
    if (byAll && e.nfilters > 0) return false;
  }
  return true;
}

// CheckMatchesResources (pkg/utils/match/match.go:26-76) of a PolicyException's match block with empty admission
// info: true when the exception applies. Differs from match_rule in that a statement with neither any nor all
// matches everything (MM_EXC_ALL), the user info of a statement is checked (never satisfied in background scans, so
// a statement carrying roles / clusterRoles / subjects fails), a statement with an empty resource description and no
// user info fails ("statement cannot be empty", :89-91), and the namespace selector is skipped for a resource with
// an empty kind (:186; the compiler clears FF_KINDS_STAR on exception filters)
KYV_HD bool match_exception(const View& v, uint32_t mode, uint32_t filters, uint32_t nfilters, const ResView& rv,
                            const LabelSet& nsl, bool* nd) {
  if (mode == MM_EXC_ALL) return true;
  if (mode == MM_ANY) {
    for (uint32_t i = 0; i < nfilters; i++) {
      const Filter& f = v.filters[filters + i];
      if ((f.flags & FF_ZERO_RD) && !(f.flags & FF_USERINFO)) continue;
      if (condition_block(v, f, rv, nsl, true, nd)) return true;
    }
    return false;
  }
  bool ok = true;  // MM_ALL: every statement's errors are collected (no early exit)
  for (uint32_t i = 0; i < nfilters; i++) {
    const Filter& f = v.filters[filters + i];
    if ((f.flags & FF_ZERO_RD) && !(f.flags & FF_USERINFO)) { ok = false; continue; }
    if (!condition_block(v, f, rv, nsl, true, nd)) ok = false;
  }
  return ok;
}

// ---------------------------------------------------------------- pattern walk
enum FrameKind : uint8_t { F_MAP = 1, F_AOM = 2, F_POS = 3, F_EXIST = 4 };
struct Frame {     // 16 bytes
  uint32_t pn;     // pnode (F_EXIST: entry index)
  uint32_t rn;     // resource node
  uint16_t i, j;
  uint8_t kind, st;
  uint16_t pad;
};
enum FrameSt : uint8_t { FS_APPLY = 1, FS_SKIP = 2 };  // bits 2..4 carry the skip-error phrase mask

// error classes (anchor/error.go): code + phrase mask of the error text
enum ErrCode : uint8_t { EC_NONE = 0, EC_COND = 1, EC_GLOBAL = 2, EC_NEG = 3 };
enum Phrase : uint8_t { PH_COND = 1, PH_GLOBAL = 2, PH_NEG = 4 };

struct Ret {
  bool err;
  uint8_t code;   // typed code or EC_NONE (untyped)
  uint8_t mask;   // phrases contained in Error()
  uint32_t tmpl;  // returned path template (NONE == "")
};

KYV_HD bool ret_is_skip(const Ret& r) {
  return r.code != EC_NONE ? (r.code == EC_COND || r.code == EC_GLOBAL) : (r.mask & (PH_COND | PH_GLOBAL)) != 0;
}
KYV_HD bool ret_is_neg(const Ret& r) { return r.code != EC_NONE ? r.code == EC_NEG : (r.mask & PH_NEG) != 0; }

struct PatOut {
  uint8_t status;       // ST_PASS / ST_FAIL / ST_SKIP / ST_ERROR / ST_FALLBACK / ST_PANIC / ST_ND
  uint32_t tmpl;
  uint64_t idx;         // MAX_IDX packed u16 array indices (register-resident, no dynamic indexing)
  uint32_t key0, key1;  // resolved metadata wildcard keys (MAX_SLOTS == 2)
};
static_assert(MAX_IDX == 4 && MAX_SLOTS == 2, "PatOut packing");

// two metadata-key slots held in registers
struct Keys {
  uint32_t k0, k1;
  KYV_HD uint32_t get(uint32_t s) const { return s ? k1 : k0; }
  KYV_HD void set(uint32_t s, uint32_t val) { if (s) k1 = val; else k0 = val; }
};

// frame stack accessor: lane-strided (LDS on device, local array on host)
struct Stack {
  Frame* base;
  uint32_t stride;
  int cap;          // frames available per lane
  KYV_HD Frame& at(int d) const { return base[(uint32_t)d * stride]; }
};

KYV_HD Ret mkerr(uint8_t code, uint8_t mask, uint32_t tmpl) { Ret r; r.err = true; r.code = code; r.mask = mask; r.tmpl = tmpl; return r; }
KYV_HD Ret ok_ret() { Ret r; r.err = false; r.code = EC_NONE; r.mask = 0; r.tmpl = NONE; return r; }

// The keys of a labels / annotations map L that glob pattern gp matches: the first one and how many. Four entries per
// step, their key words first and then (a pattern with a glob-mask bit) their mask words, as independent loads: an
// entry at a time was a chain of two dependent loads per annotation (round 6: C3's app-armor rules, one rule 0.63 ms
// over 7 M pods)
KYV_HD __attribute__((always_inline)) void meta_wild_scan(const View& v, NodeTab R, const Node& L, uint32_t gp,
                                                         uint32_t* hit, uint32_t* n) {
  const uint32_t f = v.str_flags[gp];
  const uint32_t gi1 = (f & SF_GLOBBY) ? (f >> SF_GIDX_SHIFT) & 0xFFu : 0u;
  const bool mask = gi1 && v.str_gmask;
  for (uint32_t i = 0; i < L.b; i += 4) {
    uint32_t k[4], m[4];
#pragma unroll
    for (uint32_t j = 0; j < 4; j++) k[j] = i + j < L.b ? node_key(R[L.a + i + j]) : NONE;
#pragma unroll
    for (uint32_t j = 0; j < 4; j++)
      m[j] = mask && k[j] != NONE ? v.str_gmask[(size_t)k[j] * v.gmask_words + (gi1 - 1) / 32] : 0u;
#pragma unroll
    for (uint32_t j = 0; j < 4; j++) {
      if (i + j >= L.b) break;
      const bool g = mask ? (k[j] == gp || ((m[j] >> ((gi1 - 1) % 32)) & 1u)) : glob_sid(v, gp, k[j]);
      if (g) { if (*hit == NONE) *hit = k[j]; (*n)++; }
    }
  }
}

// ExpandInMetadata at one map level (wildcards.go:62-83): resolves wildcard keys into slots; returns a
// status override (ST_PANIC / ST_ND / ST_FALLBACK) or ST_NONE.
KYV_BIG uint8_t expand_meta(const View& v, const MetaSite& ms, NodeTab R, uint32_t rn, const ResHeader& h, Keys& keys) {
  uint32_t meta = map_find(R, rn, KSID(METADATA));
  // slots default to "unresolved" (the pattern key itself, stored in the pool after the glob sid)
  for (uint32_t i = 0; i < ms.nwild_l; i++) keys.set(ms.slot_l + i, v.pool[ms.wild_l + 2 * i + 1]);
  for (uint32_t i = 0; i < ms.nwild_a; i++) keys.set(ms.slot_a + i, v.pool[ms.wild_a + 2 * i + 1]);
  if (meta == NONE || node_type(R[meta]) == N_NULL) return ST_NONE;
  if (node_type(R[meta]) != N_MAP) return ST_PANIC;
  if (h.flags & RF_ANCHORISH) return ST_FALLBACK;
  for (int tag = 0; tag < 2; tag++) {
    if (!(tag == 0 ? ms.has_labels : ms.has_ann)) continue;
    uint32_t lm = map_find(R, meta, tag == 0 ? KSID(LABELS) : KSID(ANNOTATIONS));
    if (lm == NONE || node_type(R[lm]) == N_NULL) continue;
    if (node_type(R[lm]) != N_MAP) return ST_PANIC;
    const Node& L = R[lm];
    for (uint32_t i = 0; i < L.b; i++) if (node_type(R[L.a + i]) != N_STR) return ST_PANIC;
    uint32_t wild = tag == 0 ? ms.wild_l : ms.wild_a, nw = tag == 0 ? ms.nwild_l : ms.nwild_a;
    uint32_t slot0 = tag == 0 ? ms.slot_l : ms.slot_a;
    for (uint32_t w = 0; w < nw; w++) {
      uint32_t hit = NONE, n = 0;
      meta_wild_scan(v, R, L, v.pool[wild + 2 * w], &hit, &n);
      if (n > 1) return ST_ND;
      if (n == 1) keys.set(slot0 + w, hit);
    }
  }
  return ST_NONE;
}

// expand_meta at the resource root from what the flattener already knows: the metadata shape flags and the
// header's labels / annotations nodes (maps of strings), so no map of the metadata is searched again
KYV_HD uint8_t expand_meta_root(const View& v, const MetaSite& ms, NodeTab R, const ResHeader& h, Keys& keys) {
  for (uint32_t i = 0; i < ms.nwild_l; i++) keys.set(ms.slot_l + i, v.pool[ms.wild_l + 2 * i + 1]);
  for (uint32_t i = 0; i < ms.nwild_a; i++) keys.set(ms.slot_a + i, v.pool[ms.wild_a + 2 * i + 1]);
  KYV_ACCT_ADD(0, 8);  // header: flags, labels / annotations node
  if (h.flags & RF_META_NONE) return ST_NONE;
  if (h.flags & RF_META_NOTMAP) return ST_PANIC;
  if (h.flags & RF_ANCHORISH) return ST_FALLBACK;
  for (int tag = 0; tag < 2; tag++) {
    if (!(tag == 0 ? ms.has_labels : ms.has_ann)) continue;
    if (h.flags & (tag == 0 ? RF_LAB_BAD : RF_ANN_BAD)) return ST_PANIC;
    const uint32_t lm = tag == 0 ? h.labels : h.ann;  // NONE: absent or null
    if (lm == NONE) continue;
    const Node& L = R[lm];
    uint32_t wild = tag == 0 ? ms.wild_l : ms.wild_a, nw = tag == 0 ? ms.nwild_l : ms.nwild_a;
    uint32_t slot0 = tag == 0 ? ms.slot_l : ms.slot_a;
    for (uint32_t w = 0; w < nw; w++) {
      uint32_t hit = NONE, n = 0;
      meta_wild_scan(v, R, L, v.pool[wild + 2 * w], &hit, &n);
      if (n > 1) return ST_ND;
      if (n == 1) keys.set(slot0 + w, hit);
    }
  }
  return ST_NONE;
}

// MatchPattern (validate.go:31-56) for one compiled pattern; a walk deeper than the stack ends in ST_FALLBACK.
// rn0: the node the pattern validates (the resource root, or a foreach element); dyn: the values of the pattern's
// element variables (L_DYN leaves), foreach patterns only
KYV_FN_PATTERN void eval_pattern(const View& v, uint32_t root, NodeTab R, const ResHeader& h, const RuleDesc& rd, Stack stk,
                         PatOut& out, uint32_t rn0 = 0, const Val* dyn = nullptr) {
  uint64_t seen = 0, found = 0;
  Keys keys{NONE, NONE};
  out.idx = 0;
  int sp = 0;
  Ret ret = ok_ret();
  bool fb = false;
  // action: 0 enter, 1 next, 2 return
  int action = 0;
  uint32_t epn = root, ern = rn0;  // enter arguments
  for (;;) {
    if (action == 0) {
      const PNode& P = v.pn[epn];
      uint32_t rt = ern == NONE ? 0xFF : node_type(R[ern]);
      if (P.kind == P_MAP) {
        if (rt != N_MAP) { ret = mkerr(EC_NONE, 0, P.tmpl); action = 2; continue; }
        // AnchorMap.CheckAnchorInResource (anchormap.go:30-44)
        for (uint32_t e = 0; e < P.n; e++) {
          const PEntry& E = v.pe[P.first + e];
          if (E.abit != 0xFF) {
            uint64_t b = 1ull << E.abit;
            seen |= b;
            if (!(found & b)) {
              uint32_t key = (E.flags & EF_WILD) ? keys.get(E.slot) : E.key;
              if (map_find(R, ern, key) != NONE) found |= b;
            }
          }
        }
        if (P.flags & PF_META) {
          uint8_t o = expand_meta(v, v.metas[rd.meta_sites + P.meta], R, ern, h, keys);
          if (o != ST_NONE) { if (o == ST_FALLBACK) KYV_WHY(FBW_META); out.status = o; return; }
        }
        if (sp >= stk.cap) { KYV_WHY(FBW_DEPTH); out.status = ST_FALLBACK; return; }
        Frame& f = stk.at(sp++);
        f.kind = F_MAP; f.pn = epn; f.rn = ern; f.i = 0; f.j = 0; f.st = 0;
        action = 1;
        continue;
      }
      if (P.kind == P_LEAF) {
        const Leaf& L = v.leaves[P.first];
        bool okv = true;
        const bool dl = L.type == L_DYN;
        if (dl && !dyn) { KYV_WHY(FBW_VALUE); out.status = ST_FALLBACK; return; }
        if (rt == N_ARR) {
          const Node& A = R[ern];
          for (uint32_t i = 0; i < A.b && okv; i++)
            okv = dl ? leaf_match_dyn(v, dyn[L.exact], value_of(v, R, A.a + i), &fb) : leaf_match(v, L, value_of(v, R, A.a + i), &fb);
        } else {
          okv = dl ? leaf_match_dyn(v, dyn[L.exact], value_of(v, R, ern), &fb) : leaf_match(v, L, value_of(v, R, ern), &fb);
        }
        if (fb) { KYV_WHY(FBW_VALUE); out.status = ST_FALLBACK; return; }
        ret = okv ? ok_ret() : mkerr(EC_NONE, 0, P.tmpl);
        action = 2;
        continue;
      }
      // arrays
      if (rt != N_ARR) { ret = mkerr(EC_NONE, 0, P.tmpl); action = 2; continue; }
      if (P.kind == P_ARR_EMPTY) { ret = mkerr(EC_NONE, 0, P.tmpl); action = 2; continue; }
      if (P.kind == P_ARR_SCALAR) {
        const Leaf& L = v.leaves[v.pn[P.first].first];
        const Node& A = R[ern];
        bool okv = true;
        const bool dl = L.type == L_DYN;
        if (dl && !dyn) { KYV_WHY(FBW_VALUE); out.status = ST_FALLBACK; return; }
        for (uint32_t i = 0; i < A.b && okv; i++)
          okv = dl ? leaf_match_dyn(v, dyn[L.exact], value_of(v, R, A.a + i), &fb) : leaf_match(v, L, value_of(v, R, A.a + i), &fb);
        if (fb) { KYV_WHY(FBW_VALUE); out.status = ST_FALLBACK; return; }
        ret = okv ? ok_ret() : mkerr(EC_NONE, 0, P.tmpl);
        action = 2;
        continue;
      }
      if (P.kind == P_ARR_POS && R[ern].b < P.n) { ret = mkerr(EC_NONE, 0, NONE); action = 2; continue; }
      if (sp >= stk.cap) { KYV_WHY(FBW_DEPTH); out.status = ST_FALLBACK; return; }
      Frame& f = stk.at(sp++);
      f.kind = P.kind == P_ARR_MAPS ? F_AOM : F_POS;
      f.pn = epn; f.rn = ern; f.i = 0; f.j = 0; f.st = 0;
      action = 1;
      continue;
    }
    if (action == 1) {  // next step of the top frame
      Frame& f = stk.at(sp - 1);
      if (f.kind == F_MAP) {
        const PNode& P = v.pn[f.pn];
        if (f.i == P.n) { sp--; ret = ok_ret(); action = 2; continue; }
        const PEntry& E = v.pe[P.first + f.i];
        f.i++;
        uint32_t key = (E.flags & EF_WILD) ? keys.get(E.slot) : E.key;
        uint32_t c = map_find(R, f.rn, key);
        switch (E.handler) {
          case H_NEGATION:
            if (c != NONE) { ret = mkerr(EC_NEG, PH_NEG, E.tmpl); sp--; action = 2; }
            continue;
          case H_EQUALITY: case H_GLOBAL:
            if (c != NONE) { epn = E.child; ern = c; action = 0; }
            continue;
          case H_CONDITION:
            if (c != NONE) { epn = E.child; ern = c; action = 0; }
            else { ret = mkerr(EC_COND, PH_COND, E.tmpl); sp--; action = 2; }
            continue;
          case H_STAR:
            if (c != NONE && node_type(R[c]) != N_NULL) continue;
            ret = mkerr(EC_NONE, 0, P.tmpl);  // returns dh.path (the parent path)
            sp--; action = 2;
            continue;
          case H_EXISTENCE: case H_EXIST_BADPAT:
            if (c == NONE) continue;
            if (node_type(R[c]) != N_ARR || E.handler == H_EXIST_BADPAT) { ret = mkerr(EC_NONE, 0, E.tmpl); sp--; action = 2; continue; }
            if (sp >= stk.cap) { KYV_WHY(FBW_DEPTH); out.status = ST_FALLBACK; return; }
            {
              Frame& g = stk.at(sp++);
              g.kind = F_EXIST; g.pn = P.first + f.i - 1; g.rn = c; g.i = 0; g.j = 0; g.st = 0;
            }
            continue;
          default:  // H_DEFAULT
            epn = E.child; ern = c; action = 0;
            continue;
        }
      }
      if (f.kind == F_AOM || f.kind == F_POS) {
        const PNode& P = v.pn[f.pn];
        uint32_t n = f.kind == F_AOM ? R[f.rn].b : P.n;
        if (f.i == n) {
          sp--;
          if ((f.st & FS_SKIP) && !(f.st & FS_APPLY)) ret = mkerr(EC_NONE, (uint8_t)(f.st >> 2), P.tmpl);
          else ret = ok_ret();
          action = 2;
          continue;
        }
        if (f.kind == F_AOM) {
          uint32_t sh = 16u * P.level;
          out.idx = (out.idx & ~(0xFFFFull << sh)) | ((uint64_t)f.i << sh);
          epn = P.first;
        }
        else epn = v.pool[P.first + f.i];
        ern = R[f.rn].a + f.i;
        f.i++;
        action = 0;
        continue;
      }
      // F_EXIST: entry index in f.pn; pattern maps in pool[E.child .. +n]
      {
        const PEntry& E = v.pe[f.pn];
        uint32_t npat = v.pool[E.child];
        if (f.j == npat) { sp--; ret = ok_ret(); action = 2; continue; }
        if (f.i == R[f.rn].b) { sp--; ret = mkerr(EC_NONE, 0, E.tmpl); action = 2; continue; }
        epn = v.pool[E.child + 1 + f.j];
        ern = R[f.rn].a + f.i;
        f.i++;
        action = 0;
        continue;
      }
    }
    // action == 2: deliver ret to the frame below
    if (sp == 0) break;
    Frame& f = stk.at(sp - 1);
    if (f.kind == F_MAP) {
      if (!ret.err) { action = 1; continue; }
      const PEntry& E = v.pe[v.pn[f.pn].first + f.i - 1];
      if (E.handler == H_CONDITION) { ret.code = EC_COND; ret.mask |= PH_COND; }
      else if (E.handler == H_GLOBAL) { ret.code = EC_GLOBAL; ret.mask |= PH_GLOBAL; }
      sp--;
      continue;  // propagate
    }
    if (f.kind == F_AOM || f.kind == F_POS) {
      if (ret.err) {
        if (ret_is_skip(ret)) { f.st |= FS_SKIP | (uint8_t)(ret.mask << 2); action = 1; continue; }
        sp--;
        continue;  // propagate
      }
      f.st |= FS_APPLY;
      action = 1;
      continue;
    }
    // F_EXIST
    if (ret.err) { action = 1; continue; }  // try the next resource element
    f.j++;
    f.i = 0;
    action = 1;
  }
  out.key0 = keys.k0;
  out.key1 = keys.k1;
  if (!ret.err) { out.status = ST_PASS; out.tmpl = NONE; return; }
  if (ret_is_skip(ret)) { out.status = ST_SKIP; out.tmpl = NONE; return; }
  if (ret_is_neg(ret)) { out.status = ST_FAIL; out.tmpl = ret.tmpl; return; }
  if (seen & ~found) { out.status = ST_ERROR; out.tmpl = NONE; return; }
  out.tmpl = ret.tmpl;
  out.status = ret.tmpl == NONE ? ST_ERROR : ST_FAIL;
}

}  // namespace kyv
