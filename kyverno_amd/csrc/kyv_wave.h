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
//  * resource node rows are read with global (not flat) loads, map keys by binary search on the key dword.
//
// Every per-lane side effect (return value, anchor map, array indices, metadata keys) happens only for lanes
// inside the step's mask, so each lane sees exactly the sequence of operations the per-lane walk performs.
#pragma once
#include "kyv_eval.h"

namespace kyv {

#define KYV_AS_CONST __attribute__((address_space(4)))
#define KYV_AS_GLOBAL __attribute__((address_space(1)))

// word-wise loads so that uniform addresses become s_load (constant AS) and per-lane ones global_load
template <class T>
__device__ __forceinline__ T sld(const T* p) {
  static_assert(sizeof(T) % 4 == 0, "sld: 4-byte multiple");
  T out;
  uint32_t* o = (uint32_t*)&out;
  const KYV_AS_CONST uint32_t* q = (const KYV_AS_CONST uint32_t*)p;
#pragma unroll
  for (int i = 0; i < (int)(sizeof(T) / 4); i++) o[i] = q[i];
  return out;
}
__device__ __forceinline__ uint32_t sld32(const uint32_t* p) { return *(const KYV_AS_CONST uint32_t*)p; }
typedef uint32_t kyv_u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ Node gnode(const Node* p) {
  const KYV_AS_GLOBAL kyv_u32x4* q = (const KYV_AS_GLOBAL kyv_u32x4*)p;
  kyv_u32x4 x = *q;
  Node n;
  n.tk = x.x; n.a = x.y; n.b = x.z; n.c = x.w;
  return n;
}
__device__ __forceinline__ uint32_t gtk(const Node* p) { return *(const KYV_AS_GLOBAL uint32_t*)p; }
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

__device__ __forceinline__ Val wvalue_of(const View& v, const Node* R, uint32_t rn) {
  Val x;
  x.wsid = NONE; x.nsid = NONE; x.sid = NONE; x.i = 0; x.f = 0;
  if (rn == NONE) { x.t = 0xFF; x.nsid = SID_ZERO; return x; }
  Node n = gnode(R + rn);
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

// per-lane part of a spilled frame: child range of the map / array node + array-frame state
struct LaneFrame {
  uint32_t a;     // first child row
  uint32_t bst;   // child count (low 16) | FrameSt bits << 16
};
// uniform part of a spilled frame
struct UFrame {
  uint32_t kind, pn, i, j;
  uint64_t alive, cmask, search;
  uint64_t pad;
};
static_assert(sizeof(UFrame) == 48, "UFrame");

struct WaveWalker {
  LaneFrame* lf;   // LDS, [cap][64]
  UFrame* uf;      // LDS, [cap]
  int cap;

  __device__ void run(const View& v, uint32_t root, bool walk, const Node* R, const ResHeader* hp, const RuleDesc& rd,
                      PatOut& out) {
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
    const uint32_t meta_base = rd.meta_sites;

    int sp = 0;
    // top frame (uniform)
    uint32_t t_kind = 0, t_pn = 0, t_i = 0, t_j = 0;
    uint64_t t_alive = 0, t_cmask = 0, t_search = 0;
    // top frame (per lane)
    uint32_t t_a = 0, t_b = 0, t_st = 0;

    int action = 0;
    uint32_t epn = root, ern = 0;

#define KYV_PUSH(KIND, PN, ALIVE, A, B)                                                     \
  do {                                                                                      \
    if (sp > 0) {                                                                           \
      if (lane == 0) {                                                                      \
        UFrame& u = uf[sp - 1];                                                             \
        u.kind = t_kind; u.pn = t_pn; u.i = t_i; u.j = t_j;                                 \
        u.alive = t_alive; u.cmask = t_cmask; u.search = t_search;                          \
      }                                                                                     \
      LaneFrame& l = lf[(uint32_t)(sp - 1) * 64u + lane];                                   \
      l.a = t_a; l.bst = (t_b & 0xFFFFu) | (t_st << 16);                                   \
    }                                                                                       \
    t_kind = (KIND); t_pn = (PN); t_i = 0; t_j = 0;                                         \
    t_alive = (ALIVE); t_cmask = 0; t_search = (ALIVE);                                     \
    t_a = (A); t_b = (B); t_st = 0;                                                         \
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
      t_a = l.a; t_b = l.bst & 0xFFFFu; t_st = l.bst >> 16;                                 \
    }                                                                                       \
  } while (0)

    for (;;) {
      if (action == 0) {
        // ---------------------------------------------------------------- enter epn for lanes in emask
        const PNode P = sld(v.pn + epn);
        const bool in = (emask & lbit) != 0;
        uint32_t rt = 0xFF;
        Node rnode{0, 0, 0, 0};
        if (in && ern != NONE) { rnode = gnode(R + ern); rt = node_type(rnode); }
        if (P.kind == P_MAP) {
          uint64_t bad = wballot(in && rt != N_MAP);
          if (bad & lbit) ret = mkerr(EC_NONE, 0, P.tmpl);
          uint64_t go = emask & ~bad;
          if (go) {
            // AnchorMap.CheckAnchorInResource (anchormap.go:30-44)
            for (uint32_t e = 0; e < P.n; e++) {
              const PEntry E = sld(v.pe + P.first + e);
              if (E.abit != 0xFF && (go & lbit)) {
                uint64_t b = 1ull << E.abit;
                seen |= b;
                if (!(found & b)) {
                  uint32_t key = (E.flags & EF_WILD) ? keys.get(E.slot) : E.key;
                  if (wmap_find(R, rnode.a, rnode.b, key) != NONE) found |= b;
                }
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
            KYV_PUSH(F_MAP, epn, go, rnode.a, rnode.b);
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
          for (uint32_t i = 0; i < cnt && okv; i++) okv = leaf_match(v, L, wvalue_of(v, R, each ? rnode.a + i : ern), &fb);
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
          KYV_PUSH(P.kind == P_ARR_MAPS ? F_AOM : F_POS, epn, go, rnode.a, rnode.b);
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
          uint32_t c = NONE;
          if (al) {
            uint32_t key = (E.flags & EF_WILD) ? keys.get(E.slot) : E.key;
            c = wmap_find(R, t_a, t_b, key);
          }
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
              if (ent) { t_cmask = ent; emask = ent; epn = E.child; ern = c; action = 0; }
              continue;
            }
            case H_CONDITION: {
              uint64_t pres = wballot(al && c != NONE);
              uint64_t absent = alive & ~pres;
              if (absent & lbit) ret = mkerr(EC_COND, PH_COND, E.tmpl);
              t_alive &= ~absent;
              if (pres) { t_cmask = pres; emask = pres; epn = E.child; ern = c; action = 0; }
              continue;
            }
            case H_STAR: {
              bool isnull = false;
              if (al && c != NONE) isnull = node_type(gnode(R + c)) == N_NULL;
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
                KYV_PUSH(F_EXIST, P.first + t_i - 1, ex, cn.a, cn.b);
              }
              continue;
            }
            default: {  // H_DEFAULT: recurse on resourceMap[k] (absent -> nil)
              t_cmask = alive; emask = alive; epn = E.child; ern = c; action = 0;
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
          if (search & lbit) ern = t_a + t_i;
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

}  // namespace kyv
