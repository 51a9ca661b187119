// The evaluation kernels that read per-resource data (match phase, PodSecurity, interpreted walk), in a header so
// that they are compiled twice: into the product library (kyv_engine.hip) and, with KYV_ACCT defined and the
// namespace renamed, into the byte-accounting build (kyv_acct.hip) whose loads and stores count the algorithmic
// bytes of SURVEY §8(d) (kyv_eval.h KYV_ACCT_ADD). Same source, so the accounting run executes exactly the
// product's control flow.
#pragma once
#include "kyv_pss.h"
#include "kyv_wave.h"

namespace kyv {

constexpr int BLOCK = 64;        // one wave per workgroup; LDS = depth * 64 * 16 B
constexpr int RECS_PER_PAIR = MAX_ALTS;

#ifndef KYV_WPE
#define KYV_WPE 4
#endif

// Phase 1 (match_eval): one lane per resource, the rule loop uniform across the wave. Kind gate, match /
// exclude program, dispatch; verdicts that need no pattern walk are final here (incl. PodSecurity). Pairs
// that need the walk are appended to the rule's work list (wave ballot + one atomic per wave and rule).
// Two instantiations: kJ = false for rules without JMESPath operands or foreach (the register budget of the
// plain match / condition / PodSecurity code), kJ = true for the rest (projection lists live in scratch)
#ifndef KYV_MATCH_WPE
#define KYV_MATCH_WPE 4  // C2 A/B: 1.50 ms unbounded (3 waves), 1.40 at 4, 1.47 at 5, 1.53 at 6
#endif
template <bool kJ>
__global__ void __launch_bounds__(BLOCK) __attribute__((amdgpu_waves_per_eu(KYV_MATCH_WPE))) match_kernel(const View* __restrict__ vp, DevOut o, WorkLists wl,
                                                      const uint32_t* __restrict__ mrules, uint32_t nm) {
  const View& v = *vp;
  const uint32_t lane = threadIdx.x;
  const uint32_t r = blockIdx.x * BLOCK + lane;
  const bool active = r < v.nres;
  const uint32_t* gate = active ? v.gate + (size_t)v.hdr[r].kclass * v.gate_words : nullptr;
  if (active) KYV_ACCT_ADD(0, 4);  // header: kind class
  for (uint32_t mi = 0; mi < nm; mi++) {  // rules that need this phase (direct-walk rules are decided in the walk)
    const uint32_t k = mrules[mi];
    const bool gated = active && ((gate[k >> 5] >> (k & 31)) & 1u);
    if (!__ballot(gated)) continue;  // status bytes are pre-set to ST_NONE, PSS masks to 0
    uint32_t pf = 0;
    bool walk = false;
    const uint8_t st = pair_dispatch<kJ>(v, gated, r, k, &pf, &walk);
    const unsigned long long wm = __ballot(walk);
    const RuleDesc& rdk = v.rules[k];
    if (rdk.kind == RK_PATTERN || rdk.kind == RK_ANYPATTERN) {  // this wave's work list for rule k
      const size_t list = (size_t)(k - o.rule_lo) * wl.nwaves + blockIdx.x;
      if (walk) {
        const ResHeader& h = v.hdr[r];
        wl.items[list * WAVE + __popcll(wm & ((1ull << lane) - 1))] =
            make_uint2(r | ((h.flags & RF_ROOT_MAP) ? ITEM_ROOT_MAP : 0u), h.root);
        KYV_ACCT_ADD(0, 8);  // header: flags, root
        KYV_ACCT_ADD(1, 8);  // work-list item
      }
      if (lane == 0) { wl.cnt[list] = (uint8_t)__popcll(wm); KYV_ACCT_ADD(1, 1); }
    }
    if (gated && !walk && st != ST_NONE) {
      o.status[(size_t)k * v.nres + r] = st;
      const uint32_t ps = o.pss_slot[k];
      if (ps != NONE && pf) o.pss_fails[(size_t)ps * v.nres + r] = pf;
      KYV_ACCT_ADD(1, 1 + ((ps != NONE && pf) ? 4 : 0));
    }
  }
}

// Deny rules whose conditions need no JMESPath (plain request.object operands; C5's 50 deny / precondition policies):
// pair_match, then the preconditions and deny programs of validateDeny (validation.go:281-288, 437-464), without
// the PodSecurity call and work-list code of match_kernel's dispatch, whose call frame and register need spilled the
// rule loop (C5 round 4: match_kernel<false> 4.47 ms, 5.3 GB of scratch writes per evaluation)
#ifndef KYV_NO_KERNELS  // (kyv_engine.hip launches the kernels through kyv_launch.inc)
__global__ void __launch_bounds__(BLOCK) __attribute__((amdgpu_waves_per_eu(KYV_MATCH_WPE)))
match_deny_kernel(const View* __restrict__ vp, DevOut o, const uint32_t* __restrict__ mrules, uint32_t nm) {
  const View& v = *vp;
  const uint32_t lane = threadIdx.x;
  const uint32_t r = blockIdx.x * BLOCK + lane;
  const bool active = r < v.nres;
  const uint32_t* gate = active ? v.gate + (size_t)v.hdr[r].kclass * v.gate_words : nullptr;
  if (active) KYV_ACCT_ADD(0, 4);  // header: kind class
  (void)lane;
  for (uint32_t mi = 0; mi < nm; mi++) {
    const uint32_t k = mrules[mi];
    const bool gated = active && ((gate[k >> 5] >> (k & 31)) & 1u);
    if (!__ballot(gated)) continue;
    if (!gated) continue;
    const RuleDesc& rd = v.rules[k];
    uint8_t st = ST_NONE;
    if (pair_match(v, r, rd, &st)) {
      const NodeTab R{v.nodes + v.hdr[r].root};
      KYV_ACCT_ADD(0, 4);  // header: root
      uint32_t ec, es, eg;
      // preconditions (pass 0, when the rule has them) then the deny program (pass 1): one inlined evaluation site
      for (uint32_t pass = rd.pre != NONE ? 0u : 1u; pass < 2; pass++) {
        const int c = eval_prog_inl<false>(v, R, pass ? rd.root : rd.pre, &ec, &es, &eg, NONE, r);
        if (c == CR_FB) { st = (KYV_WHY(FBW_COND), ST_FALLBACK); break; }
        if (c == CR_PANIC) { st = ST_PANIC; break; }
        if (pass == 0) {
          if (c == CP_ERROR) { st = ST_ERROR | ST_MARK_PRE; break; }
          if (c == CR_FALSE) { st = ST_SKIP | ST_MARK_PRE; break; }
        } else {
          st = c == CP_ERROR ? ST_ERROR : c == CR_TRUE ? ST_FAIL : ST_PASS;
        }
      }
    }
    if (st != ST_NONE) { o.status[(size_t)k * v.nres + r] = st; KYV_ACCT_ADD(1, 1); }
  }
}
#endif

// Staged match records of match_rec_kernel. Every wave runs a rule loop, so a rule's match program read from the rule
// descriptors was a chain of dependent uniform loads (rule list -> RuleDesc -> Filter -> KindDesc / pattern sids ->
// pattern flags -> the string's glob mask) paid by every wave for every rule (C4 round 4: wait 0.85). The host lays
// each rule's match block out as one fixed-size record (kinds, name / names / namespaces patterns with their glob-mask
// bit resolved); a wave reads it with scalar loads and evaluates it against the lane's resource facts (kind, name,
// namespace and their glob-mask words) held in registers. A filter with annotations or selectors, or one whose matching
// kind carries a group / version, runs condition_block's tail itself after the record's checks passed; a rule the
// record cannot hold (exceptions, more than MREC_F filters / 4 kinds / 2 names / 2 namespaces, a glob without a mask)
// runs pair_match in match_walk_generic_kernel.
constexpr uint32_t MREC_F = 3, MREC_LABELS = 8, PAT_MASK = 0x80000000u;
// MR_EMPTY: empty_may_match; MR_ECONST: the empty-OldResource retry's outcome is a constant of the rule (no filter can
// reach a namespace selector for a kind-less resource), precomputed on the host as MR_EMATCH / MR_END (matched /
// nondeterministic); MR_FASTEVAL: every filter is decided by the branch-free path (kinds without group / version,
// tails covered by the lane tail facts)
enum MRecBits : uint32_t { MR_FAST = 1u, MR_MASKS = 2u, MR_EMPTY = 4u, MR_ECONST = 8u, MR_EMATCH = 16u, MR_END = 32u,
                           MR_FASTEVAL = 64u };
constexpr uint32_t MRF_KPACK = 1u << 29;  // the filter's kinds are packed: sid | (group / version atom + 1) << 24
struct MRecFilter {   // 48 bytes
  uint32_t idx;       // Filter index (condition_block of a tail filter)
  uint32_t bits;      // [0,16) FilterFlag, [16,19) kinds, [19,21) names, 21 name, [22,24) namespaces,
                      // [24,28) kind i has a group / version, 28 tail (annotations / selector / namespace selector),
                      // 29 MRF_KPACK
  uint32_t kinds[4];  // kind sids (NONE: "*")
  uint32_t pats[5];   // name, names[2], namespaces[2]: PAT_MASK | glob-mask index + 1, or the exact sid
  uint32_t pad;
};
struct MRec {         // 160 bytes
  uint32_t k;         // rule
  uint32_t bits;      // MRecBits | match mode << 8 | exclude mode << 16 | match filters << 24 | exclude filters << 28
  uint32_t kind, flags;  // RuleDesc.kind / .flags
  MRecFilter f[MREC_F];  // match filters, then exclude filters
};
static_assert(sizeof(MRec) == 160, "match record size");

enum MFactFlag : uint32_t { MF_ISNS = 1u, MF_KIND_EMPTY = 2u };
struct MFacts {       // the lane's resource: what condition_block compares, and the glob-mask words of its strings
  uint32_t gk, rname, rns, fl;
  uint32_t n0, n1, n2, n3;  // mask words of rname
  uint32_t s0, s1, s2, s3;  // mask words of rns
};
KYV_HD bool mf_bit(uint32_t m0, uint32_t m1, uint32_t m2, uint32_t m3, uint32_t g) {
  const uint32_t w = g >> 5;
  const uint32_t x = w == 0 ? m0 : w == 1 ? m1 : w == 2 ? m2 : m3;
  return (x >> (g & 31u)) & 1u;
}
// glob_sid(pattern, s) for a record pattern: the mask bit (which holds pattern == s too), or sid equality for a
// pattern without '*' / '?' / non-ASCII runes
KYV_HD bool pat_name(const MFacts& mf, uint32_t p) {
  return (p & PAT_MASK) ? mf_bit(mf.n0, mf.n1, mf.n2, mf.n3, (p & 0xFFu) - 1u) : p == mf.rname;
}
KYV_HD bool pat_ns(const MFacts& mf, uint32_t p) {
  return (p & PAT_MASK) ? mf_bit(mf.s0, mf.s1, mf.s2, mf.s3, (p & 0xFFu) - 1u) : p == mf.rns;
}

// condition_block (kyv_eval.h:500-539) after its kinds / name / namespace checks: annotations, selector (over the
// lane's labels, staged in LDS), namespace selector, user info
KYV_HD bool cb_tail(const View& v, const Filter& f, const ResView& rv, const LabelSet& labels, const LabelSet& nsl,
                    bool uic, bool* nd, uint32_t fl) {
  if (f.nann) {
    LabelSet as{rv.R, rv.h ? rv.h->ann : NONE, nullptr, 0};
    const uint32_t n = ls_count(as);
    for (uint32_t q = 0; q < f.nann; q++) {
      const uint32_t kp = v.pool[f.ann + 2 * q], vp = v.pool[f.ann + 2 * q + 1];
      bool m = false;
      for (uint32_t i = 0; i < n && !m; i++) m = glob_sid(v, kp, ls_key(as, i)) && glob_sid(v, vp, ls_val(as, i));
      if (!m) return false;
    }
  }
  if ((f.flags & FF_HAS_SEL) && check_selector(v, v.sels[f.sel], labels, nd) != 1) return false;
  if ((f.flags & FF_HAS_NSSEL) && !(fl & MF_ISNS) && (!(fl & MF_KIND_EMPTY) || (f.flags & FF_KINDS_STAR))) {
    if (check_selector(v, v.sels[f.sel + 1], nsl, nd) != 1) return false;
  }
  return !(uic && (f.flags & FF_USERINFO));
}

// Lane tail facts (round 5). The tail of a filter (annotations, selector, namespace selector: condition_block after its
// kinds / name / namespace checks) was evaluated per (rule, resource) from the resource's label and annotation maps,
// each test a chain of dependent loads (label row -> its string's glob-mask word); C4 (10,440 rules) spent ~3,000 SIMD
// cycles per (wave, rule) there. The slice's tail filters are reduced on the host to a few ruleset-wide facts -- label
// values of the most used selector keys (slots), namespace-label values of the namespace-selector keys, the outcome
// of each distinct wildcard selector requirement (ReplaceInSelector, pkg/utils/wildcards/wildcards.go:13-50) and of
// each distinct annotation pair -- which every lane computes once from its resource (tail_facts); a covered filter
// (MRecFilter.pad = 1 + its TailProg) then tests registers. Filters with anything else keep cb_tail.
constexpr uint32_t TF_SLOTS = 8, TF_NSSLOTS = 4, TF_WILD = 16, TF_ANN = 32, TF_GV = 16;
struct TailCfg {  // per slice (scalar loads)
  uint32_t nslot, nnsslot, nwild, nann;
  uint32_t slot[TF_SLOTS];      // label keys read by exact-key requirements
  uint32_t nsslot[TF_NSSLOTS];  // namespace-label keys of the namespace selectors
  uint32_t wkey[TF_WILD], wval[TF_WILD], wrkey[TF_WILD], wrval[TF_WILD];  // wildcard requirements (SelReq RQ_WILD)
  uint32_t akey[TF_ANN], aval[TF_ANN];  // annotation (key glob, value glob) pairs
  uint32_t ngv;
  uint32_t gvmode[TF_GV], gvg[TF_GV], gvv[TF_GV];  // group / version refinements of record kinds (KindDesc)
  // how each atom's key / value pattern is tested against a string (glob_sid, kyv_eval.h): TC_EXACT | sid compare
  // (a pattern without '*' / '?'), TC_MASK | glob-mask bit (< 32: one mask word), else the pattern sid for glob_sid
  uint32_t wkc[TF_WILD], wvc[TF_WILD], akc[TF_ANN], avc[TF_ANN];
  uint32_t onemask;  // the batch keeps one glob-mask word per string: TC_MASK codes are valid
};
enum TailCode : uint32_t { TC_EXACT = 0x40000000u, TC_MASK = 0x80000000u };
// a covered tail filter, flattened so one group of scalar loads fetches it: the annotation atoms that must all match
// and the selector / namespace-selector requirements with their slot or atom and literal values
constexpr uint32_t TP_REQ = 4, TP_VALS = 4;
struct SelProg {
  uint32_t n;                       // requirements; NONE: statically invalid selector (error)
  uint32_t req[TP_REQ];             // op | slot or atom << 8 | nvals << 16
  uint32_t vals[TP_REQ][TP_VALS];   // exact requirements' values
};
struct TailProg {                   // 48 words
  uint32_t ann;
  SelProg sel, nssel;
  uint32_t pad[5];
};
static_assert(sizeof(TailProg) == 192, "tail program size");
struct TailTab {
  const TailCfg* cfg;
  const TailProg* prog;
};
// the facts of one resource (or of the empty OldResource: no labels, no annotations, the lane's namespace labels)
struct LaneTail {
  uint32_t sv[TF_SLOTS];    // label value of slot key (NONE: absent)
  uint32_t nv[TF_NSSLOTS];  // namespace-label value of namespace slot key
  uint32_t wno, werr, wnd;  // wildcard requirement a: bit a = selector result 0 / error / nondeterministic
  uint32_t ann;             // annotation atom a: bit a = some annotation matches both globs
  uint32_t gv;              // kind refinement a: bit a = the resource's group / version satisfy it (kinds_match)
};
template <int N>
KYV_HD __attribute__((always_inline)) uint32_t pick(const uint32_t (&a)[N], uint32_t i) {  // a[i], i uniform, no scratch
  uint32_t x = NONE;
#pragma unroll
  for (int j = 0; j < N; j++) x = i == (uint32_t)j ? a[j] : x;
  return x;
}
KYV_HD uint32_t tf_ld(const uint32_t* p) {
#if defined(__HIP_DEVICE_COMPILE__)
  return sld32(p);
#else
  return *p;
#endif
}
// glob_sid(pattern, s) through an atom's test code, the string's glob-mask word `m` loaded once by the caller
KYV_HD __attribute__((always_inline)) bool tc_test(const View& v, uint32_t code, uint32_t pat, uint32_t s, uint32_t m) {
  if (code & TC_MASK) return (m >> (code & 31u)) & 1u;
  if (code & TC_EXACT) return s == pat;
  return glob_sid(v, pat, s);
}
KYV_HD __attribute__((always_inline)) uint32_t mask0(const View& v, uint32_t s) {
  return v.str_gmask ? v.str_gmask[(size_t)s * v.gmask_words] : 0u;
}
// the facts of labels `ls`, annotations `as`, namespace labels `nsl` (CheckSelector's requirement loop per wildcard
// requirement, as check_selector in kyv_eval.h). Each label / annotation string's mask word is loaded once and every
// atom tested against it (round 5: an atom loop calling glob_sid reloaded it per atom -- a dependent global load per
// (atom, annotation) pair)
KYV_HD void tail_facts(const View& v, const TailCfg* c, const LabelSet& ls, const LabelSet& as, const LabelSet& nsl,
                       const ResHeader* h, LaneTail& t) {
  const uint32_t nslot = tf_ld(&c->nslot), nns = tf_ld(&c->nnsslot), nw = tf_ld(&c->nwild), na = tf_ld(&c->nann);
  const bool one = tf_ld(&c->onemask) != 0 && v.str_gmask && v.gmask_words == 1;
  const uint32_t nl = ls_count(ls);
#pragma unroll
  for (uint32_t s = 0; s < TF_SLOTS; s++) t.sv[s] = NONE;
#pragma unroll
  for (uint32_t s = 0; s < TF_NSSLOTS; s++) t.nv[s] = NONE;
  // wildcard requirements over the labels: per atom the hit count and whether hits are valid label pairs
  uint32_t hit1 = 0, hit2 = 0, valid = 0, invalid = 0;  // bit a: >= 1 hit, >= 2 hits, a valid hit, an invalid hit
  for (uint32_t i = 0; i < nl; i++) {
    const uint32_t k = ls_key(ls, i), val = ls_val(ls, i);
#pragma unroll
    for (uint32_t q = 0; q < TF_SLOTS; q++)
      if (q < nslot && t.sv[q] == NONE && k == tf_ld(&c->slot[q])) t.sv[q] = val;  // ls_find: the first such label
    if (!nw) continue;
    const uint32_t km = one ? mask0(v, k) : 0u, vm = one ? mask0(v, val) : 0u;
    const bool ok = (v.str_flags[k] & SF_LKEY) && (v.str_flags[val] & SF_LVAL);
    for (uint32_t a = 0; a < nw; a++) {
      const uint32_t kc = one ? tf_ld(&c->wkc[a]) : 0u, vc = one ? tf_ld(&c->wvc[a]) : 0u;
      if (tc_test(v, kc, tf_ld(&c->wkey[a]), k, km) && tc_test(v, vc, tf_ld(&c->wval[a]), val, vm)) {
        const uint32_t bit = 1u << a;
        hit2 |= hit1 & bit;
        hit1 |= bit;
        if (ok) valid |= bit; else invalid |= bit;
      }
    }
  }
  const uint32_t nn = ls_count(nsl);
  for (uint32_t i = 0; i < nn && nns; i++) {
    const uint32_t k = ls_key(nsl, i);
#pragma unroll
    for (uint32_t q = 0; q < TF_NSSLOTS; q++)
      if (q < nns && t.nv[q] == NONE && k == tf_ld(&c->nsslot[q])) t.nv[q] = ls_val(nsl, i);
  }
  t.wno = t.werr = 0;
  t.wnd = hit2 & valid & invalid;
  for (uint32_t a = 0; a < nw; a++) {
    const uint32_t bit = 1u << a;
    if (!(hit1 & bit)) {
      const uint32_t rk = tf_ld(&c->wrkey[a]), rv = tf_ld(&c->wrval[a]);
      if (rk == NONE) t.werr |= bit;
      else {
        const uint32_t i = ls_find(ls, rk);
        if (!(i != NONE && ls_val(ls, i) == rv)) t.wno |= bit;
      }
    } else if ((invalid & bit) && !(valid & bit)) {
      t.werr |= bit;
    }
  }
  // kinds_match's group / version refinement of kind entry a (kyv_eval.h), for this resource
  t.gv = 0;
  const uint32_t ngv = tf_ld(&c->ngv);
  for (uint32_t a = 0; a < ngv; a++) {
    const uint32_t mode = tf_ld(&c->gvmode[a]), kg = tf_ld(&c->gvg[a]), kv = tf_ld(&c->gvv[a]);
    const uint32_t g = h ? h->group : SID_EMPTY, ver = h ? h->version : SID_EMPTY, gvs = h ? h->gv : SID_EMPTY;
    bool r;
    if (mode == 1) r = kg == g && kv == ver;
    else if (mode == 2) {
      const uint32_t ln = v.str_len[kg], sn = v.str_len[gvs];
      r = sn >= ln && bytes_eq(sbytes(v, gvs), sbytes(v, kg), ln);
    } else r = false;
    if (r) t.gv |= 1u << a;
  }
  t.ann = 0;
  const uint32_t nan = ls_count(as);
  for (uint32_t i = 0; i < nan && na; i++) {
    const uint32_t k = ls_key(as, i), val = ls_val(as, i);
    const uint32_t km = one ? mask0(v, k) : 0u, vm = one ? mask0(v, val) : 0u;
    for (uint32_t a = 0; a < na; a++) {
      const uint32_t kc = one ? tf_ld(&c->akc[a]) : 0u, vc = one ? tf_ld(&c->avc[a]) : 0u;
      if (tc_test(v, kc, tf_ld(&c->akey[a]), k, km) && tc_test(v, vc, tf_ld(&c->aval[a]), val, vm)) t.ann |= 1u << a;
    }
  }
}

// check_selector (kyv_eval.h) from the facts over a selector program: *r_out 1 match, 0 no, -1 error (per lane) and
// *nd as check_selector raises it: requirements after an erroring wildcard requirement are not evaluated; branch-free
// per lane, the program's fields uniform
KYV_HD __attribute__((always_inline)) void sel_prog(const SelProg& sp, const LaneTail& t, bool ns, int* r_out, bool* nd) {
  if (sp.n == NONE) { *r_out = -1; return; }
  bool err = false, no = false, n = false;
#pragma unroll
  for (uint32_t q = 0; q < TP_REQ; q++) {
    if (q >= sp.n) continue;
    const uint32_t op = sp.req[q] & 0xFFu, m = (sp.req[q] >> 8) & 0xFFu, nv = sp.req[q] >> 16;
    if (op == RQ_WILD) {
      n = n | (!err & (((t.wnd >> m) & 1u) != 0));
      no = no | (((t.wno >> m) & 1u) != 0);
      err = err | (((t.werr >> m) & 1u) != 0);
      continue;
    }
    const uint32_t val = ns ? pick(t.nv, m) : pick(t.sv, m);
    const bool has = val != NONE;
    bool inset = false;
#pragma unroll
    for (uint32_t k = 0; k < TP_VALS; k++)
      if (k < nv) inset = inset | (sp.vals[q][k] == val);
    inset = inset & has;
    const bool ok = (op == RQ_EQ || op == RQ_IN) ? inset : op == RQ_NOTIN ? (!has | !inset) : op == RQ_EXISTS ? has : !has;
    no = no | !ok;
  }
  *nd = *nd | n;
  *r_out = err ? -1 : no ? 0 : 1;
}
KYV_HD __attribute__((always_inline)) SelProg ld_selprog(const SelProg* p) {
#if defined(__HIP_DEVICE_COMPILE__)
  return sld(p);
#else
  return *p;
#endif
}
// cb_tail (above) of a covered filter (program pi), from the lane's facts; *fnd: the nondeterminism cb_tail would raise
KYV_HD __attribute__((always_inline)) bool tail_prog(const TailTab& tt, uint32_t pi, uint32_t b, const LaneTail& t,
                                                     uint32_t fl, bool uic, bool* fnd) {
  const TailProg* tp = tt.prog + pi;
  const uint32_t ann = tf_ld(&tp->ann);
  const bool annok = (t.ann & ann) == ann;
  bool sok = true, n1 = false;
  if (b & FF_HAS_SEL) {
    int r;
    sel_prog(ld_selprog(&tp->sel), t, false, &r, &n1);
    sok = r == 1;
  }
  bool nsok = true, n2 = false, nscond = false;
  if (b & FF_HAS_NSSEL) {
    nscond = !(fl & MF_ISNS) & (!(fl & MF_KIND_EMPTY) | ((b & FF_KINDS_STAR) != 0));
    int r;
    sel_prog(ld_selprog(&tp->nssel), t, true, &r, &n2);
    nsok = !nscond | (r == 1);
  }
  *fnd = annok & (n1 | (sok & nscond & n2));
  return annok & sok & nsok & !(uic && (b & FF_USERINFO));
}

// condition_block (kyv_eval.h) of a record filter: kinds, name, names and namespaces from the record and the lane's
// facts (a kind with a group / version that equals the resource's: kinds_match decides), then the tail. Loops over the
// record's fixed-size arrays are unrolled with static indices: the record stays in scalar registers (a dynamic index
// would copy it to per-lane scratch)
KYV_HD __attribute__((always_inline)) bool cb_rec(const View& v, const MRecFilter& F, const MFacts& mf, const ResView& rv, const LabelSet& labels,
                   const LabelSet& nsl, bool uic, bool* nd, const TailTab& tt, const LaneTail& lt) {
  const uint32_t b = F.bits;
  const uint32_t nk = (b >> 16) & 7u;
  if (nk) {
    bool ok = false, gv = false;
#pragma unroll
    for (uint32_t i = 0; i < 4; i++) {
      if (i < nk && !ok) {
        const uint32_t kd = (F.kinds[i] != NONE && (b & MRF_KPACK)) ? F.kinds[i] & 0xFFFFFFu : F.kinds[i];
        if (kd == NONE) ok = true;
        else if (kd == mf.gk) { ok = true; gv = (b >> (24 + i)) & 1u; }
      }
    }
    if (gv) ok = kinds_match(v, v.filters[F.idx], rv.h);
    if (!ok) return false;
  }
  if (((b >> 21) & 1u) && !pat_name(mf, F.pats[0])) return false;
  const uint32_t nn = (b >> 19) & 3u;
  if (nn && !(pat_name(mf, F.pats[1]) || (nn > 1 && pat_name(mf, F.pats[2])))) return false;
  const uint32_t ns = (b >> 22) & 3u;
  if (ns && !(pat_ns(mf, F.pats[3]) || (ns > 1 && pat_ns(mf, F.pats[4])))) return false;
  if ((b >> 28) & 1u) {
    if (F.pad) {
      bool fnd;
      const bool c = tail_prog(tt, F.pad - 1, b, lt, mf.fl, uic, &fnd);
      *nd = *nd | fnd;
      return c;
    }
    return cb_tail(v, v.filters[F.idx], rv, labels, nsl, uic, nd, mf.fl);
  }
  return !(uic && (b & FF_USERINFO));
}

// The record's header words (k, bits, kind, flags) and its filter slots are read with scalar loads from the record
// array (wave-uniform addresses) where they are needed: a local copy of the whole record indexed by the slot number
// would live in per-lane scratch memory
struct MRecHead { uint32_t k, bits, kind, flags; };

// match_rule (kyv_eval.h) over a record: slot j of the record's filters is match filter j (j < nmf) or exclude filter
// j - nmf, visited in order with match_rule's short-circuits (a filter is not evaluated once the block's outcome is
// known, so its nondeterminism flag is not raised either): ANY stops at the first matching filter, ALL / plain at the
// first failing one (a filter without resource description fails it); a failed match block ends the rule before its
// exclude block; exclude ANY / plain excludes on the first excluding filter, exclude ALL only when every filter excludes
KYV_HD __attribute__((always_inline)) bool match_rule_rec(const View& v, const MRec* Rp, uint32_t bits, const MFacts& mf,
                                                          const ResView& rv, const LabelSet& labels, const LabelSet& nsl,
                                                          bool* nd, const TailTab& tt, const LaneTail& lt) {
  const uint32_t mm = (bits >> 8) & 0xFFu, em = (bits >> 16) & 0xFFu, nmf = (bits >> 24) & 0xFu, nef = bits >> 28;
  const bool any = mm == MM_ANY, all = mm == MM_ALL || mm == MM_PLAIN;
  if (!any && !all) return false;
  const bool eany = em == MM_ANY || em == MM_PLAIN, eall = em == MM_ALL;
  bool one = false, failed = false, excluded = false, byAll = true;
  const uint32_t n = nmf + nef;
#pragma unroll 1
  for (uint32_t j = 0; j < n; j++) {
    const bool ism = j < nmf;
    if (ism) {
      if (any ? one : failed) continue;
    } else {
      if (any ? !one : failed) break;  // the match block failed: the exclude block is not evaluated
      if (eany ? excluded : (!eall || !byAll)) break;
    }
#if defined(__HIP_DEVICE_COMPILE__)
    const MRecFilter F = sld(&Rp->f[j]);
#else
    const MRecFilter F = Rp->f[j];
#endif
    const bool skip = ism ? (F.bits & FF_ZERO_RD) != 0 : ((F.bits & FF_ZERO_RD) && !(F.bits & FF_USERINFO));
    const bool c = !skip && cb_rec(v, F, mf, rv, labels, nsl, !ism, nd, tt, lt);
    if (ism) {
      if (any) { if (c) one = true; }
      else if (!c) failed = true;
    } else if (eany) {
      if (c) excluded = true;
    } else if (!c) {
      byAll = false;
    }
  }
  if (any ? !one : failed) return false;
  if (eany && excluded) return false;
  if (eall && byAll && nef > 0) return false;
  return true;
}

// pair_match (kyv_pss.h) of a record rule (compiled match block, no exceptions); a rule whose match may accept the
// empty OldResource (MR_EMPTY, validation.go:606) retries against it: the facts of the empty resource (mf0: kind,
// name and namespace "", no labels, no annotations)
KYV_HD __attribute__((always_inline)) bool pair_match_rec(const View& v, const MRec* Rp, const MRecHead& H, const MFacts& mf,
                                                          const ResView& rv, const LabelSet& labels, const LabelSet& nsl,
                                                          const MFacts& mf0, uint8_t* st, const TailTab& tt,
                                                          const LaneTail& lt, const LaneTail& lt0) {
  bool nd = false;
  if (!(H.flags & RD_GATE_EXACT)) {
    KYV_ACCT_ADD(0, 16);  // header words the match program compares (model, as pair_match)
    bool m = match_rule_rec(v, Rp, H.bits, mf, rv, labels, nsl, &nd, tt, lt);
    if (!m && (H.bits & MR_EMPTY))
      m = match_rule_rec(v, Rp, H.bits, mf0, ResView{rv.R, nullptr}, LabelSet{NodeTab{nullptr}, 0, nullptr, 0}, nsl, &nd,
                         tt, lt0);
    if (!m) { *st = ST_NONE; return false; }
  }
  if (nd) { *st = ST_ND; return false; }
  if ((H.kind & 0xFFu) == RK_FALLBACK) { *st = ST_FALLBACK; return false; }
  return true;
}

// ---- branch-free record evaluation (round 5). The general path above decides a filter with a divergent branch per
// test (exec-mask juggling dominated the C4 match kernel: ~650 instructions per (wave, rule), 40 % of them exec-mask
// and spill moves). For MR_FASTEVAL records every per-lane condition is a boolean combined with & / |; branches remain
// only on the record's uniform fields. The short-circuits of match_rule / condition_block / check_selector are kept as
// masks: a filter's or requirement's nondeterminism flag counts only on lanes where the reference would have evaluated
// it.
// condition_block of a record filter (uic: an exclude filter), branch-free per lane; *fnd: its nondeterminism
KYV_HD __attribute__((always_inline)) bool filt_fast(const MRecFilter& F, const MFacts& mf, const TailTab& tt,
                                                     const LaneTail& t, bool uic, bool* fnd) {
  const uint32_t b = F.bits, nk = (b >> 16) & 7u;
  bool kok = nk == 0;
#pragma unroll
  for (uint32_t i = 0; i < 4; i++)
    if (i < nk) {
      const uint32_t kd = F.kinds[i];
      if (kd == NONE) kok = true;
      else if (!(b & MRF_KPACK)) kok = kok | (kd == mf.gk);  // (MR_FASTEVAL: no group / version kinds then)
      else if (!((b >> (24 + i)) & 1u)) kok = kok | ((kd & 0xFFFFFFu) == mf.gk);
      else kok = kok | (((kd & 0xFFFFFFu) == mf.gk) & (((t.gv >> ((kd >> 24) - 1)) & 1u) != 0));  // sid | (atom + 1) << 24
    }
  bool nok = true;
  if ((b >> 21) & 1u) nok = pat_name(mf, F.pats[0]);
  const uint32_t nn = (b >> 19) & 3u;
  if (nn) nok = nok & (pat_name(mf, F.pats[1]) | (nn > 1 && pat_name(mf, F.pats[2])));
  bool sok = true;
  const uint32_t ns = (b >> 22) & 3u;
  if (ns) sok = pat_ns(mf, F.pats[3]) | (ns > 1 && pat_ns(mf, F.pats[4]));
  const bool head = kok & nok & sok;
  *fnd = false;
  if (!((b >> 28) & 1u)) return head & !(uic && (b & FF_USERINFO));
  bool tnd;
  const bool c = tail_prog(tt, F.pad - 1, b, t, mf.fl, uic, &tnd);
  *fnd = head & tnd;
  return head & c;
}
// match_rule over an MR_FASTEVAL record (filter slots F[0..2]), branch-free per lane
KYV_HD __attribute__((always_inline)) bool match_fast(const View& v, uint32_t bits, const MRecFilter* F, const MFacts& mf,
                                                      const TailTab& tt, const LaneTail& t, bool* nd) {
  const uint32_t mm = (bits >> 8) & 0xFFu, em = (bits >> 16) & 0xFFu, nmf = (bits >> 24) & 0xFu, nef = bits >> 28;
  const bool any = mm == MM_ANY, all = mm == MM_ALL || mm == MM_PLAIN;
  if (!any && !all) return false;
  bool one = false, failed = false, n = false;
#pragma unroll
  for (uint32_t j = 0; j < MREC_F; j++) {
    if (j < nmf) {
      const bool zero = (F[j].bits & FF_ZERO_RD) != 0;
      const bool ev = any ? !one : !failed;  // the reference reaches this filter
      bool c = false;
      if (!zero) {
        bool fnd;
        c = filt_fast(F[j], mf, tt, t, false, &fnd);
        n = n | (ev & fnd);
      }
      if (any) one = one | (ev & c);
      else failed = failed | (ev & (zero | !c));
    }
  }
  const bool matched = any ? one : !failed;
  const bool eany = em == MM_ANY || em == MM_PLAIN, eall = em == MM_ALL;
  bool excluded = false, byAll = true;
#pragma unroll
  for (uint32_t j = 0; j < MREC_F; j++) {
    if (j >= nmf && j < nmf + nef && (eany || eall)) {
      const bool skip = (F[j].bits & FF_ZERO_RD) && !(F[j].bits & FF_USERINFO);
      const bool ev = matched & (eany ? !excluded : byAll);
      bool c = false;
      if (!skip) {
        bool fnd;
        c = filt_fast(F[j], mf, tt, t, true, &fnd);
        n = n | (ev & fnd);
      }
      if (eany) excluded = excluded | (ev & c);
      else byAll = byAll & !(ev & !c);
    }
  }
  *nd = *nd | n;
  return matched & !(eany & excluded) & !(eall & byAll & (nef > 0));
}

// Pattern / anyPattern rules without preconditions (and compile-time fallback rules): the match phase is only
// pair_match (kind gate, match / exclude program, PolicyException candidates) and the work-list append, so these
// kernels carry none of the dispatch code (conditions, PodSecurity calls) whose register need made the rule loop
// of match_kernel spill every iteration (C4: 10,440 rules per wave, 252 GB of scratch writes per evaluation).
// match_rec_kernel takes the rules as staged match records (above) through a kind index;
// match_walk_generic_kernel the rules whose match block does not fit a record (pair_match; one kernel for both needs
// both match programs' registers: 111 VGPRs, 4 waves/SIMD).
// kWpe: occupancy target (KYV_MATCHW_WPE = 4 / 6 / 8 at run time; 4 by default)
KYV_HD void match_walk_append(const View& v, DevOut& o, WorkLists& wl, uint32_t k, uint32_t rkind, uint32_t r, bool gated,
                              bool m, uint8_t st, uint32_t hflags, uint32_t hroot) {
  const uint32_t lane = threadIdx.x;
  bool walk = false;
  if (m) {  // a matched pattern pair: walk it (RF_MAGIC: the CPU engine)
    if (hflags & RF_MAGIC) st = ST_FALLBACK;
    else walk = true;
  }
  const unsigned long long wm = __ballot(walk);
  if (rkind == RK_PATTERN || rkind == RK_ANYPATTERN) {
    const size_t list = (size_t)(k - o.rule_lo) * wl.nwaves + blockIdx.x;
    if (walk) {
      wl.items[list * WAVE + __popcll(wm & ((1ull << lane) - 1))] =
          make_uint2(r | ((hflags & RF_ROOT_MAP) ? ITEM_ROOT_MAP : 0u), hroot);
      KYV_ACCT_ADD(1, 8);  // work-list item
    }
    if (lane == 0) { wl.cnt[list] = (uint8_t)__popcll(wm); KYV_ACCT_ADD(1, 1); }
  }
  if (gated && !walk && st != ST_NONE) { o.status[(size_t)k * v.nres + r] = st; KYV_ACCT_ADD(1, 1); }
}

// Shape rules (jit.cpp, round 5): pattern rules whose compiled pattern is one of the ruleset's deduplicated shapes
// (structurally identical patterns: same keys, handlers, leaves, path templates and columns; C4's 10,440 rules use 15)
// get their walk verdict from the shape tables (ShapeTab, kyv_wave.h), computed once per (shape, resource) by
// kyv_jit_shapes: a matched pair's verdict byte is its shape's, and a FAIL pair's staged failing-path record is its
// shape's record (the record carries no rule: StageRec). The pair is decided here; no work-list item, no walk.
constexpr uint32_t SHAPE_REGS = 16;  // shape verdicts a lane keeps in registers (4 words of bytes)
KYV_HD void mrec_shape_out(const View& v, DevOut& o, const ShapeTab& sh, uint32_t s, bool wide, uint32_t k, uint32_t r,
                           bool gated, bool m, uint8_t st, uint32_t hflags, uint32_t w, const uint32_t (&sv)[4]) {
  const uint32_t lane = threadIdx.x & (WAVE - 1);
  bool rec = false;
  if (m) {
    if (hflags & RF_MAGIC) {
      st = ST_FALLBACK;  // pattern pairs on such resources go to the CPU engine (as match_walk_append)
    } else {
      st = s < SHAPE_REGS ? (uint8_t)(pick(sv, s >> 2) >> (8 * (s & 3))) : sh.st[(size_t)s * v.nres + r];
      rec = (st & 7u) == ST_FAIL;
      KYV_ACCT_ADD(0, 1 + (rec ? sizeof(FailRec) : 0));  // the shape's verdict (and record) for this resource
    }
  }
  const unsigned long long rm = __ballot(rec);
  if (rm) {
    FailRec* chunk = o.stage + o.rbase[k - o.rule_lo] + (size_t)w * WAVE;  // chunk (k, w): one alternative
    if (rec) {
      const uint32_t at = (uint32_t)__popcll(rm & ((1ull << lane) - 1));
      FailRec f = sh.rec[(size_t)s * v.nres + r];
      if (wide) {  // a rule with metadata-expansion sites: whole records (resolved keys), as the walk stages them
        f.rule = k;
        chunk[at] = f;
        KYV_ACCT_ADD(2, sizeof(FailRec));
      } else {
        StageRec x;
        x.tmpl = f.tmpl;
        x.lane_alt = lane | ((uint32_t)f.alt << 8);
        for (int i = 0; i < MAX_IDX; i++) x.idx[i] = f.idx[i];
        reinterpret_cast<StageRec*>(chunk)[at] = x;
        KYV_ACCT_ADD(2, sizeof(StageRec));
      }
    }
    if (lane == 0) { o.rcnt[(size_t)(k - o.rule_lo) * sh.nwaves + w] = (uint16_t)__popcll(rm); KYV_ACCT_ADD(1, 2); }
  }
  if (gated && st != ST_NONE) { o.status[(size_t)k * v.nres + r] = st; KYV_ACCT_ADD(1, 1); }
}

// Kind index of a slice's match records (round 5): records recs[off[c], off[c + 1]) are (copies of) those whose rule's
// kind gate admits kind class c (policycache's kind -> policies index, pkg/policycache/store.go:96-170, at compile time)
struct MRecIndex {
  const uint32_t* off;  // [nclass + 1]
  const MRec* recs;     // the records of class c at [off[c], off[c + 1])
};

// A resource's match facts (round 5): what the record path compares (MFacts) and its lane tail facts, computed once
// per evaluation by facts_kernel (the tail configuration is ruleset-wide) and read by every slice's match_rec_kernel
struct ResFacts {
  MFacts mf;
  LaneTail lt;
  uint32_t hflags, hroot, pad;
};
static_assert(sizeof(ResFacts) == 128, "resource facts size");

// the lane's record-path facts (kind, name, namespace, their glob-mask words)
template <int kMW>
KYV_HD __attribute__((always_inline)) MFacts res_mfacts(const View& v, const ResHeader& h) {
  MFacts mf{};
  const uint32_t name = h.name, kind = h.kind;
  mf.gk = h.gvk_kind;
  mf.rname = name == SID_EMPTY ? h.gen_name : name;
  const bool isNs = v.str_len[kind] == 9 && bytes_eq(sbytes(v, kind), (const uint8_t*)"Namespace", 9);
  mf.rns = isNs ? name : h.ns;
  mf.fl = (isNs ? MF_ISNS : 0u) | (kind == SID_EMPTY ? MF_KIND_EMPTY : 0u);
  if (v.str_gmask) {  // (records with a glob-mask pattern are only built when the batch has masks)
    const uint32_t gw = v.gmask_words;
    const uint32_t* a = v.str_gmask + (size_t)mf.rname * gw;
    const uint32_t* b = v.str_gmask + (size_t)mf.rns * gw;
    mf.n0 = a[0]; mf.s0 = b[0];
    if (kMW > 1) {
      if (gw > 1) { mf.n1 = a[1]; mf.s1 = b[1]; }
      if (gw > 2) { mf.n2 = a[2]; mf.s2 = b[2]; }
      if (gw > 3) { mf.n3 = a[3]; mf.s3 = b[3]; }
    }
  }
  return mf;
}
KYV_HD LabelSet res_nsl(const View& v, const ResHeader& h) {
  LabelSet nsl{NodeTab{nullptr}, 0, nullptr, 0};
  if (h.nsl != NONE) { nsl.kv = v.nsl_kv + 2 * v.nsl_off[h.nsl]; nsl.n = v.nsl_off[h.nsl + 1] - v.nsl_off[h.nsl]; }
  return nsl;
}
template <int kMW>
__global__ void __launch_bounds__(256) facts_kernel(const View* __restrict__ vp, const TailCfg* __restrict__ cfg,
                                                    ResFacts* __restrict__ out) {
  const View& v = *vp;
  const uint32_t r = blockIdx.x * 256u + threadIdx.x;
  if (r >= v.nres) return;
  const ResHeader& h = v.hdr[r];
  KYV_ACCT_ADD(0, 48);  // header fields, label / annotation / namespace-label rows (model)
  ResFacts f;
  f.mf = res_mfacts<kMW>(v, h);
  const NodeTab R{v.nodes + h.root};
  tail_facts(v, cfg, LabelSet{R, h.labels, nullptr, 0}, LabelSet{R, h.ann, nullptr, 0}, res_nsl(v, h), &h, f.lt);
  f.hflags = h.flags;
  f.hroot = h.root;
  f.pad = 0;
  out[r] = f;
  KYV_ACCT_ADD(1, sizeof(ResFacts));
}

// Pattern / anyPattern rules without preconditions whose match block fits a staged record (MRec). One lane per
// resource, one wave per workgroup; the lane holds its resource's facts (kind, name, namespace and their glob-mask
// words) in registers and its labels in LDS. The rule loop is kind-indexed: a wave whose resources share one kind class
// (kind-major batches: all but the waves at class boundaries) walks only the records of that class (C4: ~40 % of the
// rules for a Pod wave); a mixed wave walks every record with a per-lane kind-gate test. Records come through scalar
// loads (wave-uniform addresses: the scalar cache and L2 serve every wave of the class from one copy), so a rule's
// kinds / name / namespace checks are register compares and its selector / annotation tail a scan of LDS. Matched pairs
// of shape rules are decided here from the shape tables (mrec_shape_out), the rest go to the walk's work lists.
// kWpe: occupancy target (KYV_MATCHW_WPE); kMW: glob-mask words held per string (1 when the ruleset has <= 32 bits)
template <int kWpe, int kMW>
__global__ void __launch_bounds__(BLOCK) __attribute__((amdgpu_waves_per_eu(kWpe)))
match_rec_kernel(const View* __restrict__ vp, DevOut o, WorkLists wl, const MRec* __restrict__ recs, uint32_t nm,
                 MRecIndex ix, ShapeTab sh, TailTab tt, const ResFacts* __restrict__ facts) {
  // the lane's labels (key, value sid pairs; stride 2 * MREC_LABELS + 1 words: no bank conflicts), when it has at most
  // MREC_LABELS of them
  __shared__ uint32_t s_lab[BLOCK * (2 * MREC_LABELS + 1)];
  const View& v = *vp;
  const uint32_t lane = threadIdx.x;
  const uint32_t w = blockIdx.x;
  const uint32_t r = w * BLOCK + lane;
  const bool active = r < v.nres;
  const ResHeader* hp = active ? &v.hdr[r] : nullptr;
  const uint32_t cls = active ? hp->kclass : 0u;
  const uint32_t hflags = active ? hp->flags : 0u;
  const uint32_t hroot = active ? hp->root : 0u;
  if (active) KYV_ACCT_ADD(0, 12);  // header: kind class, flags, root
  const uint32_t c0 = __builtin_amdgcn_readfirstlane(cls);
  const bool uni = __ballot(active && cls != c0) == 0;  // (lane 0 is active whenever any lane is)
  const uint32_t* gate = active ? v.gate + (size_t)cls * v.gate_words : nullptr;
  // the lane's facts: from the per-evaluation facts table, else computed here
  MFacts mf{};
  LaneTail lt{};
  bool have = false;
  if (facts && active) {
    const ResFacts F = facts[r];
    KYV_ACCT_ADD(0, sizeof(ResFacts));
    mf = F.mf;
    lt = F.lt;
    have = true;
  } else if (active) {
    mf = res_mfacts<kMW>(v, *hp);
  }
  const LabelSet nsl = active ? res_nsl(v, *hp) : LabelSet{NodeTab{nullptr}, 0, nullptr, 0};
  // the empty OldResource's facts (uniform): every string "", its glob-mask words those of the empty string
  MFacts mf0{};
  mf0.gk = mf0.rname = mf0.rns = SID_EMPTY;
  mf0.fl = MF_KIND_EMPTY;
  if (v.str_gmask) {
    const uint32_t gw = v.gmask_words;
    const uint32_t* a = v.str_gmask + (size_t)SID_EMPTY * gw;
    mf0.n0 = mf0.s0 = a[0];
    if (kMW > 1) {
      if (gw > 1) mf0.n1 = mf0.s1 = a[1];
      if (gw > 2) mf0.n2 = mf0.s2 = a[2];
      if (gw > 3) mf0.n3 = mf0.s3 = a[3];
    }
  }
  const ResView rv{NodeTab{v.nodes + hroot}, hp};
  LabelSet labels{rv.R, hp ? hp->labels : NONE, nullptr, 0};
  {
    const uint32_t nl = ls_count(labels);
    if (active && nl <= MREC_LABELS) {
      uint32_t* kv = s_lab + lane * (2 * MREC_LABELS + 1);
      for (uint32_t i = 0; i < nl; i++) { kv[2 * i] = ls_key(labels, i); kv[2 * i + 1] = ls_val(labels, i); }
      labels = LabelSet{NodeTab{nullptr}, 0, kv, nl};
    }
  }
  if (!__ballot(active)) return;
  // the lane's tail facts (unless read above), and the empty OldResource's: no labels or annotations, the lane's
  // namespace labels
  const LabelSet none{NodeTab{nullptr}, 0, nullptr, 0};
  if (!have) tail_facts(v, tt.cfg, labels, LabelSet{rv.R, hp ? hp->ann : NONE, nullptr, 0}, nsl, hp, lt);
  LaneTail lt0;
  tail_facts(v, tt.cfg, none, none, none, nullptr, lt0);
#pragma unroll
  for (uint32_t q = 0; q < TF_NSSLOTS; q++) lt0.nv[q] = lt.nv[q];
  // this resource's verdicts of the first SHAPE_REGS shapes, one byte each (loaded once, read per matched pair)
  uint32_t sv[4] = {0, 0, 0, 0};
  if (active)
#pragma unroll
    for (uint32_t q = 0; q < SHAPE_REGS; q++)
      if (q < sh.nshapes) sv[q >> 2] |= (uint32_t)sh.st[(size_t)q * v.nres + r] << (8 * (q & 3));
  const uint32_t i0 = uni ? sld32(ix.off + c0) : 0u, i1 = uni ? sld32(ix.off + c0 + 1) : nm;
  const MRec* base = uni ? ix.recs : recs;
  for (uint32_t i = i0; i < i1; i++) {
    const MRec* Rp = base + i;
    const MRecHead H = sld(reinterpret_cast<const MRecHead*>(Rp));
    const uint32_t k = H.k;
    const bool gated = active && (uni || ((gate[k >> 5] >> (k & 31)) & 1u));
    if (!__ballot(gated)) continue;
    uint8_t st = ST_NONE;
    bool m;
    if ((H.bits & MR_FASTEVAL) && (!(H.bits & MR_EMPTY) || (H.bits & MR_ECONST)) && !(H.flags & RD_GATE_EXACT)) {
      // branch-free path: the record's filter slots with scalar loads (independent: one latency)
      const uint32_t nf = ((H.bits >> 24) & 0xFu) + (H.bits >> 28);
      MRecFilter F[MREC_F];
#pragma unroll
      for (uint32_t j = 0; j < MREC_F; j++)
        if (j < nf) F[j] = sld(&Rp->f[j]);
      KYV_ACCT_ADD(0, 16);  // header words the match program compares (model, as pair_match)
      bool nd = false;
      bool mt = match_fast(v, H.bits, F, mf, tt, lt, &nd);
      if (H.bits & MR_EMPTY) {  // the retry against the empty OldResource: a constant of the rule
        nd = nd | (!mt & ((H.bits & MR_END) != 0));
        mt = mt | ((H.bits & MR_EMATCH) != 0);
      }
      st = !mt ? (uint8_t)ST_NONE : nd ? (uint8_t)ST_ND : (H.kind & 0xFFu) == RK_FALLBACK ? (uint8_t)ST_FALLBACK : (uint8_t)ST_NONE;
      m = gated & mt & !nd & ((H.kind & 0xFFu) != RK_FALLBACK);
      if (!gated) st = ST_NONE;
    } else {
      m = gated && pair_match_rec(v, Rp, H, mf, rv, labels, nsl, mf0, &st, tt, lt, lt0);
    }
    const uint32_t shape = (H.kind >> 8) & 0x7FFFu;  // 1 + shape of a shape rule, else 0; bit 23: wide records
    if (shape) mrec_shape_out(v, o, sh, shape - 1, (H.kind >> 23) & 1u, k, r, gated, m, st, hflags, w, sv);
    else match_walk_append(v, o, wl, k, H.kind & 0xFFu, r, gated, m, st, hflags, hroot);
  }
}

template <int kWpe>
__global__ void __launch_bounds__(BLOCK) __attribute__((amdgpu_waves_per_eu(kWpe)))
match_walk_generic_kernel(const View* __restrict__ vp, DevOut o, WorkLists wl, const uint32_t* __restrict__ mrules,
                          uint32_t nm) {
  const View& v = *vp;
  const uint32_t lane = threadIdx.x;
  const uint32_t r = blockIdx.x * BLOCK + lane;
  const bool active = r < v.nres;
  const uint32_t* gate = active ? v.gate + (size_t)v.hdr[r].kclass * v.gate_words : nullptr;
  const uint32_t hflags = active ? v.hdr[r].flags : 0u;
  const uint32_t hroot = active ? v.hdr[r].root : 0u;
  if (active) KYV_ACCT_ADD(0, 12);  // header: kind class, flags, root
  (void)lane;
  for (uint32_t mi = 0; mi < nm; mi++) {
    const uint32_t k = mrules[mi];
    const bool gated = active && ((gate[k >> 5] >> (k & 31)) & 1u);
    if (!__ballot(gated)) continue;
    const RuleDesc& rdk = v.rules[k];
    uint8_t st = ST_NONE;
    const bool m = gated && pair_match(v, r, rdk, &st);
    match_walk_append(v, o, wl, k, rdk.kind, r, gated, m, st, hflags, hroot);
  }
}

// Pattern / anyPattern rules with preconditions and no JMESPath operands (C5): pair_match, checkPreconditions
// (validation.go:281-288), then the work-list append -- without the PodSecurity / deny dispatch code of match_kernel,
// whose register need spilled its rule loop (C5 round 4: match_kernel<false> 166 VGPRs + 176 B of scratch per lane;
// 4.1 GB of scratch writes per evaluation in the match phase)
// kJ: the preconditions hold JMESPath operands (rules the compiled condition kernels do not take; the interpreter's
// projection lists live in scratch, so these rules get their own instantiation instead of match_kernel<true>)
template <int kWpe, bool kJ = false>
__global__ void __launch_bounds__(BLOCK) __attribute__((amdgpu_waves_per_eu(kWpe)))
match_pre_kernel(const View* __restrict__ vp, DevOut o, WorkLists wl, const uint32_t* __restrict__ mrules, uint32_t nm) {
  const View& v = *vp;
  const uint32_t r = blockIdx.x * BLOCK + threadIdx.x;
  const bool active = r < v.nres;
  const uint32_t* gate = active ? v.gate + (size_t)v.hdr[r].kclass * v.gate_words : nullptr;
  const uint32_t hflags = active ? v.hdr[r].flags : 0u;
  const uint32_t hroot = active ? v.hdr[r].root : 0u;
  if (active) KYV_ACCT_ADD(0, 12);  // header: kind class, flags, root
  for (uint32_t mi = 0; mi < nm; mi++) {
    const uint32_t k = mrules[mi];
    const bool gated = active && ((gate[k >> 5] >> (k & 31)) & 1u);
    if (!__ballot(gated)) continue;
    const RuleDesc& rd = v.rules[k];
    uint8_t st = ST_NONE;
    bool m = false;
    if (gated && pair_match(v, r, rd, &st)) {
      uint32_t ec, es, eg;
      const int c = eval_prog_inl<kJ>(v, NodeTab{v.nodes + hroot}, rd.pre, &ec, &es, &eg, NONE, r);
      if (c == CR_FB) st = (KYV_WHY(FBW_COND), ST_FALLBACK);
      else if (c == CR_PANIC) st = ST_PANIC;
      else if (c == CP_ERROR) st = ST_ERROR | ST_MARK_PRE;
      else if (c == CR_FALSE) st = ST_SKIP | ST_MARK_PRE;
      else m = true;
    }
    match_walk_append(v, o, wl, k, rd.kind, r, gated, m, st, hflags, hroot);
  }
}

// PodSecurity rules (without preconditions): one lane per resource over the match waves [w0, w0 + grid) of the rule's
// kind gate, the match and the path-column checks inlined. The per-container checks (pss_container_facts) run with
// one container per lane across the wave -- the 64 pods' container lists concatenated, a lane's facts OR-ed into its
// pod's word in LDS -- instead of each lane walking its pod's containers one after the other (the longest chain of
// dependent loads in the kernel); each lane then combines its pod's facts with the pod-level checks. Pairs the column
// form does not cover
// (exclusion sub-pods, resources without path columns) are marked ST_PSS_MAP and finished by pss_map_kernel: the map
// walk (eval_pss) is a call whose frame and spills would otherwise sit in this kernel's scratch and write traffic
// (round 3 C2 profile: 13x write amplification). kExact: the rule's match block is its kind gate (RD_GATE_EXACT), no
// match program compiled in; kWpe: occupancy target (KYV_PSS_WPE = 4 / 6 / 8 at run time; 8 by default: 41 VGPRs, no
// scratch). kPre (round 5): the rule has preconditions without JMESPath operands, evaluated inline first
// (checkPreconditions, validation.go:281-288) -- C5's PodSecurity rules behind preconditions ran in match_kernel<false>
// with eval_pss as a call (its frame in scratch memory)
template <bool kExact, int kWpe, bool kPre = false>
__global__ void __launch_bounds__(BLOCK) __attribute__((amdgpu_waves_per_eu(kWpe)))
pss_kernel(const View* __restrict__ vp, DevOut o, uint32_t k, uint32_t w0) {
  // the wave's containers, one per lane (lists of all 64 pods concatenated): per list the pods' counts, exclusive
  // prefix and first element row; per pod its resource root, pod position and the OR of its containers' facts
  __shared__ uint32_t s_pre[PSS_NLISTS][BLOCK], s_eb[PSS_NLISTS][BLOCK];
  __shared__ uint32_t s_root[BLOCK], s_pos[BLOCK], s_fact[BLOCK];
  const View& v = *vp;
  const uint32_t lane = threadIdx.x;
  const uint32_t r = (w0 + blockIdx.x) * BLOCK + lane;
  const bool gated = r < v.nres && ((v.gate[(size_t)v.hdr[r].kclass * v.gate_words + (k >> 5)] >> (k & 31)) & 1u);
  if (r < v.nres) KYV_ACCT_ADD(0, 4);  // header: kind class
  if (!__ballot(gated)) return;
  const RuleDesc& rd = v.rules[k];
  const PssDesc& pd = v.pss[rd.root];
  uint8_t st = ST_NONE;
  uint32_t pf = 0;
  bool m;
  if constexpr (kExact) {
    m = rd.kind == RK_PSS;  // pair_match of a kind-gate rule: matched (a fallback rule never gets here)
  } else {
    m = gated && pair_match(v, r, rd, &st);
  }
  if constexpr (kPre) {
    if (gated && m) {  // the precondition program first; only a true outcome reaches the PodSecurity checks
      uint32_t ec, es, eg;
      KYV_ACCT_ADD(0, 4);  // header: root
      const int c = eval_prog_inl<false>(v, NodeTab{v.nodes + v.hdr[r].root}, rd.pre, &ec, &es, &eg, NONE, r);
      if (c != CR_TRUE) {
        m = false;
        st = c == CR_FB ? (uint8_t)(KYV_WHY(FBW_COND), ST_FALLBACK)
           : c == CR_PANIC ? (uint8_t)ST_PANIC
           : c == CP_ERROR ? (uint8_t)(ST_ERROR | ST_MARK_PRE) : (uint8_t)(ST_SKIP | ST_MARK_PRE);
      }
    }
  }
  const uint32_t* T = nullptr;
  uint32_t hroot = 0;
  if (gated && m) {
    const ResHeader& h = v.hdr[r];
    KYV_ACCT_ADD(0, 12);  // header: root, node count, flags
    hroot = h.root;
    st = pss_cols_table(v, pd, h, &T);
  }
  // round 6: in kind-major batches the pods of a wave share their pod position, so their column table T is one
  // pointer: taken as a wave-uniform value, the table words and column offsets the checks look up are scalar loads
  // (scalar cache) instead of per-lane vector loads in front of every column read (C2: wait 0.92)
  const unsigned long long tmask = __ballot(T != nullptr);
  const uint32_t* Tu = nullptr;
  bool tuni = false;
  if (tmask) {
    const uint64_t tb = (uint64_t)(uintptr_t)T;
    const uint64_t first = __shfl(tb, __ffsll((long long)tmask) - 1);
    tuni = __ballot(T != nullptr && tb != first) == 0;
    const uint32_t lo32 = __builtin_amdgcn_readfirstlane((uint32_t)first);
    const uint32_t hi32 = __builtin_amdgcn_readfirstlane((uint32_t)(first >> 32));
    Tu = (const uint32_t*)(uintptr_t)(((uint64_t)hi32 << 32) | lo32);
  }
  uint32_t tot[PSS_NLISTS];
#pragma unroll
  for (uint32_t l = 0; l < PSS_NLISTS; l++) {
    uint32_t cnt = 0, eb = 0;
    if (T) {
      uint32_t lc;
      if (tuni) lc = Tu[PC_LISTS + l * PCL_COUNT + PCL_LEN];
      else lc = T[PC_LISTS + l * PCL_COUNT + PCL_LEN];
      if (lc != NONE) {
        KYV_ACCT_ADD(0, 8);
        const uint32_t co = tuni ? sld32(v.col_off + __builtin_amdgcn_readfirstlane(lc)) : v.col_off[lc];
        const uint64_t ln = v.colv[(size_t)co + r];  // (count, row of element 0)
        if ((uint32_t)ln != NONE) { cnt = (uint32_t)ln; eb = (uint32_t)(ln >> 32); }
      }
    }
    uint32_t incl = cnt;  // inclusive prefix over the wave
#pragma unroll
    for (uint32_t d = 1; d < BLOCK; d <<= 1) {
      const uint32_t y = __shfl_up(incl, d);
      if (lane >= d) incl += y;
    }
    s_pre[l][lane] = incl - cnt;
    s_eb[l][lane] = eb;
    tot[l] = __shfl(incl, BLOCK - 1);
  }
  s_root[lane] = hroot;
  s_pos[lane] = T ? (uint32_t)((T - (v.pool + pd.cols)) / PC_COUNT) : 0u;
  s_fact[lane] = 0;
  __syncthreads();
  // the checks of every container of the wave, a container per lane (its facts OR-ed into its pod's word)
  const uint32_t ncont = tot[0] + tot[1] + tot[2];
  for (uint32_t base = 0; base < ncont; base += BLOCK) {
    const uint32_t s = base + lane;
    if (s < ncont) {
      const uint32_t l = s < tot[0] ? 0u : s < tot[0] + tot[1] ? 1u : 2u;
      const uint32_t q = s - (l == 0 ? 0u : l == 1 ? tot[0] : tot[0] + tot[1]);
      uint32_t lo = 0, hi = BLOCK - 1;  // the last pod whose list starts at or before q
      while (lo < hi) {
        const uint32_t mid = (lo + hi + 1) >> 1;
        if (s_pre[l][mid] <= q) lo = mid; else hi = mid - 1;
      }
      const uint32_t er = s_eb[l][lo] + (q - s_pre[l][lo]);
      uint32_t f;
      if (tuni) {
        // one table for the wave's pods (kind-major batch): the three lists' column offsets as scalar loads, the
        // lane's list selected, so each container field is one vector load (round 6; per-lane table words and
        // column offsets were two dependent gathers in front of every field)
        const uint32_t* T0 = Tu + PC_LISTS;
        auto co = [&](uint32_t F) -> uint32_t {
          const uint32_t c0 = sld32(T0 + F), c1 = sld32(T0 + PCL_COUNT + F), c2 = sld32(T0 + 2 * PCL_COUNT + F);
          const uint32_t o0 = c0 == NONE ? NONE : sld32(v.col_off + c0);
          const uint32_t o1 = c1 == NONE ? NONE : sld32(v.col_off + c1);
          const uint32_t o2 = c2 == NONE ? NONE : sld32(v.col_off + c2);
          return l == 0 ? o0 : l == 1 ? o1 : o2;
        };
        f = pss_container_facts_g(v, NodeTab{v.nodes + s_root[lo]}, co, er);
      } else {
        const uint32_t* L = v.pool + pd.cols + s_pos[lo] * PC_COUNT + PC_LISTS + l * PCL_COUNT;
        f = pss_container_facts(v, NodeTab{v.nodes + s_root[lo]}, L, er);
      }
      atomicOr(&s_fact[lo], f);
    }
  }
  __syncthreads();
  if (T) {
    const uint32_t mask = (pd.flags & PSS_BASELINE) ? ~PSS_RESTRICTED_SLOTS : 0xFFFFFFFFu;
    if (tuni) {
      auto po = [&](uint32_t X) -> uint32_t {  // the shared table's column offsets: scalar loads
        const uint32_t c = sld32(Tu + X);
        return c == NONE ? NONE : sld32(v.col_off + c);
      };
      pf = pss_checks_cols_g(v, NodeTab{v.nodes + hroot}, r, Tu, po, s_fact[lane], true) & mask;
    }
    else pf = pss_checks_cols(v, NodeTab{v.nodes + hroot}, r, T, s_fact[lane], true) & mask;
    st = pf ? ST_FAIL : ST_PASS;
  }
  if (gated && st != ST_NONE) {
    o.status[(size_t)k * v.nres + r] = st;
    const uint32_t ps = o.pss_slot[k];
    if (ps != NONE && pf) o.pss_fails[(size_t)ps * v.nres + r] = pf;
    KYV_ACCT_ADD(1, 1 + ((ps != NONE && pf) ? 4 : 0));
  }
}

// The PodSecurity pairs pss_kernel marked ST_PSS_MAP (same grid): the map walk with the typed pod view, exclusion
// sub-pods included (eval_pss, validation.go:535-566 + pkg/pss/evaluate.go:83-108)
#ifndef KYV_NO_KERNELS
__global__ void __launch_bounds__(BLOCK) pss_map_kernel(const View* __restrict__ vp, DevOut o, uint32_t k, uint32_t w0) {
  const View& v = *vp;
  const uint32_t r = (w0 + blockIdx.x) * BLOCK + threadIdx.x;
  if (r >= v.nres) return;
  const uint8_t s0 = o.status[(size_t)k * v.nres + r];
  KYV_ACCT_ADD(0, 1);  // the pair's status byte
  if (s0 != ST_PSS_MAP) return;
  const ResHeader& h = v.hdr[r];
  uint32_t pf = 0;
  const uint8_t st = eval_pss(v, v.pss[v.rules[k].root], NodeTab{v.nodes + h.root}, h, &pf, r);
  o.status[(size_t)k * v.nres + r] = st;
  const uint32_t ps = o.pss_slot[k];
  if (ps != NONE && pf) o.pss_fails[(size_t)ps * v.nres + r] = pf;
  KYV_ACCT_ADD(1, 1 + ((ps != NONE && pf) ? 4 : 0));
}
#endif

// Phase 2 (pattern_eval): each wave takes chunks of 64 work items of ONE rule (grid-stride over all rules'
// chunks), so every lane walks the same compiled pattern over a different resource with the wave-uniform
// walker; verdict bytes as in phase 1, failing-path records staged in the chunk's own slots.
#ifndef KYV_NO_KERNELS
__global__ void __launch_bounds__(BLOCK) __attribute__((amdgpu_waves_per_eu(KYV_WPE)))
walk_kernel(const View* __restrict__ vp, DevOut o, WorkLists wl, ChunkMap cm, int depth) {
  extern __shared__ uint4 lds_raw[];  // [depth] UFrame, then [depth][BLOCK] LaneFrame
  WaveWalker wk{(LaneFrame*)((UFrame*)lds_raw + depth), (UFrame*)lds_raw, depth, false};
  walk_chunks(*vp, o, wl, cm, wk);
}
#endif

}  // namespace kyv
