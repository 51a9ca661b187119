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
      int c = CR_TRUE;
      if (rd.pre != NONE) c = eval_prog<false>(v, R, rd.pre, &ec, &es, &eg, NONE, r);
      if (c == CR_FB) st = (KYV_WHY(FBW_COND), ST_FALLBACK);
      else if (c == CR_PANIC) st = ST_PANIC;
      else if (c == CP_ERROR) st = ST_ERROR | ST_MARK_PRE;
      else if (c == CR_FALSE) st = ST_SKIP | ST_MARK_PRE;
      else {
        c = eval_prog<false>(v, R, rd.root, &ec, &es, &eg, NONE, r);
        st = c == CR_FB ? (KYV_WHY(FBW_COND), ST_FALLBACK) : c == CR_PANIC ? ST_PANIC : c == CP_ERROR ? ST_ERROR
           : c == CR_TRUE ? ST_FAIL : ST_PASS;
      }
    }
    if (st != ST_NONE) { o.status[(size_t)k * v.nres + r] = st; KYV_ACCT_ADD(1, 1); }
  }
}

// Staged match records of match_walk_kernel. Every wave runs the same rule loop, so a rule's match program was a chain
// of dependent uniform loads (rule list -> RuleDesc -> Filter -> KindDesc / pattern sids -> pattern flags -> the
// string's glob mask) paid by every wave for every rule: the C4 loop (10,440 rules) was latency-bound (wait 0.85).
// The host lays each rule's match block out as one fixed-size record (kinds, name / names / namespaces patterns with
// their glob-mask bit resolved); a wave copies MREC_CHUNK records into LDS with one coalesced load and evaluates them
// against the lane's resource facts (kind, name, namespace and their glob-mask words) held in registers. A filter with
// annotations or selectors, or one whose matching kind carries a group / version, runs condition_block itself after
// the record's checks passed; a rule the record cannot hold (exceptions, the empty-OldResource retry, more than
// MREC_F filters / 4 kinds / 2 names / 2 namespaces, a glob without a mask) runs pair_match.
constexpr uint32_t MREC_F = 3, MREC_CHUNK = 16, MREC_LABELS = 8, PAT_MASK = 0x80000000u;
enum MRecBits : uint32_t { MR_FAST = 1u, MR_MASKS = 2u, MR_EMPTY = 4u };  // MR_EMPTY: empty_may_match
struct MRecFilter {   // 48 bytes
  uint32_t idx;       // Filter index (condition_block of a tail filter)
  uint32_t bits;      // [0,16) FilterFlag, [16,19) kinds, [19,21) names, 21 name, [22,24) namespaces,
                      // [24,28) kind i has a group / version, 28 tail (annotations / selector / namespace selector)
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

// condition_block (kyv_eval.h) of a record filter: kinds, name, names and namespaces from the record and the lane's
// facts (a kind with a group / version that equals the resource's: kinds_match decides), then the tail
KYV_HD bool cb_rec(const View& v, const MRecFilter& F, const MFacts& mf, const ResView& rv, const LabelSet& labels,
                   const LabelSet& nsl, bool uic, bool* nd) {
  const uint32_t b = F.bits;
  const uint32_t nk = (b >> 16) & 7u;
  if (nk) {
    bool ok = false, gv = false;
    for (uint32_t i = 0; i < nk && !ok; i++) {
      const uint32_t kd = F.kinds[i];
      if (kd == NONE) ok = true;
      else if (kd == mf.gk) { ok = true; gv = (b >> (24 + i)) & 1u; }
    }
    if (gv) ok = kinds_match(v, v.filters[F.idx], rv.h);
    if (!ok) return false;
  }
  if (((b >> 21) & 1u) && !pat_name(mf, F.pats[0])) return false;
  const uint32_t nn = (b >> 19) & 3u;
  if (nn && !(pat_name(mf, F.pats[1]) || (nn > 1 && pat_name(mf, F.pats[2])))) return false;
  const uint32_t ns = (b >> 22) & 3u;
  if (ns && !(pat_ns(mf, F.pats[3]) || (ns > 1 && pat_ns(mf, F.pats[4])))) return false;
  if ((b >> 28) & 1u) return cb_tail(v, v.filters[F.idx], rv, labels, nsl, uic, nd, mf.fl);
  return !(uic && (b & FF_USERINFO));
}

// match_rule (kyv_eval.h) over a record
KYV_HD bool match_rule_rec(const View& v, const MRec& R, const MFacts& mf, const ResView& rv, const LabelSet& labels,
                           const LabelSet& nsl, bool* nd) {
  const uint32_t mm = (R.bits >> 8) & 0xFFu, em = (R.bits >> 16) & 0xFFu, nmf = (R.bits >> 24) & 0xFu, nef = R.bits >> 28;
  bool failed = false;
  if (mm == MM_ANY) {
    bool one = false;
    for (uint32_t i = 0; i < nmf && !one; i++)
      if (!(R.f[i].bits & FF_ZERO_RD) && cb_rec(v, R.f[i], mf, rv, labels, nsl, false, nd)) one = true;
    if (!one) failed = true;
  } else if (mm == MM_ALL || mm == MM_PLAIN) {
    for (uint32_t i = 0; i < nmf && !failed; i++)
      if ((R.f[i].bits & FF_ZERO_RD) || !cb_rec(v, R.f[i], mf, rv, labels, nsl, false, nd)) failed = true;
  } else {
    failed = true;
  }
  if (failed) return false;
  if (em == MM_ANY || em == MM_PLAIN) {
    for (uint32_t i = 0; i < nef; i++) {
      const MRecFilter& F = R.f[nmf + i];
      if ((F.bits & FF_ZERO_RD) && !(F.bits & FF_USERINFO)) continue;
      if (cb_rec(v, F, mf, rv, labels, nsl, true, nd)) return false;
    }
  } else if (em == MM_ALL) {
    bool byAll = true;
    for (uint32_t i = 0; i < nef && byAll; i++) {
      const MRecFilter& F = R.f[nmf + i];
      const bool excl = !((F.bits & FF_ZERO_RD) && !(F.bits & FF_USERINFO)) && cb_rec(v, F, mf, rv, labels, nsl, true, nd);
      if (!excl) byAll = false;
    }
    if (byAll && nef > 0) return false;
  }
  return true;
}

// pair_match (kyv_pss.h) of a record rule (compiled match block, no exceptions); a rule whose match may accept the
// empty OldResource (MR_EMPTY, validation.go:606) retries against it: the facts of the empty resource (mf0: kind,
// name and namespace "", no labels, no annotations)
KYV_HD bool pair_match_rec(const View& v, const MRec& R, const MFacts& mf, const ResView& rv, const LabelSet& labels,
                           const LabelSet& nsl, const MFacts& mf0, uint8_t* st) {
  bool nd = false;
  if (!(R.flags & RD_GATE_EXACT)) {
    KYV_ACCT_ADD(0, 16);  // header words the match program compares (model, as pair_match)
    bool m = match_rule_rec(v, R, mf, rv, labels, nsl, &nd);
    if (!m && (R.bits & MR_EMPTY))
      m = match_rule_rec(v, R, mf0, ResView{rv.R, nullptr}, LabelSet{NodeTab{nullptr}, 0, nullptr, 0}, nsl, &nd);
    if (!m) { *st = ST_NONE; return false; }
  }
  if (nd) { *st = ST_ND; return false; }
  if (R.kind == RK_FALLBACK) { *st = ST_FALLBACK; return false; }
  return true;
}

// Pattern / anyPattern rules without preconditions (and compile-time fallback rules): the match phase is only
// pair_match (kind gate, match / exclude program, PolicyException candidates) and the work-list append, so these
// kernels carry none of the dispatch code (conditions, PodSecurity calls) whose register need made the rule loop
// of match_kernel spill every iteration (C4: 10,440 rules per wave, 252 GB of scratch writes per evaluation).
// match_walk_kernel takes the rules as staged match records (above), MREC_CHUNK at a time through LDS;
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

// kMW: glob-mask words held per string (1 when the ruleset has at most 32 mask bits, else 4)
template <int kWpe, int kMW>
__global__ void __launch_bounds__(BLOCK) __attribute__((amdgpu_waves_per_eu(kWpe)))
match_walk_kernel(const View* __restrict__ vp, DevOut o, WorkLists wl, const MRec* __restrict__ recs, uint32_t nm) {
  __shared__ MRec s_rec[MREC_CHUNK];
  // the lane's labels (key, value sid pairs; stride 2 * MREC_LABELS + 1 words: no bank conflicts), when it has at most
  // MREC_LABELS of them
  __shared__ uint32_t s_lab[BLOCK * (2 * MREC_LABELS + 1)];
  const View& v = *vp;
  const uint32_t lane = threadIdx.x;
  const uint32_t r = blockIdx.x * BLOCK + lane;
  const bool active = r < v.nres;
  const uint32_t* gate = active ? v.gate + (size_t)v.hdr[r].kclass * v.gate_words : nullptr;
  const uint32_t hflags = active ? v.hdr[r].flags : 0u;
  const uint32_t hroot = active ? v.hdr[r].root : 0u;
  if (active) KYV_ACCT_ADD(0, 12);  // header: kind class, flags, root
  MFacts mf{};
  LabelSet nsl{NodeTab{nullptr}, 0, nullptr, 0};
  const ResHeader* hp = active ? &v.hdr[r] : nullptr;
  if (active) {
    const ResHeader& h = *hp;
    const uint32_t name = h.name, kind = h.kind;
    mf.gk = h.gvk_kind;
    mf.rname = name == SID_EMPTY ? h.gen_name : name;
    const bool isNs = v.str_len[kind] == 9 && bytes_eq(sbytes(v, kind), (const uint8_t*)"Namespace", 9);
    mf.rns = isNs ? name : h.ns;
    mf.fl = (isNs ? MF_ISNS : 0u) | (kind == SID_EMPTY ? MF_KIND_EMPTY : 0u);
    if (v.str_gmask) {  // (records with a glob-mask pattern are only built when the batch has masks)
      const uint32_t w = v.gmask_words;
      const uint32_t* a = v.str_gmask + (size_t)mf.rname * w;
      const uint32_t* b = v.str_gmask + (size_t)mf.rns * w;
      mf.n0 = a[0]; mf.s0 = b[0];
      if (kMW > 1) {
        if (w > 1) { mf.n1 = a[1]; mf.s1 = b[1]; }
        if (w > 2) { mf.n2 = a[2]; mf.s2 = b[2]; }
        if (w > 3) { mf.n3 = a[3]; mf.s3 = b[3]; }
      }
    }
    if (h.nsl != NONE) { nsl.kv = v.nsl_kv + 2 * v.nsl_off[h.nsl]; nsl.n = v.nsl_off[h.nsl + 1] - v.nsl_off[h.nsl]; }
  }
  // the empty OldResource's facts (uniform): every string "", its glob-mask words those of the empty string
  MFacts mf0{};
  mf0.gk = mf0.rname = mf0.rns = SID_EMPTY;
  mf0.fl = MF_KIND_EMPTY;
  if (v.str_gmask) {
    const uint32_t w = v.gmask_words;
    const uint32_t* a = v.str_gmask + (size_t)SID_EMPTY * w;
    mf0.n0 = mf0.s0 = a[0];
    if (kMW > 1) {
      if (w > 1) mf0.n1 = mf0.s1 = a[1];
      if (w > 2) mf0.n2 = mf0.s2 = a[2];
      if (w > 3) mf0.n3 = mf0.s3 = a[3];
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
  for (uint32_t c0 = 0; c0 < nm; c0 += MREC_CHUNK) {
    const uint32_t n = nm - c0 < MREC_CHUNK ? nm - c0 : MREC_CHUNK;
    __syncthreads();  // the previous chunk's records are read
    {
      const uint32_t* src = (const uint32_t*)(recs + c0);
      uint32_t* dst = (uint32_t*)s_rec;
      for (uint32_t i = lane; i < n * (uint32_t)(sizeof(MRec) / 4); i += BLOCK) dst[i] = src[i];
    }
    __syncthreads();
    // the chunk's kind-gate bits, loaded together (independent loads: one latency per chunk, not one per rule)
    uint32_t gm = 0;
    if (active) {
#pragma unroll 8
      for (uint32_t j = 0; j < MREC_CHUNK; j++)
        if (j < n) {
          const uint32_t k = s_rec[j].k;
          gm |= ((gate[k >> 5] >> (k & 31)) & 1u) << j;
        }
    }
    for (uint32_t j = 0; j < n; j++) {
      const MRec& R = s_rec[j];
      const uint32_t k = __builtin_amdgcn_readfirstlane(R.k);
      const bool gated = (gm >> j) & 1u;
      if (!__ballot(gated)) continue;
      uint8_t st = ST_NONE;
      const bool m = gated && pair_match_rec(v, R, mf, rv, labels, nsl, mf0, &st);
      match_walk_append(v, o, wl, k, __builtin_amdgcn_readfirstlane(R.kind), r, gated, m, st, hflags, hroot);
    }
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
template <int kWpe>
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
      const int c = eval_prog<false>(v, NodeTab{v.nodes + hroot}, rd.pre, &ec, &es, &eg, NONE, r);
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
// scratch)
template <bool kExact, int kWpe>
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
  const uint32_t* T = nullptr;
  uint32_t hroot = 0;
  if (gated && m) {
    const ResHeader& h = v.hdr[r];
    KYV_ACCT_ADD(0, 12);  // header: root, node count, flags
    hroot = h.root;
    st = pss_cols_table(v, pd, h, &T);
  }
  uint32_t tot[PSS_NLISTS];
#pragma unroll
  for (uint32_t l = 0; l < PSS_NLISTS; l++) {
    uint32_t cnt = 0, eb = 0;
    if (T) {
      const uint32_t* L = T + PC_LISTS + l * PCL_COUNT;
      if (L[PCL_LEN] != NONE) {
        KYV_ACCT_ADD(0, 8);
        const uint64_t ln = v.colv[(size_t)v.col_off[L[PCL_LEN]] + r];  // (count, row of element 0)
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
      const uint32_t* L = v.pool + pd.cols + s_pos[lo] * PC_COUNT + PC_LISTS + l * PCL_COUNT;
      const uint32_t f = pss_container_facts(v, NodeTab{v.nodes + s_root[lo]}, L, s_eb[l][lo] + (q - s_pre[l][lo]));
      atomicOr(&s_fact[lo], f);
    }
  }
  __syncthreads();
  if (T) {
    const uint32_t mask = (pd.flags & PSS_BASELINE) ? ~PSS_RESTRICTED_SLOTS : 0xFFFFFFFFu;
    pf = pss_checks_cols(v, NodeTab{v.nodes + hroot}, r, T, s_fact[lane], true) & mask;
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

// Phase 2 (pattern_eval): each wave takes chunks of 64 work items of ONE rule (grid-stride over all rules'
// chunks), so every lane walks the same compiled pattern over a different resource with the wave-uniform
// walker; verdict bytes as in phase 1, failing-path records staged in the chunk's own slots.
__global__ void __launch_bounds__(BLOCK) __attribute__((amdgpu_waves_per_eu(KYV_WPE)))
walk_kernel(const View* __restrict__ vp, DevOut o, WorkLists wl, ChunkMap cm, int depth) {
  extern __shared__ uint4 lds_raw[];  // [depth] UFrame, then [depth][BLOCK] LaneFrame
  WaveWalker wk{(LaneFrame*)((UFrame*)lds_raw + depth), (UFrame*)lds_raw, depth, false};
  walk_chunks(*vp, o, wl, cm, wk);
}

}  // namespace kyv
