// Fused walk (device only): one wave per match wave of 64 resources walks every direct pattern rule of a compiled
// group back to back (jit.cpp JitFused<g>, kernel kyv_jit_fused_<g>).
//
// The per-chunk schedule (walk_chunks, kyv_wave.h) gives each wave ONE (rule, match wave) pair: the schedule slot,
// the rule descriptor, the resources' header words and their kind-gate word are loaded again for every rule, a chain
// of dependent loads in front of every walk. Here a wave loads its 64 headers and kind-gate words once and then runs
// the group's rules in order; per rule only the uniform gate test, the rule's own column preload and walk remain.
// Same per-pair semantics as walk_chunks for RD_GATE_EXACT rules: gated lanes walk (validate.go:31-247 via the
// generated pattern code), an RF_MAGIC resource gets ST_FALLBACK, verdict bytes and staged failing-path records go
// to the same places (status[k][r], chunk (k, w) staging slots, rcnt[k - rule_lo][w]).
#pragma once
#include "kyv_wave.h"

namespace kyv {

#ifndef KYV_FUSED_GW
#define KYV_FUSED_GW 8  // kind-gate words a fused wave keeps in registers (rulesets of <= 256 rules)
#endif

template <class Fused>
__device__ __forceinline__ void walk_fused(const View& v, DevOut o, uint32_t nwaves, Fused& f) {
  const uint32_t lane = threadIdx.x & (WAVE - 1);
  for (uint32_t w = blockIdx.x; w < nwaves; w += gridDim.x) {
    const uint32_t r = w * WAVE + lane;
    const bool active = r < v.nres;
    uint32_t hflags = 0, hroot = 0, cls = 0;
    if (active) {
      const ResHeader* h = v.hdr + r;
      hflags = gld32(&h->flags);
      hroot = gld32(&h->root);
      cls = gld32(&h->kclass);
      KYV_ACCT_ADD(0, 12);  // header: flags, root, kind class
    }
    // the wave's kind-gate words: one scalar load each when every active lane has the same kind class (kind-major
    // batches: all but the waves at kind boundaries), else per lane
    const uint32_t c0 = __builtin_amdgcn_readfirstlane(active ? cls : 0u);
    const bool uniform = __ballot(active && cls != c0) == 0;
    uint32_t gw[KYV_FUSED_GW];
#pragma unroll
    for (uint32_t i = 0; i < KYV_FUSED_GW; i++) {
      gw[i] = 0;
      if (i < v.gate_words) {
        if (uniform) gw[i] = sld32(v.gate + (size_t)c0 * v.gate_words + i);
        else if (active) gw[i] = gld32(v.gate + (size_t)cls * v.gate_words + i);
      }
    }
    f.run(v, o, nwaves, w, r, active, hflags, hroot, gw);
  }
}

// Shape tables (round 5): one record slot per (shape, resource); the shape walk emits at most one record per lane
// (a pattern rule: one alternative), kept whole (resolved metadata keys included) for the match phase, which copies
// it into the staging chunk of every matched FAIL pair of the shape's rules (kyv_kernels.h mrec_shape_out)
struct ShapeSink {
  FailRec* at;
  __device__ __forceinline__ void emit(bool has, const FailRec& f) {
    if (!has) return;
    *at = f;
    KYV_ACCT_ADD(1, sizeof(FailRec));
  }
};

// kyv_jit_shapes: one wave per match wave (grid-stride), its resources' header words loaded once, then every shape
// the wave's kind classes need (jit.cpp JitShapes: the verdict byte of each gated lane, its record where FAIL)
template <class Shapes>
__device__ __forceinline__ void walk_shapes(const View& v, const ShapeOut& so, Shapes& f) {
  const uint32_t lane = threadIdx.x & (WAVE - 1);
  for (uint32_t w = blockIdx.x; w < so.nwaves; w += gridDim.x) {
    const uint32_t r = w * WAVE + lane;
    const bool active = r < v.nres;
    uint32_t hflags = 0, hroot = 0, cls = 0;
    if (active) {
      const ResHeader* h = v.hdr + r;
      hflags = gld32(&h->flags);
      hroot = gld32(&h->root);
      cls = gld32(&h->kclass);
      KYV_ACCT_ADD(0, 12);  // header: flags, root, kind class
    }
    f.run(v, so, r, active, hflags, hroot, cls);
  }
}

}  // namespace kyv
