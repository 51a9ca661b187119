// Byte-accounting build of the evaluation kernels (SURVEY §8(d) algorithmic bytes, bench.py `roofline`): the same
// kernel source as the product (kyv_kernels.h) compiled with KYV_ACCT, so every per-resource load and result store
// adds its bytes to device counters (kyv_eval.h KYV_ACCT_ADD). The namespace is renamed so both builds link into one
// library without sharing a symbol; kyv_engine.hip runs these only in an explicit accounting evaluation.
// the label-selector check inlined into the statically compiled kernels: as an out-of-line call its callee-saved
// registers went through scratch for every (resource, rule) pair with a selector (C4 round 4: 220 GB of scratch
// writes per evaluation in match_walk_kernel; inlined: 86 VGPRs, no scratch)
#define KYV_SEL_INLINE 1
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>

#define KYV_ACCT 1
#define kyv kyv_acct
#include "kyv_kernels.h"
#undef kyv
#include "kyv_acct.h"

namespace kyvacct {
namespace {
template <class T>
T as(const void* p) {
  T x;
  memcpy(&x, p, sizeof x);
  return x;
}
void check(hipError_t e) {
  if (e != hipSuccess) throw std::runtime_error(std::string("HIP error (accounting kernels): ") + hipGetErrorString(e));
}
}  // namespace

void match(bool kj, unsigned grid, hipStream_t s, const void* view, const void* devout, const void* wl,
           const uint32_t* mrules, uint32_t nm) {
  using namespace kyv_acct;
  auto kf = kj ? match_kernel<true> : match_kernel<false>;
  hipLaunchKernelGGL(kf, dim3(grid), dim3(BLOCK), 0, s, (const View*)view, as<DevOut>(devout), as<WorkLists>(wl), mrules, nm);
  check(hipGetLastError());
}
void match_rec(int wpe, bool mw1, unsigned grid, hipStream_t s, const void* view, const void* devout, const void* wl,
               const void* recs, uint32_t nm, const void* index, const void* shapes, const void* tails,
               const void* facts) {
  using namespace kyv_acct;
  auto kf = wpe == 8 ? (mw1 ? match_rec_kernel<8, 1> : match_rec_kernel<8, 4>)
          : wpe == 6 ? (mw1 ? match_rec_kernel<6, 1> : match_rec_kernel<6, 4>)
          : wpe == 4 ? (mw1 ? match_rec_kernel<4, 1> : match_rec_kernel<4, 4>)
                     : (mw1 ? match_rec_kernel<5, 1> : match_rec_kernel<5, 4>);
  hipLaunchKernelGGL(kf, dim3(grid), dim3(BLOCK), 0, s, (const View*)view, as<DevOut>(devout), as<WorkLists>(wl),
                     (const MRec*)recs, nm, as<MRecIndex>(index), as<ShapeTab>(shapes), as<TailTab>(tails),
                     (const ResFacts*)facts);
  check(hipGetLastError());
}
void facts(bool mw1, unsigned grid, hipStream_t s, const void* view, const void* cfg, void* out) {
  using namespace kyv_acct;
  hipLaunchKernelGGL(mw1 ? facts_kernel<1> : facts_kernel<4>, dim3(grid), dim3(256), 0, s, (const View*)view,
                     (const TailCfg*)cfg, (ResFacts*)out);
  check(hipGetLastError());
}
void match_walk_generic(int wpe, unsigned grid, hipStream_t s, const void* view, const void* devout, const void* wl,
                        const uint32_t* mrules, uint32_t nm) {
  using namespace kyv_acct;
  auto kf = wpe == 8 ? match_walk_generic_kernel<8> : wpe == 6 ? match_walk_generic_kernel<6> : match_walk_generic_kernel<4>;
  hipLaunchKernelGGL(kf, dim3(grid), dim3(BLOCK), 0, s, (const View*)view, as<DevOut>(devout), as<WorkLists>(wl), mrules, nm);
  check(hipGetLastError());
}
void match_pre(unsigned grid, hipStream_t s, const void* view, const void* devout, const void* wl, const uint32_t* mrules,
               uint32_t nm) {
  using namespace kyv_acct;
  hipLaunchKernelGGL(match_pre_kernel<KYV_MATCH_WPE>, dim3(grid), dim3(BLOCK), 0, s, (const View*)view, as<DevOut>(devout),
                     as<WorkLists>(wl), mrules, nm);
  check(hipGetLastError());
}
void match_pre_j(unsigned grid, hipStream_t s, const void* view, const void* devout, const void* wl, const uint32_t* mrules,
                 uint32_t nm) {
  using namespace kyv_acct;
  hipLaunchKernelGGL((match_pre_kernel<KYV_MATCH_WPE, true>), dim3(grid), dim3(BLOCK), 0, s, (const View*)view,
                     as<DevOut>(devout), as<WorkLists>(wl), mrules, nm);
  check(hipGetLastError());
}
void pss(bool exact, int wpe, unsigned grid, hipStream_t s, const void* view, const void* devout, uint32_t k, uint32_t w0) {
  using namespace kyv_acct;
  auto kf = exact ? (wpe == 4 ? pss_kernel<true, 4> : wpe == 6 ? pss_kernel<true, 6> : pss_kernel<true, 8>)
                  : (wpe == 4 ? pss_kernel<false, 4> : wpe == 6 ? pss_kernel<false, 6> : pss_kernel<false, 8>);
  hipLaunchKernelGGL(kf, dim3(grid), dim3(BLOCK), 0, s, (const View*)view, as<DevOut>(devout), k, w0);
  check(hipGetLastError());
}
void match_deny(unsigned grid, hipStream_t s, const void* view, const void* devout, const uint32_t* mrules, uint32_t nm) {
  using namespace kyv_acct;
  hipLaunchKernelGGL(match_deny_kernel, dim3(grid), dim3(BLOCK), 0, s, (const View*)view, as<DevOut>(devout), mrules, nm);
  check(hipGetLastError());
}
void pss_map(unsigned grid, hipStream_t s, const void* view, const void* devout, uint32_t k, uint32_t w0) {
  using namespace kyv_acct;
  hipLaunchKernelGGL(pss_map_kernel, dim3(grid), dim3(BLOCK), 0, s, (const View*)view, as<DevOut>(devout), k, w0);
  check(hipGetLastError());
}
void walk(unsigned grid, size_t lds, hipStream_t s, const void* view, const void* devout, const void* wl, const void* cm,
          int depth) {
  using namespace kyv_acct;
  hipLaunchKernelGGL(walk_kernel, dim3(grid), dim3(BLOCK), lds, s, (const View*)view, as<DevOut>(devout),
                     as<WorkLists>(wl), as<ChunkMap>(cm), depth);
  check(hipGetLastError());
}
unsigned long long* counters() {
  void* p = nullptr;
  check(hipGetSymbolAddress(&p, HIP_SYMBOL(kyv_acct::kyv_acct_bytes)));
  return (unsigned long long*)p;
}
}  // namespace kyvacct
