// Byte-accounting build of the evaluation kernels -- its JMESPath instantiations (match_kernel<true>,
// match_pre_kernel<.., true>; the rest: kyv_acct.hip) (SURVEY §8(d) algorithmic bytes, bench.py `roofline`): the same
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
#define KYV_NO_KERNELS 1                    // (the non-template kernels: kyv_acct.hip)
#define kyv_acct_bytes kyv_acct_bytes_j     // this code object's own counters (an extern "C" device symbol)
#define kyv kyv_acct_j
#include "kyv_kernels.h"
#undef kyv
#include "kyv_acct.h"

#define KYV_LAUNCH_PART 2
#define KYV_LNS kyvacct
#define KYV_KNS kyv_acct_j
#define KYV_LNS_NAME "accounting kernels"
#include "kyv_launch.inc"

namespace kyvacct {
unsigned long long* counters_j() {
  void* p = nullptr;
  check(hipGetSymbolAddress(&p, HIP_SYMBOL(kyv_acct_j::kyv_acct_bytes)));
  return (unsigned long long*)p;
}
}  // namespace kyvacct
