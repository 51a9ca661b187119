// The JMESPath instantiations (match_kernel<true>, match_pre_kernel<.., true>) of the product build; the other
// evaluation kernels: kyv_prod.hip.
// The product build of the evaluation kernels of kyv_kernels.h (match phase, PodSecurity, interpreted walk) and their
// launch shims (kyv_launch.inc, namespace kyvprod): compiled in a translation unit of its own, beside its byte-accounting
// twin (kyv_acct.hip), so the host engine (kyv_engine.hip) compiles no evaluation kernel.
// the label-selector check inlined into the statically compiled kernels: as an out-of-line call its callee-saved
// registers went through scratch for every (resource, rule) pair with a selector (C4 round 4: 220 GB of scratch
// writes per evaluation in match_walk_kernel; inlined: 86 VGPRs, no scratch)
#define KYV_SEL_INLINE 1
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>

#define KYV_NO_KERNELS 1  // (the non-template kernels: kyv_prod.hip)
#include "kyv_kernels.h"
#include "kyv_acct.h"

#define KYV_LAUNCH_PART 2
#define KYV_LNS kyvprod
#define KYV_KNS kyv
#define KYV_LNS_NAME "evaluation kernels"
#include "kyv_launch.inc"
