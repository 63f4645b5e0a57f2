// Device code of the resident propagation kernel (nlspn_resident.h) for the geometries
// beyond 3x3: 1x17 (K = 16, two pixels per thread: the C5 stress config's taps) and 5x5
// (K = 24, a pixel per thread).  Its own translation unit, so it compiles in parallel with
// the 3x3 builds (nlspn_kern_resident.hip); launched from nlspn_capi.hip.
#include "nlspn_resident.h"

namespace nlspn {
// 1x17: the 576-thread builds (compile-time pitch; GROUPS for several image groups per
// launch, the C5 shape: 16 images in 4 groups of 4) and the run-time-thread-count builds.
// The step-1 form only (FIRST = false): a thread's raw-plane loads are 4 B or less, and the
// prologue's loads from HBM cost C5 more than step 1 does (nlspn_capi.hip plan_resident).
#define NLSPN_RES_INST_W(T)                                                                            \
    template __global__ void prop_resident_kernel<T, 1, 17, kResMaxNT, kResSMax, 0, false, false>(ResArgs);   \
    template __global__ void prop_resident_kernel<T, 1, 17, kResMaxNT, kResSMax, 576, false, false>(ResArgs); \
    template __global__ void prop_resident_kernel<T, 1, 17, kResMaxNT, kResSMax, 576, true, false>(ResArgs);  \
    template __global__ void prop_resident_kernel<T, 1, 17, kResMaxNT, kResSMax, 0, true, false>(ResArgs);    \
    template __global__ void prop_resident_kernel<T, 5, 5, kResMaxNT, kResSMax, 0, false, false>(ResArgs);
NLSPN_RES_INST_W(float)
NLSPN_RES_INST_W(__half)
}  // namespace nlspn
