// Device code of the resident propagation kernel (nlspn_resident.h), compiled as its
// own translation unit so its code-generation flags can differ from the rest of the
// library (see Makefile) and so it rebuilds in parallel with nlspn_capi.hip.  The
// host stubs instantiated here are launched from nlspn_capi.hip.
#include "nlspn_resident.h"

namespace nlspn {
// The 3x3 geometry (the reference default; quads per thread); the wider geometries' builds
// are nlspn_kern_resident_wide.hip.
// NTC: compile-time thread counts of the shapes the bench configs plan (C2 NYU B=8:
// 576; one NYU image, C1: 128), so the LDS row addresses fold into immediates;
// 0 = any other shape (thread count read at run time).  GROUPS = true: several image
// groups in turn in one launch (C3 KITTI B=4: 576 threads; others: run-time count).
#define NLSPN_RES_INST(T, F)                                                                \
    template __global__ void prop_resident_kernel<T, 3, 3, kResMaxNT, kResSMax, 0, false, F>(ResArgs);   \
    template __global__ void prop_resident_kernel<T, 3, 3, kResMaxNT, kResSMax, 576, false, F>(ResArgs); \
    template __global__ void prop_resident_kernel<T, 3, 3, kResMaxNT, kResSMax, 128, false, F>(ResArgs); \
    template __global__ void prop_resident_kernel<T, 3, 3, kResMaxNT, kResSMax, 576, true, F>(ResArgs);
// F: the forward prologue and iteration 1 inside the launch (ResArgs kResFirst), or after step 1
NLSPN_RES_INST(float, true)
NLSPN_RES_INST(__half, true)
NLSPN_RES_INST(float, false)
NLSPN_RES_INST(__half, false)
// the run-time-thread-count GROUPS build: the step-1 form only (its prologue form held scratch
// reloads in the iteration loop; the planner keeps step 1 for such merged launches)
template __global__ void prop_resident_kernel<float, 3, 3, kResMaxNT, kResSMax, 0, true, false>(ResArgs);
template __global__ void prop_resident_kernel<__half, 3, 3, kResMaxNT, kResSMax, 0, true, false>(ResArgs);
// the split-quad builds (small 3x3 parts, C1; step-1 form): four threads per quad at 320
// threads, two at 192
template __global__ void prop_resident_kernel<float, 3, 3, kResMaxNT, kResSMax, 192, false, false, 2>(ResArgs);
template __global__ void prop_resident_kernel<__half, 3, 3, kResMaxNT, kResSMax, 192, false, false, 2>(ResArgs);
template __global__ void prop_resident_kernel<float, 3, 3, kResMaxNT, kResSMax, 320, false, false, 1>(ResArgs);
template __global__ void prop_resident_kernel<__half, 3, 3, kResMaxNT, kResSMax, 320, false, false, 1>(ResArgs);
template __global__ void prop_resident_kernel<float, 3, 3, kResMaxNT, kResSMax, 320, false, true, 1>(ResArgs);
template __global__ void prop_resident_kernel<__half, 3, 3, kResMaxNT, kResSMax, 320, false, true, 1>(ResArgs);
}  // namespace nlspn
