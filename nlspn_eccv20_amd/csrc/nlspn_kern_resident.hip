// Device code of the resident propagation kernel (nlspn_resident.h), compiled as its
// own translation unit so its code-generation flags can differ from the rest of the
// library (see Makefile) and so it rebuilds in parallel with nlspn_capi.hip.  The
// host stubs instantiated here are launched from nlspn_capi.hip.
#include "nlspn_resident.h"

namespace nlspn {
template __global__ void prop_resident_kernel<float, kResMaxNT, 2>(ResArgs);
template __global__ void prop_resident_kernel<__half, kResMaxNT, 2>(ResArgs);
}  // namespace nlspn
