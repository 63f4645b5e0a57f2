// Device code of the GRU-mode convolutions (nlspn_gconv.h), their own translation unit.
// Launched from nlspn_capi.hip (nlspn_gconv); the configurations are NLSPN_GC_CONFIGS.
#include "nlspn_gconv.h"

namespace nlspn {
#define NLSPN_GC_INST(id, ...) template __global__ void gconv_kernel<__VA_ARGS__>(GconvArgs);
NLSPN_GC_CONFIGS(NLSPN_GC_INST)
template __global__ void gsmall_kernel<16>(GconvArgs, const float *);
}  // namespace nlspn
