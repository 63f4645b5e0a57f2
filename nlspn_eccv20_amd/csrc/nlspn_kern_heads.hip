// Device code of the head-epilogue convolution kernel (nlspn_heads.h), its own
// translation unit (it rebuilds in parallel with nlspn_capi.hip).  Launched from
// nlspn_capi.hip.
#include "nlspn_heads.h"

namespace nlspn {
#define NLSPN_HD_INST(MB)                                    \
    template __global__ void heads_kernel<MB, true>(HeadsArgs);  \
    template __global__ void heads_kernel<MB, false>(HeadsArgs);
NLSPN_HD_INST(1)
NLSPN_HD_INST(2)
NLSPN_HD_INST(3)
NLSPN_HD_INST(5)
// ablation variants (NLSPN_HEADS_DBG bits 1, 2; tools/head_ablate.py)
template __global__ void heads_kernel<1, true, 1>(HeadsArgs);
template __global__ void heads_kernel<1, true, 2>(HeadsArgs);
template __global__ void heads_kernel<1, true, 3>(HeadsArgs);
// the fused propagation prologue (nlspn_head_epilogue_prologue)
template __global__ void heads_kernel<1, true, 0, true>(HeadsArgs);
template __global__ void heads_kernel<1, false, 0, true>(HeadsArgs);
}  // namespace nlspn
