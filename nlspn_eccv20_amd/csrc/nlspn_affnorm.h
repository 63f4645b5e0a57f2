// Standalone affinity normalisation kernel (the forward prologue itself is fused
// into the first propagation iteration, nlspn_step.h FIRST).
#pragma once

#include "nlspn_common.h"

namespace nlspn {


// Standalone affinity normalisation (NLSPNModel._affinity_normalization + _aff_insert),
// used where the affinity changes per iteration (GRU refinement, nlspnmodel.py:373).
template <typename T, int K, int PX>
__global__ void __launch_bounds__(256) affnorm_kernel(const T *aff_raw, long long aff_bs, const float *gamma_p,
                                                     T *aff_out, long long HW, int B, int kind) {
    constexpr int REF = K / 2;
    const long long gpb = HW / PX, ngroups = (long long)B * gpb;
    const float gamma = *gamma_p;
    for (long long g = (long long)blockIdx.x * blockDim.x + threadIdx.x; g < ngroups;
         g += (long long)gridDim.x * blockDim.x) {
        const long long b = g / gpb, p = (g - b * gpb) * PX;
        float t[K][PX], o[PX];
#pragma unroll
        for (int k = 0; k < K; ++k) Vec<T, PX>::load(aff_raw + b * aff_bs + k * HW + p, t[k]);
        normalize_taps<K, PX>(t, o, kind, gamma);
        T *ao = aff_out + b * (K + 1) * HW + p;
#pragma unroll
        for (int c = 0; c < K + 1; ++c) {
            if (c == REF) Vec<T, PX>::store(ao + c * HW, o);
            else Vec<T, PX>::store(ao + c * HW, t[c < REF ? c : c - 1]);
        }
    }
}

}  // namespace nlspn
