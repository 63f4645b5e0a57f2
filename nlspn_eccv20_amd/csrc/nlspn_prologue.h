// Propagation prologue: everything nlspnmodel.py does once before the loop, in
// one elementwise pass over the head outputs:
//   _off_insert            (src/model/nlspnmodel.py:252-259, called :324)   [optional]
//   _affinity_normalization(:179-201) + _aff_insert (:261-269), called :325
//   mask_fix, confidence blend (:328-334)
//   k == 1 blend + clamp of pred_init (:341-348) -> p0 (workspace)
#pragma once

#include "nlspn_common.h"

namespace nlspn {

struct PrologueArgs {
    const void *pred_init, *dep, *conf, *aff_raw, *off_raw;
    const float *gamma;   // device, 1 float (aff_scale_const)
    void *aff_out;        // (K+1) planes per batch item, contiguous
    void *off_out;        // 2(K+1) planes per batch item or null
    void *conf_out;       // or null (iff conf null)
    void *p0;             // B planes
    long long aff_bs, off_bs;
    long long HW;
    int B, kind;
    unsigned flags;
};

enum { kAffAS = 0, kAffASS = 1, kAffTC = 2, kAffTGASS = 3 };

// _affinity_normalization (nlspnmodel.py:179-201) on K raw taps in place, and the
// reference-tap weight 1 - sum (_aff_insert :262-263) into `ref`; per pixel e.
template <int K, int PX>
__device__ __forceinline__ void normalize_taps(float (&t)[K][PX], float (&ref)[PX], int kind, float gamma) {
#pragma unroll
    for (int e = 0; e < PX; ++e) {
        if (kind == kAffTC) {            // :182-183
#pragma unroll
            for (int k = 0; k < K; ++k) t[k][e] = tanhf(t[k][e]) / gamma;
        } else if (kind == kAffTGASS) {  // :184-185
            const float den = gamma + 1e-8f;
#pragma unroll
            for (int k = 0; k < K; ++k) t[k][e] = tanhf(t[k][e]) / den;
        }
        float s = 0.f;                   // :190-191
#pragma unroll
        for (int k = 0; k < K; ++k) s += fabsf(t[k][e]);
        s = s + 1e-4f;
        if ((kind == kAffASS || kind == kAffTGASS) && s < 1.0f) s = 1.0f;  // :193-194
        if (kind != kAffTC) {            // :196-197
#pragma unroll
            for (int k = 0; k < K; ++k) t[k][e] = t[k][e] / s;
        }
        float sum = 0.f;                 // :262-263
#pragma unroll
        for (int k = 0; k < K; ++k) sum += t[k][e];
        ref[e] = 1.0f - sum;
    }
}

template <typename T, int K, int PX>
__global__ void __launch_bounds__(256) prologue_kernel(PrologueArgs a) {
    constexpr int REF = K / 2;
    const long long HW = a.HW, gpb = HW / PX, ngroups = (long long)a.B * gpb;
    const bool preserve = (a.flags & 0x1u) != 0, clip = (a.flags & 0x2u) != 0;
    const float gamma = *a.gamma;
    for (long long g = (long long)blockIdx.x * blockDim.x + threadIdx.x; g < ngroups;
         g += (long long)gridDim.x * blockDim.x) {
        const long long b = g / gpb, p = (g - b * gpb) * PX;

        // affinity normalisation, per pixel over the K planes
        float t[K][PX];
        const T *ar = static_cast<const T *>(a.aff_raw) + b * a.aff_bs + p;
#pragma unroll
        for (int k = 0; k < K; ++k) Vec<T, PX>::load(ar + k * HW, t[k]);
        float o[PX];
        normalize_taps<K, PX>(t, o, a.kind, gamma);
        T *ao = static_cast<T *>(a.aff_out) + b * (K + 1) * HW + p;
#pragma unroll
        for (int c = 0; c < K + 1; ++c) {
            if (c == REF) Vec<T, PX>::store(ao + c * HW, o);
            else Vec<T, PX>::store(ao + c * HW, t[c < REF ? c : c - 1]);
        }

        // _off_insert: zero (dh, dw) pair at the reference tap
        if (a.off_out) {
            const T *orw = static_cast<const T *>(a.off_raw) + b * a.off_bs + p;
            T *oo = static_cast<T *>(a.off_out) + b * 2 * (K + 1) * HW + p;
#pragma unroll
            for (int c = 0; c < K + 1; ++c) {
                float v0[PX], v1[PX];
                if (c == REF) {
#pragma unroll
                    for (int e = 0; e < PX; ++e) v0[e] = v1[e] = 0.f;
                } else {
                    const int k = c < REF ? c : c - 1;
                    Vec<T, PX>::load(orw + (2 * k) * HW, v0);
                    Vec<T, PX>::load(orw + (2 * k + 1) * HW, v1);
                }
                Vec<T, PX>::store(oo + (2 * c) * HW, v0);
                Vec<T, PX>::store(oo + (2 * c + 1) * HW, v1);
            }
        }

        // mask_fix / confidence / first blend
        const long long q = b * HW + p;
        float pi[PX], d[PX] = {0}, m[PX] = {0};
        Vec<T, PX>::load(static_cast<const T *>(a.pred_init) + q, pi);
        if (preserve) {
            Vec<T, PX>::load(static_cast<const T *>(a.dep) + q, d);
#pragma unroll
            for (int e = 0; e < PX; ++e) m[e] = d[e] > 0.f ? 1.f : 0.f;
        }
        if (a.conf) {
            float c[PX];
            Vec<T, PX>::load(static_cast<const T *>(a.conf) + q, c);
            if (preserve) {
#pragma unroll
                for (int e = 0; e < PX; ++e) c[e] = (1.0f - m[e]) * c[e] + m[e];
            }
            Vec<T, PX>::store(static_cast<T *>(a.conf_out) + q, c);
        }
#pragma unroll
        for (int e = 0; e < PX; ++e) {
            float v = pi[e];
            if (preserve) v = (1.0f - m[e]) * v + m[e] * d[e];
            if (clip) v = clamp0(v);
            pi[e] = v;
        }
        Vec<T, PX>::store(static_cast<T *>(a.p0) + q, pi);
    }
}

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
