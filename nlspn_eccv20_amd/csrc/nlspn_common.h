// Shared device helpers for the NLSPN HIP kernels (gfx950 / CDNA4).
#pragma once

#include <hip/hip_fp16.h>
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace nlspn {

constexpr int kNumXcd = 8;  // MI355X: 8 XCDs, blocks dealt round-robin (b, b+8 share one)

// Experiment switches (the NLSPN_RES_DBG / NLSPN_S2D_DBG / NLSPN_HEADS_DBG ablation bits,
// which make results wrong on purpose, and NLSPN_RES_GUARD=0) exist only in the
// experiments build (make exp: lib/exp/libnlspn_hip_exp.so, loaded through
// NLSPN_LIB_PATH for A/B runs and the abort-path tests).  In the product library the
// environment is not read for them and every dbg branch folds away.
#ifndef NLSPN_EXPERIMENTS
#define NLSPN_EXPERIMENTS 0
#endif
constexpr bool kExperiments = NLSPN_EXPERIMENTS != 0;
__host__ __device__ constexpr unsigned exp_dbg(unsigned d) { return kExperiments ? d : 0u; }

// Element load/store with fp32 math regardless of storage type.
template <typename T> __device__ __forceinline__ float ld(const T *p);
template <> __device__ __forceinline__ float ld<float>(const float *p) { return *p; }
template <> __device__ __forceinline__ float ld<__half>(const __half *p) { return __half2float(*p); }

template <typename T> __device__ __forceinline__ void st(T *p, float v);
template <> __device__ __forceinline__ void st<float>(float *p, float v) { *p = v; }
template <> __device__ __forceinline__ void st<__half>(__half *p, float v) { *p = __float2half(v); }

// PX contiguous elements <-> float[PX]; PX>1 variants need PX*sizeof(T) alignment.
template <typename T, int PX> struct Vec;

template <> struct Vec<float, 1> {
    static __device__ __forceinline__ void load(const float *p, float (&v)[1]) { v[0] = *p; }
    static __device__ __forceinline__ void store(float *p, const float (&v)[1]) { *p = v[0]; }
};
template <> struct Vec<float, 4> {
    static __device__ __forceinline__ void load(const float *p, float (&v)[4]) {
        const float4 q = *reinterpret_cast<const float4 *>(p);
        v[0] = q.x; v[1] = q.y; v[2] = q.z; v[3] = q.w;
    }
    static __device__ __forceinline__ void store(float *p, const float (&v)[4]) {
        *reinterpret_cast<float4 *>(p) = make_float4(v[0], v[1], v[2], v[3]);
    }
};
template <> struct Vec<float, 2> {
    static __device__ __forceinline__ void load(const float *p, float (&v)[2]) {
        const float2 q = *reinterpret_cast<const float2 *>(p);
        v[0] = q.x; v[1] = q.y;
    }
    static __device__ __forceinline__ void store(float *p, const float (&v)[2]) {
        *reinterpret_cast<float2 *>(p) = make_float2(v[0], v[1]);
    }
};
template <> struct Vec<__half, 2> {
    static __device__ __forceinline__ void load(const __half *p, float (&v)[2]) {
        const float2 f = __half22float2(*reinterpret_cast<const __half2 *>(p));
        v[0] = f.x; v[1] = f.y;
    }
    static __device__ __forceinline__ void store(__half *p, const float (&v)[2]) {
        *reinterpret_cast<__half2 *>(p) = __floats2half2_rn(v[0], v[1]);
    }
};
template <> struct Vec<__half, 1> {
    static __device__ __forceinline__ void load(const __half *p, float (&v)[1]) { v[0] = __half2float(*p); }
    static __device__ __forceinline__ void store(__half *p, const float (&v)[1]) { *p = __float2half(v[0]); }
};
template <> struct Vec<__half, 4> {
    static __device__ __forceinline__ void load(const __half *p, float (&v)[4]) {
        const uint2 q = *reinterpret_cast<const uint2 *>(p);
        const __half2 a = *reinterpret_cast<const __half2 *>(&q.x);
        const __half2 b = *reinterpret_cast<const __half2 *>(&q.y);
        const float2 fa = __half22float2(a), fb = __half22float2(b);
        v[0] = fa.x; v[1] = fa.y; v[2] = fb.x; v[3] = fb.y;
    }
    static __device__ __forceinline__ void store(__half *p, const float (&v)[4]) {
        uint2 q;
        __half2 a = __floats2half2_rn(v[0], v[1]);
        __half2 b = __floats2half2_rn(v[2], v[3]);
        q.x = *reinterpret_cast<uint32_t *>(&a);
        q.y = *reinterpret_cast<uint32_t *>(&b);
        *reinterpret_cast<uint2 *>(p) = q;
    }
};

// ---- raw buffer access (cdna_hip_programming.md §5.5 T8): one wave-uniform
// descriptor per batch item, a 32-bit per-lane byte offset shared by every plane,
// and the plane offset in an SGPR (soffset).  Compared with flat 64-bit
// per-lane addresses this frees ~2 VGPRs per in-flight plane.  num_records is
// the 2 GiB maximum: each descriptor spans one batch item's planes (host checks).
using rsrc_t = __amdgpu_buffer_rsrc_t;

__device__ __forceinline__ rsrc_t make_rsrc(const void *base) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(base), (short)0, 0x7fffffff, 0x00020000);
}

// NOTE (hipcc / ROCm 7.2, gfx950): extracting elements of a raw_buffer_load_b64/
// b96/b128 result one by one with __builtin_bit_cast(float, q[i]) miscompiles —
// the load is narrowed to a single dword while the other lanes of the vector are
// still read (garbage).  Bit-cast the WHOLE vector to a float/half vector first;
// that form emits buffer_load_dwordx2/x4 correctly.
constexpr unsigned kNT = 2u;  // buffer-instruction cache policy: nt (streaming, non-temporal)

typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

template <typename T, int PX> struct BVec;

template <> struct BVec<float, 1> {
    static __device__ __forceinline__ void load(rsrc_t r, unsigned vo, unsigned so, float (&v)[1]) {
        v[0] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, vo, so, 0));
    }
    template <unsigned AUX = 0>
    static __device__ __forceinline__ void store(rsrc_t r, unsigned vo, unsigned so, const float (&v)[1]) {
        __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v[0]), r, vo, so, AUX);
    }
};
template <> struct BVec<float, 2> {
    static __device__ __forceinline__ void load(rsrc_t r, unsigned vo, unsigned so, float (&v)[2]) {
        const f32x2 q = __builtin_bit_cast(f32x2, __builtin_amdgcn_raw_buffer_load_b64(r, vo, so, 0));
        v[0] = q[0]; v[1] = q[1];
    }
    template <unsigned AUX = 0>
    static __device__ __forceinline__ void store(rsrc_t r, unsigned vo, unsigned so, const float (&v)[2]) {
        const f32x2 q = {v[0], v[1]};
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, q), r, vo, so, AUX);
    }
};
template <> struct BVec<float, 4> {
    static __device__ __forceinline__ void load(rsrc_t r, unsigned vo, unsigned so, float (&v)[4]) {
        const f32x4 q = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, vo, so, 0));
        v[0] = q[0]; v[1] = q[1]; v[2] = q[2]; v[3] = q[3];
    }
    template <unsigned AUX = 0>
    static __device__ __forceinline__ void store(rsrc_t r, unsigned vo, unsigned so, const float (&v)[4]) {
        const f32x4 q = {v[0], v[1], v[2], v[3]};
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, q), r, vo, so, AUX);
    }
};
template <> struct BVec<__half, 1> {
    static __device__ __forceinline__ void load(rsrc_t r, unsigned vo, unsigned so, float (&v)[1]) {
        v[0] = (float)__builtin_bit_cast(_Float16, __builtin_amdgcn_raw_buffer_load_b16(r, vo, so, 0));
    }
    template <unsigned AUX = 0>
    static __device__ __forceinline__ void store(rsrc_t r, unsigned vo, unsigned so, const float (&v)[1]) {
        __builtin_amdgcn_raw_buffer_store_b16(__builtin_bit_cast(unsigned short, (_Float16)v[0]), r, vo, so, AUX);
    }
};
template <> struct BVec<__half, 2> {
    static __device__ __forceinline__ void load(rsrc_t r, unsigned vo, unsigned so, float (&v)[2]) {
        const f16x2 q = __builtin_bit_cast(f16x2, __builtin_amdgcn_raw_buffer_load_b32(r, vo, so, 0));
        v[0] = (float)q[0]; v[1] = (float)q[1];
    }
    template <unsigned AUX = 0>
    static __device__ __forceinline__ void store(rsrc_t r, unsigned vo, unsigned so, const float (&v)[2]) {
        const f16x2 q = {(_Float16)v[0], (_Float16)v[1]};
        __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, q), r, vo, so, AUX);
    }
};
template <> struct BVec<__half, 4> {
    static __device__ __forceinline__ void load(rsrc_t r, unsigned vo, unsigned so, float (&v)[4]) {
        const f16x4 q = __builtin_bit_cast(f16x4, __builtin_amdgcn_raw_buffer_load_b64(r, vo, so, 0));
        v[0] = (float)q[0]; v[1] = (float)q[1]; v[2] = (float)q[2]; v[3] = (float)q[3];
    }
    template <unsigned AUX = 0>
    static __device__ __forceinline__ void store(rsrc_t r, unsigned vo, unsigned so, const float (&v)[4]) {
        const f16x4 q = {(_Float16)v[0], (_Float16)v[1], (_Float16)v[2], (_Float16)v[3]};
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, q), r, vo, so, AUX);
    }
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

// torch.clamp(x, min=0) (NaN propagates).
__device__ __forceinline__ float clamp0(float v) { return v < 0.f ? 0.f : v; }

// Bijective XCD-aware remap (cdna_hip_programming.md §5.5 T1): consecutive
// logical tiles land on the same XCD so neighbouring tiles' halo reads of the
// previous iteration's depth hit that XCD's L2.  Speed only, never correctness.
__device__ __forceinline__ int xcd_remap(int bid, int nblk) {
    const int q = nblk / kNumXcd, r = nblk % kNumXcd;
    const int xcd = bid % kNumXcd, slot = bid / kNumXcd;
    const int base = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
    return base + slot;
}

// Inverse of xcd_remap: the block index that xcd_remap maps to logical index L.  L is clamped
// into [0, nblk): the resident kernel indexes its sync lines by the result, and an index from
// outside the grid (a negative neighbour band, the likely cause of round 5's one
// illegal-address fault in a dropped neighbour-wait form) must not address
// past the workspace.  (For nblk < kNumXcd the else branch would divide by q = 0.)
__device__ __forceinline__ int xcd_unmap(int L, int nblk) {
    L = min(max(L, 0), nblk - 1);
    const int q = nblk / kNumXcd, r = nblk % kNumXcd;
    int xcd, slot;
    if (L < r * (q + 1)) {
        xcd = L / (q + 1);
        slot = L - xcd * (q + 1);
    } else {
        const int L2 = L - r * (q + 1);
        xcd = r + L2 / q;
        slot = L2 - (xcd - r) * q;
    }
    return slot * kNumXcd + xcd;
}

}  // namespace nlspn
