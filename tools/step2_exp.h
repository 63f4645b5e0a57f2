// EXPERIMENT (tools/step_bench only, not part of the library): one propagation
// iteration (steps t >= 2) for config C5's shape (1x17 taps, fp16), two horizontal
// pixels per lane, a branch-free tap path, and finally a persistent software-
// pipelined form.  Measured (profiles/r02/c5_step_experiments.txt): bit-identical to
// prop_step_kernel but never faster — the tap phase is LDS-bound (random-offset
// bilinear gather, ~3.5-way bank conflicts) and does not overlap the HBM stream; the
// pipelined form cannot keep two tiles' 57 loads per wave in flight (vmcnt counts to 63)
// and runs at half speed.
//
// Same arithmetic as prop_step_kernel (nlspn_step.h; bit-identical outputs), with
// the instruction count cut where that kernel is issue-bound (DESIGN §3.1, C5 at
// VALU ~60 %):
//   * every streamed plane is loaded once per PIXEL PAIR (fp16: one 4-byte load,
//     fp32: one 8-byte load) and kept packed until its tap consumes it;
//   * no branches in pass A: every tap computes its fractional parts, weights and
//     window index; a tap outside (-1,H) x (-1,W) (or NaN: the reference's .cuh:180
//     test) is redirected to a 2x2 block of zeros with weights (1,0,0,0), so it
//     contributes +0 exactly as the reference's val = 0; a valid tap whose footprint
//     leaves the window (h >= wy0 and h < wy0 + WH - 1 is floor(h) in
//     [wy0, wy0 + WH - 2]) takes an inline slow path from global memory with the
//     reference's per-corner checks (rare);
//   * taps are accumulated as they come, in the reference's order, so no per-tap
//     column array is held (the register budget goes to loads in flight);
//   * the window is stored as horizontal pairs (f[r][c], f[r][c+1]), so each row of a
//     footprint is ONE 8-byte ds_read_b64 at a plain cell index (two reads per tap).
#pragma once

#include "../nlspn_eccv20_amd/csrc/nlspn_step.h"

namespace nlspn {

// A horizontal pixel pair of one plane, as loaded (converted where consumed).
template <typename T> struct Pair;
// add(q, p, y) = (float)q[p] + y and mul(q, p, v) = (float)q[p] * v, each rounded
// once as the separate convert and add/multiply are (the conversion is exact).  For
// fp16 storage each is ONE v_fma_mix_f32 reading the half in place (q*1 + y, and
// v*q + (-0): an exact product plus -0 keeps the product's rounding and zero sign).
template <> struct Pair<float> {
    using raw = f32x2;
    static __device__ __forceinline__ raw load(rsrc_t r, unsigned vo, unsigned so) {
        return __builtin_bit_cast(f32x2, __builtin_amdgcn_raw_buffer_load_b64(r, vo, so, 0));
    }
    static __device__ __forceinline__ float get(raw q, int p) { return q[p]; }
    static __device__ __forceinline__ float add(raw q, int p, float y) { return q[p] + y; }
    static __device__ __forceinline__ float mul(raw q, int p, float v) { return v * q[p]; }
};
template <> struct Pair<__half> {
    using raw = f16x2;
    static __device__ __forceinline__ raw load(rsrc_t r, unsigned vo, unsigned so) {
        return __builtin_bit_cast(f16x2, __builtin_amdgcn_raw_buffer_load_b32(r, vo, so, 0));
    }
    static __device__ __forceinline__ float get(raw q, int p) { return (float)q[p]; }
    static __device__ __forceinline__ float add(raw q, int p, float y) {
        const unsigned u = __builtin_bit_cast(unsigned, q);
        float d;
        if (p == 0) asm("v_fma_mix_f32 %0, %1, 1.0, %2 op_sel_hi:[1,0,0]" : "=v"(d) : "v"(u), "v"(y));
        else asm("v_fma_mix_f32 %0, %1, 1.0, %2 op_sel:[1,0,0] op_sel_hi:[1,0,0]" : "=v"(d) : "v"(u), "v"(y));
        return d;
    }
    static __device__ __forceinline__ float mul(raw q, int p, float v) {
        const unsigned u = __builtin_bit_cast(unsigned, q);
        const float nz = -0.0f;
        float d;
        if (p == 0) asm("v_fma_mix_f32 %0, %1, %2, %3 op_sel_hi:[1,0,0]" : "=v"(d) : "v"(u), "v"(v), "v"(nz));
        else asm("v_fma_mix_f32 %0, %1, %2, %3 op_sel:[1,0,0] op_sel_hi:[1,0,0]" : "=v"(d) : "v"(u), "v"(v), "v"(nz));
        return d;
    }
};

// The largest float below v >= 0 (h > below(v) is h >= v; for v = 0 the negative
// denormal, or -0 where denormals flush — then h = 0 takes the slow path, still exact).
__device__ __forceinline__ float below(float v) {
    return v > 0.f ? __int_as_float(__float_as_int(v) - 1) : __int_as_float(0x80000001);
}

// 4 staged elements of a window row, as loaded (converted when the window is written).
template <typename T> struct SRaw;
template <> struct SRaw<float> {
    using raw = f32x4;
    static __device__ __forceinline__ raw load(rsrc_t r, unsigned vo) {
        return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, vo, 0u, 0));
    }
    static __device__ __forceinline__ float get(raw q, int e) { return q[e]; }
};
template <> struct SRaw<__half> {
    using raw = f16x4;
    static __device__ __forceinline__ raw load(rsrc_t r, unsigned vo) {
        return __builtin_bit_cast(f16x4, __builtin_amdgcn_raw_buffer_load_b64(r, vo, 0u, 0));
    }
    static __device__ __forceinline__ float get(raw q, int e) { return (float)q[e]; }
};

// Everything one tile loads: the window's p and conf (staged into LDS), and per
// pixel pair the K affinities, 2K offsets and dep (held in registers until the taps).
template <typename T, int K, int SIT>
struct TileLoads {
    typename SRaw<T>::raw sp[SIT], sc[SIT];
    typename Pair<T>::raw ar[K], oh[K], ow[K], dr;
};

// The persistent, software-pipelined form: each workgroup walks a contiguous run of
// tiles (neighbouring tiles share its XCD's L2 for the halo) and issues tile n+1's
// loads before it computes tile n, so the tap phase (LDS-bound: a bilinear gather at
// random offsets is ~3.5-way bank-conflicted) overlaps the next tile's HBM stream
// instead of alternating with it.  Two register sets (unrolled by two) and two LDS
// windows; one barrier per tile.
// KH x KW taps, TH x TW tile (TW/2 lanes per row), window radii RY / RX (RX % 4 == 0).
// Requires W % 4 == 0 and pair-aligned planes (the host checks).  Not the FIRST step
// (the prologue stays in prop_step_kernel).
// DBG (experiments, tools/step_bench only; 0 in the library): 1 = no staging loads
// (zero window), 2 = no taps (loads consumed by a plain sum), 3 = both.
template <typename T, int KH, int KW, int TH, int TW, int RY, int RX, int DBG = 0>
__global__ void __launch_bounds__(TH * TW / 2) prop_step2_kernel(StepArgs a) {
    constexpr int PX = 2, NT = TH * TW / PX;
    constexpr int KK = KH * KW, REF = KK / 2, K = KK - 1;
    constexpr int PH = (KH - 1) / 2, PW = (KW - 1) / 2;
    constexpr int WH = TH + 2 * RY, WW = TW + 2 * RX, WC = WH * WW;
    constexpr int TPR = TW / PX;
    constexpr int SV = 4, WV = WW / SV, NV = WH * WV, SIT = (NV + NT - 1) / NT;
    constexpr int ZC = WC + 1;  // pair cells ZC, ZC+WW: zeros (the redirect of invalid taps)
    constexpr int PS = ZC + WW + 1;  // pairs per window buffer
    static_assert(NT % 64 == 0 && RX % 4 == 0 && WW % 4 == 0 && RY > PH && RX > PW, "tile / window shape");
    constexpr unsigned ES = sizeof(T);
    // Two windows as horizontal pairs: P[1 + r*WW + c] = (f[r][c], f[r][c+1]), so each
    // row of a footprint is ONE aligned ds_read_b64 at a plain cell index, the
    // footprint's second row an immediate offset from the first.
    __shared__ __attribute__((aligned(16))) float2 Pbuf[2 * PS];
    if (threadIdx.x < 4) Pbuf[(threadIdx.x >> 1) * PS + ZC + (threadIdx.x & 1) * WW] = make_float2(0.f, 0.f);

    const int H = a.H, W = a.W;
    const long long HW = (long long)H * W;
    const unsigned plane_bytes = (unsigned)HW * ES;
    const bool has_conf = a.conf != nullptr;
    const bool preserve = (a.flags & kPreserve) != 0;
    const bool clip = (a.flags & kAlwaysClip) != 0;
    const float Hf = (float)H, Wf = (float)W;
    const int ly = threadIdx.x / TPR, lx = (threadIdx.x % TPR) * PX;
    const int ntiles = a.B * a.tiles_y * a.tiles_x;
    const int t_lo = (int)((long long)blockIdx.x * ntiles / gridDim.x);
    const int t_hi = (int)((long long)(blockIdx.x + 1) * ntiles / gridDim.x);

    // tile -> (image, tile origin)
    auto tile_at = [&](int t, int &b, int &x0, int &y0) {
        x0 = (t % a.tiles_x) * TW;
        t /= a.tiles_x;
        y0 = (t % a.tiles_y) * TH;
        b = t / a.tiles_y;
    };
    auto issue = [&](int t, TileLoads<T, K, SIT> &L) {
        int b, x0, y0;
        tile_at(t, b, x0, y0);
        const int wy0 = y0 - RY, wx0 = x0 - RX;
        const T *pbase = static_cast<const T *>(a.p_in) + b * HW;
        const rsrc_t rp = make_rsrc(pbase);
        const rsrc_t rc = make_rsrc(has_conf ? static_cast<const T *>(a.conf) + b * HW : pbase);
#pragma unroll
        for (int it = 0; it < SIT; ++it) {  // the window's p and conf first, clamped addresses
            const int i = threadIdx.x + it * NT;
            const int ii = i < NV ? i : NV - 1;
            const int r = ii / WV, c = (ii - r * WV) * SV;
            int gy = wy0 + r, gx = wx0 + c;
            gy = gy < 0 ? 0 : (gy > H - 1 ? H - 1 : gy);
            gx = gx < 0 ? 0 : (gx > W - SV ? W - SV : gx);
            const unsigned q = (unsigned)(gy * W + gx) * ES;
            if (!(DBG & 1)) {
                L.sp[it] = SRaw<T>::load(rp, q);
                if (has_conf) L.sc[it] = SRaw<T>::load(rc, q);
            }
        }
        const int y = y0 + ly, xb = x0 + lx;
        const unsigned vpix = ((y < H && xb < W) ? (unsigned)(y * W + xb) : 0u) * ES;
        const rsrc_t ra = make_rsrc(static_cast<const T *>(a.aff) + b * a.aff_bs);
        const rsrc_t ro = make_rsrc(static_cast<const T *>(a.off) + b * a.off_bs);
#pragma unroll
        for (int k = 0; k < K; ++k) {  // then the per-pair planes, in tap order
            const int tt = k < REF ? k : k + 1;
            const unsigned c = a.off_raw ? k : tt;
            L.ar[k] = Pair<T>::load(ra, vpix, (unsigned)tt * plane_bytes);
            L.oh[k] = Pair<T>::load(ro, vpix, (2 * c) * plane_bytes);
            L.ow[k] = Pair<T>::load(ro, vpix, (2 * c + 1) * plane_bytes);
        }
        if (preserve) L.dr = Pair<T>::load(make_rsrc(static_cast<const T *>(a.dep) + b * HW), vpix, 0u);
    };
    // f = p * conf' into window buffer P (waits for the staging loads only)
    auto stage = [&](int t, const TileLoads<T, K, SIT> &L, float2 *P) {
        int b, x0, y0;
        tile_at(t, b, x0, y0);
        const int wy0 = y0 - RY, wx0 = x0 - RX;
        float *pf = reinterpret_cast<float *>(P);
#pragma unroll
        for (int it = 0; it < SIT; ++it) {
            const int i = threadIdx.x + it * NT;
            if (i < NV) {
                const int r = i / WV, c = (i - r * WV) * SV;
                const int gy = wy0 + r, gx = wx0 + c;
                const bool in = gy >= 0 && gy < H && gx >= 0 && gx < W;  // zero outside the image
                float v[SV];
#pragma unroll
                for (int e = 0; e < SV; ++e) {
                    const float pv = (DBG & 1) ? 0.f : SRaw<T>::get(L.sp[it], e);
                    const float f = has_conf && !(DBG & 1) ? pv * SRaw<T>::get(L.sc[it], e) : pv;
                    v[e] = in ? f : 0.f;
                }
                const int li = 1 + r * WW + c;
                pf[2 * li - 1] = v[0];                                                          // P[li-1].y
                *reinterpret_cast<float4 *>(&pf[2 * li]) = make_float4(v[0], v[1], v[1], v[2]);  // P[li], P[li+1]
                *reinterpret_cast<float2 *>(&pf[2 * li + 4]) = make_float2(v[2], v[3]);         // P[li+2]
                pf[2 * li + 6] = v[3];                                                          // P[li+3].x
            }
        }
    };
    // taps of tile t from window P, blend, clamp, store
    auto compute = [&](int t, const TileLoads<T, K, SIT> &L, const float2 *P) {
        int b, x0, y0;
        tile_at(t, b, x0, y0);
        const int wy0 = y0 - RY, wx0 = x0 - RX;
        const int y = y0 + ly, xb = x0 + lx;
        if (!(y < H && xb < W)) return;  // W % 2 == 0: a pair is all-in or all-out
        const unsigned vpix = (unsigned)(y * W + xb) * ES;
        const T *pbase = static_cast<const T *>(a.p_in) + b * HW;
        const rsrc_t rp = make_rsrc(pbase);
        const rsrc_t rc = make_rsrc(has_conf ? static_cast<const T *>(a.conf) + b * HW : pbase);
        const rsrc_t rd = make_rsrc(preserve ? static_cast<const T *>(a.dep) + b * HW : pbase);
        // take = valid (.cuh:180: h > -1, h < H, ...) AND footprint in the window (h >= wy0,
        // h < wy0 + WH - 1: floor(h) in [wy0, wy0 + WH - 2]) as ONE open interval per
        // axis: h > lo (lo = -1, or the float just below wy0 when wy0 >= 0) and h < hi
        const float fy_lo = wy0 >= 0 ? below((float)wy0) : -1.f;
        const float fy_hi = fminf((float)(wy0 + WH - 1), Hf);
        const float fx_lo = wx0 >= 0 ? below((float)wx0) : -1.f;
        const float fx_hi = fminf((float)(wx0 + WW - 1), Wf);
        const int lbase = 1 - (wy0 * WW + wx0);
        const float zh = (float)(wy0 + WH), zw = (float)wx0;  // (zh*WW + zw) + lbase == ZC
        // Taps in index order, accumulated as they come (the reference's summation order,
        // .cu:108-114 with the all-ones weight), the reference tap (K/2, zero offset)
        // weighted 1 - sum (nlspnmodel.py:262-263) in its place; a valid tap whose
        // footprint leaves the window takes the rare slow path (global memory, the
        // reference's per-corner checks) inline.
        float acc[PX], aref[PX];
#pragma unroll
        for (int p = 0; p < PX; ++p) {
            float s = 0.f;
#pragma unroll
            for (int k = 0; k < K; ++k) s = Pair<T>::add(L.ar[k], p, s);
            aref[p] = 1.0f - s;
            acc[p] = 0.f;
        }
        if (DBG & 2) {  // experiment: consume every load, no taps
#pragma unroll
            for (int k = 0; k < K; ++k)
#pragma unroll
                for (int p = 0; p < PX; ++p)
                    acc[p] += Pair<T>::get(L.ar[k], p) + Pair<T>::get(L.oh[k], p) * Pair<T>::get(L.ow[k], p) +
                              P[1 + (ly + RY) * WW + lx + p + RX].x;
        }
#pragma unroll
        for (int k = 0; k < (DBG & 2 ? 0 : K); ++k) {
            const int tt = k < REF ? k : k + 1;
            const int i = tt / KW, j = tt % KW;
            if (k == REF) {
#pragma unroll
                for (int p = 0; p < PX; ++p) acc[p] += P[1 + (ly + RY) * WW + lx + p + RX].x * aref[p];
            }
#pragma unroll
            for (int p = 0; p < PX; ++p) {
                // modulated_deform_im2col_cuda.cuh:178-179 + mdmcn_im2col_bilinear :24-54
                const float h_im = Pair<T>::add(L.oh[k], p, (float)(y - PH + i));
                const float w_im = Pair<T>::add(L.ow[k], p, (float)(xb + p - PW + j));
                const bool take = h_im > fy_lo && h_im < fy_hi && w_im > fx_lo && w_im < fx_hi;
                // not taken: the integer point (wy0 + WH, wx0), whose footprint is the
                // zero pairs ZC / ZC + WW, weights (1, 0, 0, 0): v = +0 (val = 0)
                const float hs = take ? h_im : zh, ws = take ? w_im : zw;
                const float fh = floorf(hs), fw = floorf(ws);
                const float lh = hs - fh, lw = ws - fw;
                const float hh = 1.f - lh, hw = 1.f - lw;
                const float w1 = hh * hw, w2 = hh * lw, w3 = lh * hw, w4 = lh * lw;
                const int li = (int)__builtin_fmaf(fh, (float)WW, fw) + lbase;  // exact: integers < 2^24
                const float2 s01 = P[li], s23 = P[li + WW];
                float v = (w1 * s01.x + w2 * s01.y + w3 * s23.x + w4 * s23.y);
                if (__builtin_expect(!take, 0) && h_im > -1.f && w_im > -1.f && h_im < Hf && w_im < Wf) {
                    const int h_low = (int)floorf(h_im), w_low = (int)floorf(w_im), h_high = h_low + 1,
                              w_high = w_low + 1;
                    const float slh = h_im - (float)h_low, slw = w_im - (float)w_low;
                    const float shh = 1.f - slh, shw = 1.f - slw;
                    const int r0 = h_low * W, r1 = h_high * W;
                    const float v1 = (h_low >= 0 && w_low >= 0)
                                         ? fetch_f<T, false>(rp, rc, rd, has_conf, preserve, clip, (r0 + w_low) * ES)
                                         : 0.f;
                    const float v2 = (h_low >= 0 && w_high <= W - 1)
                                         ? fetch_f<T, false>(rp, rc, rd, has_conf, preserve, clip, (r0 + w_high) * ES)
                                         : 0.f;
                    const float v3 = (h_high <= H - 1 && w_low >= 0)
                                         ? fetch_f<T, false>(rp, rc, rd, has_conf, preserve, clip, (r1 + w_low) * ES)
                                         : 0.f;
                    const float v4 = (h_high <= H - 1 && w_high <= W - 1)
                                         ? fetch_f<T, false>(rp, rc, rd, has_conf, preserve, clip, (r1 + w_high) * ES)
                                         : 0.f;
                    const float sw1 = shh * shw, sw2 = shh * slw, sw3 = slh * shw, sw4 = slh * slw;
                    v = (sw1 * v1 + sw2 * v2 + sw3 * v3 + sw4 * v4);
                }
                acc[p] += Pair<T>::mul(L.ar[k], p, v);  // .cuh:189 col = val * mask, summed in tap order
            }
        }
        // preserve-input blend (:355-357), clamp (:359-361), final clamp (:375-377)
        float o[PX], fin[PX];
#pragma unroll
        for (int p = 0; p < PX; ++p) {
            float v = acc[p];
            if (preserve) {
                const float d = Pair<T>::get(L.dr, p);
                const float m = d > 0.f ? 1.f : 0.f;
                v = (1.0f - m) * v + m * d;
            }
            if (clip) v = clamp0(v);
            o[p] = v;
            fin[p] = clip ? v : clamp0(v);
        }
        BVec<T, PX>::store(make_rsrc(static_cast<T *>(a.p_out) + b * HW), vpix, 0u, o);
        if (a.pred_out) BVec<T, PX>::store(make_rsrc(static_cast<T *>(a.pred_out) + b * HW), vpix, 0u, fin);
    };

    // ---- the pipeline: loads of tile n+1 in flight while tile n computes
    TileLoads<T, K, SIT> L0, L1;
    if (t_lo >= t_hi) return;
    issue(t_lo, L0);
    stage(t_lo, L0, Pbuf);
    lds_barrier();
    for (int t = t_lo; t < t_hi; t += 2) {
        if (t + 1 < t_hi) issue(t + 1, L1);
        compute(t, L0, Pbuf);
        if (t + 1 >= t_hi) break;
        stage(t + 1, L1, Pbuf + PS);
        lds_barrier();  // window t+1 written; every read of window t done
        if (t + 2 < t_hi) issue(t + 2, L0);
        compute(t + 1, L1, Pbuf + PS);
        if (t + 2 >= t_hi) break;
        stage(t + 2, L0, Pbuf);
        lds_barrier();
    }
}

}  // namespace nlspn
