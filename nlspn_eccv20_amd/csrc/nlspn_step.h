// One fused NLSPN propagation iteration for gfx950 (CDNA4).
//
// Replaces, per iteration, the reference's
//   new_pred*confidence                          (src/model/nlspnmodel.py:351)
//   _propagate_once(...)                          (:203-226) -> DCN forward
//     modulated_deformable_im2col_gpu_kernel      (.../cuda/modulated_deform_im2col_cuda.cuh:127-194)
//     at::addmm(bias, columns^T, weight^T)        (.../cuda/modulated_deform_conv_cuda.cu:108-114)
//   preserve-input blend + optional clamp         (:355-361)   [+ final clamp :375-377 on the last]
// with one launch, no `columns` buffer and no GEMM (the NLSPN weight is all ones).
//
// Structure (one 256-thread workgroup per TH x TW output tile, PX pixels per thread):
//   1. issue the tile's streamed loads first — K normalised-affinity planes,
//      2K offset planes and dep — 16-B (fp32) / 8-B (fp16) per lane, coalesced;
//   2. stage f = p_in * conf for the tile + halo window into LDS (fp32), zero
//      outside the image (= the reference's zero-padded bilinear) or replicate-
//      clamped for the no-offset branch;
//   3. per tap, bilinear-sample f from LDS; taps whose 2x2 footprint leaves the
//      window (learned offsets are unbounded) fall back to L2/global reads with
//      the reference's per-corner checks — correctness never depends on HALO;
//   4. accumulate taps in index order with the reference tap (index K/2) weighted
//      1 - sum(others); blend, clamp, store p_out (and pred on the last step).
// Summation and bilinear arithmetic follow the reference's operation order; the
// file is compiled with -ffp-contract=off so it issues exactly the IEEE sequence
// the C oracle does (bit-identical iterations given identical inputs).
#pragma once

#include "nlspn_common.h"

namespace nlspn {

struct StepArgs {
    const void *p_in;   // B planes
    const void *conf;   // B planes or null (conf_prop off)
    const void *dep;    // B planes or null (preserve off)
    const void *aff;    // normalised affinity, (K+1) planes per batch item
    const void *off;    // offsets (null: no-offset branch)
    void *p_out;        // B planes
    void *pred_out;     // B planes or null
    long long aff_bs;   // batch strides in elements
    long long off_bs;
    int B, H, W;
    int tiles_x, tiles_y;
    int off_raw;        // 1: raw (2K planes, ref tap implicit), 0: inserted (2(K+1) planes)
    unsigned flags;     // NLSPN_PRESERVE_INPUT | NLSPN_ALWAYS_CLIP
};

constexpr unsigned kPreserve = 0x1u;
constexpr unsigned kAlwaysClip = 0x2u;

template <typename T>
__device__ __forceinline__ float fetch_f(const T *__restrict__ pin, const T *__restrict__ cf, long long q) {
    float v = ld(pin + q);
    if (cf) v = v * ld(cf + q);
    return v;
}

// KH x KW taps; TH x TW tile; PX px per thread; window radii RY/RX; SV = staging
// vector width (4 requires W % 4 == 0 and RX % 4 == 0); PRE = preload offsets
// before the staging barrier.
template <typename T, int KH, int KW, int TH, int TW, int PX, int RY, int RX, int SV, bool OFFSET, bool PRE>
__global__ void __launch_bounds__(TH * TW / PX) prop_step_kernel(StepArgs a) {
    constexpr int NT = TH * TW / PX;
    constexpr int KK = KH * KW, REF = KK / 2, K = KK - 1;
    constexpr int PH = (KH - 1) / 2, PW = (KW - 1) / 2;
    constexpr int WH = TH + 2 * RY, WW = TW + 2 * RX;
    constexpr int TPR = TW / PX;
    static_assert(TW % PX == 0 && NT % 64 == 0, "tile/thread shape");
    static_assert(OFFSET || (KH == 3 && KW == 3 && RY == 1 && RX == 1), "no-offset branch is 3x3 replicate");
    static_assert(!OFFSET || (RY > PH && RX > PW), "window must cover the tap base grid");
    static_assert(SV == 1 || (RX % 4 == 0 && WW % 4 == 0), "vector staging alignment");
    __shared__ __attribute__((aligned(16))) float win[WH * WW];

    const int H = a.H, W = a.W;
    const long long HW = (long long)H * W;
    int tile = xcd_remap(blockIdx.x, gridDim.x);
    const int tx = tile % a.tiles_x;
    tile /= a.tiles_x;
    const int ty = tile % a.tiles_y;
    const int b = tile / a.tiles_y;
    const int x0 = tx * TW, y0 = ty * TH;
    const int wy0 = y0 - RY, wx0 = x0 - RX;

    const T *__restrict__ pin = static_cast<const T *>(a.p_in) + b * HW;
    const T *__restrict__ cf = a.conf ? static_cast<const T *>(a.conf) + b * HW : nullptr;
    const bool preserve = (a.flags & kPreserve) != 0;
    const bool clip = (a.flags & kAlwaysClip) != 0;

    const int ly = threadIdx.x / TPR, lx = (threadIdx.x % TPR) * PX;
    const int y = y0 + ly, xb = x0 + lx;
    const bool active = (y < H) && (xb < W);  // PX>1 requires W % PX == 0: groups are all-in or all-out
    const long long pix = (long long)y * W + xb;

    // ---- 1. streamed per-pixel loads (issued before staging so they overlap it)
    float av[K][PX];
    float dh[PRE ? K : 1][PX], dw[PRE ? K : 1][PX];
    float dv[PX];
    const T *__restrict__ offb = nullptr;
    if (active) {
        const T *__restrict__ ab = static_cast<const T *>(a.aff) + b * a.aff_bs + pix;
#pragma unroll
        for (int k = 0; k < K; ++k) Vec<T, PX>::load(ab + (long long)(k < REF ? k : k + 1) * HW, av[k]);
        if (OFFSET) {
            offb = static_cast<const T *>(a.off) + b * a.off_bs + pix;
            if (PRE) {
#pragma unroll
                for (int k = 0; k < K; ++k) {
                    const int c = a.off_raw ? k : (k < REF ? k : k + 1);
                    Vec<T, PX>::load(offb + (long long)(2 * c) * HW, dh[PRE ? k : 0]);
                    Vec<T, PX>::load(offb + (long long)(2 * c + 1) * HW, dw[PRE ? k : 0]);
                }
            }
        }
        if (preserve) Vec<T, PX>::load(static_cast<const T *>(a.dep) + b * HW + pix, dv);
    }

    // ---- 2. stage f = p * conf over the window
    if (OFFSET) {
        if (SV == 4) {
            constexpr int WW4 = WW / 4;
            for (int i = threadIdx.x; i < WH * WW4; i += NT) {
                const int r = i / WW4, c4 = (i - r * WW4) * 4;
                const int gy = wy0 + r, gx = wx0 + c4;
                float v[4] = {0.f, 0.f, 0.f, 0.f};
                if (gy >= 0 && gy < H && gx >= 0 && gx < W) {
                    const long long q = (long long)gy * W + gx;
                    Vec<T, 4>::load(pin + q, v);
                    if (cf) {
                        float c[4];
                        Vec<T, 4>::load(cf + q, c);
#pragma unroll
                        for (int e = 0; e < 4; ++e) v[e] = v[e] * c[e];
                    }
                }
                *reinterpret_cast<float4 *>(&win[r * WW + c4]) = make_float4(v[0], v[1], v[2], v[3]);
            }
        } else {
            for (int i = threadIdx.x; i < WH * WW; i += NT) {
                const int r = i / WW, c = i - r * WW;
                const int gy = wy0 + r, gx = wx0 + c;
                float v = 0.f;
                if (gy >= 0 && gy < H && gx >= 0 && gx < W) v = fetch_f(pin, cf, (long long)gy * W + gx);
                win[i] = v;
            }
        }
    } else {
        // F.pad(feat, (1,1,1,1), mode="replicate") (nlspnmodel.py:210)
        for (int i = threadIdx.x; i < WH * WW; i += NT) {
            const int r = i / WW, c = i - r * WW;
            int gy = wy0 + r, gx = wx0 + c;
            gy = gy < 0 ? 0 : (gy > H - 1 ? H - 1 : gy);
            gx = gx < 0 ? 0 : (gx > W - 1 ? W - 1 : gx);
            win[i] = fetch_f(pin, cf, (long long)gy * W + gx);
        }
    }
    __syncthreads();
    if (!active) return;  // no barrier below

    // ---- 3. taps, in index order; reference tap weight = 1 - sum(others) (nlspnmodel.py:262-263)
    float aref[PX], acc[PX];
#pragma unroll
    for (int p = 0; p < PX; ++p) {
        float s = 0.f;
#pragma unroll
        for (int k = 0; k < K; ++k) s += av[k][p];
        aref[p] = 1.0f - s;
        acc[p] = 0.f;
    }
    const float Hf = (float)H, Wf = (float)W;
#pragma unroll
    for (int t = 0; t < KK; ++t) {
        const int i = t / KW, j = t % KW;
        if (t == REF) {
            // zero offset, integer sample point: the bilinear weight is exactly (1,0,0,0)
#pragma unroll
            for (int p = 0; p < PX; ++p) acc[p] += win[(ly + RY) * WW + lx + p + RX] * aref[p];
            continue;
        }
        const int k = t < REF ? t : t - 1;
        if (!OFFSET) {
#pragma unroll
            for (int p = 0; p < PX; ++p) acc[p] += win[(ly + RY + i - 1) * WW + lx + p + RX + j - 1] * av[k][p];
            continue;
        }
        float tdh[PX], tdw[PX];
        if (PRE) {
#pragma unroll
            for (int p = 0; p < PX; ++p) { tdh[p] = dh[PRE ? k : 0][p]; tdw[p] = dw[PRE ? k : 0][p]; }
        } else {
            const int c = a.off_raw ? k : t;
            Vec<T, PX>::load(offb + (long long)(2 * c) * HW, tdh);
            Vec<T, PX>::load(offb + (long long)(2 * c + 1) * HW, tdw);
        }
#pragma unroll
        for (int p = 0; p < PX; ++p) {
            // modulated_deform_im2col_cuda.cuh:178-189 + mdmcn_im2col_bilinear :24-54
            const float h_im = (float)(y - PH + i) + tdh[p];
            const float w_im = (float)(xb + p - PW + j) + tdw[p];
            float val = 0.f;
            if (h_im > -1.f && w_im > -1.f && h_im < Hf && w_im < Wf) {
                const int h_low = (int)floorf(h_im), w_low = (int)floorf(w_im);
                const float lh = h_im - (float)h_low, lw = w_im - (float)w_low;
                const float hh = 1.f - lh, hw = 1.f - lw;
                const int ry = h_low - wy0, rx = w_low - wx0;
                float v1, v2, v3, v4;
                if ((unsigned)ry < (unsigned)(WH - 1) && (unsigned)rx < (unsigned)(WW - 1)) {
                    const float *s = &win[ry * WW + rx];
                    v1 = s[0];
                    v2 = s[1];
                    v3 = s[WW];
                    v4 = s[WW + 1];
                } else {
                    const int h_high = h_low + 1, w_high = w_low + 1;
                    const long long r0 = (long long)h_low * W, r1 = (long long)h_high * W;
                    v1 = (h_low >= 0 && w_low >= 0) ? fetch_f(pin, cf, r0 + w_low) : 0.f;
                    v2 = (h_low >= 0 && w_high <= W - 1) ? fetch_f(pin, cf, r0 + w_high) : 0.f;
                    v3 = (h_high <= H - 1 && w_low >= 0) ? fetch_f(pin, cf, r1 + w_low) : 0.f;
                    v4 = (h_high <= H - 1 && w_high <= W - 1) ? fetch_f(pin, cf, r1 + w_high) : 0.f;
                }
                const float w1 = hh * hw, w2 = hh * lw, w3 = lh * hw, w4 = lh * lw;
                val = (w1 * v1 + w2 * v2 + w3 * v3 + w4 * v4);
            }
            acc[p] += val * av[k][p];
        }
    }

    // ---- 4. preserve-input blend (:355-357), clamp (:359-361), final clamp (:375-377)
    float o[PX], fin[PX];
#pragma unroll
    for (int p = 0; p < PX; ++p) {
        float v = acc[p];
        if (preserve) {
            const float m = dv[p] > 0.f ? 1.f : 0.f;
            v = (1.0f - m) * v + m * dv[p];
        }
        if (clip) v = clamp0(v);
        o[p] = v;
        fin[p] = clip ? v : clamp0(v);
    }
    Vec<T, PX>::store(static_cast<T *>(a.p_out) + b * HW + pix, o);
    if (a.pred_out) Vec<T, PX>::store(static_cast<T *>(a.pred_out) + b * HW + pix, fin);
}

}  // namespace nlspn
