// Backward of the fused NLSPN propagation for gfx950 (CDNA4), fp32.
//
// What the reference gets from autograd over nlspnmodel.py:323-381, with the
// DCNv2 backward (src/model/deformconv/src/cuda/modulated_deform_conv_cuda.cu:124-280)
// for each of the T DCN calls:
//   grad_mask   = sum col * bilinear            (col2im_coord mval, .cuh:304-307)
//   grad_offset = coordinate_weight * col * mask (col2im_coord val,  .cuh:309-312, :84-125)
//   grad_input  = bilinear weight * col * mask   (col2im, atomicAdd scatter, .cuh:196-254)
// with col = grad_output (NLSPN's DCN weight is all ones), plus torch autograd of
// the confidence product, blends, clamps, _aff_insert and the affinity normalisation.
//
// One launch per iteration, t = T..1 (bwd_step_kernel), then one finishing
// elementwise launch (bwd_final_kernel):
//   * the iteration's output pixel owns its dL/d(affinity) and dL/d(offset)
//     accumulators (plain read-modify-write across the T launches, no atomics;
//     step T initialises them, so nothing is cleared beforehand); dL/d(affinity)
//     is kept as G_k = dL/daff_k - dL/daff_ref (K planes, _aff_insert folded in);
//   * step 1 finishes each pixel's affinity gradient in place: the normalisation
//     backward runs on the final G and writes grad_aff_raw directly;
//   * the scatter of dL/df_{t-1} to the 4 bilinear corners of every tap goes to an
//     LDS window (ds_add_f32) covering the tile + halo; the window is flushed once
//     with global float atomics (non-zero in-image cells only) and taps that leave
//     the window add to global memory directly.  Float atomics make the last bits
//     of dL/df order-dependent, as in the reference's col2im.
//   * dL/df buffers ping-pong between iterations; each step zeroes the cells it
//     consumed, so no memset is needed between launches.
#pragma once

#include "nlspn_step.h"

namespace nlspn {

struct BwdArgs {
    const float *p_in;      // p_{t-1} (FIRST: pred_init)
    const float *p_out;     // p_t (pred_inter[t-1])
    const float *conf;      // FIRST: raw conf; else conf' (forward conf_out); null = conf_prop off
    const float *conf_eff;  // conf' (forward conf_out) for the own-pixel product, or null
    const float *dep;
    const float *aff;       // normalised affinity (forward aff_out), (K+1) planes per item
    const float *off;       // raw offsets (2K planes per item) or null (no-offset branch)
    const float *g_pred;    // dL/dpred (used when t == T) or null
    const float *g_inter;   // dL/dpred_inter[t-1] or null
    float *gf_read;         // dL/df_t   (scattered by step t+1); zeroed after use
    float *gf_write;        // dL/df_{t-1} (scattered here)
    float *g_aff;           // K planes per item: G_k = dL/daff_k - dL/daff_ref, accumulated
    float *g_off;           // 2K planes per item (raw layout), accumulated = grad_off_raw
    float *g_conf;          // dL/dconf' plane, accumulated (null iff conf null)
    long long off_bs;
    int B, H, W, tiles_x, tiles_y;
    int last;               // t == T: accumulators are initialised, not read
    int g_aff_ins;          // 1: g_aff has the inserted (K+1)-plane layout (step-level backward; tap
                            //    K/2 untouched), 0: K planes (G form)
    unsigned flags;
    // FIRST only: affinity-normalisation backward fused in (per pixel, G final)
    const float *aff_raw;   // raw head affinity, K planes per item at aff_raw_bs
    long long aff_raw_bs;
    const float *gamma;
    float *grad_aff_raw;    // K planes per item, batch stride gaff_bs (0: K*H*W)
    long long gaff_bs, goff_bs;  // batch strides of grad_aff_raw / g_off in elements (0: contiguous)
    float *gamma_part;      // one partial dL/dgamma per workgroup (TGASS), or null
    int kind;
    // two-pass form (SPLIT): this iteration's dL/dout plane, written for bwd_coef_kernel
    float *go_out;          // plane of item 0; item b at go_out + b * go_bs
    long long go_bs;
};

__device__ __forceinline__ float bld(rsrc_t r, unsigned vo, unsigned so) {
    return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, vo, so, 0));
}
__device__ __forceinline__ void bst(rsrc_t r, unsigned vo, unsigned so, float v) {
    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v), r, vo, so, 0);
}

// Bilinear corners of f_{t-1} at (hs, ws) (caller checked validity): from the LDS
// window when the 2x2 footprint lies inside it, else from global memory with the
// reference's per-corner checks (.cuh:24-54).
template <bool FIRST, int WH, int WW>
__device__ __forceinline__ bool tap_corners(float hs, float ws, int wy0, int wx0, int H, int W, const float *win,
                                            rsrc_t rp, rsrc_t rc, rsrc_t rd, bool has_conf, bool preserve, bool clip,
                                            int &hl, int &wl, float (&v)[4]) {
    hl = (int)floorf(hs);
    wl = (int)floorf(ws);
    const int ry = hl - wy0, rx = wl - wx0;
    if ((unsigned)ry < (unsigned)(WH - 1) && (unsigned)rx < (unsigned)(WW - 1)) {
        const float *s = &win[ry * WW + rx];
        v[0] = s[0]; v[1] = s[1]; v[2] = s[WW]; v[3] = s[WW + 1];
        return true;
    }
    constexpr unsigned ES = 4;
    const int r0 = hl * W, r1 = (hl + 1) * W;
    v[0] = (hl >= 0 && wl >= 0) ? fetch_f<float, FIRST>(rp, rc, rd, has_conf, preserve, clip, (r0 + wl) * ES) : 0.f;
    v[1] = (hl >= 0 && wl + 1 <= W - 1) ? fetch_f<float, FIRST>(rp, rc, rd, has_conf, preserve, clip, (r0 + wl + 1) * ES) : 0.f;
    v[2] = (hl + 1 <= H - 1 && wl >= 0) ? fetch_f<float, FIRST>(rp, rc, rd, has_conf, preserve, clip, (r1 + wl) * ES) : 0.f;
    v[3] = (hl + 1 <= H - 1 && wl + 1 <= W - 1) ? fetch_f<float, FIRST>(rp, rc, rd, has_conf, preserve, clip, (r1 + wl + 1) * ES) : 0.f;
    return false;
}

// Backward of _affinity_normalization + _aff_insert for one pixel (nlspnmodel.py:
// 179-201, :261-269): G_k = dL/daff_k - dL/daff_ref (aff_ref = 1 - sum aff_k);
//   u = tanh(a)/(gamma+1e-8) [TGASS] | tanh(a)/gamma [TC] | a [AS/ASS];
//   s = sum|u| + 1e-4, s = 1 where s < 1 [ASS/TGASS; no gradient there]; aff = u/s [not TC].
template <int K>
__device__ __forceinline__ float aff_norm_backward(const float (&G)[K], const float (&ar)[K], float gamma, int kind,
                                                   float (&ga)[K]) {
    float u[K], th[K], s = 0.f, dot = 0.f, gsum = 0.f;
#pragma unroll
    for (int k = 0; k < K; ++k) {
        th[k] = tanhf(ar[k]);
        u[k] = kind == kAffTC ? th[k] / gamma : (kind == kAffTGASS ? th[k] / (gamma + 1e-8f) : ar[k]);
        s += fabsf(u[k]);
    }
    s = s + 1e-4f;
    const bool clamped = (kind == kAffASS || kind == kAffTGASS) && s < 1.0f;
    const float se = clamped ? 1.0f : s;
#pragma unroll
    for (int k = 0; k < K; ++k) dot += G[k] * u[k];
#pragma unroll
    for (int k = 0; k < K; ++k) {
        float gu;
        if (kind == kAffTC) {
            gu = G[k];
        } else {
            gu = G[k] / se;
            if (!clamped) {
                const float sg = u[k] > 0.f ? 1.f : (u[k] < 0.f ? -1.f : 0.f);
                gu += -dot / (se * se) * sg;
            }
        }
        float g = gu;
        if (kind == kAffTC) {
            g = gu * (1.f - th[k] * th[k]) / gamma;
        } else if (kind == kAffTGASS) {
            const float dd = gamma + 1e-8f;
            g = gu * (1.f - th[k] * th[k]) / dd;
            gsum += -gu * th[k] / (dd * dd);
        }
        ga[k] = g;
    }
    return gsum;
}

// One backward iteration.  Every global load of the step is issued before the
// first store (the compiler cannot reorder a buffer load above a buffer store it
// cannot prove disjoint, so a read-modify-write per plane would cost one memory
// round trip each): window staging, the tap planes, the own-pixel planes and —
// for K <= 8 — the dL/daff and dL/doffset accumulators.  Larger K accumulate in
// registers and read-modify-write in chunks of 8 planes.
// DIAG: diagnostic knobs for tools/bwd_bench (0 in the library; non-zero values
// produce wrong gradients): 1 = no window flush, 4 = no accumulator read-modify-write,
// 8 = no scatter at all (SPLIT: neither the LDS window adds nor the direct atomics), 16 = the
// window adds as LDS f64 atomics (timing only: the flush still reads fixed point).
// SPLIT (two-pass form, offsets): the step only produces dL/dout (written to go_out) and
// scatters dL/df_{t-1}; the dL/daff and dL/doffset terms, which need f_{t-1} at every
// tap, are computed for all T iterations afterwards by bwd_coef_kernel.  Without the
// clamp's mask recomputation a SPLIT step stages no window and reads no accumulator.
template <int KH, int KW, int TH, int TW, int RY, int RX, int SV, bool OFFSET, bool FIRST, int DIAG = 0,
          bool SPLIT = false>
__global__ void __launch_bounds__(TH * TW) bwd_step_kernel(BwdArgs a) {
    constexpr int NT = TH * TW;
    constexpr int KK = KH * KW, REF = KK / 2, K = KK - 1;
    constexpr int PH = (KH - 1) / 2, PW = (KW - 1) / 2;
    constexpr int WH = TH + 2 * RY, WW = TW + 2 * RX;
    static_assert(NT % 64 == 0, "tile shape");
    static_assert(OFFSET || (KH == 3 && KW == 3 && RY == 1 && RX == 1), "no-offset branch is 3x3 replicate");
    static_assert(!OFFSET || (RY > PH && RX > PW), "window must cover the tap base grid");
    static_assert(SV == 1 || (OFFSET && RX % 4 == 0 && WW % 4 == 0), "vector staging alignment");
    constexpr int WV = WW / SV, NV = WH * WV, SIT = (NV + NT - 1) / NT;
    constexpr int NC = WH * WW, CIT = (NC + NT - 1) / NT;
    constexpr unsigned ES = 4;
    constexpr bool HOIST = K <= 8;
    constexpr int KO = OFFSET ? 2 * K : 1;
    static_assert(!SPLIT || OFFSET, "the two-pass form is for the offset branch");
    __shared__ __attribute__((aligned(16))) float win[NC];   // f_{t-1} over the window
    __shared__ unsigned long long gacc[NC];                 // scatter accumulator for dL/df_{t-1} (fixed point)
    __shared__ float red[NT / 64], redm[NT / 64];

    const int H = a.H, W = a.W;
    const long long HW = (long long)H * W;
    int tile = xcd_remap(blockIdx.x, gridDim.x);
    const int tx = tile % a.tiles_x;
    tile /= a.tiles_x;
    const int ty = tile % a.tiles_y;
    const int b = tile / a.tiles_y;
    const int x0 = tx * TW, y0 = ty * TH;
    const int wy0 = y0 - RY, wx0 = x0 - RX;

    const bool has_conf = a.conf != nullptr;
    const bool preserve = (a.flags & kPreserve) != 0;
    const bool clip = (a.flags & kAlwaysClip) != 0;
    const bool last = a.last != 0;
    const float *pbase = a.p_in + b * HW;
    const rsrc_t rp = make_rsrc(pbase);
    const rsrc_t rc = make_rsrc(has_conf ? a.conf + b * HW : pbase);
    const rsrc_t rd = make_rsrc(preserve ? a.dep + b * HW : pbase);

    const int ly = threadIdx.x / TW, lx = threadIdx.x % TW;
    const int y = y0 + ly, x = x0 + lx;
    const bool active = (y < H) && (x < W);
    const unsigned vpix = (active ? (unsigned)(y * W + x) : 0u) * ES, plane_bytes = (unsigned)HW * ES;

    // ---- 1. all loads: window staging, tap planes, own pixel, accumulators
    const bool need_win = !SPLIT || clip;  // SPLIT: f_{t-1} only for the clamp's mask
    float sp[SIT][SV], sc[SIT][SV], sd[FIRST ? SIT : 1][SV];
    bool sin[SIT];
#pragma unroll
    for (int it = 0; it < SIT && need_win; ++it) {
        const int i = threadIdx.x + it * NT;
        const int ii = i < NV ? i : NV - 1;
        const int r = ii / WV, c = (ii - r * WV) * SV;
        int gy = wy0 + r, gx = wx0 + c;
        if (OFFSET) sin[it] = i < NV && gy >= 0 && gy < H && gx >= 0 && gx < W;
        else sin[it] = i < NV;
        gy = gy < 0 ? 0 : (gy > H - 1 ? H - 1 : gy);
        gx = gx < 0 ? 0 : (gx > W - SV ? W - SV : gx);
        const unsigned q = (unsigned)(gy * W + gx) * ES;
        BVec<float, SV>::load(rp, q, 0u, sp[it]);
        if (has_conf) BVec<float, SV>::load(rc, q, 0u, sc[it]);
        if (FIRST && preserve) BVec<float, SV>::load(rd, q, 0u, sd[FIRST ? it : 0]);
    }
    const rsrc_t ra = make_rsrc(a.aff + b * (K + 1) * HW);
    const rsrc_t ro = make_rsrc(OFFSET ? a.off + b * a.off_bs : a.aff);
    float av[K], dh[OFFSET ? K : 1], dw[OFFSET ? K : 1];
#pragma unroll
    for (int k = 0; k < K; ++k) {
        av[k] = bld(ra, vpix, (unsigned)(k < REF ? k : k + 1) * plane_bytes);
        if (OFFSET) {
            dh[k] = bld(ro, vpix, (2u * k) * plane_bytes);
            dw[k] = bld(ro, vpix, (2u * k + 1) * plane_bytes);
        }
    }
    const rsrc_t rgc = make_rsrc(has_conf ? a.g_conf + b * HW : a.gf_read);
    const rsrc_t rgf = make_rsrc(a.gf_read + b * HW);
    float dv = 0.f, gfr = 0.f, pt = 0.f, ce = 1.f, gi = 0.f, gpr = 0.f, gcv = 0.f;
    if (preserve) dv = bld(rd, vpix, 0u);
    if (!last) gfr = bld(rgf, vpix, 0u);
    if (has_conf || (last && a.g_pred && !clip)) pt = bld(make_rsrc(a.p_out + b * HW), vpix, 0u);
    if (has_conf) ce = bld(make_rsrc(a.conf_eff + b * HW), vpix, 0u);
    if (has_conf && !last) gcv = bld(rgc, vpix, 0u);
    if (a.g_inter) gi = bld(make_rsrc(a.g_inter + b * HW), vpix, 0u);
    if (last && a.g_pred) gpr = bld(make_rsrc(a.g_pred + b * HW), vpix, 0u);
    const bool gins = a.g_aff_ins != 0;
    const rsrc_t rga = make_rsrc(a.g_aff + b * (gins ? K + 1 : K) * HW);
    auto gplane = [&](int k) { return (unsigned)(gins && k >= REF ? k + 1 : k) * plane_bytes; };
    const rsrc_t rgo = make_rsrc(OFFSET ? a.g_off + b * (a.goff_bs ? a.goff_bs : 2LL * K * HW) : a.g_aff);
    float cG[K], cO[KO];
#pragma unroll
    for (int k = 0; k < K; ++k) cG[k] = (HOIST && !SPLIT && !last && !(DIAG & 4)) ? bld(rga, vpix, gplane(k)) : 0.f;
#pragma unroll
    for (int k = 0; k < KO; ++k)
        cO[k] = (OFFSET && HOIST && !SPLIT && !last && !(DIAG & 4)) ? bld(rgo, vpix, (unsigned)k * plane_bytes) : 0.f;

    // ---- 2. stage f_{t-1}, zero the scatter window
#pragma unroll
    for (int it = 0; it < SIT && need_win; ++it) {
        const int i = threadIdx.x + it * NT;
        if (i < NV) {
            float v[SV];
#pragma unroll
            for (int e = 0; e < SV; ++e) {
                const float f = make_f<FIRST>(sp[it][e], has_conf ? sc[it][e] : 1.f,
                                              FIRST && preserve ? sd[FIRST ? it : 0][e] : 0.f, has_conf, preserve, clip);
                v[e] = sin[it] ? f : 0.f;
            }
            const int r = i / WV, c = (i - r * WV) * SV;
            if constexpr (SV == 4)
                *reinterpret_cast<float4 *>(&win[r * WW + c]) = make_float4(v[0], v[1], v[2], v[3]);
            else
                win[r * WW + c] = v[0];
        }
    }
#pragma unroll
    for (int it = 0; it < CIT; ++it) {
        const int i = threadIdx.x + it * NT;
        if (i < NC) gacc[i] = 0ull;
    }
    lds_barrier();

    // ---- per pixel: dL/dp_t (the next step's scatter through f_t = p_t * conf', plus
    //      direct grads), the clamp mask, dL/dout = go
    const float Hf = (float)H, Wf = (float)W;
    auto tap_pos = [&](int k, float &hs, float &ws) {
        const int t = k < REF ? k : k + 1;
        const int i = t / KW, j = t % KW;
        if (OFFSET) {
            hs = (float)(y - PH + i) + dh[k];
            ws = (float)(x - PW + j) + dw[k];
        } else {
            int yy = y + i - 1, xx = x + j - 1;
            yy = yy < 0 ? 0 : (yy > H - 1 ? H - 1 : yy);
            xx = xx < 0 ? 0 : (xx > W - 1 ? W - 1 : xx);
            hs = (float)yy;
            ws = (float)xx;
        }
    };
    const float fown = need_win ? win[(ly + RY) * WW + lx + RX] : 0.f;
    float asum = 0.f;
#pragma unroll
    for (int k = 0; k < K; ++k) asum += av[k];
    const float aref = 1.0f - asum;
    float go = 0.f, mass = 0.f;
    if (active) {
        float g = has_conf ? gfr * ce : gfr;
        if (a.g_inter) g += gi;
        if (last && a.g_pred) g += clip ? gpr : (pt >= 0.f ? gpr : 0.f);  // pred = clamp(p_T, 0)
        if (has_conf) bst(rgc, vpix, 0u, gcv + gfr * pt);
        bst(rgf, vpix, 0u, 0.f);  // consumed: ready for reuse as a scatter target
        if (clip) {
            // recompute the forward value for the clamp mask (torch clamp passes the gradient where x >= 0)
            float val[K];
#pragma unroll
            for (int k = 0; k < K; ++k) {
                float hs, ws;
                tap_pos(k, hs, ws);
                val[k] = 0.f;
                if (hs > -1.f && ws > -1.f && hs < Hf && ws < Wf) {
                    int hl, wl;
                    float v[4];
                    tap_corners<FIRST, WH, WW>(hs, ws, wy0, wx0, H, W, win, rp, rc, rd, has_conf, preserve, clip, hl, wl, v);
                    const float lh = hs - (float)hl, lw = ws - (float)wl, hh = 1.f - lh, hw = 1.f - lw;
                    val[k] = (hh * hw * v[0] + hh * lw * v[1] + lh * hw * v[2] + lh * lw * v[3]);
                }
            }
            float acc = 0.f;
#pragma unroll
            for (int t = 0; t < KK; ++t) acc += t == REF ? fown * aref : val[t < REF ? t : t - 1] * av[t < REF ? t : t - 1];
            float pre = acc;
            if (preserve) {
                const float m = dv > 0.f ? 1.f : 0.f;
                pre = (1.0f - m) * acc + m * dv;
            }
            if (!(pre >= 0.f)) g = 0.f;
        }
        go = preserve ? (1.0f - (dv > 0.f ? 1.f : 0.f)) * g : g;
        if (SPLIT) bst(make_rsrc(a.go_out + b * a.go_bs), vpix, 0u, go);
        // bound on everything this pixel scatters: |go| (|a_ref| + sum |a_k|), bilinear weights <= 1
        float as = fabsf(aref);
#pragma unroll
        for (int k = 0; k < K; ++k) as += fabsf(av[k]);
        mass = fabsf(go) * as;
    }

    // ---- the tile's scatter scale.  dL/df_{t-1} is accumulated in LDS as 64-bit
    // fixed point (ds_add_u64: integer LDS atomics run at ~3x the rate of ds_add_f32
    // on gfx950, tools/bwd_bench), scaled by 2^sh so the tile's total scattered mass
    // stays below 2^59: every float contribution converts exactly up to a rounding
    // of 2^-sh (~2^-59 of the tile's mass), and the window sums are exact, so they do
    // not depend on arrival order.  Non-finite mass: plain float global atomics.
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) mass += __shfl_xor(mass, o, 64);
    if ((threadIdx.x & 63) == 0) redm[threadIdx.x >> 6] = mass;
    lds_barrier();
    float tot = 0.f;
#pragma unroll
    for (int i = 0; i < NT / 64; ++i) tot += redm[i];
    const bool exact = tot < 3.0e38f;  // finite (NaN compares false); 0 scatters nothing
    const int sh = exact && tot > 0.f ? 58 - ilogbf(tot) : 0;

    float gsum = 0.f;
    if (active) {
        // ---- taps: dL/daff (G form), dL/doffset (coordinate weights, .cuh:84-125),
        //      and the col2im scatter of dL/df_{t-1} (.cuh:196-254)
        float *gfw = a.gf_write + b * HW;
        auto add_win = [&](int cell, float v) {
            if constexpr ((DIAG & 16) != 0)  // (tools/bwd_bench: LDS f64 atomic adds instead, timing only)
                atomicAdd(reinterpret_cast<double *>(&gacc[cell]), (double)v);
            else
                atomicAdd(&gacc[cell], (unsigned long long)__float2ll_rn(ldexpf(v, sh)));
        };
        if (exact) add_win((ly + RY) * WW + lx + RX, go * aref);  // reference tap: integer point, weight 1
        else atomicAdd(&gfw[y * W + x], go * aref);
        if constexpr (SPLIT && (DIAG & 8)) {
        } else if constexpr (SPLIT) {
            // scatter only: the corner weights of every valid tap (.cuh:196-254)
#pragma unroll
            for (int k = 0; k < K; ++k) {
                float hs, ws;
                tap_pos(k, hs, ws);
                if (hs > -1.f && ws > -1.f && hs < Hf && ws < Wf) {
                    const int hl = (int)floorf(hs), wl = (int)floorf(ws);
                    const float lh = hs - (float)hl, lw = ws - (float)wl, hh = 1.f - lh, hw = 1.f - lw;
                    const float w1 = hh * hw, w2 = hh * lw, w3 = lh * hw, w4 = lh * lw;
                    const float top = go * av[k];
                    const bool inwin = (unsigned)(hl - wy0) < (unsigned)(WH - 1) && (unsigned)(wl - wx0) < (unsigned)(WW - 1);
                    if (inwin && exact) {
                        const int c0 = (hl - wy0) * WW + (wl - wx0);
                        add_win(c0, w1 * top);
                        add_win(c0 + 1, w2 * top);
                        add_win(c0 + WW, w3 * top);
                        add_win(c0 + WW + 1, w4 * top);
                    } else {
                        const float wts[4] = {w1, w2, w3, w4};
#pragma unroll
                        for (int cnr = 0; cnr < 4; ++cnr) {
                            const int hy = hl + (cnr >> 1), wx = wl + (cnr & 1);
                            if (hy >= 0 && hy <= H - 1 && wx >= 0 && wx <= W - 1) atomicAdd(&gfw[hy * W + wx], wts[cnr] * top);
                        }
                    }
                }
            }
        } else {
    #pragma unroll
            for (int k = 0; k < K; ++k) {
                float hs, ws;
                tap_pos(k, hs, ws);
                float val = 0.f;
                if (hs > -1.f && ws > -1.f && hs < Hf && ws < Wf) {
                    int hl, wl;
                    float v[4];
                    const bool inwin = tap_corners<FIRST, WH, WW>(hs, ws, wy0, wx0, H, W, win, rp, rc, rd, has_conf,
                                                                  preserve, clip, hl, wl, v);
                    const float lh = hs - (float)hl, lw = ws - (float)wl, hh = 1.f - lh, hw = 1.f - lw;
                    const float w1 = hh * hw, w2 = hh * lw, w3 = lh * hw, w4 = lh * lw;
                    val = (w1 * v[0] + w2 * v[1] + w3 * v[2] + w4 * v[3]);
                    const float top = go * av[k];
                    if (OFFSET) {
                        float cwh = 0.f, cww = 0.f;
                        cwh += -1 * hw * v[0];
                        cwh += -1 * lw * v[1];
                        cwh += hw * v[2];
                        cwh += lw * v[3];
                        cww += -1 * hh * v[0];
                        cww += hh * v[1];
                        cww += -1 * lh * v[2];
                        cww += lh * v[3];
                        cO[2 * k] += cwh * go * av[k];
                        cO[2 * k + 1] += cww * go * av[k];
                    }
                    if (inwin && exact) {
                        // out-of-image cells of the window are dropped by the flush (as the reference's checks)
                        const int c0 = (hl - wy0) * WW + (wl - wx0);
                        add_win(c0, w1 * top);
                        add_win(c0 + 1, w2 * top);
                        add_win(c0 + WW, w3 * top);
                        add_win(c0 + WW + 1, w4 * top);
                    } else {
                        const float wts[4] = {w1, w2, w3, w4};
    #pragma unroll
                        for (int cnr = 0; cnr < 4; ++cnr) {
                            const int hy = hl + (cnr >> 1), wx = wl + (cnr & 1);
                            if (hy >= 0 && hy <= H - 1 && wx >= 0 && wx <= W - 1) atomicAdd(&gfw[hy * W + wx], wts[cnr] * top);
                        }
                    }
                }
                cG[k] += go * (val - fown);
            }
        }

        // ---- accumulators
        if (!SPLIT && !HOIST && !last) {
#pragma unroll
            for (int c0 = 0; c0 < K; c0 += 8) {
                float t8[8];
#pragma unroll
                for (int i = 0; i < 8; ++i) t8[i] = c0 + i < K ? bld(rga, vpix, gplane(c0 + i)) : 0.f;
#pragma unroll
                for (int i = 0; i < 8; ++i) if (c0 + i < K) cG[c0 + i] = t8[i] + cG[c0 + i];
            }
            if (OFFSET) {
#pragma unroll
                for (int c0 = 0; c0 < KO; c0 += 8) {
                    float t8[8];
#pragma unroll
                    for (int i = 0; i < 8; ++i) t8[i] = c0 + i < KO ? bld(rgo, vpix, (unsigned)(c0 + i) * plane_bytes) : 0.f;
#pragma unroll
                    for (int i = 0; i < 8; ++i) if (c0 + i < KO) cO[c0 + i] = t8[i] + cO[c0 + i];
                }
            }
        }
        if (OFFSET && !SPLIT && !(DIAG & 4)) {
#pragma unroll
            for (int k = 0; k < KO; ++k) bst(rgo, vpix, (unsigned)k * plane_bytes, cO[k]);
        }
        if (!SPLIT && FIRST) {
            // G is final for this pixel: normalisation backward -> grad_aff_raw, dL/dgamma partial
            const rsrc_t rar = make_rsrc(a.aff_raw + b * a.aff_raw_bs);
            float ar[K], ga[K];
#pragma unroll
            for (int k = 0; k < K; ++k) ar[k] = bld(rar, vpix, (unsigned)k * plane_bytes);
            gsum = aff_norm_backward<K>(cG, ar, *a.gamma, a.kind, ga);
            const rsrc_t rout = make_rsrc(a.grad_aff_raw + b * (a.gaff_bs ? a.gaff_bs : (long long)K * HW));
#pragma unroll
            for (int k = 0; k < K; ++k) bst(rout, vpix, (unsigned)k * plane_bytes, ga[k]);
        } else if (!SPLIT && !(DIAG & 4)) {
#pragma unroll
            for (int k = 0; k < K; ++k) bst(rga, vpix, gplane(k), cG[k]);
        }
    }
    if (FIRST && !SPLIT && a.gamma_part) {
        for (int o = 32; o > 0; o >>= 1) gsum += __shfl_down(gsum, o, 64);
        if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = gsum;
    }
    lds_barrier();
    if (FIRST && !SPLIT && a.gamma_part && threadIdx.x == 0) {
        float s = 0.f;
#pragma unroll
        for (int i = 0; i < NT / 64; ++i) s += red[i];
        a.gamma_part[blockIdx.x] = s;
    }
    // ---- flush the scatter window (in-image, non-zero cells) with global float atomics
    if ((DIAG & 1) || !exact) return;
    float *gfw = a.gf_write + b * HW;
#pragma unroll
    for (int it = 0; it < CIT; ++it) {
        const int i = threadIdx.x + it * NT;
        if (i < NC) {
            const int r = i / WW, c = i - r * WW;
            const int gy = wy0 + r, gx = wx0 + c;
            const long long q = (long long)gacc[i];
            if (q != 0 && gy >= 0 && gy < H && gx >= 0 && gx < W) atomicAdd(&gfw[gy * W + gx], ldexpf((float)q, -sh));
        }
    }
}

// Second pass of the two-pass backward (offset branch): dL/daff and dL/doffset of all T
// iterations, after the SPLIT steps wrote every iteration's dL/dout.  A workgroup owns
// the same tile as the steps and loops t = T..1: it stages f_{t-1} into its LDS window,
// reads the own pixel's dL/dout_t and adds each tap's terms to register accumulators —
// the one-pass step's arithmetic in the same order (its accumulators start at 0 at
// t = T and are summed t = T..1), so the results are bit-identical to it.  The affinity
// and offset planes are read once (the one-pass form re-reads them and read-modify-
// writes 24 accumulator planes per iteration).  Step 1's normalisation backward and
// dL/dgamma partial run at the end.
// dL/dout_t is stored in the gradient outputs themselves (plane t-1 of grad_off_raw's
// 2K planes, then of grad_aff_raw's K; T <= 3K): a pixel's dL/dout values are read only
// by its own thread, before that thread writes its gradients over them.
#ifndef NLSPN_BWD_COEF_WAVES
#define NLSPN_BWD_COEF_WAVES 1
#endif
struct BwdCoefArgs {
    const float *pred_init, *pred_inter, *conf, *conf_eff, *dep, *aff, *off, *aff_raw, *gamma;
    float *g_off, *grad_aff_raw, *gamma_part;
    long long off_bs, aff_raw_bs, goff_bs, gaff_bs, N;  // batch strides resolved (non-zero)
    int B, H, W, tiles_x, tiles_y, T, kind;
    unsigned flags;
};

// conf' (iteration-invariant) is staged into an LDS window once; iterations t >= 2 load only
// p_{t-1} and form f = p * conf' from it (half the staging loads; measured within noise of
// staging both, profiles/r06/ab_bwd_resident_v1.json).  Issuing the next iteration's p loads
// before the taps (one register window, 105 VGPRs; or capped at 5 waves, 9 VGPRs spilled)
// measured 5 % / 2 % slower (profiles/r06/ab_bwd_pf_t18_rejected.json).
// The coefficient sums contract into fused multiply-adds (the file is built with
// -ffp-contract=off for the forward's exact IEEE sequence; the backward is checked to float
// rounding, 1e-4 against the fp64 oracle and 1e-6 against the one-pass form): 0.4627 vs 0.4757
// ms per C2 backward (profiles/r06/ab_bwd_pass2_fma.jsonl).
template <int KH, int KW, int TH, int TW, int RY, int RX, int SV>
__global__ void __launch_bounds__(TH * TW, NLSPN_BWD_COEF_WAVES) bwd_coef_kernel(BwdCoefArgs a) {
#pragma clang fp contract(fast)
    constexpr int NT = TH * TW;
    constexpr int KK = KH * KW, REF = KK / 2, K = KK - 1;
    constexpr int PH = (KH - 1) / 2, PW = (KW - 1) / 2;
    constexpr int WH = TH + 2 * RY, WW = TW + 2 * RX;
    constexpr int WV = WW / SV, NV = WH * WV, SIT = (NV + NT - 1) / NT;
    constexpr unsigned ES = 4;
    static_assert(RY > PH && RX > PW, "window must cover the tap base grid");
    static_assert(SV == 1 || (RX % 4 == 0 && WW % 4 == 0), "vector staging alignment");
    __shared__ __attribute__((aligned(16))) float win[WH * WW];
    __shared__ __attribute__((aligned(16))) float cwin[WH * WW];  // conf', invariant
    __shared__ float red[NT / 64];

    const int H = a.H, W = a.W;
    const long long HW = (long long)H * W;
    int tile = xcd_remap(blockIdx.x, gridDim.x);
    const int tx = tile % a.tiles_x;
    tile /= a.tiles_x;
    const int ty = tile % a.tiles_y;
    const int b = tile / a.tiles_y;
    const int x0 = tx * TW, y0 = ty * TH;
    const int wy0 = y0 - RY, wx0 = x0 - RX;
    const bool has_conf = a.conf != nullptr;
    const bool preserve = (a.flags & kPreserve) != 0;
    const bool clip = (a.flags & kAlwaysClip) != 0;
    const int ly = threadIdx.x / TW, lx = threadIdx.x % TW;
    const int y = y0 + ly, x = x0 + lx;
    const bool active = (y < H) && (x < W);
    const unsigned vpix = (active ? (unsigned)(y * W + x) : 0u) * ES, plane_bytes = (unsigned)HW * ES;
    const float Hf = (float)H, Wf = (float)W;

    const rsrc_t ra = make_rsrc(a.aff + b * (K + 1) * HW);
    const rsrc_t ro = make_rsrc(a.off + b * a.off_bs);
    float av[K], dh[K], dw[K], cG[K], cO[2 * K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
        av[k] = bld(ra, vpix, (unsigned)(k < REF ? k : k + 1) * plane_bytes);
        dh[k] = bld(ro, vpix, (2u * k) * plane_bytes);
        dw[k] = bld(ro, vpix, (2u * k + 1) * plane_bytes);
        cG[k] = 0.f;
        cO[2 * k] = cO[2 * k + 1] = 0.f;
    }
    const rsrc_t rgo = make_rsrc(a.g_off + b * a.goff_bs);
    const rsrc_t rgr = make_rsrc(a.grad_aff_raw + b * a.gaff_bs);
    const bool cw = has_conf;  // (conf_prop off: f = p, nothing to keep)
    if (cw) {  // conf' over the window (zero outside the image), once
        const rsrc_t rc = make_rsrc(a.conf_eff + b * HW);
#pragma unroll
        for (int it = 0; it < SIT; ++it) {
            const int i = threadIdx.x + it * NT;
            const int ii = i < NV ? i : NV - 1;
            const int r = ii / WV, c = (ii - r * WV) * SV;
            int gy = wy0 + r, gx = wx0 + c;
            const bool in = i < NV && gy >= 0 && gy < H && gx >= 0 && gx < W;
            gy = gy < 0 ? 0 : (gy > H - 1 ? H - 1 : gy);
            gx = gx < 0 ? 0 : (gx > W - SV ? W - SV : gx);
            float v[SV];
            BVec<float, SV>::load(rc, (unsigned)(gy * W + gx) * ES, 0u, v);
            if (i < NV) {
#pragma unroll
                for (int e = 0; e < SV; ++e) cwin[r * WW + c + e] = in ? v[e] : 0.f;
            }
        }
        // (each thread reads back only the cells it wrote: the staging below maps cells alike)
    }

    const auto taps = [&](auto first_c, rsrc_t rp, rsrc_t rc, rsrc_t rd, float go) {
        constexpr bool FIRST = decltype(first_c)::value;
        // the taps' geometry is t-invariant: opaque moves keep the compiler from hoisting
        // every tap's weights and addresses out of the t loop (187 VGPRs, 2 waves per SIMD)
#pragma unroll
        for (int k = 0; k < K; ++k) asm volatile("" : "+v"(dh[k]), "+v"(dw[k]));
        if (active) {
            const float fown = win[(ly + RY) * WW + lx + RX];
#pragma unroll
            for (int k = 0; k < K; ++k) {
                const int tt = k < REF ? k : k + 1;
                const int i = tt / KW, jj = tt % KW;
                const float hs = (float)(y - PH + i) + dh[k];
                const float ws = (float)(x - PW + jj) + dw[k];
                float val = 0.f;
                if (hs > -1.f && ws > -1.f && hs < Hf && ws < Wf) {
                    int hl, wl;
                    float v[4];
                    tap_corners<FIRST, WH, WW>(hs, ws, wy0, wx0, H, W, win, rp, rc, rd, has_conf, preserve, clip, hl, wl, v);
                    const float lh = hs - (float)hl, lw = ws - (float)wl, hh = 1.f - lh, hw = 1.f - lw;
                    const float w1 = hh * hw, w2 = hh * lw, w3 = lh * hw, w4 = lh * lw;
                    val = (w1 * v[0] + w2 * v[1] + w3 * v[2] + w4 * v[3]);
                    float cwh = 0.f, cww = 0.f;
                    cwh += -1 * hw * v[0];
                    cwh += -1 * lw * v[1];
                    cwh += hw * v[2];
                    cwh += lw * v[3];
                    cww += -1 * hh * v[0];
                    cww += hh * v[1];
                    cww += -1 * lh * v[2];
                    cww += lh * v[3];
                    cO[2 * k] += cwh * go * av[k];
                    cO[2 * k + 1] += cww * go * av[k];
                }
                cG[k] += go * (val - fown);
            }
        }
    };
    const auto iter = [&](auto first_c, int t) {
        constexpr bool FIRST = decltype(first_c)::value;
        const float *pbase = FIRST ? a.pred_init + b * HW : a.pred_inter + (size_t)(t - 2) * a.N + b * HW;
        const rsrc_t rp = make_rsrc(pbase);
        const rsrc_t rc = make_rsrc(has_conf ? (FIRST ? a.conf : a.conf_eff) + b * HW : pbase);
        const rsrc_t rd = make_rsrc(preserve ? a.dep + b * HW : pbase);
        // stage f_{t-1} (bwd_step_kernel's staging)
        float sp[SIT][SV], sc[SIT][SV], sd[FIRST ? SIT : 1][SV];
        bool sin[SIT];
#pragma unroll
        for (int it = 0; it < SIT; ++it) {
            const int i = threadIdx.x + it * NT;
            const int ii = i < NV ? i : NV - 1;
            const int r = ii / WV, c = (ii - r * WV) * SV;
            int gy = wy0 + r, gx = wx0 + c;
            sin[it] = i < NV && gy >= 0 && gy < H && gx >= 0 && gx < W;
            gy = gy < 0 ? 0 : (gy > H - 1 ? H - 1 : gy);
            gx = gx < 0 ? 0 : (gx > W - SV ? W - SV : gx);
            const unsigned q = (unsigned)(gy * W + gx) * ES;
            BVec<float, SV>::load(rp, q, 0u, sp[it]);
            if (has_conf && (FIRST || !cw)) BVec<float, SV>::load(rc, q, 0u, sc[it]);
            if (FIRST && preserve) BVec<float, SV>::load(rd, q, 0u, sd[FIRST ? it : 0]);
        }
        // this iteration's dL/dout at the own pixel (plane t-1 of the dL/dout store)
        const int j = t - 1;
        const float go = active ? (j < 2 * K ? bld(rgo, vpix, (unsigned)j * plane_bytes)
                                             : bld(rgr, vpix, (unsigned)(j - 2 * K) * plane_bytes))
                                : 0.f;
#pragma unroll
        for (int it = 0; it < SIT; ++it) {
            const int i = threadIdx.x + it * NT;
            if (i < NV) {
                float v[SV];
                const int r = i / WV, c = (i - r * WV) * SV;
#pragma unroll
                for (int e = 0; e < SV; ++e) {
                    // (cw: conf' from the LDS window, the same product p * conf')
                    const float cc = has_conf ? (!FIRST && cw ? cwin[r * WW + c + e] : sc[it][e]) : 1.f;
                    const float f = make_f<FIRST>(sp[it][e], cc, FIRST && preserve ? sd[FIRST ? it : 0][e] : 0.f,
                                                  has_conf, preserve, clip);
                    v[e] = sin[it] ? f : 0.f;
                }
                if constexpr (SV == 4)
                    *reinterpret_cast<float4 *>(&win[r * WW + c]) = make_float4(v[0], v[1], v[2], v[3]);
                else
                    win[r * WW + c] = v[0];
            }
        }
        lds_barrier();
        taps(first_c, rp, rc, rd, go);
        __syncthreads();  // the window is restaged by the next iteration
    };
#pragma unroll 1
    for (int t = a.T; t >= 2; --t) iter(std::false_type{}, t);
    iter(std::true_type{}, 1);

    float gsum = 0.f;
    if (active) {
#pragma unroll
        for (int k = 0; k < 2 * K; ++k) bst(rgo, vpix, (unsigned)k * plane_bytes, cO[k]);
        const rsrc_t rar = make_rsrc(a.aff_raw + b * a.aff_raw_bs);
        float ar[K], ga[K];
#pragma unroll
        for (int k = 0; k < K; ++k) ar[k] = bld(rar, vpix, (unsigned)k * plane_bytes);
        gsum = aff_norm_backward<K>(cG, ar, *a.gamma, a.kind, ga);
#pragma unroll
        for (int k = 0; k < K; ++k) bst(rgr, vpix, (unsigned)k * plane_bytes, ga[k]);
    }
    if (a.gamma_part) {
        for (int o = 32; o > 0; o >>= 1) gsum += __shfl_down(gsum, o, 64);
        if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = gsum;
        lds_barrier();
        if (threadIdx.x == 0) {
            float s = 0.f;
#pragma unroll
            for (int i = 0; i < NT / 64; ++i) s += red[i];
            a.gamma_part[blockIdx.x] = s;
        }
    }
}

// Finishing pass (after step 1 has scattered dL/df_0 completely):
//   f_0 = p_0 * conf', p_0 = clamp(blend(pred_init)) (nlspnmodel.py:341-348, :351),
//   conf' = (1-m) conf + m (:333-334) -> grad_pred_init, grad_conf;
// workgroup 0 also sums step 1's per-workgroup dL/dgamma partials in a fixed order.
__global__ void __launch_bounds__(256) bwd_final_kernel(
    const float *pred_init, const float *dep, const float *conf, const float *conf_eff, const float *gf0,
    const float *g_conf_acc, float *grad_pred_init, float *grad_conf, long long N, unsigned flags,
    const float *gamma_part, int n_part, float *grad_gamma) {
    const bool preserve = (flags & kPreserve) != 0, clip = (flags & kAlwaysClip) != 0;
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < N; i += (long long)gridDim.x * blockDim.x) {
        const float d = preserve ? dep[i] : 0.f;
        const float m = d > 0.f ? 1.f : 0.f;
        float pre = pred_init[i];
        if (preserve) pre = (1.0f - m) * pre + m * d;
        const float p0 = clip ? clamp0(pre) : pre;
        const float gfi = gf0[i];
        float g = conf ? gfi * conf_eff[i] : gfi;
        if (clip && !(pre >= 0.f)) g = 0.f;
        grad_pred_init[i] = preserve ? (1.0f - m) * g : g;
        if (conf) {
            const float gc = g_conf_acc[i] + gfi * p0;
            grad_conf[i] = preserve ? (1.0f - m) * gc : gc;
        }
    }
    if (grad_gamma && blockIdx.x == 0) {
        __shared__ float red[4];
        float s = 0.f;
        for (int i = threadIdx.x; i < n_part; i += 256) s += gamma_part[i];
        for (int o = 32; o > 0; o >>= 1) s += __shfl_down(s, o, 64);
        if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
        __syncthreads();
        if (threadIdx.x == 0) *grad_gamma = red[0] + red[1] + red[2] + red[3];
    }
}

// Step-level backward, after bwd_step_kernel has scattered dL/df (f = feat * conf) for
// one prop_step (nlspnmodel.py:350-361): grad_feat = dL/df * conf, grad_conf =
// dL/df * feat, and tap K/2 of the (K+1)-plane affinity gradient = 0 (the kernels
// recompute that tap as 1 - sum of the others, so it does not enter the output).
__global__ void __launch_bounds__(256) bwd_step_io_kernel(const float *feat, const float *conf, const float *gf,
                                                           float *grad_feat, float *grad_conf, float *grad_aff,
                                                           long long HW, int B, int K) {
    const long long N = (long long)B * HW;
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < N; i += (long long)gridDim.x * blockDim.x) {
        const float g = gf[i];
        grad_feat[i] = conf ? g * conf[i] : g;
        if (conf) grad_conf[i] = g * feat[i];
        const long long b = i / HW, q = i - b * HW;
        grad_aff[(b * (K + 1) + K / 2) * HW + q] = 0.f;
    }
}

// Backward of nlspn_affinity_normalize (_affinity_normalization + _aff_insert,
// nlspnmodel.py:179-201, :261-269) for a (K+1)-plane gradient of its output:
// G_k = g[k] - g[K/2], then aff_norm_backward; one dL/dgamma partial per workgroup.
template <int K>
__global__ void __launch_bounds__(256) affnorm_bwd_kernel(const float *aff_raw, long long aff_bs, const float *gamma_p,
                                                          const float *grad_aff, float *grad_aff_raw,
                                                          float *gamma_part, long long HW, int B, int kind) {
    constexpr int REF = K / 2;
    const float gamma = *gamma_p;
    const long long N = (long long)B * HW;
    float gsum = 0.f;
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < N; i += (long long)gridDim.x * blockDim.x) {
        const long long b = i / HW, q = i - b * HW;
        const float *gin = grad_aff + b * (K + 1) * HW + q;
        const float gref = gin[REF * HW];
        float G[K], ar[K], ga[K];
#pragma unroll
        for (int k = 0; k < K; ++k) {
            G[k] = gin[(k < REF ? k : k + 1) * HW] - gref;
            ar[k] = aff_raw[b * aff_bs + k * HW + q];
        }
        gsum += aff_norm_backward<K>(G, ar, gamma, kind, ga);
#pragma unroll
        for (int k = 0; k < K; ++k) grad_aff_raw[(b * K + k) * HW + q] = ga[k];
    }
    if (gamma_part) {
        __shared__ float red[4];
        for (int o = 32; o > 0; o >>= 1) gsum += __shfl_down(gsum, o, 64);
        if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = gsum;
        __syncthreads();
        if (threadIdx.x == 0) gamma_part[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
    }
}

// Fixed-order sum of n partials into *out (one workgroup).
__global__ void __launch_bounds__(256) sum_partials_kernel(const float *part, int n, float *out) {
    __shared__ float red[4];
    float s = 0.f;
    for (int i = threadIdx.x; i < n; i += 256) s += part[i];
    for (int o = 32; o > 0; o >>= 1) s += __shfl_down(s, o, 64);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) *out = red[0] + red[1] + red[2] + red[3];
}

}  // namespace nlspn
