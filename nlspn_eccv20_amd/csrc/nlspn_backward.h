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
// launch (bwd_final_kernel):
//   * the iteration's output pixel owns its dL/d(affinity) and dL/d(offset)
//     accumulators (plain read-modify-write across the T launches, no atomics);
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
    float *g_aff;           // (K+1) planes per item, accumulated
    float *g_off;           // 2K planes per item (raw layout), accumulated
    float *g_conf;          // dL/dconf' plane, accumulated (null iff conf null)
    long long off_bs;
    int B, H, W, tiles_x, tiles_y;
    int last;               // t == T
    unsigned flags;
};

template <int KH, int KW, int TH, int TW, int RY, int RX, int SV, bool OFFSET, bool FIRST>
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
    __shared__ __attribute__((aligned(16))) float win[NC];   // f_{t-1} over the window
    __shared__ float gwin[NC];                              // scatter accumulator for dL/df_{t-1}

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
    const float *pbase = a.p_in + b * HW;
    const rsrc_t rp = make_rsrc(pbase);
    const rsrc_t rc = make_rsrc(has_conf ? a.conf + b * HW : pbase);
    const rsrc_t rd = make_rsrc(preserve ? a.dep + b * HW : pbase);

    const int ly = threadIdx.x / TW, lx = threadIdx.x % TW;
    const int y = y0 + ly, x = x0 + lx;
    const bool active = (y < H) && (x < W);
    const unsigned pix = active ? (unsigned)(y * W + x) : 0u;
    const unsigned vpix = pix * ES, plane_bytes = (unsigned)HW * ES;

    // ---- staging loads of the window (as in the forward), then own-pixel loads
    float sp[SIT][SV], sc[SIT][SV], sd[FIRST ? SIT : 1][SV];
    bool sin[SIT];
#pragma unroll
    for (int it = 0; it < SIT; ++it) {
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
    float av[K][1], dh[K][1], dw[K][1];
    const rsrc_t ra = make_rsrc(a.aff + b * (K + 1) * HW);
    const rsrc_t ro = make_rsrc(OFFSET ? a.off + b * a.off_bs : a.aff);
#pragma unroll
    for (int k = 0; k < K; ++k) {
        BVec<float, 1>::load(ra, vpix, (unsigned)(k < REF ? k : k + 1) * plane_bytes, av[k]);
        if (OFFSET) {
            BVec<float, 1>::load(ro, vpix, (2u * k) * plane_bytes, dh[k]);
            BVec<float, 1>::load(ro, vpix, (2u * k + 1) * plane_bytes, dw[k]);
        }
    }
    float dv[1] = {0.f}, gfr[1], pt[1] = {0.f}, ce[1] = {1.f}, gi[1] = {0.f}, gpr[1] = {0.f};
    if (preserve) BVec<float, 1>::load(rd, vpix, 0u, dv);
    BVec<float, 1>::load(make_rsrc(a.gf_read + b * HW), vpix, 0u, gfr);
    if (has_conf) {
        BVec<float, 1>::load(make_rsrc(a.p_out + b * HW), vpix, 0u, pt);
        BVec<float, 1>::load(make_rsrc(a.conf_eff + b * HW), vpix, 0u, ce);
    } else if (a.last && a.g_pred && !clip) {
        BVec<float, 1>::load(make_rsrc(a.p_out + b * HW), vpix, 0u, pt);
    }
    if (a.g_inter) BVec<float, 1>::load(make_rsrc(a.g_inter + b * HW), vpix, 0u, gi);
    if (a.last && a.g_pred) BVec<float, 1>::load(make_rsrc(a.g_pred + b * HW), vpix, 0u, gpr);

    // ---- stage f_{t-1}, zero the scatter window
#pragma unroll
    for (int it = 0; it < SIT; ++it) {
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
        if (i < NC) gwin[i] = 0.f;
    }
    lds_barrier();

    if (active) {
        // ---- dL/dp_t from the next step's scatter (f_t = p_t * conf') and the direct grads
        float g = has_conf ? gfr[0] * ce[0] : gfr[0];
        if (a.g_inter) g += gi[0];
        if (a.last && a.g_pred) g += clip ? gpr[0] : (pt[0] >= 0.f ? gpr[0] : 0.f);  // pred = clamp(p_T, 0)
        if (has_conf) {
            const rsrc_t rgc = make_rsrc(a.g_conf + b * HW);
            float gc[1];
            BVec<float, 1>::load(rgc, vpix, 0u, gc);
            gc[0] += gfr[0] * pt[0];
            BVec<float, 1>::store(rgc, vpix, 0u, gc);
        }
        const float zero[1] = {0.f};
        BVec<float, 1>::store(make_rsrc(a.gf_read + b * HW), vpix, 0u, zero);  // consumed: ready for reuse

        // ---- forward recompute of the taps (values, corners) for the clamp mask and grads
        const float Hf = (float)H, Wf = (float)W;
        float val[K], asum = 0.f;
        bool valid[K];
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const int t = k < REF ? k : k + 1;
            const int i = t / KW, j = t % KW;
            asum += av[k][0];
            float hs, ws;
            if (OFFSET) {
                hs = (float)(y - PH + i) + dh[k][0];
                ws = (float)(x - PW + j) + dw[k][0];
            } else {
                int yy = y + i - 1, xx = x + j - 1;
                yy = yy < 0 ? 0 : (yy > H - 1 ? H - 1 : yy);
                xx = xx < 0 ? 0 : (xx > W - 1 ? W - 1 : xx);
                hs = (float)yy;
                ws = (float)xx;
            }
            valid[k] = hs > -1.f && ws > -1.f && hs < Hf && ws < Wf;
            float v = 0.f;
            if (valid[k]) {
                const int hl = (int)floorf(hs), wl = (int)floorf(ws);
                const float lh = hs - (float)hl, lw = ws - (float)wl, hh = 1.f - lh, hw = 1.f - lw;
                float v1, v2, v3, v4;
                const int ry = hl - wy0, rx = wl - wx0;
                if ((unsigned)ry < (unsigned)(WH - 1) && (unsigned)rx < (unsigned)(WW - 1)) {
                    const float *s = &win[ry * WW + rx];
                    v1 = s[0]; v2 = s[1]; v3 = s[WW]; v4 = s[WW + 1];
                } else {
                    const int r0 = hl * W, r1 = (hl + 1) * W;
                    v1 = (hl >= 0 && wl >= 0) ? fetch_f<float, FIRST>(rp, rc, rd, has_conf, preserve, clip, (r0 + wl) * ES) : 0.f;
                    v2 = (hl >= 0 && wl + 1 <= W - 1) ? fetch_f<float, FIRST>(rp, rc, rd, has_conf, preserve, clip, (r0 + wl + 1) * ES) : 0.f;
                    v3 = (hl + 1 <= H - 1 && wl >= 0) ? fetch_f<float, FIRST>(rp, rc, rd, has_conf, preserve, clip, (r1 + wl) * ES) : 0.f;
                    v4 = (hl + 1 <= H - 1 && wl + 1 <= W - 1) ? fetch_f<float, FIRST>(rp, rc, rd, has_conf, preserve, clip, (r1 + wl + 1) * ES) : 0.f;
                }
                const float w1 = hh * hw, w2 = hh * lw, w3 = lh * hw, w4 = lh * lw;
                v = (w1 * v1 + w2 * v2 + w3 * v3 + w4 * v4);
                // coordinate weights, mdmcn_get_coordinate_weight (.cuh:84-125); corners
                // outside the image are zero in the window / fetch, as the checks there
                if (OFFSET) {
                    float cwh = 0.f, cww = 0.f;
                    cwh += -1 * hw * v1;
                    cwh += -1 * lw * v2;
                    cwh += hw * v3;
                    cwh += lw * v4;
                    cww += -1 * hh * v1;
                    cww += hh * v2;
                    cww += -1 * lh * v3;
                    cww += lh * v4;
                    dh[k][0] = cwh;  // reuse the offset registers for the coordinate weights
                    dw[k][0] = cww;
                }
            }
            val[k] = v;
        }
        const float fown = win[(ly + RY) * WW + lx + RX];
        const float aref = 1.0f - asum;
        if (clip) {
            float acc = 0.f;
#pragma unroll
            for (int t = 0; t < KK; ++t) acc += t == REF ? fown * aref : val[t < REF ? t : t - 1] * av[t < REF ? t : t - 1][0];
            float pre = acc;
            if (preserve) {
                const float m = dv[0] > 0.f ? 1.f : 0.f;
                pre = (1.0f - m) * acc + m * dv[0];
            }
            if (!(pre >= 0.f)) g = 0.f;  // clamp(min=0) passes the gradient where x >= 0
        }
        const float go = preserve ? (1.0f - (dv[0] > 0.f ? 1.f : 0.f)) * g : g;

        // ---- per-pixel accumulators: dL/d(aff) (K+1 planes), dL/d(offset) (2K planes)
        const rsrc_t rga = make_rsrc(a.g_aff + b * (K + 1) * HW);
        const rsrc_t rgo = make_rsrc(OFFSET ? a.g_off + b * 2 * K * HW : a.g_aff);
#pragma unroll
        for (int c = 0; c < K + 1; ++c) {
            float ga[1];
            BVec<float, 1>::load(rga, vpix, (unsigned)c * plane_bytes, ga);
            ga[0] += go * (c == REF ? fown : val[c < REF ? c : c - 1]);
            BVec<float, 1>::store(rga, vpix, (unsigned)c * plane_bytes, ga);
        }
        if (OFFSET) {
#pragma unroll
            for (int k = 0; k < K; ++k) {
                if (!valid[k]) continue;
                float g2[1], g3[1];
                BVec<float, 1>::load(rgo, vpix, (2u * k) * plane_bytes, g2);
                BVec<float, 1>::load(rgo, vpix, (2u * k + 1) * plane_bytes, g3);
                g2[0] += dh[k][0] * go * av[k][0];
                g3[0] += dw[k][0] * go * av[k][0];
                BVec<float, 1>::store(rgo, vpix, (2u * k) * plane_bytes, g2);
                BVec<float, 1>::store(rgo, vpix, (2u * k + 1) * plane_bytes, g3);
            }
        }

        // ---- scatter dL/df_{t-1} (col2im): LDS window, global atomics outside it
        float *gfw = a.gf_write + b * HW;
        atomicAdd(&gwin[(ly + RY) * WW + lx + RX], go * aref);  // reference tap, weight (1,0,0,0)
#pragma unroll
        for (int k = 0; k < K; ++k) {
            if (!valid[k]) continue;
            const int t = k < REF ? k : k + 1;
            const int i = t / KW, j = t % KW;
            float hs, ws;
            if (OFFSET) {
                // recompute the sample point from the raw offsets (dh/dw now hold coordinate weights)
                float o1[1], o2[1];
                BVec<float, 1>::load(ro, vpix, (2u * k) * plane_bytes, o1);
                BVec<float, 1>::load(ro, vpix, (2u * k + 1) * plane_bytes, o2);
                hs = (float)(y - PH + i) + o1[0];
                ws = (float)(x - PW + j) + o2[0];
            } else {
                int yy = y + i - 1, xx = x + j - 1;
                yy = yy < 0 ? 0 : (yy > H - 1 ? H - 1 : yy);
                xx = xx < 0 ? 0 : (xx > W - 1 ? W - 1 : xx);
                hs = (float)yy;
                ws = (float)xx;
            }
            const float top = go * av[k][0];
            const int hl = (int)floorf(hs), wl = (int)floorf(ws);
            const float lh = hs - (float)hl, lw = ws - (float)wl, hh = 1.f - lh, hw = 1.f - lw;
            const float wts[4] = {hh * hw, hh * lw, lh * hw, lh * lw};
            const int ry = hl - wy0, rx = wl - wx0;
            const bool inwin = (unsigned)ry < (unsigned)(WH - 1) && (unsigned)rx < (unsigned)(WW - 1);
#pragma unroll
            for (int cnr = 0; cnr < 4; ++cnr) {
                const int hy = hl + (cnr >> 1), wx = wl + (cnr & 1);
                if (hy < 0 || hy > H - 1 || wx < 0 || wx > W - 1) continue;
                const float v = wts[cnr] * top;
                if (inwin) atomicAdd(&gwin[(ry + (cnr >> 1)) * WW + rx + (cnr & 1)], v);
                else atomicAdd(&gfw[hy * W + wx], v);
            }
        }
    }
    lds_barrier();
    // ---- flush the scatter window (in-image, non-zero cells) with global atomics
    float *gfw = a.gf_write + b * HW;
#pragma unroll
    for (int it = 0; it < CIT; ++it) {
        const int i = threadIdx.x + it * NT;
        if (i < NC) {
            const int r = i / WW, c = i - r * WW;
            const int gy = wy0 + r, gx = wx0 + c;
            const float v = gwin[i];
            if (v != 0.f && gy >= 0 && gy < H && gx >= 0 && gx < W) atomicAdd(&gfw[gy * W + gx], v);
        }
    }
}

// Finishing pass: p_0 / conf' / affinity-normalisation backward.
//   f_0 = p_0 * conf', p_0 = clamp(blend(pred_init)) (nlspnmodel.py:341-348, :351)
//   conf' = (1-m) conf + m (:333-334)
//   aff_ref = 1 - sum(aff) (_aff_insert :262-263); _affinity_normalization (:179-201):
//   u = tanh(a)/(gamma+1e-8) [TGASS] | tanh(a)/gamma [TC] | a [AS/ASS];
//   s = sum|u| + 1e-4, s = 1 where s < 1 [ASS/TGASS; no gradient there]; aff = u / s [not TC].
template <int K>
__global__ void __launch_bounds__(256) bwd_final_kernel(
    const float *pred_init, const float *dep, const float *conf, const float *conf_eff, const float *aff_raw,
    long long aff_bs, const float *gamma_p, const float *gf0, const float *g_aff, const float *g_conf_acc,
    float *grad_pred_init, float *grad_conf, float *grad_aff_raw, float *grad_gamma, long long HW, int B, int kind,
    unsigned flags) {
    constexpr int REF = K / 2;
    const bool preserve = (flags & kPreserve) != 0, clip = (flags & kAlwaysClip) != 0;
    const float gamma = *gamma_p;
    const long long N = (long long)B * HW;
    float gsum = 0.f;
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < N; i += (long long)gridDim.x * blockDim.x) {
        const long long b = i / HW, q = i - b * HW;
        const float d = preserve ? dep[i] : 0.f;
        const float m = d > 0.f ? 1.f : 0.f;
        float pre = pred_init[i];
        if (preserve) pre = (1.0f - m) * pre + m * d;
        const float p0 = clip ? clamp0(pre) : pre;
        float g = conf ? gf0[i] * conf_eff[i] : gf0[i];
        if (clip && !(pre >= 0.f)) g = 0.f;
        grad_pred_init[i] = preserve ? (1.0f - m) * g : g;
        if (conf) {
            const float gc = g_conf_acc[i] + gf0[i] * p0;
            grad_conf[i] = preserve ? (1.0f - m) * gc : gc;
        }
        // aff: G_k = g_aff[k] - g_aff[ref]; normalisation backward
        const float gref = g_aff[(b * (K + 1) + REF) * HW + q];
        float u[K], th[K], G[K], s = 0.f, dot = 0.f;
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const float av = aff_raw[b * aff_bs + k * HW + q];
            th[k] = tanhf(av);
            u[k] = kind == kAffTC ? th[k] / gamma : (kind == kAffTGASS ? th[k] / (gamma + 1e-8f) : av);
            s += fabsf(u[k]);
            G[k] = g_aff[(b * (K + 1) + (k < REF ? k : k + 1)) * HW + q] - gref;
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
            float ga = gu;
            if (kind == kAffTC) {
                ga = gu * (1.f - th[k] * th[k]) / gamma;
            } else if (kind == kAffTGASS) {
                const float dd = gamma + 1e-8f;
                ga = gu * (1.f - th[k] * th[k]) / dd;
                gsum += -gu * th[k] / (dd * dd);
            }
            grad_aff_raw[(b * K + k) * HW + q] = ga;
        }
    }
    if (grad_gamma && kind == kAffTGASS) {
        // wave reduction, then one atomic per wave
        for (int off = 32; off > 0; off >>= 1) gsum += __shfl_down(gsum, off, 64);
        if ((threadIdx.x & 63) == 0) atomicAdd(grad_gamma, gsum);
    }
}

}  // namespace nlspn
