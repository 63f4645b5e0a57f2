// Generic modulated DCNv2 forward (seam 2: the reference's `DCN` module entry
// DCN.modulated_deform_conv_forward, src/model/deformconv/src/vision.cpp:9).
//
// The reference runs im2col into a (C*kh*kw, B*Ho*Wo) `columns` buffer
// (cuda/modulated_deform_im2col_cuda.cuh:127-194) and then one addmm per group
// (cuda/modulated_deform_conv_cuda.cu:90-116).  Here each thread owns one output
// element and gathers its (C/group)*kh*kw bilinear samples directly: no columns
// buffer, no GEMM (NLSPN's use has C = Cout = 1, where the "GEMM" is a 9-term
// sum).  Sum order = the im2col row order (channel-major, then tap), then + bias,
// as addmm(bias, columns^T, weight^T) defines it.
#pragma once

#include "nlspn_common.h"

namespace nlspn {

struct MdcnArgs {
    const void *input, *weight, *bias, *offset, *mask;
    void *output;
    int B, C, H, W, Cout, kh, kw, sh, sw, ph, pw, dh, dw, group, dg, Ho, Wo;
};

template <typename T>
__device__ __forceinline__ float mdcn_bilinear(const T *im, int H, int W, float h, float w) {
    // modulated_deform_im2col_cuda.cuh:24-54
    const int h_low = (int)floorf(h), w_low = (int)floorf(w);
    const int h_high = h_low + 1, w_high = w_low + 1;
    const float lh = h - (float)h_low, lw = w - (float)w_low;
    const float hh = 1.f - lh, hw = 1.f - lw;
    float v1 = 0.f, v2 = 0.f, v3 = 0.f, v4 = 0.f;
    if (h_low >= 0 && w_low >= 0) v1 = ld(im + (long long)h_low * W + w_low);
    if (h_low >= 0 && w_high <= W - 1) v2 = ld(im + (long long)h_low * W + w_high);
    if (h_high <= H - 1 && w_low >= 0) v3 = ld(im + (long long)h_high * W + w_low);
    if (h_high <= H - 1 && w_high <= W - 1) v4 = ld(im + (long long)h_high * W + w_high);
    const float w1 = hh * hw, w2 = hh * lw, w3 = lh * hw, w4 = lh * lw;
    return (w1 * v1 + w2 * v2 + w3 * v3 + w4 * v4);
}

template <typename T>
__global__ void __launch_bounds__(256) mdcn_forward_kernel(MdcnArgs a) {
    const long long HoWo = (long long)a.Ho * a.Wo, HW = (long long)a.H * a.W;
    const long long total = (long long)a.B * a.Cout * HoWo;
    const int KK = a.kh * a.kw;
    const int cpg = a.C / a.group, opg = a.Cout / a.group, cpdg = a.C / a.dg;
    const T *in = static_cast<const T *>(a.input);
    const T *wt = static_cast<const T *>(a.weight);
    const T *off = static_cast<const T *>(a.offset);
    const T *msk = static_cast<const T *>(a.mask);
    for (long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
         idx += (long long)gridDim.x * blockDim.x) {
        const long long q = idx % HoWo;
        const int wo = (int)(q % a.Wo), ho = (int)(q / a.Wo);
        const int co = (int)((idx / HoWo) % a.Cout);
        const int b = (int)(idx / HoWo / a.Cout);
        const int g = co / opg;
        const int h_in = ho * a.sh - a.ph, w_in = wo * a.sw - a.pw;
        float acc = 0.f;
        for (int cl = 0; cl < cpg; ++cl) {
            const int ci = g * cpg + cl;
            const int dgi = ci / cpdg;
            const T *im = in + ((long long)b * a.C + ci) * HW;
            const T *ob = off + ((long long)b * a.dg + dgi) * 2 * KK * HoWo + q;
            const T *mb = msk + ((long long)b * a.dg + dgi) * KK * HoWo + q;
            const T *wr = wt + ((long long)co * cpg + cl) * KK;
            for (int i = 0; i < a.kh; ++i)
                for (int j = 0; j < a.kw; ++j) {
                    const int t = i * a.kw + j;
                    const float oh = ld(ob + (long long)(2 * t) * HoWo);
                    const float ow = ld(ob + (long long)(2 * t + 1) * HoWo);
                    const float m = ld(mb + (long long)t * HoWo);
                    const float h_im = (float)(h_in + i * a.dh) + oh;
                    const float w_im = (float)(w_in + j * a.dw) + ow;
                    float val = 0.f;
                    if (h_im > -1.f && w_im > -1.f && h_im < (float)a.H && w_im < (float)a.W)
                        val = mdcn_bilinear(im, a.H, a.W, h_im, w_im);
                    const float col = val * m;  // .cuh:189
                    acc += col * ld(wr + t);     // .cu:112 addmm row x weight
                }
        }
        if (a.bias) acc = acc + ld(static_cast<const T *>(a.bias) + co);
        st(static_cast<T *>(a.output) + idx, acc);
    }
}

// ------------------------------------------------------------------ backward
// DCN.modulated_deform_conv_backward (vision.cpp:10; modulated_deform_conv_cuda.cu:
// 124-280).  The reference materialises columns = weight_g^T . grad_output_g (an
// at::mm per group), then runs col2im_coord (.cuh:256-328: grad_offset, grad_mask),
// col2im (.cuh:196-254: grad_input, float atomics) and im2col again for
// grad_weight (+ addmv for grad_bias).  Here:
//   mdcn_bwd_data_kernel: one thread per (b, deformable group, tap, output pixel);
//     for each channel of the group it forms that column entry directly
//     (sum over the group's output channels), accumulates grad_offset / grad_mask
//     in the reference's channel order, and scatters grad_input with float
//     atomics — col2im's candidate loop and its pad_w := pad_h call (.cuh:371)
//     reproduced, so the result is the reference's, quirk included;
//   mdcn_bwd_weight_kernel: one workgroup per weight element (co, cl, t), a
//     deterministic tree reduction over (b, pixel) of grad_output * im2col value;
//     workgroups past the weight count reduce grad_bias.
struct MdcnBwdArgs {
    const float *input, *weight, *offset, *mask, *grad_out;
    float *grad_in, *grad_off, *grad_mask, *grad_w, *grad_b;
    int B, C, H, W, Cout, kh, kw, sh, sw, ph, pw, dh, dw, group, dg, Ho, Wo;
};

// mdmcn_get_gradient_weight (.cuh:57-81)
__device__ __forceinline__ float mdcn_grad_weight(float ah, float aw, int h, int w, int H, int W) {
    if (ah <= -1.f || ah >= (float)H || aw <= -1.f || aw >= (float)W) return 0.f;
    const int hl = (int)floorf(ah), wl = (int)floorf(aw), hh = hl + 1, wh = wl + 1;
    float weight = 0.f;
    if (h == hl && w == wl) weight = ((float)(h + 1) - ah) * ((float)(w + 1) - aw);
    if (h == hl && w == wh) weight = ((float)(h + 1) - ah) * (aw + 1.f - (float)w);
    if (h == hh && w == wl) weight = (ah + 1.f - (float)h) * ((float)(w + 1) - aw);
    if (h == hh && w == wh) weight = (ah + 1.f - (float)h) * (aw + 1.f - (float)w);
    return weight;
}

// mdmcn_get_coordinate_weight (.cuh:84-125)
__device__ __forceinline__ float mdcn_coord_weight(float h, float w, int H, int W, const float *im, int dir) {
    if (h <= -1.f || h >= (float)H || w <= -1.f || w >= (float)W) return 0.f;
    const int hl = (int)floorf(h), wl = (int)floorf(w), hh = hl + 1, wh = wl + 1;
    float weight = 0.f;
    if (dir == 0) {
        if (hl >= 0 && wl >= 0) weight += -1.f * ((float)(wl + 1) - w) * im[(long long)hl * W + wl];
        if (hl >= 0 && wh <= W - 1) weight += -1.f * (w - (float)wl) * im[(long long)hl * W + wh];
        if (hh <= H - 1 && wl >= 0) weight += ((float)(wl + 1) - w) * im[(long long)hh * W + wl];
        if (hh <= H - 1 && wh <= W - 1) weight += (w - (float)wl) * im[(long long)hh * W + wh];
    } else {
        if (hl >= 0 && wl >= 0) weight += -1.f * ((float)(hl + 1) - h) * im[(long long)hl * W + wl];
        if (hl >= 0 && wh <= W - 1) weight += ((float)(hl + 1) - h) * im[(long long)hl * W + wh];
        if (hh <= H - 1 && wl >= 0) weight += -1.f * (h - (float)hl) * im[(long long)hh * W + wl];
        if (hh <= H - 1 && wh <= W - 1) weight += (h - (float)hl) * im[(long long)hh * W + wh];
    }
    return weight;
}

__global__ void __launch_bounds__(256) mdcn_bwd_data_kernel(MdcnBwdArgs a) {
    const long long P = (long long)a.Ho * a.Wo, HW = (long long)a.H * a.W;
    const int KK = a.kh * a.kw, cpg = a.C / a.group, opg = a.Cout / a.group, cpdg = a.C / a.dg;
    const long long total = (long long)a.B * a.dg * KK * P;
    for (long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
         idx += (long long)gridDim.x * blockDim.x) {
        const long long p = idx % P;
        const int t = (int)((idx / P) % KK);
        const int dgi = (int)((idx / P / KK) % a.dg);
        const int b = (int)(idx / P / KK / a.dg);
        const int ho = (int)(p / a.Wo), wo = (int)(p % a.Wo), i = t / a.kw, j = t % a.kw;
        const long long ob = ((long long)(b * a.dg + dgi) * 2 * KK) * P + p;
        const float oh = a.offset[ob + (long long)(2 * t) * P], ow = a.offset[ob + (long long)(2 * t + 1) * P];
        const float m = a.mask[((long long)(b * a.dg + dgi) * KK + t) * P + p];
        const float ih0 = (float)(ho * a.sh - a.ph + i * a.dh) + oh;
        const float iw0 = (float)(wo * a.sw - a.pw + j * a.dw) + ow;
        const float iwq = (float)(wo * a.sw - a.ph + j * a.dw) + ow;  // col2im's w with pad_h (.cuh:371)
        const bool valid = !(ih0 <= -1.f || iw0 <= -1.f || ih0 >= (float)a.H || iw0 >= (float)a.W);
        const float ih = valid ? ih0 : -2.f, iw = valid ? iw0 : -2.f;
        float vh = 0.f, vw = 0.f, mval = 0.f;
        for (int cnt = 0; cnt < cpdg; ++cnt) {
            const int c = dgi * cpdg + cnt, g = c / cpg, cl = c % cpg;
            float cv = 0.f;  // columns[c*KK + t][b, p] (.cu:213-220)
            for (int ol = 0; ol < opg; ++ol) {
                const int co = g * opg + ol;
                cv += a.weight[((long long)co * cpg + cl) * KK + t] * a.grad_out[((long long)b * a.Cout + co) * P + p];
            }
            const float *im = a.input + ((long long)b * a.C + c) * HW;
            if (valid) mval += cv * mdcn_bilinear(im, a.H, a.W, ih, iw);  // .cuh:306-309
            vh += mdcn_coord_weight(ih, iw, a.H, a.W, im, 0) * cv * m;   // .cuh:313-315
            vw += mdcn_coord_weight(ih, iw, a.H, a.W, im, 1) * cv * m;
            // col2im (.cuh:226-252): candidates around the truncated point
            const float top = cv * m;
            const int ch = (int)ih0, cw = (int)iwq;
            float *gi = a.grad_in + ((long long)b * a.C + c) * HW;
            for (int dy = -2; dy <= 2; ++dy)
                for (int dx = -2; dx <= 2; ++dx) {
                    const int y = ch + dy, x = cw + dx;
                    if (y >= 0 && y < a.H && x >= 0 && x < a.W && fabsf(ih0 - (float)y) < 1.f &&
                        fabsf(iwq - (float)x) < 1.f) {
                        const float weight = mdcn_grad_weight(ih0, iwq, y, x, a.H, a.W);
                        atomicAdd(gi + (long long)y * a.W + x, weight * top);
                    }
                }
        }
        a.grad_off[ob + (long long)(2 * t) * P] = vh;
        a.grad_off[ob + (long long)(2 * t + 1) * P] = vw;
        a.grad_mask[((long long)(b * a.dg + dgi) * KK + t) * P + p] = mval;
    }
}

__global__ void __launch_bounds__(256) mdcn_bwd_weight_kernel(MdcnBwdArgs a) {
    __shared__ float red[256];
    const long long P = (long long)a.Ho * a.Wo;
    const int KK = a.kh * a.kw, cpg = a.C / a.group, opg = a.Cout / a.group, cpdg = a.C / a.dg;
    const long long nw = (long long)a.Cout * cpg * KK;
    const long long e = blockIdx.x;
    const long long n = (long long)a.B * P;
    float s = 0.f;
    if (e < nw) {  // grad_weight[co, cl, t] = sum_{b,p} grad_out * im2col value (.cu:262-270)
        const int t = (int)(e % KK), cl = (int)((e / KK) % cpg), co = (int)(e / KK / cpg);
        const int c = (co / opg) * cpg + cl, dgi = c / cpdg, i = t / a.kw, j = t % a.kw;
        for (long long q = threadIdx.x; q < n; q += blockDim.x) {
            const int b = (int)(q / P);
            const long long p = q % P;
            const int ho = (int)(p / a.Wo), wo = (int)(p % a.Wo);
            const long long ob = ((long long)(b * a.dg + dgi) * 2 * KK) * P + p;
            const float h_im = (float)(ho * a.sh - a.ph + i * a.dh) + a.offset[ob + (long long)(2 * t) * P];
            const float w_im = (float)(wo * a.sw - a.pw + j * a.dw) + a.offset[ob + (long long)(2 * t + 1) * P];
            float val = 0.f;
            if (h_im > -1.f && w_im > -1.f && h_im < (float)a.H && w_im < (float)a.W)
                val = mdcn_bilinear(a.input + ((long long)b * a.C + c) * a.H * a.W, a.H, a.W, h_im, w_im);
            const float col = val * a.mask[((long long)(b * a.dg + dgi) * KK + t) * P + p];
            s += a.grad_out[((long long)b * a.Cout + co) * P + p] * col;
        }
    } else {  // grad_bias[co] = sum_{b,p} grad_out (.cu:271)
        const int co = (int)(e - nw);
        for (long long q = threadIdx.x; q < n; q += blockDim.x)
            s += a.grad_out[((long long)(q / P) * a.Cout + co) * P + q % P];
    }
    red[threadIdx.x] = s;
    __syncthreads();
    for (int w = blockDim.x / 2; w > 0; w >>= 1) {
        if ((int)threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        if (e < nw) a.grad_w[e] = red[0];
        else a.grad_b[e - nw] = red[0];
    }
}

}  // namespace nlspn
