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
//
// Arithmetic type A: float for float / half storage, double for double (the
// reference dispatches float and double, AT_DISPATCH_FLOATING_TYPES at .cu:93 and
// .cu:221; double is what gradcheck runs in).
#pragma once

#include "nlspn_common.h"

namespace nlspn {

struct MdcnArgs {
    const void *input, *weight, *bias, *offset, *mask;
    void *output;
    int B, C, H, W, Cout, kh, kw, sh, sw, ph, pw, dh, dw, group, dg, Ho, Wo;
};

// storage T -> arithmetic A, and back
template <typename A, typename T> __device__ __forceinline__ A ldc(const T *p) { return (A)p[0]; }
template <> __device__ __forceinline__ float ldc<float, __half>(const __half *p) { return __half2float(*p); }
template <typename T, typename A> __device__ __forceinline__ void stc(T *p, A v) { *p = (T)v; }
template <> __device__ __forceinline__ void stc<__half, float>(__half *p, float v) { *p = __float2half(v); }

template <typename A, typename T>
__device__ __forceinline__ A mdcn_bilinear(const T *im, int H, int W, A h, A w) {
    // modulated_deform_im2col_cuda.cuh:24-54
    const int h_low = (int)floor(h), w_low = (int)floor(w);
    const int h_high = h_low + 1, w_high = w_low + 1;
    const A lh = h - (A)h_low, lw = w - (A)w_low;
    const A hh = (A)1 - lh, hw = (A)1 - lw;
    A v1 = 0, v2 = 0, v3 = 0, v4 = 0;
    if (h_low >= 0 && w_low >= 0) v1 = ldc<A>(im + (long long)h_low * W + w_low);
    if (h_low >= 0 && w_high <= W - 1) v2 = ldc<A>(im + (long long)h_low * W + w_high);
    if (h_high <= H - 1 && w_low >= 0) v3 = ldc<A>(im + (long long)h_high * W + w_low);
    if (h_high <= H - 1 && w_high <= W - 1) v4 = ldc<A>(im + (long long)h_high * W + w_high);
    const A w1 = hh * hw, w2 = hh * lw, w3 = lh * hw, w4 = lh * lw;
    return (w1 * v1 + w2 * v2 + w3 * v3 + w4 * v4);
}

template <typename T, typename A>
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
        A acc = 0;
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
                    const A oh = ldc<A>(ob + (long long)(2 * t) * HoWo);
                    const A ow = ldc<A>(ob + (long long)(2 * t + 1) * HoWo);
                    const A m = ldc<A>(mb + (long long)t * HoWo);
                    const A h_im = (A)(h_in + i * a.dh) + oh;
                    const A w_im = (A)(w_in + j * a.dw) + ow;
                    A val = 0;
                    if (h_im > (A)-1 && w_im > (A)-1 && h_im < (A)a.H && w_im < (A)a.W)
                        val = mdcn_bilinear<A>(im, a.H, a.W, h_im, w_im);
                    const A col = val * m;      // .cuh:189
                    acc += col * ldc<A>(wr + t);  // .cu:112 addmm row x weight
                }
        }
        if (a.bias) acc = acc + ldc<A>(static_cast<const T *>(a.bias) + co);
        stc(static_cast<T *>(a.output) + idx, acc);
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
template <typename A>
struct MdcnBwdArgs {
    const A *input, *weight, *offset, *mask, *grad_out;
    A *grad_in, *grad_off, *grad_mask, *grad_w, *grad_b;
    int B, C, H, W, Cout, kh, kw, sh, sw, ph, pw, dh, dw, group, dg, Ho, Wo;
};

// mdmcn_get_gradient_weight (.cuh:57-81)
template <typename A>
__device__ __forceinline__ A mdcn_grad_weight(A ah, A aw, int h, int w, int H, int W) {
    if (ah <= (A)-1 || ah >= (A)H || aw <= (A)-1 || aw >= (A)W) return 0;
    const int hl = (int)floor(ah), wl = (int)floor(aw), hh = hl + 1, wh = wl + 1;
    A weight = 0;
    if (h == hl && w == wl) weight = ((A)(h + 1) - ah) * ((A)(w + 1) - aw);
    if (h == hl && w == wh) weight = ((A)(h + 1) - ah) * (aw + (A)1 - (A)w);
    if (h == hh && w == wl) weight = (ah + (A)1 - (A)h) * ((A)(w + 1) - aw);
    if (h == hh && w == wh) weight = (ah + (A)1 - (A)h) * (aw + (A)1 - (A)w);
    return weight;
}

// mdmcn_get_coordinate_weight (.cuh:84-125)
template <typename A>
__device__ __forceinline__ A mdcn_coord_weight(A h, A w, int H, int W, const A *im, int dir) {
    if (h <= (A)-1 || h >= (A)H || w <= (A)-1 || w >= (A)W) return 0;
    const int hl = (int)floor(h), wl = (int)floor(w), hh = hl + 1, wh = wl + 1;
    A weight = 0;
    if (dir == 0) {
        if (hl >= 0 && wl >= 0) weight += (A)-1 * ((A)(wl + 1) - w) * im[(long long)hl * W + wl];
        if (hl >= 0 && wh <= W - 1) weight += (A)-1 * (w - (A)wl) * im[(long long)hl * W + wh];
        if (hh <= H - 1 && wl >= 0) weight += ((A)(wl + 1) - w) * im[(long long)hh * W + wl];
        if (hh <= H - 1 && wh <= W - 1) weight += (w - (A)wl) * im[(long long)hh * W + wh];
    } else {
        if (hl >= 0 && wl >= 0) weight += (A)-1 * ((A)(hl + 1) - h) * im[(long long)hl * W + wl];
        if (hl >= 0 && wh <= W - 1) weight += ((A)(hl + 1) - h) * im[(long long)hl * W + wh];
        if (hh <= H - 1 && wl >= 0) weight += (A)-1 * (h - (A)hl) * im[(long long)hh * W + wl];
        if (hh <= H - 1 && wh <= W - 1) weight += (h - (A)hl) * im[(long long)hh * W + wh];
    }
    return weight;
}

template <typename A>
__global__ void __launch_bounds__(256) mdcn_bwd_data_kernel(MdcnBwdArgs<A> a) {
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
        const A oh = a.offset[ob + (long long)(2 * t) * P], ow = a.offset[ob + (long long)(2 * t + 1) * P];
        const A m = a.mask[((long long)(b * a.dg + dgi) * KK + t) * P + p];
        const A ih0 = (A)(ho * a.sh - a.ph + i * a.dh) + oh;
        const A iw0 = (A)(wo * a.sw - a.pw + j * a.dw) + ow;
        const A iwq = (A)(wo * a.sw - a.ph + j * a.dw) + ow;  // col2im's w with pad_h (.cuh:371)
        const bool valid = !(ih0 <= (A)-1 || iw0 <= (A)-1 || ih0 >= (A)a.H || iw0 >= (A)a.W);
        const A ih = valid ? ih0 : (A)-2, iw = valid ? iw0 : (A)-2;
        A vh = 0, vw = 0, mval = 0;
        for (int cnt = 0; cnt < cpdg; ++cnt) {
            const int c = dgi * cpdg + cnt, g = c / cpg, cl = c % cpg;
            A cv = 0;  // columns[c*KK + t][b, p] (.cu:213-220)
            for (int ol = 0; ol < opg; ++ol) {
                const int co = g * opg + ol;
                cv += a.weight[((long long)co * cpg + cl) * KK + t] * a.grad_out[((long long)b * a.Cout + co) * P + p];
            }
            const A *im = a.input + ((long long)b * a.C + c) * HW;
            if (valid) mval += cv * mdcn_bilinear<A>(im, a.H, a.W, ih, iw);  // .cuh:306-309
            vh += mdcn_coord_weight(ih, iw, a.H, a.W, im, 0) * cv * m;   // .cuh:313-315
            vw += mdcn_coord_weight(ih, iw, a.H, a.W, im, 1) * cv * m;
            // col2im (.cuh:226-252): candidates around the truncated point
            const A top = cv * m;
            const int ch = (int)ih0, cw = (int)iwq;
            A *gi = a.grad_in + ((long long)b * a.C + c) * HW;
            for (int dy = -2; dy <= 2; ++dy)
                for (int dx = -2; dx <= 2; ++dx) {
                    const int y = ch + dy, x = cw + dx;
                    if (y >= 0 && y < a.H && x >= 0 && x < a.W && fabs(ih0 - (A)y) < (A)1 &&
                        fabs(iwq - (A)x) < (A)1) {
                        const A weight = mdcn_grad_weight<A>(ih0, iwq, y, x, a.H, a.W);
                        atomicAdd(gi + (long long)y * a.W + x, weight * top);
                    }
                }
        }
        a.grad_off[ob + (long long)(2 * t) * P] = vh;
        a.grad_off[ob + (long long)(2 * t + 1) * P] = vw;
        a.grad_mask[((long long)(b * a.dg + dgi) * KK + t) * P + p] = mval;
    }
}

template <typename A>
__global__ void __launch_bounds__(256) mdcn_bwd_weight_kernel(MdcnBwdArgs<A> a) {
    __shared__ A red[256];
    const long long P = (long long)a.Ho * a.Wo;
    const int KK = a.kh * a.kw, cpg = a.C / a.group, opg = a.Cout / a.group, cpdg = a.C / a.dg;
    const long long nw = (long long)a.Cout * cpg * KK;
    const long long e = blockIdx.x;
    const long long n = (long long)a.B * P;
    A s = 0;
    if (e < nw) {  // grad_weight[co, cl, t] = sum_{b,p} grad_out * im2col value (.cu:262-270)
        const int t = (int)(e % KK), cl = (int)((e / KK) % cpg), co = (int)(e / KK / cpg);
        const int c = (co / opg) * cpg + cl, dgi = c / cpdg, i = t / a.kw, j = t % a.kw;
        for (long long q = threadIdx.x; q < n; q += blockDim.x) {
            const int b = (int)(q / P);
            const long long p = q % P;
            const int ho = (int)(p / a.Wo), wo = (int)(p % a.Wo);
            const long long ob = ((long long)(b * a.dg + dgi) * 2 * KK) * P + p;
            const A h_im = (A)(ho * a.sh - a.ph + i * a.dh) + a.offset[ob + (long long)(2 * t) * P];
            const A w_im = (A)(wo * a.sw - a.pw + j * a.dw) + a.offset[ob + (long long)(2 * t + 1) * P];
            A val = 0;
            if (h_im > (A)-1 && w_im > (A)-1 && h_im < (A)a.H && w_im < (A)a.W)
                val = mdcn_bilinear<A>(a.input + ((long long)b * a.C + c) * a.H * a.W, a.H, a.W, h_im, w_im);
            const A col = val * a.mask[((long long)(b * a.dg + dgi) * KK + t) * P + p];
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
