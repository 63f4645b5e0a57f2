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

}  // namespace nlspn
