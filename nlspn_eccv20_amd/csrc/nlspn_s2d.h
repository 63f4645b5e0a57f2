// S2D sparse-depth encoder front (src/model/nlspnmodel.py:406-462), fused: the
// min/max-pool pyramid over the sparse depth and the two 1x1 conv + ReLU layers
// (pool_convs) in one pass, written straight into the 17-channel input of the
// 3x3 conv that follows (channels 0..15 = pool_convs output, 16 = dep: the
// reference's torch.cat([dep_feat, dep], 1), :459).
//
// Per pixel, over the (2r+1)^2 window of radius r (stride 1, the implicit -inf
// padding of nn.MaxPool2d(s, 1, s // 2): out-of-image cells never win):
//   min pools r = 1..4 (:441-447): -maxpool(where(dep == 0, -999, -dep)), then 999
//                                  -> 0; i.e. the min over in-image cells of
//                                  (dep != 0 ? dep : 999), 999 mapped to 0;
//   max pools r = 5, 6 (:449-452): the max over in-image cells of dep.
// The 1x1 convs sum their input channels in index order from the bias; MIOpen's
// order is not specified, so parity with the torch module is to a tolerance.
//
// Work decomposition: a 16 x 64 tile per 256-thread workgroup; thread t takes column
// t % 64 of rows t / 64 + 4e (e = 0..3), so every store instruction writes 64
// consecutive pixels of a plane; the tile's dep window (halo 6) staged once in LDS.  HBM: 4 B read +
// 68 B written per pixel (72 B/px, byte-bound); the pool window re-reads hit LDS.
#pragma once

#include "nlspn_common.h"

namespace nlspn {

struct S2DArgs {
    const float *dep;   // B x H x W
    const float *w1;    // 8 x 6   (pool_convs[0] conv weight, (8, 6, 1, 1))
    const float *b1;    // 8
    const float *w2;    // 16 x 8  (pool_convs[1] conv weight, (16, 8, 1, 1))
    const float *b2;    // 16
    float *out;         // B x 17 x H x W
    float *pyr;         // B x 6 x H x W (the pool pyramid, for the weight gradients), or null
    int B, H, W;
    int tiles_x, tiles_y;
};

constexpr int kS2DTH = 16, kS2DTW = 64, kS2DR = 6;

__global__ void __launch_bounds__(256) s2d_pyramid_kernel(S2DArgs a) {
    constexpr int TH = kS2DTH, TW = kS2DTW, R = kS2DR, WH = TH + 2 * R, WW = TW + 2 * R;
    constexpr float NEG = -3.402823466e38f;  // "no cell": loses every max
    __shared__ float win[WH * WW];
    __shared__ float wts[8 * 6 + 8 + 16 * 8 + 16];
    const int H = a.H, W = a.W;
    int tile = blockIdx.x;
    const int tx = tile % a.tiles_x;
    tile /= a.tiles_x;
    const int ty = tile % a.tiles_y;
    const int b = tile / a.tiles_y;
    const int x0 = tx * TW, y0 = ty * TH;
    const long long HW = (long long)H * W;
    const float *dep = a.dep + b * HW;

    for (int i = threadIdx.x; i < 8 * 6 + 8 + 16 * 8 + 16; i += 256) {
        float v;
        if (i < 48) v = a.w1[i];
        else if (i < 56) v = a.b1[i - 48];
        else if (i < 184) v = a.w2[i - 56];
        else v = a.b2[i - 184];
        wts[i] = v;
    }
    for (int i = threadIdx.x; i < WH * WW; i += 256) {  // out-of-image cells: 0, never read
        const int r = i / WW, c = i % WW, gy = y0 - R + r, gx = x0 - R + c;
        win[i] = (gy >= 0 && gy < H && gx >= 0 && gx < W) ? dep[(long long)gy * W + gx] : 0.0f;
    }
    __syncthreads();

    const int lx = threadIdx.x % TW, x = x0 + lx;
    if (x >= W) return;  // no barrier below
    const float *w1 = wts, *b1 = wts + 48, *w2 = wts + 56, *b2 = wts + 184;
#pragma unroll 1
    for (int e = 0; e < TH / 4; ++e) {
        const int ly = threadIdx.x / TW + 4 * e, y = y0 + ly;
        if (y >= H) break;
        // ring by ring: the running min (masked) for r <= 4, the running max for r <= 6
        float mn = 999.0f, mx = NEG, pyr[6];
#pragma unroll
        for (int r = 0; r <= R; ++r) {
            for (int dy = -r; dy <= r; ++dy) {
                if (y + dy < 0 || y + dy >= H) continue;  // the pools' -inf padding
                const int step = (dy == -r || dy == r) ? 1 : 2 * r;  // full edge rows, else the two side cells
                for (int dx = -r; dx <= r; dx += step) {
                    if (x + dx < 0 || x + dx >= W) continue;
                    const float v = win[(ly + R + dy) * WW + lx + R + dx];
                    if (r <= 4) mn = fminf(mn, v != 0.0f ? v : 999.0f);
                    mx = fmaxf(mx, v);
                }
            }
            if (r >= 1 && r <= 4) pyr[r - 1] = mn == 999.0f ? 0.0f : mn;
            if (r >= 5) pyr[r - 1] = mx;
        }
        // pool_convs (:455): two 1x1 conv + bias + ReLU, input channels in index order
        float h1[8];
#pragma unroll
        for (int o = 0; o < 8; ++o) {
            float s = b1[o];
#pragma unroll
            for (int c = 0; c < 6; ++c) s += w1[o * 6 + c] * pyr[c];
            h1[o] = fmaxf(s, 0.0f);
        }
        const long long px = (long long)y * W + x;
        float *out = a.out + (long long)b * 17 * HW + px;
#pragma unroll
        for (int o = 0; o < 16; ++o) {
            float s = b2[o];
#pragma unroll
            for (int c = 0; c < 8; ++c) s += w2[o * 8 + c] * h1[c];
            out[o * HW] = fmaxf(s, 0.0f);
        }
        out[16 * HW] = win[(ly + R) * WW + lx + R];  // :459 torch.cat([dep_feat, dep], 1)
        if (a.pyr) {
            float *pp = a.pyr + (long long)b * 6 * HW + px;
#pragma unroll
            for (int c = 0; c < 6; ++c) pp[c * HW] = pyr[c];
        }
    }
}

}  // namespace nlspn
