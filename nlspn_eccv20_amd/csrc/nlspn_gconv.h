// GRU-mode convolutions (the reference's forced default, src/config.py:225-228):
// every convolution of one GRU-mode iteration (nlspnmodel.py:365-373) —
//   dep_feat = encode_dep(new_pred / max_depth)   3x3 stride-2 convs + bias + ReLU   (:134-138)
//   aff_feat = encode_aff(aff)  (first update)    3x3 stride-2 convs + bias, ReLU / Tanh (:127-132)
//   aff_feat = GRU(h=aff_feat, x=dep_feat)        ConvGRU, three 3x3 convs         (:386-403)
//   aff      = decode_aff(aff_feat)               3x3 stride-2 transposed convs    (:140-143)
//                                                 + the _clip_as crop (:237-250)
// as implicit GEMMs on the f32-input matrix cores (v_mfma_f32_16x16x4_f32: f32 operands,
// exact f32 products, f32 accumulation; only the summation order differs from a
// sequential f32 convolution), NCHW in and out, with bias and activation in the epilogue —
// no torch.cat, no layout conversions, no separate bias / ReLU / sigmoid / tanh kernels.
//
// The ConvGRU as two launches (the candidate needs r at the neighbouring pixels):
//   GRU1: output channels 0..127 z = sigmoid(convz(cat(h, x))), 128..255 r = sigmoid(convr(..))
//         stored as r*h, 256..383 qx = convq's x half + bias (its K runs over x only);
//   GRU2: q = tanh(convq's r*h half + qx); h' = (1 - z) h + z q.
//
// GEMM: D[co][px] = sum_k W[co][k] X[k][px], k = (input channel, tap).  A workgroup of 4
// waves (WGM x WGN) owns 16*WM*WGM output channels x 16*WN*WGN pixels; a wave owns WM x WN
// 16x16 blocks (lane l: A[co = l & 15][k = l >> 4], B[k = l >> 4][px = l & 15], so a k-step
// is 4 input channels at one tap).  Pixels: the output grid (a transposed conv: one output
// phase's grid, = the input grid) is cut into column bands of width bw, and a band into flat
// row-major runs of NPX pixels — no tile columns wasted on a 38-pixel-wide 1/8-scale image.
// Per chunk of CC input channels the workgroup stages the packed weights [ci][tap][co] and
// the input window (the rows / columns its pixels' taps reach, zero outside the image = the
// zero padding) in LDS by LDS-DMA loads (no staging registers, no LDS store instructions);
// the next chunk's loads land in the other LDS stage while the current chunk computes.  The LDS window pitch XP is a compile-time constant, so every
// operand read is one ds_read_b32 with an immediate offset from a per-lane base.
#pragma once

#include "nlspn_common.h"

namespace nlspn {

constexpr int kGcNT = 256;  // threads per workgroup (4 waves)
constexpr int kGcCP = 16;   // packed input channels: a multiple of this (every chunk size CC divides it)
enum { kGcS1 = 0, kGcS2 = 1, kGcT2 = 2 };         // 3x3 pad 1 stride 1 / stride 2; transposed stride 2 (pad 1, output pad 1)
enum { kGcEpiAct = 0, kGcEpiGru1 = 1, kGcEpiGru2 = 2, kGcEpiAff = 3 };
enum { kGcActNone = 0, kGcActRelu = 1, kGcActTanh = 2 };

struct GconvArgs {
    const float *x0, *x1;  // inputs (B, c0, Hi, Wi) and (B, c1, Hi, Wi): channels [0, c0) and [c0, c0 + c1)
    const float *w;        // packed weights [phase][co_tile][cin_pad][ntap][WGco] (phase: transposed only)
    const float *bias;     // [co_tiles * WGco] (zero past cout)
    float *y;              // kGcEpiAct: (B, cout, ohs, ows)
    // ConvGRU (kGcEpiGru*): h the hidden state (B, hc, Ho, Wo); z, r*h and qx of GRU1
    const float *h;
    float *zb, *rhb, *qxb;
    float *hout;           // GRU2: h'
    int c0, c1, cin_pad;   // cin_pad = roundup(c0 + c1, kGcCP)
    int B, Hi, Wi, Ho, Wo;
    int ohs, ows;          // stored rows / columns of y (the crop: rows >= ohs / columns >= ows are not stored)
    int cout, co_tiles;
    int gh, gw;            // the pixel grid tiled (convolutions: Ho x Wo; transposed: Hi x Wi per phase)
    int bw, nbands, tpb;   // band width, bands, tiles per band (of the widest band)
    int npx;               // pixels per tile (<= NPX: a narrow band's tile must fit the window rows)
    int act;               // kGcAct*
    float in_div;          // inputs divided by it (encode_dep: max_depth, :366): the VALU kernel only, 1 for the MFMA kernels
    int hc;                // GRU hidden channels
    // kGcEpiAff (decode_aff's last layer, K = 8 raw taps): y is the normalised affinity with the
    // reference tap inserted, (B, K + 1, ohs, ows), of kind aff_kind (kAff*) with *gamma
    const float *gamma;
    int aff_kind;
};

typedef float f32x4v __attribute__((ext_vector_type(4)));

// taps of a transposed stride-2 pad-1 3x3 conv landing on output phase (py, px): kernel row ky
// reaches output row oy = 2 iy - 1 + ky, so oy = 2 qy + py takes ky = 1 (py = 0, iy = qy) or
// ky = 0 / 2 (py = 1, iy = qy + 1 / qy)
__host__ __device__ constexpr int gc_ntap(int mode, int phase) {
    return mode != kGcT2 ? 9 : ((phase >> 1) ? 2 : 1) * ((phase & 1) ? 2 : 1);
}
// the tap's kernel row / column (ky, kx) and its window offset (dy, dx) for tap index t
template <int MODE, int PH>
__device__ __forceinline__ constexpr void gc_tap(int t, int &ky, int &kx, int &dy, int &dx) {
    if constexpr (MODE != kGcT2) {
        ky = t / 3; kx = t % 3; dy = ky; dx = kx;
    } else {
        constexpr int py = PH >> 1, px = PH & 1, nx = px ? 2 : 1;
        const int ty = t / nx, tx = t % nx;
        ky = py ? 2 * ty : 1;   // py = 1: ky 0 then 2
        kx = px ? 2 * tx : 1;
        dy = (py + 1 - ky) / 2;  // window row offset (iy - qy)
        dx = (px + 1 - kx) / 2;
    }
}

// LDS channel strides.  The four lane groups (k rows) of an operand read sit one channel
// stride apart; a ds_read_b32 serves lanes 0-31 and 32-63 in turn over 32 banks, so groups 0 / 1
// (and 2 / 3) must not share banks: a weight row or a stride-1 window row (16 consecutive
// words) needs a stride = 16 (mod 32), a stride-2 window row (16 even words) an odd stride.
__host__ __device__ constexpr int gc_wcs(int ntap, int wgco) { return ntap * wgco + (16 - (ntap * wgco) % 32 + 32) % 32; }
__host__ __device__ constexpr int gc_xcs(int mode, int xr, int xp) {
    return mode == kGcS2 ? xr * xp + 1 - (xr * xp) % 2 : xr * xp + (16 - (xr * xp) % 32 + 32) % 32;
}
__host__ __device__ constexpr int gc_round(int v, int m) { return (v + m - 1) / m * m; }

template <int MODE, int WM, int WN, int WGM, int WGN, int XR, int XP, int CC, int EPI>
struct GcCfg {
    static constexpr int WGCO = 16 * WM * WGM, NPX = 16 * WN * WGN;
    static constexpr int NTMAX = MODE == kGcT2 ? 4 : 9;
    static constexpr int XCS = gc_xcs(MODE, XR, XP);
    // One LDS stage = a chunk's weights [CC][WCS] then its input window [CC][XCS], each region
    // rounded up to whole LDS-DMA rounds of the workgroup (256 lanes x 16 B weights, x 4 B
    // window: every lane's write lands inside the stage).
    static constexpr int WST = gc_round(CC * gc_wcs(NTMAX, WGCO), 4 * kGcNT);
    static constexpr int XST = gc_round(CC * XCS, kGcNT);
    static constexpr int STAGE = WST + XST;
    static constexpr int LDS_FLOATS = 2 * STAGE;  // two stages: chunk k computes while k + 1 lands
    static constexpr int WREG = WST / (4 * kGcNT), XREG = XST / kGcNT;  // LDS-DMA loads per lane per chunk
};

template <int MODE, int WM, int WN, int WGM, int WGN, int XR, int XP, int CC, int EPI, int PH>
__device__ __forceinline__ void gconv_body(const GconvArgs &a, float *lds, int wgi) {
    using Cfg = GcCfg<MODE, WM, WN, WGM, WGN, XR, XP, CC, EPI>;
    constexpr int WGCO = Cfg::WGCO, NPX = Cfg::NPX, XCS = Cfg::XCS;
    constexpr int NTAP = gc_ntap(MODE, PH);
    constexpr int WCS = gc_wcs(NTAP, WGCO);  // (this phase's taps only)
    constexpr int S = MODE == kGcS2 ? 2 : 1;
    // stage s: weights at lds + s STAGE, window after them
    float *Ws = lds;
    float *Xs = lds + Cfg::WST;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int wm = wv % WGM, wn = wv / WGM;
    const int l16 = lane & 15, lg = lane >> 4;

    // workgroup -> (co tile, image, band, tile); the phase is PH
    const int cot = wgi % a.co_tiles;
    int rest = wgi / a.co_tiles;
    const int tile = rest % a.tpb;
    rest /= a.tpb;
    const int band = rest % a.nbands;
    const int b = rest / a.nbands;
    const int bx0 = band * a.bw, bwi = min(a.bw, a.gw - bx0);
    const int npx = a.npx;
    const int f0 = tile * npx;
    if (f0 >= a.gh * bwi) return;  // (the narrower last band has fewer tiles)
    const int ra = f0 / bwi, rb = min(a.gh - 1, (f0 + npx - 1) / bwi);
    // the window: input rows iy0 .. iy0 + nrows - 1, columns ix0 .. ix0 + ncols - 1
    const int iy0 = MODE == kGcT2 ? ra : S * ra - 1;
    const int ix0 = MODE == kGcT2 ? bx0 : S * bx0 - 1;
    const int nrows = MODE == kGcT2 ? rb - ra + 2 : S * (rb - ra) + 3;
    const int ncols = MODE == kGcT2 ? bwi + 1 : S * (bwi - 1) + 3;

    // per n-block: this lane's pixel (grid row gy, column gx) and its window base
    int gyv[WN], gxv[WN], xb[WN];
#pragma unroll
    for (int n = 0; n < WN; ++n) {
        const int jj = 16 * (wn * WN + n) + l16;
        const int f = f0 + min(jj, npx - 1);
        const int gy = f / bwi, gx = bx0 + (f - gy * bwi);
        gyv[n] = jj < npx ? gy : a.gh;  // (past the tile: not stored)
        gxv[n] = gx;
        // (a pixel past the grid reads a clamped in-window cell; its result is not stored)
        const int ry = min(gy, rb) - ra;
        xb[n] = lg * XCS + (S * ry) * XP + S * (gx - bx0);
    }
    const int wb = lg * WCS + wm * (16 * WM) + l16;

    // the K range: GRU1's qx tile (co 2hc .. 3hc - 1) runs over x's channels only
    int cs = 0;
    if constexpr (EPI == kGcEpiGru1) cs = (cot * WGCO >= 2 * a.hc) ? a.c0 : 0;
    // (chunks up to the last input channel: the packing pads the channels to kGcCP, a chunk of
    // CC < kGcCP channels past the last one is skipped, not read)
    const int ce = min(a.cin_pad, (a.c0 + a.c1 + CC - 1) / CC * CC);
    const long long HWi = (long long)a.Hi * a.Wi;
    // (transposed: the phases' taps are packed one after another, 1 + 2 + 2 + 4 = 9)
    constexpr int TAP0 = MODE == kGcT2 ? (PH == 0 ? 0 : PH == 1 ? 1 : PH == 2 ? 3 : 5) : 0;
    const float *wsrc = a.w + (long long)a.cin_pad * WGCO * ((long long)TAP0 * a.co_tiles + (long long)cot * NTAP);

    // Staging: LDS-DMA (buffer / global loads that write LDS directly, no registers).  Lane l
    // of wave w's i-th load writes stage word (i * 256 + 64 w + l) (x 4 words for the weights),
    // so the source of every LDS position is computed once: a window word's byte offset within
    // a chunk's channels (0x80000000 for a pad word or a cell outside the window or the image:
    // the buffer load returns 0 = the zero padding; a chunk is one buffer descriptor whose size
    // ends at the source's last channel, so the chunk's padding channels read 0 too), a weight
    // quad's float offset within the chunk's contiguous weights (pad quads reload quad 0 into
    // the pad: never read).
    unsigned xoff[Cfg::XREG];
#pragma unroll
    for (int i = 0; i < Cfg::XREG; ++i) {
        const int p = tid + i * kGcNT;
        const int c = p / XCS, rem = p - c * XCS;
        const int row = rem / XP, col = rem - row * XP;
        const int iy = iy0 + row, ix = ix0 + col;
        const bool ok = c < CC && rem < XR * XP && row < nrows && col < ncols && (unsigned)iy < (unsigned)a.Hi &&
                        (unsigned)ix < (unsigned)a.Wi;
        xoff[i] = ok ? (unsigned)(((long long)c * HWi + (long long)iy * a.Wi + ix) * 4) : 0x80000000u;
    }
    int woff[Cfg::WREG];
#pragma unroll
    for (int i = 0; i < Cfg::WREG; ++i) {
        const int p = 4 * (tid + i * kGcNT);
        const int c = p / WCS, rem = p - c * WCS;
        woff[i] = c < CC && rem < NTAP * WGCO ? c * NTAP * WGCO + rem : 0;
    }
    typedef __attribute__((address_space(3))) void lds_t;
    auto issue_chunk = [&](int c0, const int stage) __attribute__((always_inline)) {
        const float *wc = wsrc + (long long)c0 * NTAP * WGCO;
        float *Wd = Ws + stage * Cfg::STAGE + 4 * 64 * wv, *Xd = Xs + stage * Cfg::STAGE + 64 * wv;
#pragma unroll
        for (int i = 0; i < Cfg::WREG; ++i)
            __builtin_amdgcn_global_load_lds(wc + woff[i], (lds_t *)(Wd + 4 * kGcNT * i), 16, 0, 0);
        // (a chunk past the last channel — possible only within the 16-channel packing pad, which
        // the loop bound below excludes — would read nothing: an empty descriptor on x0)
        const bool s0 = c0 < a.c0;
        const int nch = s0 ? a.c0 - c0 : a.c1 - (c0 - a.c0);
        const bool any = nch > 0 && (s0 || a.x1 != nullptr);
        const float *base = !any ? a.x0
                            : s0 ? a.x0 + ((long long)b * a.c0 + c0) * HWi
                                 : a.x1 + ((long long)b * a.c1 + (c0 - a.c0)) * HWi;
        const int nrec = any ? (int)(nch * HWi * 4) : 0;
        const rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc(const_cast<float *>(base), (short)0, nrec, 0x00020000);
#pragma unroll
        for (int i = 0; i < Cfg::XREG; ++i)
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rx, (lds_t *)(Xd + kGcNT * i), 4, xoff[i], 0, 0, 0);
    };

    f32x4v acc[WM][WN];
#pragma unroll
    for (int m = 0; m < WM; ++m)
#pragma unroll
        for (int n = 0; n < WN; ++n) acc[m][n] = f32x4v{0.f, 0.f, 0.f, 0.f};

    auto compute = [&](const int stage) __attribute__((always_inline)) {
        const float *Wc = Ws + stage * Cfg::STAGE, *Xc = Xs + stage * Cfg::STAGE;
        // the chunk's k-steps j = (4-channel group c4, tap t), software pipelined by hand: the
        // operands of step j + 1 are read while the MFMAs of step j issue (scheduling barriers
        // keep the compiler from sinking the reads next to their use and then waiting on an LDS
        // round trip before every MFMA group)
        constexpr int NS = (CC / 4) * NTAP;
        float av[2][WM], bv[2][WN];
        auto fetch = [&](const int j, const int slot) __attribute__((always_inline)) {
            const int c4 = j / NTAP, t = j % NTAP;
            int ky, kx, dy, dx;
            gc_tap<MODE, PH>(t, ky, kx, dy, dx);
            (void)ky; (void)kx;
#pragma unroll
            for (int m = 0; m < WM; ++m) av[slot][m] = Wc[wb + 4 * c4 * WCS + t * WGCO + 16 * m];
#pragma unroll
            for (int n = 0; n < WN; ++n) bv[slot][n] = Xc[xb[n] + 4 * c4 * XCS + dy * XP + dx];
        };
        fetch(0, 0);
#pragma unroll
        for (int j = 0; j < NS; ++j) {
            const int cur = j & 1;
            if (j + 1 < NS) fetch(j + 1, cur ^ 1);
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int m = 0; m < WM; ++m)
#pragma unroll
                for (int n = 0; n < WN; ++n)
                    acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[cur][m], bv[cur][n], acc[m][n], 0, 0, 0);
            __builtin_amdgcn_sched_barrier(0);
        }
    };
    issue_chunk(cs, 0);
    __syncthreads();  // (waits for the loads: vmcnt(0), then the barrier)
    // one barrier per chunk: chunk k + 1's loads go to the other stage — last read by chunk
    // k - 1, which every wave finished before the previous barrier — and land while chunk k
    // computes; the barrier after it waits for them.
    auto step = [&](const int c0, const int stage) __attribute__((always_inline)) {
        if (c0 + CC < ce) issue_chunk(c0 + CC, stage ^ 1);
        compute(stage);
        __syncthreads();
    };
    for (int c0 = cs; c0 < ce; c0 += 2 * CC) {  // (two chunks per trip: the stages are compile-time)
        step(c0, 0);
        if (c0 + CC < ce) step(c0 + CC, 1);
    }

    // epilogue: lane l, register r of block (m, n) holds output channel co = co0 + 16 m + 4 (l >> 4) + r
    // of this lane's pixel of block n.  Per n-block every global operand (bias; GRU: h, z, qx) is
    // loaded first, then combined and stored: one memory round trip per block, not per element.
    // Lanes past the grid or the crop use an in-range pixel and skip the store.
    const int co0 = cot * WGCO + wm * (16 * WM);
    const long long HWo = (long long)a.Ho * a.Wo;
    float bv[WM][4];
#pragma unroll
    for (int m = 0; m < WM; ++m)
#pragma unroll
        for (int r = 0; r < 4; ++r) bv[m][r] = a.bias[co0 + 16 * m + 4 * lg + r];  // (padded to the co tiles)
    const int hc = a.hc;
    const int gate = EPI == kGcEpiGru1 ? (cot * WGCO) / hc : 0;  // GRU1: 0 z, 1 r, 2 qx (uniform per tile)
#pragma unroll
    for (int n = 0; n < WN; ++n) {
        const int gy = gyv[n], gx = gxv[n];
        int oy = gy, ox = gx;
        if constexpr (MODE == kGcT2) {
            oy = 2 * gy + (PH >> 1);
            ox = 2 * gx + (PH & 1);
        }
        const bool ok = gy < a.gh && oy < a.ohs && ox < a.ows;
        const long long pix = ok ? (long long)oy * a.Wo + ox : 0;
        if constexpr (EPI == kGcEpiAct) {
            const long long pixs = ok ? (long long)oy * a.ows + ox : 0;
            const long long HWs = (long long)a.ohs * a.ows;
#pragma unroll
            for (int m = 0; m < WM; ++m)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int co = co0 + 16 * m + 4 * lg + r;
                    float u = acc[m][n][r] + bv[m][r];
                    if (a.act == kGcActRelu) u = u < 0.f ? 0.f : u;  // (NaN kept, as torch's ReLU)
                    else if (a.act == kGcActTanh) u = tanhf(u);
                    if (ok && co < a.cout) a.y[((long long)b * a.cout + co) * HWs + pixs] = u;
                }
        } else if constexpr (EPI == kGcEpiGru1) {
            float hv[WM][4];
            const long long ob = ((long long)b * hc + (co0 - gate * hc)) * HWo + pix;  // channel co0 of the gate
            if (gate == 1) {
#pragma unroll
                for (int m = 0; m < WM; ++m)
#pragma unroll
                    for (int r = 0; r < 4; ++r) hv[m][r] = a.h[ob + (long long)(16 * m + 4 * lg + r) * HWo];
            }
            float *dst = gate == 0 ? a.zb : gate == 1 ? a.rhb : a.qxb;
#pragma unroll
            for (int m = 0; m < WM; ++m)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const float u = acc[m][n][r] + bv[m][r];
                    float o;
                    if (gate == 0) o = 1.f / (1.f + expf(-u));                    // z
                    else if (gate == 1) o = (1.f / (1.f + expf(-u))) * hv[m][r];  // r * h
                    else o = u;                                                    // convq's x half + bias
                    if (ok) dst[ob + (long long)(16 * m + 4 * lg + r) * HWo] = o;
                }
        } else if constexpr (EPI == kGcEpiAff) {
            // _affinity_normalization + _aff_insert (nlspnmodel.py:179-201, :261-269) on the raw
            // taps as they leave the accumulators: the same float values the two-kernel path
            // stores and affnorm_kernel reloads, through the same normalize_taps, so bit-equal.
            // Channels 0-3 sit in lane group 0, 4-7 in group 1 (same pixel, lane ^ 16): one
            // exchange gives both groups all eight taps; group 0 stores planes 0-4, group 1 5-8.
            static_assert(WM == 1 && WGM == 1, "kGcEpiAff: one 16-channel block holds the K = 8 taps");
            float u[4], v[4], t[8][1], ref[1];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                u[r] = acc[0][n][r] + bv[0][r];
                if (a.act == kGcActRelu) u[r] = u[r] < 0.f ? 0.f : u[r];
                else if (a.act == kGcActTanh) u[r] = tanhf(u[r]);
            }
#pragma unroll
            for (int r = 0; r < 4; ++r) v[r] = __shfl_xor(u[r], 16, 64);
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                t[r][0] = lg == 0 ? u[r] : v[r];
                t[4 + r][0] = lg == 0 ? v[r] : u[r];
            }
            normalize_taps<8, 1>(t, ref, a.aff_kind, *a.gamma);
            const long long HWs = (long long)a.ohs * a.ows;
            const long long pixs = ok ? (long long)oy * a.ows + ox : 0;
            float *yb = a.y + (long long)b * 9 * HWs + pixs;
            if (ok && lg == 0) {
#pragma unroll
                for (int c = 0; c < 4; ++c) yb[c * HWs] = t[c][0];
                yb[4 * HWs] = ref[0];
            } else if (ok && lg == 1) {
#pragma unroll
                for (int c = 5; c < 9; ++c) yb[c * HWs] = t[c - 1][0];
            }
        } else {  // kGcEpiGru2
            float qv[WM][4], zv[WM][4], hv[WM][4];
            const long long ob = ((long long)b * hc + co0) * HWo + pix;
#pragma unroll
            for (int m = 0; m < WM; ++m)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const long long o = ob + (long long)(16 * m + 4 * lg + r) * HWo;
                    qv[m][r] = a.qxb[o];
                    zv[m][r] = a.zb[o];
                    hv[m][r] = a.h[o];
                }
#pragma unroll
            for (int m = 0; m < WM; ++m)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const float q = tanhf(acc[m][n][r] + qv[m][r]);
                    const float z = zv[m][r];
                    if (ok) a.hout[ob + (long long)(16 * m + 4 * lg + r) * HWo] = (1.f - z) * hv[m][r] + z * q;  // :402
                }
        }
    }
}

// GRU1's output-channel tiles differ in cost: z and r run K over h and x, qx over x alone (half).
// One workgroup per (co tile, pixel tile) left the CUs unevenly loaded (every workgroup is
// resident at once, so a CU's finish time is its summed work: 3.5 heavy-tile units on the most
// loaded CUs against 2.8 on average).  A qx workgroup takes TWO consecutive pixel tiles instead,
// so every workgroup costs the same.  (The pixel tiles of a GRU1 launch: gc_rest_count.)
__host__ __device__ inline int gc_gru1_heavy_cots(const GconvArgs &a, int wgco) { return (2 * a.hc) / wgco; }
__host__ __device__ inline int gc_rest_count(const GconvArgs &a) { return a.B * a.nbands * a.tpb; }
__host__ __device__ inline int gc_gru1_wgs(const GconvArgs &a, int wgco) {
    const int nh = gc_gru1_heavy_cots(a, wgco), nr = gc_rest_count(a);
    return nh * nr + (a.co_tiles - nh) * ((nr + 1) / 2);
}

template <int MODE, int WM, int WN, int WGM, int WGN, int XR, int XP, int CC, int EPI>
__global__ void __launch_bounds__(kGcNT) gconv_kernel(GconvArgs a) {
    extern __shared__ __attribute__((aligned(16))) float gc_lds[];
    if constexpr (EPI == kGcEpiGru1) {
        using Cfg = GcCfg<MODE, WM, WN, WGM, WGN, XR, XP, CC, EPI>;
        const int nh = gc_gru1_heavy_cots(a, Cfg::WGCO), nr = gc_rest_count(a);
        const int wg = xcd_remap((int)blockIdx.x, gc_gru1_wgs(a, Cfg::WGCO));
        if (wg < nh * nr) {  // z / r: one pixel tile
            gconv_body<MODE, WM, WN, WGM, WGN, XR, XP, CC, EPI, 0>(a, gc_lds, wg % nh + (wg / nh) * a.co_tiles);
        } else {             // qx: two pixel tiles in turn
            const int w = wg - nh * nr, nl = a.co_tiles - nh;
            const int cot = nh + w % nl, r0 = 2 * (w / nl);
            gconv_body<MODE, WM, WN, WGM, WGN, XR, XP, CC, EPI, 0>(a, gc_lds, cot + r0 * a.co_tiles);
            if (r0 + 1 < nr) gconv_body<MODE, WM, WN, WGM, WGN, XR, XP, CC, EPI, 0>(a, gc_lds, cot + (r0 + 1) * a.co_tiles);
        }
        return;
    }
    const int per_phase = a.co_tiles * a.B * a.nbands * a.tpb;
    const int nph = MODE == kGcT2 ? 4 : 1;
    const int wg = xcd_remap((int)blockIdx.x, per_phase * nph);  // neighbouring tiles (and co tiles) share an XCD
    const int ph = wg / per_phase, wgi = wg - ph * per_phase;
    if constexpr (MODE == kGcT2) {
        switch (ph) {
            case 0: gconv_body<MODE, WM, WN, WGM, WGN, XR, XP, CC, EPI, 0>(a, gc_lds, wgi); break;
            case 1: gconv_body<MODE, WM, WN, WGM, WGN, XR, XP, CC, EPI, 1>(a, gc_lds, wgi); break;
            case 2: gconv_body<MODE, WM, WN, WGM, WGN, XR, XP, CC, EPI, 2>(a, gc_lds, wgi); break;
            default: gconv_body<MODE, WM, WN, WGM, WGN, XR, XP, CC, EPI, 3>(a, gc_lds, wgi); break;
        }
    } else {
        gconv_body<MODE, WM, WN, WGM, WGN, XR, XP, CC, EPI, 0>(a, gc_lds, wgi);
    }
}

// The narrow first layers (encode_dep / encode_aff's first conv: 1 or 9 -> 16 channels) on the
// VALU: one thread per output pixel holds the 16 sums, reads its taps' inputs directly and the
// weights as LDS broadcasts.  As MFMA tiles their K (9 or 81 terms) would be mostly padding and
// their windows mostly empty; here they are bound by their few MB of HBM traffic (NYU B=8:
// 16 vs 34 us).  Same bias / activation epilogue.  (The 16 -> 8 transposed conv measured
// slower this way — per-lane output phases diverge — and stays on the MFMA kernel.)
constexpr int kGsNT = 256, kGsMaxW = 16 * 16 * 9;  // threads; weights held in LDS (16 x cin x 9 at most)
template <int COUT>
__global__ void __launch_bounds__(kGsNT) gsmall_kernel(GconvArgs a, const float *w) {
    // w: the module's own (cout, cin, 3, 3) layout
    __shared__ float ws[kGsMaxW];
    const int cin = a.c0;
    for (int i = threadIdx.x; i < COUT * cin * 9; i += kGsNT) ws[i] = w[i];
    __syncthreads();
    const long long npix = (long long)a.B * a.ohs * a.ows;
    const long long HWi = (long long)a.Hi * a.Wi;
    for (long long p = (long long)blockIdx.x * kGsNT + threadIdx.x; p < npix; p += (long long)gridDim.x * kGsNT) {
        const int b = (int)(p / ((long long)a.ohs * a.ows));
        const int rem = (int)(p - (long long)b * a.ohs * a.ows);
        const int oy = rem / a.ows, ox = rem - oy * a.ows;
        float acc[COUT];
#pragma unroll
        for (int co = 0; co < COUT; ++co) acc[co] = 0.f;
        const float *xb = a.x0 + (long long)b * cin * HWi;
        for (int ci = 0; ci < cin; ++ci) {
#pragma unroll
            for (int ky = 0; ky < 3; ++ky) {
                const int iy = 2 * oy - 1 + ky;
                if ((unsigned)iy >= (unsigned)a.Hi) continue;
#pragma unroll
                for (int kx = 0; kx < 3; ++kx) {
                    const int ix = 2 * ox - 1 + kx;
                    if ((unsigned)ix >= (unsigned)a.Wi) continue;
                    float v = xb[(long long)ci * HWi + (long long)iy * a.Wi + ix];
                    if (a.in_div != 1.f) v = v / a.in_div;
#pragma unroll
                    for (int co = 0; co < COUT; ++co) acc[co] = fmaf(ws[(co * cin + ci) * 9 + ky * 3 + kx], v, acc[co]);
                }
            }
        }
#pragma unroll
        for (int co = 0; co < COUT; ++co) {
            float u = acc[co] + a.bias[co];
            if (a.act == kGcActRelu) u = u < 0.f ? 0.f : u;
            else if (a.act == kGcActTanh) u = tanhf(u);
            a.y[(((long long)b * a.cout + co) * a.ohs + oy) * a.ows + ox] = u;
        }
    }
}

// The instantiated configurations: X(id, MODE, WM, WN, WGM, WGN, XR, XP, CC, EPI).  Ids 0..5, 23 and 24
// are the presets NLSPN_GC_* of include/nlspn_prop.h (23 / 24: NLSPN_GC_S2 / NLSPN_GC_GRU2 on
// 32-pixel tiles, which nlspn_gconv picks for small grids; 25: NLSPN_GC_T2_C16 with the affinity
// normalisation in its epilogue, nlspn_gconv_affnorm); the other ids >= 16 are alternative tilings of the same
// layer kinds, selectable through nlspn_gconv's layer argument for A/B timing
// (tools/gc_bench.py) and bit-compatible with the preset of their kind in layout (the packed
// weights depend only on the kind's output-channel tile, which a variant must keep).
#define NLSPN_GC_CONFIGS(X)                                        \
    X(0, kGcS2, 4, 1, 1, 4, 12, 40, 4, kGcEpiAct)                  \
    X(1, kGcS2, 1, 1, 1, 4, 10, 72, 8, kGcEpiAct)                  \
    X(2, kGcS1, 2, 2, 2, 2, 6, 40, 4, kGcEpiGru1)                  \
    X(3, kGcS1, 2, 2, 2, 2, 8, 40, 8, kGcEpiGru2)                  \
    X(4, kGcT2, 4, 1, 1, 4, 6, 40, 8, kGcEpiAct)                   \
    X(5, kGcT2, 1, 4, 1, 4, 6, 80, 8, kGcEpiAct)                   \
    X(16, kGcS1, 2, 2, 2, 2, 8, 40, 8, kGcEpiGru1)                 \
    X(17, kGcS1, 2, 2, 2, 2, 6, 40, 4, kGcEpiGru2)                 \
    X(18, kGcS1, 2, 4, 2, 2, 8, 40, 8, kGcEpiGru1)                 \
    X(20, kGcS2, 4, 1, 1, 4, 12, 40, 8, kGcEpiAct)                 \
    X(21, kGcT2, 4, 1, 1, 4, 6, 40, 4, kGcEpiAct)                  \
    X(22, kGcT2, 1, 4, 1, 4, 6, 80, 4, kGcEpiAct)                  \
    X(23, kGcS2, 2, 1, 2, 2, 8, 40, 4, kGcEpiAct)                  \
    X(24, kGcS1, 2, 1, 2, 2, 6, 40, 8, kGcEpiGru2)                 \
    X(25, kGcT2, 1, 4, 1, 4, 6, 80, 8, kGcEpiAff)

}  // namespace nlspn
