// Head epilogue: the reference's last three 3x3 convolutions of
// the decoder, nlspnmodel.py:296-315 —
//   pred_init  = ReLU(id_dec0(cat(id_fd1, fe1)))          (:297, id_dec0 :68)
//   off_aff    = off_aff_dec0(cat(off_aff_fd1, fe1))      (:301, off_aff_dec0 :74)
//   confidence = Sigmoid(cf_dec0(cat(cf_fd1, fe1)))       (:313, cf_dec0 :83-86)
// — as ONE kernel that reads the four C-channel sources (fe1 shared by all three)
// directly: no torch.cat copies, bias and activation in the epilogue.
//
// Implicit GEMM on the f32-input matrix cores (v_mfma_f32_32x32x2_f32: f32 operands,
// exact f32 products, f32 accumulation — only the summation order differs from a
// sequential f32 convolution).  D[co][px] = sum_k W[co][k] X[k][px], k = (channel,
// tap):
//   * MFMA part, M = 32*MB output channels (0..nout-1 the off_aff conv, nout the
//     id conv, nout+1 the cf conv, the rest zero), N = 32 pixels of one tile row,
//     k over fe1 (all columns) and over off_aff_fd1 (off_aff columns only);
//   * VALU part: the 1-channel id / cf convs' own decoder halves (id_fd1, cf_fd1),
//     one pixel per thread, weights from scalar registers (wave-uniform loads), issued
//     in the same loop body as the MFMAs (the matrix cores' shadow).  As MFMA columns
//     they would cost 32x their FLOPs.
// Tile: 8 rows x 32 columns, 256 threads (4 waves, 2 rows each).  The K loop runs in
// rounds of 16 channels: the round's two input windows (16 ch x 10 rows x 40 cols, zero
// outside the image = the conv's zero padding) and its packed weights are staged in
// LDS; the next round's global loads are in flight in registers while the current
// round computes.  LDS 74 KB and 239 registers: two workgroups per CU.
#pragma once

#include <type_traits>

#include "nlspn_common.h"

namespace nlspn {

constexpr int kHdTH = 8, kHdTW = 32, kHdNT = 256;  // tile rows / columns, threads
constexpr int kHdCC = 16;                            // channels per K chunk
constexpr int kHdRS = 40;                            // LDS row stride (cols x0-4 .. x0+35)
constexpr int kHdCS = (kHdTH + 2) * kHdRS + 16;      // LDS channel stride: 416 = 32 (mod 64) banks
constexpr int kHdXF4 = kHdCC * (kHdTH + 2) * (kHdRS / 4);  // float4s of one chunk's input window (1600)
constexpr int kHdXR = (kHdXF4 + kHdNT - 1) / kHdNT;        // per thread (7)

struct HeadsArgs {
    const float *fe1, *fd_oa, *fd_id, *fd_cf;  // (B,C,H,W) each; fd_id / fd_cf may be null
    const float *wm;    // packed MFMA weights [2][C][9][32*MB]: source 0 = fe1, 1 = off_aff_fd1
    const float *wv;    // packed VALU weights [2][C][9]: id conv on id_fd1, cf conv on cf_fd1
    const float *bias;  // [32*MB]: off_aff biases, id bias, cf bias, zeros
    float *off_aff;     // (B,nout,H,W)
    float *pred_init;   // (B,1,H,W) or null
    float *conf;        // (B,1,H,W) or null
    int B, C, H, W, nout, tiles_x, tiles_y;
    // The propagation prologue fused in (nlspnmodel.py:323-348; 3x3, K = 8 with offsets:
    // nout = 24, one M-block), when aff_out is set: instead of the raw off_aff planes the
    // epilogue writes the output-dict tensors — off_out = _off_insert(off) (:324),
    // aff_out = _affinity_normalization + _aff_insert (:325), conf = the blended
    // confidence (:328-334) — and p0, iteration 1's input (:341-348).  Same IEEE
    // sequence as step 1 of nlspn_propagate (bit-identical given the same conv sums).
    const float *dep;    // (B,1,H,W), or null (preserve_input off)
    const float *gamma;  // device, 1 float (aff_scale_const)
    float *aff_out;      // (B,K+1,H,W), or null: raw off_aff out
    float *off_out;      // (B,2(K+1),H,W)
    float *p0;           // (B,1,H,W)
    int kind;
    unsigned flags;      // NLSPN_PRESERVE_INPUT | NLSPN_ALWAYS_CLIP
    unsigned dbg;  // NLSPN_HEADS_DBG (ablation, timing only): 1 no VALU sums, 2 no MFMAs (both: the ABL
                   // kernels of MB=1), 4 no LDS staging
};

template <int MB> struct HdCfg {
    static constexpr int NCO = 32 * MB;
    static constexpr int WCS = 9 * NCO + ((MB % 2) ? 0 : 32);  // LDS weight channel stride: 32 (mod 64) banks
    static constexpr int WF4 = kHdCC * 9 * NCO / 4;              // float4s of one chunk's weights
    static constexpr int WR = (WF4 + kHdNT - 1) / kHdNT;
    static constexpr int LDS_FLOATS = 2 * kHdCC * kHdCS + kHdCC * WCS + 2 * kHdTH * kHdTW;  // + 2*C*9 (VALU weights)
};

typedef float f32x16 __attribute__((ext_vector_type(16)));

// The fused-prologue epilogue of one MB = 1 workgroup (HeadsArgs::aff_out set; 3x3,
// K = 8, nout = 24).  Lane (px, h) holds output channels co = (r&3) + 8(r>>2) + 4h of
// pixel px: offsets co 0..15 in r 0..7, raw affinities 16..23 in r 8..11 (h = 0:
// taps 0-3, h = 1: taps 4-7), the id conv in r 12 and the cf conv in r 13 (h = 0).
// The two halves swap their four affinities (a 32-lane xor shuffle), so both hold the
// pixel's eight in tap order and normalise them exactly as step 1 does (normalize_taps).
__device__ __forceinline__ void heads_epilogue_prologue(const HeadsArgs &a, const f32x16 (&acc)[2],
                                                        const float (&bv)[16], const float *SV, int b, int y0,
                                                        int x, int wv, int h, int l32) {
    constexpr int K = 8, REF = 4;
    const int H = a.H, W = a.W;
    const long long HW = (long long)H * W;
    const bool preserve = (a.flags & 0x1u) != 0, clip = (a.flags & 0x2u) != 0;
    const float gamma = *a.gamma;
#pragma unroll
    for (int n = 0; n < 2; ++n) {
        const int yl = 2 * wv + n, y = y0 + yl;
        if (y >= H || x >= W) continue;  // both halves of a pixel skip together
        const long long pix = (long long)y * W + x;
        float v[16];
#pragma unroll
        for (int r = 0; r < 16; ++r) v[r] = acc[n][r] + bv[r];
        // _off_insert (:252-259): raw channel c of tap c/2 -> inserted channel c + 2 past the reference tap
        float *oo = a.off_out + (long long)b * 2 * (K + 1) * HW + pix;
#pragma unroll
        for (int r = 0; r < 8; ++r) {
            const int co = (r & 3) + 8 * (r >> 2) + 4 * h;
            oo[(long long)(co + (co >= 2 * REF ? 2 : 0)) * HW] = v[r];
        }
        if (h == 0) {
            oo[(long long)(2 * REF) * HW] = 0.f;
            oo[(long long)(2 * REF + 1) * HW] = 0.f;
        }
        // _affinity_normalization + _aff_insert (:179-201, :261-269)
        float t[K][1], ref[1];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const float other = __shfl_xor(v[8 + i], 32);
            t[i][0] = h == 0 ? v[8 + i] : other;
            t[4 + i][0] = h == 0 ? other : v[8 + i];
        }
        normalize_taps<K, 1>(t, ref, a.kind, gamma);
        float *ao = a.aff_out + (long long)b * (K + 1) * HW + pix;
        if (h == 0) {
#pragma unroll
            for (int k = 0; k < 4; ++k) ao[(long long)k * HW] = t[k][0];
            ao[(long long)REF * HW] = ref[0];
        } else {
#pragma unroll
            for (int k = 4; k < K; ++k) ao[(long long)(k + 1) * HW] = t[k][0];
        }
        // pred_init, p0 and the blended confidence (:297, :313, :328-348)
        if (h == 0) {
            const float d = preserve ? a.dep[(long long)b * HW + pix] : 0.f;
            const float m = d > 0.f ? 1.f : 0.f;
            const float u = v[12] + SV[yl * kHdTW + l32];
            const float pi = u < 0.f ? 0.f : u;  // ReLU (NaN kept)
            a.pred_init[(long long)b * HW + pix] = pi;
            float p = pi;
            if (preserve) p = __fadd_rn(__fmul_rn(1.0f - m, p), __fmul_rn(m, d));
            if (clip) p = clamp0(p);
            a.p0[(long long)b * HW + pix] = p;
            if (a.conf) {
                const float uc = v[13] + SV[kHdNT + yl * kHdTW + l32];
                float c = 1.f / (1.f + expf(-uc));  // Sigmoid
                if (preserve) c = __fadd_rn(__fmul_rn(1.0f - m, c), m);
                a.conf[(long long)b * HW + pix] = c;
            }
        }
    }
}

// One input window of a chunk (16 channels x 10 rows x 40 columns) in flight in
// registers: raw bits + a per-float4 in-image mask.  Every lane loads a clamped,
// in-bounds address and the mask zeroes what lies outside the image when the window is
// written to LDS: a select right after the load would let the compiler sink the load
// into a branch and wait for it at the join (one full memory latency per load).
template <bool VEC> struct HdWin {
    u32x4 r[kHdXR];  // ext-vector types: a HIP float4 struct copy from global memory becomes
    unsigned m[kHdXR];  // a memcpy that keeps the array in scratch

    __device__ __forceinline__ void load(const float *src, long long HW, int H, int W, int y0, int x0, int tid) {
#pragma unroll
        for (int i = 0; i < kHdXR; ++i) {
            const int f = min(tid + i * kHdNT, kHdXF4 - 1);
            const int ch = f / ((kHdTH + 2) * (kHdRS / 4)), rem = f - ch * ((kHdTH + 2) * (kHdRS / 4));
            const int row = rem / (kHdRS / 4), c4 = rem - row * (kHdRS / 4);
            const int y = y0 - 1 + row, x = x0 - 4 + 4 * c4;
            const bool yin = (unsigned)y < (unsigned)H;
            const float *p = src + ch * HW + (long long)min(max(y, 0), H - 1) * W;
            if (VEC) {
                r[i] = *reinterpret_cast<const u32x4 *>(p + min(max(x, 0), W - 4));
                m[i] = (yin && (unsigned)x < (unsigned)W) ? 0xfu : 0u;
            } else {
                unsigned mm = 0;
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    r[i][j] = __builtin_bit_cast(unsigned, p[min(max(x + j, 0), W - 1)]);
                    mm |= (yin && (unsigned)(x + j) < (unsigned)W) ? (1u << j) : 0u;
                }
                m[i] = mm;
            }
        }
    }
    __device__ __forceinline__ void store(float *XL, int tid) const {
#pragma unroll
        for (int i = 0; i < kHdXR; ++i) {
            const int f = tid + i * kHdNT;
            if (f < kHdXF4) {
                const int ch = f / ((kHdTH + 2) * (kHdRS / 4)), rem = f - ch * ((kHdTH + 2) * (kHdRS / 4));
                const u32x4 mk = {(m[i] & 1u) ? ~0u : 0u, (m[i] & 2u) ? ~0u : 0u, (m[i] & 4u) ? ~0u : 0u,
                                  (m[i] & 8u) ? ~0u : 0u};
                *reinterpret_cast<u32x4 *>(&XL[ch * kHdCS + 4 * rem]) = r[i] & mk;  // rows of 40 = 10 float4
            }
        }
    }
};

// Round r (0 .. 2*C/16-1) stages three chunks of 16 channels: the MFMA source (fe1 for
// r < C/16, then off_aff_fd1), its packed weights, and the VALU source (id_fd1 for
// r < C/16, then cf_fd1).  The VALU sums (18 FMAs per channel pair) sit in the same loop
// body as the channel pair's 18 MFMAs, so they issue in the matrix cores' shadow.  An
// absent id / cf source is replaced by fe1 (valid memory) and its sum discarded: every
// round runs the same straight-line code.
template <int MB, bool VEC, int ABL = 0, bool PRO = false>
__global__ void __launch_bounds__(kHdNT) __attribute__((amdgpu_waves_per_eu(2, 2))) heads_kernel(HeadsArgs a) {
    using Cfg = HdCfg<MB>;
    constexpr int NCO = Cfg::NCO, WCS = Cfg::WCS;
    extern __shared__ float hd_lds[];
    float *XL = hd_lds;                       // [16][CS]   MFMA source window
    float *XV = XL + kHdCC * kHdCS;           // [16][CS]   VALU source window
    float *WL = XV + kHdCC * kHdCS;           // [16][WCS]  packed weights
    float *SV = WL + kHdCC * WCS;             // [2][256]   the VALU sums per pixel
    float *WVL = SV + 2 * kHdNT;              // [2][C][9]  the VALU weights (all rounds)

    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, h = lane >> 5, l32 = lane & 31;
    const int ntile = a.tiles_x * a.tiles_y * a.B;
    const int tile = xcd_remap(blockIdx.x, ntile);
    const int b = tile / (a.tiles_x * a.tiles_y), tr = tile - b * a.tiles_x * a.tiles_y;
    const int ty = tr / a.tiles_x, tx = tr - ty * a.tiles_x;
    const int y0 = ty * kHdTH, x0 = tx * kHdTW;
    const int H = a.H, W = a.W, C = a.C;
    const long long HW = (long long)H * W;
    const int nch = C / kHdCC, nr = 2 * nch;
    const float *vsrc[2] = {a.fd_id ? a.fd_id : a.fe1, a.fd_cf ? a.fd_cf : a.fe1};

    HdWin<VEC> xm, xv;
    f32x4 wr[Cfg::WR];
    auto load_round = [&](int r) __attribute__((always_inline)) {
        const int s = r < nch ? 0 : 1, cb = (r - s * nch) * kHdCC;
        const long long off = ((long long)b * C + cb) * HW;
        xm.load((s == 0 ? a.fe1 : a.fd_oa) + off, HW, H, W, y0, x0, tid);
        xv.load(vsrc[s] + off, HW, H, W, y0, x0, tid);
        const f32x4 *wsrc = reinterpret_cast<const f32x4 *>(a.wm + ((long long)s * C + cb) * 9 * NCO);
#pragma unroll
        for (int i = 0; i < Cfg::WR; ++i) wr[i] = wsrc[min(tid + i * kHdNT, Cfg::WF4 - 1)];
    };

    f32x16 acc[MB][2];
#pragma unroll
    for (int m = 0; m < MB; ++m)
#pragma unroll
        for (int n = 0; n < 2; ++n)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[m][n][r] = 0.f;
    float sv_id = 0.f, sv_cf = 0.f;  // VALU sums of this thread's pixel
    const int vrow = tid >> 5, vcol = tid & 31;

    for (int i = tid; i < 2 * C * 9; i += kHdNT) WVL[i] = a.wv[i];  // read as LDS broadcasts
    load_round(0);
    for (int r = 0; r < nr; ++r) {
        __syncthreads();  // the previous round's LDS reads are done
        if (!(exp_dbg(a.dbg) & 4u)) {
            xm.store(XL, tid);
            xv.store(XV, tid);
#pragma unroll
            for (int i = 0; i < Cfg::WR; ++i) {
                const int f = tid + i * kHdNT;
                if (f < Cfg::WF4) {
                    const int ch = f / (9 * NCO / 4), rem = f - ch * (9 * NCO / 4);
                    *reinterpret_cast<f32x4 *>(&WL[ch * WCS + 4 * rem]) = wr[i];
                }
            }
        }
        __syncthreads();
        // the next round's loads, in flight while this round computes (the last round
        // reloads round 0, unused: no branch, so no wait at a join)
        load_round(r + 1 < nr ? r + 1 : 0);
        __builtin_amdgcn_sched_barrier(0);  // keep them ahead of the compute (the scheduler sinks them otherwise)
        const int s = r < nch ? 0 : 1;
        const float *wvp = WVL + (s * C + (r - s * nch) * kHdCC) * 9;  // same address in every lane: broadcasts
        // B operand: X[k = h][px = l32] of channel 2cp+h at tap (dy,dx), rows 2wv+n;
        // A operand: W[co = 32m + l32][k = h] of the same channel and tap
        const float *xb = XL + h * kHdCS + (2 * wv) * kHdRS + l32 + 3;
        const float *wb = WL + h * WCS + l32;
        const float *xvp = XV + vrow * kHdRS + vcol + 3;
        // the round's straight-line body; the ablation variants (ABL = NLSPN_HEADS_DBG & 3)
        // are separate kernels, so no branch sits inside the MFMA stream
        auto body = [&](auto do_mfma, auto do_valu) __attribute__((always_inline)) {
            // software pipelined by hand: the LDS operands of k-step j+1 are read while
            // the MFMAs of step j issue; scheduling barriers keep the compiler from
            // sinking the reads next to their use (it does, to save registers, and then
            // every MFMA waits on an LDS round trip)
            constexpr int NS = (kHdCC / 2) * 9;  // k-steps (channel pair, tap) per round
            float av[2][MB], bv[2][2], xv[2][2], wv2[2][2];
            auto fetch = [&](int j, int slot) __attribute__((always_inline)) {
                const int cp = j / 9, t = j % 9, dy = t / 3, dx = t % 3;
                if constexpr (decltype(do_mfma)::value) {
#pragma unroll
                    for (int m = 0; m < MB; ++m) av[slot][m] = wb[2 * cp * WCS + t * NCO + 32 * m];
#pragma unroll
                    for (int n = 0; n < 2; ++n) bv[slot][n] = xb[2 * cp * kHdCS + (n + dy) * kHdRS + dx];
                }
                if constexpr (decltype(do_valu)::value) {
#pragma unroll
                    for (int e = 0; e < 2; ++e) {
                        xv[slot][e] = xvp[(2 * cp + e) * kHdCS + dy * kHdRS + dx];
                        wv2[slot][e] = wvp[(2 * cp + e) * 9 + t];
                    }
                }
            };
            float sacc[2] = {0.f, 0.f};
            fetch(0, 0);
#pragma unroll
            for (int j = 0; j < NS; ++j) {
                const int cur = j & 1;
                if (j + 1 < NS) fetch(j + 1, cur ^ 1);
                __builtin_amdgcn_sched_barrier(0);
                if constexpr (decltype(do_mfma)::value) {
#pragma unroll
                    for (int m = 0; m < MB; ++m)
#pragma unroll
                        for (int n = 0; n < 2; ++n)
                            acc[m][n] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[cur][m], bv[cur][n], acc[m][n], 0, 0, 0);
                }
                if constexpr (decltype(do_valu)::value) {
#pragma unroll
                    for (int e = 0; e < 2; ++e) sacc[e] = fmaf(xv[cur][e], wv2[cur][e], sacc[e]);
                }
                __builtin_amdgcn_sched_barrier(0);
            }
            return sacc[0] + sacc[1];
        };
        float svr;
        svr = body(std::integral_constant<bool, !(ABL & 2)>{}, std::integral_constant<bool, !(ABL & 1)>{});
        sv_id += s == 0 ? svr : 0.f;
        sv_cf += s == 1 ? svr : 0.f;
    }

    // epilogue: the VALU sums by pixel, then bias + activation and coalesced row stores
    SV[tid] = sv_id;
    SV[kHdNT + tid] = sv_cf;
    __syncthreads();
    const int x = x0 + l32;
    float bv[MB][16];  // biases of this lane's 16*MB output channels, all loads issued together
#pragma unroll
    for (int m = 0; m < MB; ++m)
#pragma unroll
        for (int r = 0; r < 16; ++r) bv[m][r] = a.bias[32 * m + (r & 3) + 8 * (r >> 2) + 4 * h];
    if constexpr (PRO) {  // the fused propagation prologue (its own instantiation: no registers for the other)
        static_assert(MB == 1, "3x3 / K = 8 only");
        heads_epilogue_prologue(a, acc[0], bv[0], SV, b, y0, x, wv, h, l32);
        return;
    }
#pragma unroll
    for (int n = 0; n < 2; ++n) {
        const int yl = 2 * wv + n, y = y0 + yl;
        if (y >= H || x >= W) continue;
        const long long pix = (long long)y * W + x;
#pragma unroll
        for (int m = 0; m < MB; ++m)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int co = 32 * m + (r & 3) + 8 * (r >> 2) + 4 * h;
                const float v = acc[m][n][r] + bv[m][r];
                if (co < a.nout) {
                    a.off_aff[((long long)b * a.nout + co) * HW + pix] = v;
                } else if (co == a.nout) {
                    if (a.pred_init) {
                        const float u = v + SV[yl * kHdTW + l32];
                        a.pred_init[(long long)b * HW + pix] = u < 0.f ? 0.f : u;  // ReLU (NaN kept)
                    }
                } else if (co == a.nout + 1) {
                    if (a.conf) {
                        const float u = v + SV[kHdNT + yl * kHdTW + l32];
                        a.conf[(long long)b * HW + pix] = 1.f / (1.f + expf(-u));  // Sigmoid
                    }
                }
            }
    }
}

// Packs the three convs' (Cout, 2C, 3, 3) weights and biases into HeadsArgs' layouts.
// One thread per packed element of wm, then wv and bias.
struct HeadsPackArgs {
    const float *w_oa, *b_oa, *w_id, *b_id, *w_cf, *b_cf;  // id / cf may be null
    float *wm, *wv, *bias;
    int C, nout, nco;
};

static __global__ void heads_pack_kernel(HeadsPackArgs a) {
    const long long nm = 2LL * a.C * 9 * a.nco, nv = 2LL * a.C * 9;
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    const int C2 = 2 * a.C;
    if (i < nm) {
        const int co = (int)(i % a.nco);
        const long long r = i / a.nco;
        const int t = (int)(r % 9), c = (int)((r / 9) % a.C), s = (int)(r / (9LL * a.C));
        // input channel of the conv: source 0 = fe1 = channels C..2C-1, source 1 = fd = 0..C-1
        const int ci = s == 0 ? a.C + c : c;
        float v = 0.f;
        if (co < a.nout) v = a.w_oa[((long long)co * C2 + ci) * 9 + t];
        else if (s == 0 && co == a.nout && a.w_id) v = a.w_id[(long long)ci * 9 + t];
        else if (s == 0 && co == a.nout + 1 && a.w_cf) v = a.w_cf[(long long)ci * 9 + t];
        a.wm[i] = v;
    } else if (i < nm + nv) {
        const long long j = i - nm;
        const int t = (int)(j % 9), c = (int)((j / 9) % a.C), s = (int)(j / (9LL * a.C));
        const float *w = s == 0 ? a.w_id : a.w_cf;
        a.wv[j] = w ? w[(long long)c * 9 + t] : 0.f;  // the decoder half: input channels 0..C-1
    } else if (i < nm + nv + a.nco) {
        const int co = (int)(i - nm - nv);
        float v = 0.f;
        if (co < a.nout) v = a.b_oa ? a.b_oa[co] : 0.f;
        else if (co == a.nout && a.b_id) v = a.b_id[0];
        else if (co == a.nout + 1 && a.b_cf) v = a.b_cf[0];
        a.bias[co] = v;
    }
}

}  // namespace nlspn
