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
// FIRST = the first iteration with the forward prologue fused in: it reads the
// raw head outputs (pred_init, conf, raw affinity, raw offsets), builds p0 and
// conf' on the fly (:328-348), normalises the affinity in-kernel
// (_affinity_normalization + _aff_insert, :179-201, :261-269) and writes the
// output-dict tensors (aff, confidence, inserted offsets) for its own pixels —
// one pass instead of a separate prologue kernel plus a first step.
//
// Structure (one workgroup per TH x TW output tile, PX pixels per thread):
//   1. issue the window's staging loads (p_in, conf [, dep]; clamped, branch-
//      free), then the tile's streamed loads — K affinity planes, 2K offset
//      planes and dep — coalesced, through wave-uniform buffer descriptors;
//   2. stage f = p * conf for the tile + halo window into LDS (fp32), zero
//      outside the image (= the reference's zero-padded bilinear) or replicate-
//      clamped for the no-offset branch; an LDS-only barrier keeps the streamed
//      loads in flight (s_waitcnt vmcnt counts in issue order, so staging waits
//      only for its own loads and each tap only for the planes it consumes);
//   3. pass A: per tap, bilinear-sample f from LDS; taps whose 2x2 footprint
//      leaves the window (learned offsets are unbounded) are flagged; pass B
//      (rare) serves them from L2/global with the reference's per-corner checks —
//      correctness never depends on the halo;
//   4. accumulate taps in index order with the reference tap (index K/2) weighted
//      1 - sum(others); blend, clamp, store p_out (and pred on the last step).
// Summation and bilinear arithmetic follow the reference's operation order; the
// file is compiled with -ffp-contract=off so it issues exactly the IEEE sequence
// the C oracle does (bit-identical iterations given identical inputs).
#pragma once

#include "nlspn_common.h"

#include <type_traits>

namespace nlspn {

struct StepArgs {
    const void *p_in;   // B planes (FIRST: pred_init)
    const void *conf;   // B planes or null (conf_prop off). FIRST: raw confidence, else conf'
    const void *dep;    // B planes or null (preserve off)
    const void *aff;    // affinity: normalised (K+1) planes per item, or FIRST: raw K planes
    const void *off;    // offsets (null: no-offset branch)
    void *p_out;        // B planes
    void *pred_out;     // B planes or null
    long long aff_bs;   // batch strides in elements
    long long off_bs;
    int B, H, W;
    int tiles_x, tiles_y;
    int off_raw;        // 1: raw (2K planes, ref tap implicit), 0: inserted (2(K+1) planes)
    unsigned flags;     // NLSPN_PRESERVE_INPUT | NLSPN_ALWAYS_CLIP
    // FIRST only
    const float *gamma;  // device, 1 float (aff_scale_const)
    void *aff_out;       // (K+1) planes per item, contiguous
    void *off_out;       // 2(K+1) planes per item, contiguous, or null
    void *conf_out;      // B planes, or null iff conf null
    int kind;            // affinity kind
    unsigned *zero_words;  // step 1: sync words of the resident kernel that follows, zeroed here
    int nzero;             //   (replaces a memset node; the kernel boundary orders it)
    void *poison;          // step 1: plane 1 (B planes), filled with the resident hand-off's poison
                           //   (nlspn_resident.h) for the own pixels, or null
};

// The resident kernel's "not yet written" plane values (nlspn_resident.h): signalling NaNs
// (quiet bit clear), which no arithmetic result is
constexpr unsigned kPoison32 = 0x7f800badu;
constexpr unsigned short kPoison16 = 0x7d0bu;

constexpr unsigned kPreserve = 0x1u;
constexpr unsigned kAlwaysClip = 0x2u;

// Source value f at a pixel.  Steps t > 1: f = p * conf'.  FIRST: p0 =
// (1-m)*pred_init + m*dep [clamped], conf' = (1-m)*conf + m, m = dep > 0
// (nlspnmodel.py:328-348), f = p0 * conf'.
template <bool FIRST>
__device__ __forceinline__ float make_f(float p, float c, float d, bool has_conf, bool preserve, bool clip) {
    if (FIRST) {
        const float m = d > 0.f ? 1.f : 0.f;
        if (preserve) {
            p = (1.0f - m) * p + m * d;
            c = (1.0f - m) * c + m;
        }
        if (clip) p = clamp0(p);
    }
    return has_conf ? p * c : p;
}

template <typename T, bool FIRST>
__device__ __forceinline__ float fetch_f(rsrc_t rp, rsrc_t rc, rsrc_t rd, bool has_conf, bool preserve, bool clip,
                                         unsigned q) {
    float v[1], c[1] = {1.f}, d[1] = {0.f};
    BVec<T, 1>::load(rp, q, 0u, v);
    if (has_conf) BVec<T, 1>::load(rc, q, 0u, c);
    if (FIRST && preserve) BVec<T, 1>::load(rd, q, 0u, d);
    return make_f<FIRST>(v[0], c[0], d[0], has_conf, preserve, clip);
}

// Workgroup barrier that orders LDS only (no global-memory release): it waits
// lgkmcnt(0) but leaves the streamed global loads in flight across the barrier,
// so their latency overlaps staging and the first taps (the full __syncthreads
// fence would drain vmcnt(0) here and serialise load and compute phases).
__device__ __forceinline__ void lds_barrier() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// a (f16, low half) * b + c in f32 with one rounding (v_fma_mix_f32; the f16 operand is
// converted exactly inside the instruction).  Inline asm: left to itself the SLP
// vectoriser pairs two of these into two converts + a v_pk_fma_f32.
__device__ __forceinline__ float fma_mix_lo(_Float16 a, float b, float c) {
    float r;
    asm("v_fma_mix_f32 %0, %1, %2, %3 op_sel_hi:[1,0,0]" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}

// fp16-storage offset steps: at least this many waves per SIMD (80 VGPRs), so that the
// tap arithmetic of some waves overlaps the plane loads of others
#ifndef NLSPN_STEP_F16_WAVES
#define NLSPN_STEP_F16_WAVES 6
#endif
constexpr int kStepF16Waves = NLSPN_STEP_F16_WAVES;
#ifndef NLSPN_STEP_PAIR
#define NLSPN_STEP_PAIR 0
#endif
// offset branch: paired window copies (ds_read_b64); A/B builds only — C5 measured 2.5 %
// slower with them (the second copy's staging writes and the copy select cost more than the
// halved footprint reads save, profiles/r04/ab_r4e_nyu_k16.txt)
constexpr bool kStepPair = NLSPN_STEP_PAIR != 0;

// KH x KW taps; TH x TW tile; PX px per thread; window radii RY/RX; SV = staging
// vector width (4 requires W % 4 == 0 and RX % 4 == 0); PRE = issue every tap's
// planes before the staging barrier (else inside pass A); FIRST = fused prologue.
template <typename T, int KH, int KW, int TH, int TW, int PX, int RY, int RX, int SV, bool OFFSET, bool PRE,
          bool FIRST>
__global__ void __launch_bounds__(TH * TW / PX, (sizeof(T) == 2 && OFFSET && !FIRST && PX == 1 && SV == 4 && KH * KW <= 17) ? kStepF16Waves : 1)
    prop_step_kernel(StepArgs a) {
    constexpr int NT = TH * TW / PX;
    constexpr int KK = KH * KW, REF = KK / 2, K = KK - 1;
    constexpr int PH = (KH - 1) / 2, PW = (KW - 1) / 2;
    constexpr int WH = TH + 2 * RY, WW = TW + 2 * RX;
    constexpr int TPR = TW / PX;
    static_assert(TW % PX == 0 && NT % 64 == 0, "tile/thread shape");
    static_assert(OFFSET || (KH == 3 && KW == 3 && RY == 1 && RX == 1), "no-offset branch is 3x3 replicate");
    static_assert(!OFFSET || (RY > PH && RX > PW), "window must cover the tap base grid");
    static_assert(SV == 1 || (OFFSET && RX % 4 == 0 && WW % 4 == 0), "vector staging alignment");
    static_assert(!FIRST || PRE, "the fused prologue normalises all K taps up front");
    constexpr int WV = WW / SV;                  // staging vectors per window row
    constexpr int NV = WH * WV;                  // staging vectors per window
    constexpr int SIT = (NV + NT - 1) / NT;      // staging vectors per thread
    constexpr unsigned ES = sizeof(T);
    constexpr int NW = NT / 64;
    // the window, then one word per wave: "this wave staged a non-finite f".  PAIR (offset
    // branch): a second copy shifted by one cell (winB[i] = win[i + 1], from WP on), so any
    // horizontal pair of a bilinear footprint is ONE 8-byte-aligned ds_read_b64 from one of
    // the two copies (the resident kernel's form) instead of a ds_read2_b32 (two 32-lane
    // passes): half the LDS instructions per footprint row.
    constexpr bool PAIR = OFFSET && kStepPair;
    constexpr int WP = (WH * WW + NW + 4) & ~3;  // copy B's base (16-B aligned), behind the flags
    __shared__ __attribute__((aligned(16))) float win[PAIR ? WP + WH * WW + 4 : WH * WW + NW];
    float *winB = win + WP;  // winB[i] = cell i + 1 (winB[-1] is padding): an odd cell's pair is 8-B aligned

    const int H = a.H, W = a.W;
    const long long HW = (long long)H * W;
    int tile = xcd_remap(blockIdx.x, gridDim.x);
    const int tx = tile % a.tiles_x;
    tile /= a.tiles_x;
    const int ty = tile % a.tiles_y;
    const int b = tile / a.tiles_y;
    const int x0 = tx * TW, y0 = ty * TH;
    const int wy0 = y0 - RY, wx0 = x0 - RX;

    if (a.zero_words && blockIdx.x == 0)  // step 1 (either form) zeroes the resident kernel's words
        for (int i = threadIdx.x; i < a.nzero; i += NT)
            __hip_atomic_store(a.zero_words + i, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const bool has_conf = a.conf != nullptr;
    const bool preserve = (a.flags & kPreserve) != 0;
    const bool clip = (a.flags & kAlwaysClip) != 0;
    const T *pbase = static_cast<const T *>(a.p_in) + b * HW;
    const rsrc_t rp = make_rsrc(pbase);
    const rsrc_t rc = make_rsrc(has_conf ? static_cast<const T *>(a.conf) + b * HW : pbase);
    const rsrc_t rd = make_rsrc(preserve ? static_cast<const T *>(a.dep) + b * HW : pbase);

    const int ly = threadIdx.x / TPR, lx = (threadIdx.x % TPR) * PX;
    const int y = y0 + ly, xb = x0 + lx;
    const bool active = (y < H) && (xb < W);  // PX>1 requires W % PX == 0: groups are all-in or all-out
    const unsigned pix = active ? (unsigned)(y * W + xb) : 0u;  // inactive lanes load pixel 0 (in bounds)
    const unsigned vpix = pix * ES;            // per-lane byte offset, shared by every plane
    const unsigned plane_bytes = (unsigned)HW * ES;

    // MIX (fp16 storage, one pixel per lane, offset steps after the first): the plane values
    // stay fp16 in registers and enter the arithmetic through v_fma_mix_f32 (f16 operands
    // converted exactly inside the instruction); see the streamed loads below.
#ifndef NLSPN_STEP_NOMIX
    constexpr bool MIX = sizeof(T) == 2 && PX == 1 && OFFSET && PRE && !FIRST;
#else
    constexpr bool MIX = false;  // A/B builds only
#endif
    // MIX staging (SV = 4): cells outside the image load from an out-of-range buffer offset,
    // which the buffer unit returns as zeros (= the zero padding, no select per cell), and
    // f = p * conf' is one v_fma_mix_f32 (an f16 x f16 product is exact in f32: fma(p, c, 0)
    // == p * c but for the sign of a zero product, which never reaches a result — the
    // bilinear sums and the tap accumulator start at +0).
#ifndef NLSPN_STEP_NOMIXS
    constexpr bool MIXS = MIX && SV == 4;
#else
    constexpr bool MIXS = false;  // A/B builds only
#endif
    constexpr unsigned kOOB = 0x80000000u;  // >= num_records (make_rsrc): reads as 0
    float sp[SIT][SV], sc[SIT][SV], sd[FIRST ? SIT : 1][SV];
    f16x4 sp16[MIXS ? SIT : 1], sc16[MIXS ? SIT : 1];
    bool sin[SIT];
    // ---- 1. staging loads (first): the window's p, conf [, dep], clamped addresses
#pragma unroll
    for (int it = 0; it < SIT; ++it) {
        const int i = threadIdx.x + it * NT;
        const int ii = i < NV ? i : NV - 1;
        const int r = ii / WV, c = (ii - r * WV) * SV;
        int gy = wy0 + r, gx = wx0 + c;
        if (OFFSET) sin[it] = i < NV && gy >= 0 && gy < H && gx >= 0 && gx < W;  // zero padding outside
        else sin[it] = i < NV;                                                   // replicate padding
        if constexpr (MIXS) {
            const unsigned q = sin[it] ? (unsigned)(gy * W + gx) * ES : kOOB;
            sp16[it] = __builtin_bit_cast(f16x4, __builtin_amdgcn_raw_buffer_load_b64(rp, q, 0u, 0));
            if (has_conf) sc16[it] = __builtin_bit_cast(f16x4, __builtin_amdgcn_raw_buffer_load_b64(rc, q, 0u, 0));
            continue;
        }
        gy = gy < 0 ? 0 : (gy > H - 1 ? H - 1 : gy);
        gx = gx < 0 ? 0 : (gx > W - SV ? W - SV : gx);
        const unsigned q = (unsigned)(gy * W + gx) * ES;
        BVec<T, SV>::load(rp, q, 0u, sp[it]);
        if (has_conf) BVec<T, SV>::load(rc, q, 0u, sc[it]);
        if (FIRST && preserve) BVec<T, SV>::load(rd, q, 0u, sd[FIRST ? it : 0]);
    }

    // ---- 2. streamed per-pixel loads: K affinity planes, 2K offset planes, dep [, conf].
    // MIX: the affinity and offset planes stay fp16: x + y as fma(x, 1, y) and col = v * a
    // as fma(v, a, 0) — the same roundings, and col's zero sign never reaches the
    // accumulator (it starts at +0) — so 3 VALU per tap fewer than converting first.
    using PT = typename std::conditional<MIX, _Float16, float>::type;
    PT av[PRE ? K : 1][PX];
    PT dh[PRE ? K : 1][PX], dw[PRE ? K : 1][PX];
    float dv[PX], cv[PX];
#pragma unroll
    for (int p = 0; p < PX; ++p) dv[p] = cv[p] = 0.f;
    const rsrc_t ra = make_rsrc(static_cast<const T *>(a.aff) + b * a.aff_bs);
    const rsrc_t ro = make_rsrc(OFFSET ? static_cast<const T *>(a.off) + b * a.off_bs : static_cast<const T *>(a.aff));
    auto load_pt = [&](rsrc_t r, unsigned so, PT (&dst)[PX]) {
        if constexpr (MIX) {
            dst[0] = __builtin_bit_cast(_Float16, __builtin_amdgcn_raw_buffer_load_b16(r, vpix, so, 0));
        } else {
            float f[PX];
            BVec<T, PX>::load(r, vpix, so, f);
#pragma unroll
            for (int p = 0; p < PX; ++p) dst[p] = f[p];
        }
    };
    if (PRE) {
#pragma unroll
        for (int k = 0; k < K; ++k) {
            // FIRST: raw affinity (K planes); otherwise the normalised (K+1)-plane layout
            const unsigned ap = FIRST ? (unsigned)k : (unsigned)(k < REF ? k : k + 1);
            load_pt(ra, ap * plane_bytes, av[PRE ? k : 0]);
            if (OFFSET) {
                const unsigned c = a.off_raw ? k : (k < REF ? k : k + 1);
                load_pt(ro, (2 * c) * plane_bytes, dh[PRE ? k : 0]);
                load_pt(ro, (2 * c + 1) * plane_bytes, dw[PRE ? k : 0]);
            }
        }
    }
    float one = 1.0f;  // opaque 1: fma(x, one, y) stays an fma (mixed precision), not an add
    asm volatile("" : "+v"(one));
    if (preserve) BVec<T, PX>::load(rd, vpix, 0u, dv);
    if (FIRST && has_conf) BVec<T, PX>::load(rc, vpix, 0u, cv);

    // ---- 3. finish staging into LDS (waits for the staging loads only)
    // Every tile notes whether its window holds a non-finite f.  Only then can
    //  * an invalid tap at exactly h == -1 / w == -1 (0 * f over the in-image row /
    //    column; edge tiles) differ from the reference's val = 0 (pass B below), and
    //  * the reference tap differ from its one-cell read: the reference samples all four
    //    corners of the integer point with weights (1, 0, 0, 0) (.cuh:37-52), so a
    //    non-finite right / lower neighbour makes it NaN (0 * inf) — the four-corner form
    //    below (offset branch only: the no-offset branch multiplies its centre cell,
    //    nlspnmodel.py:215-222).
    const bool edge_tile = wy0 < 0 || wx0 < 0;
    bool nonfin = false;
    const auto stage_store = [&](int it, const float (&v)[SV]) {
        if constexpr (OFFSET) {
#pragma unroll
            for (int e = 0; e < SV; ++e) nonfin |= !__builtin_isfinite(v[e]);
        }
        const int i = threadIdx.x + it * NT;
        const int r = i / WV, c = (i - r * WV) * SV;
        if constexpr (SV == 4)
            *reinterpret_cast<float4 *>(&win[r * WW + c]) = make_float4(v[0], v[1], v[2], v[3]);
        else
            win[r * WW + c] = v[0];
        if constexpr (PAIR) {  // copy B: cell (r, c + e) at winB[r * WW + c + e - 1]
            const int li = r * WW + c;
            if constexpr (SV == 4) {
                winB[li - 1] = v[0];
                *reinterpret_cast<float2 *>(&winB[li]) = make_float2(v[1], v[2]);  // li % 4 == 0
                winB[li + 2] = v[3];
            } else {
                winB[li - 1] = v[0];
            }
        }
    };
    if constexpr (MIXS) {  // out-of-image cells loaded as zeros: 0 * 0 = +0
        // two loops under the uniform has_conf branch (one select per cell otherwise)
        if (has_conf) {
#pragma unroll
            for (int it = 0; it < SIT; ++it) {
                if (threadIdx.x + it * NT >= NV) continue;
                float v[SV];
#pragma unroll
                for (int e = 0; e < SV; ++e) v[e] = __builtin_fmaf((float)sp16[it][e], (float)sc16[it][e], 0.0f);
                stage_store(it, v);
            }
        } else {
#pragma unroll
            for (int it = 0; it < SIT; ++it) {
                if (threadIdx.x + it * NT >= NV) continue;
                float v[SV];
#pragma unroll
                for (int e = 0; e < SV; ++e) v[e] = (float)sp16[it][e];
                stage_store(it, v);
            }
        }
    } else {
#pragma unroll
        for (int it = 0; it < SIT; ++it) {
            if (threadIdx.x + it * NT >= NV) continue;
            float v[SV];
#pragma unroll
            for (int e = 0; e < SV; ++e) {
                const float f = make_f<FIRST>(sp[it][e], has_conf ? sc[it][e] : 1.f,
                                              FIRST && preserve ? sd[FIRST ? it : 0][e] : 0.f, has_conf, preserve, clip);
                v[e] = sin[it] ? f : 0.f;
            }
            stage_store(it, v);
        }
    }
    {
        const bool wnf = __builtin_amdgcn_ballot_w64(nonfin) != 0;
        if ((threadIdx.x & 63) == 0) win[WH * WW + threadIdx.x / 64] = wnf ? 1.f : 0.f;
    }
    lds_barrier();
    if (!active) return;  // no barrier below
    bool win_nf = false;  // tile-uniform: the window holds a non-finite f
#pragma unroll
    for (int w = 0; w < NW; ++w) win_nf |= win[WH * WW + w] != 0.f;
    const bool edge_fix = edge_tile && win_nf;

    // ---- FIRST: the prologue's per-pixel outputs (normalised affinity, conf', offsets)
    float fref_a[PX];  // FIRST: reference-tap weight from the normalisation (== 1 - sum, same order)
    if constexpr (FIRST) {
        normalize_taps<K, PX>(av, fref_a, a.kind, *a.gamma);
        const rsrc_t rao = make_rsrc(static_cast<T *>(a.aff_out) + b * (K + 1) * HW);
#pragma unroll
        for (int c = 0; c < K + 1; ++c)
            BVec<T, PX>::store(rao, vpix, (unsigned)c * plane_bytes, c == REF ? fref_a : av[c < REF ? c : c - 1]);
        if (has_conf) {
            float co[PX];
#pragma unroll
            for (int p = 0; p < PX; ++p) {
                const float m = dv[p] > 0.f ? 1.f : 0.f;
                co[p] = preserve ? (1.0f - m) * cv[p] + m : cv[p];
            }
            BVec<T, PX>::store(make_rsrc(static_cast<T *>(a.conf_out) + b * HW), vpix, 0u, co);
        }
        if (OFFSET && a.off_out) {
            const rsrc_t roo = make_rsrc(static_cast<T *>(a.off_out) + b * 2 * (K + 1) * HW);
            float z[PX];
#pragma unroll
            for (int p = 0; p < PX; ++p) z[p] = 0.f;
#pragma unroll
            for (int c = 0; c < K + 1; ++c) {
                const int k = c < REF ? c : c - 1;
                // streaming (nt): the inserted offsets are an output only, never re-read here
                BVec<T, PX>::template store<kNT>(roo, vpix, (unsigned)(2 * c) * plane_bytes, c == REF ? z : dh[PRE ? k : 0]);
                BVec<T, PX>::template store<kNT>(roo, vpix, (unsigned)(2 * c + 1) * plane_bytes,
                                                 c == REF ? z : dw[PRE ? k : 0]);
            }
        }
    }

    // ---- 4. taps.  Pass A (LDS only, no divergent global loads, so the
    // compiler's vmcnt waits stay counted per tap): col[k] = bilinear * a_k for
    // every tap whose 2x2 footprint is inside the window (one range test; invalid taps
    // there sample zeros, see lo_h below); a lane with a tap outside it sets `anyout`
    // (a lane mask, no vector work per tap).  Pass B (rare): such lanes re-read their
    // offsets from cache, skip the taps pass A served (the same test on the same values),
    // test validity (invalid: col = 0 * a stands) and sample the valid ones from
    // L2/global with the reference's per-corner checks.  Then
    // accumulate in tap index order with the reference tap (K/2) weighted
    // 1 - sum(others) (nlspnmodel.py:262-263): the reference's summation order,
    // whichever pass served a tap.  col = val * a then acc += col is the same
    // IEEE sequence as acc += val * a (no contraction).
    float col[K][PX], asum[PX];
#pragma unroll
    for (int p = 0; p < PX; ++p) asum[p] = 0.f;
    const float Hf = (float)H, Wf = (float)W;
    const float yb_f = (float)(y - PH), xb_f = (float)(xb - PW);  // |values| < 2^24: exact
    // One range test per tap: the footprint rows floor(h), floor(h)+1 lie in the window iff
    // wy0 <= h < wy0 + WH - 1 (likewise w), tested as the bits of h - wy0 (an unsigned
    // compare) below those of WH - 1: a negative difference (sign bit), NaN
    // and anything >= WH - 1 fail, and rounding can only fail a tap that is in range
    // (pass B serves it exactly).  The window holds zeros outside the image, so
    // an INVALID tap (outside (-1, H) x (-1, W), .cuh:180) whose footprint is in the
    // window samples exactly +0 there — the reference's val = 0 — except at h == -1 or
    // w == -1 exactly, where the in-image row / column enters with weight 0 (0 * f, NaN
    // for a non-finite f): when an edge tile's window holds a non-finite f (edge_fix,
    // tile-uniform, from the staging) every lane runs pass B, which zeroes those taps —
    // no per-tap test on the common path (an in-loop test costs 3 VALU per tap; a re-read
    // fix-up after pass A measured 14 % slower at C5, profiles/r03/ab_step_ablation_v1.txt).
    // A tap outside the window (or NaN) goes to pass B, which tests validity first.
    const float lo_h = (float)wy0, lo_w = (float)wx0;
    constexpr unsigned kLimH = __builtin_bit_cast(unsigned, (float)(WH - 1));
    constexpr unsigned kLimW = __builtin_bit_cast(unsigned, (float)(WW - 1));
    // window byte offset of the footprint's top-left cell, from the floors in exact float
    // arithmetic (small integers): 4 (floor(h) - wy0) WW + 4 (floor(w) - wx0)
    const float wofs = -4.f * (float)(wy0 * WW + wx0);
    bool anyout = edge_fix;  // this lane has a tap outside the window (pass B)
    // small K (3x3): also a wave mask per tap (SGPRs), so pass B skips, wave-uniformly, the
    // taps no lane of the wave has outside the window (a 3x3 step's 8-cell halo leaves ~1/3
    // of its waves with some out-of-window tap at N(0, 2^2) offsets)
    constexpr bool TAPMASK = OFFSET && K * PX <= 8;
    uint64_t tapout[TAPMASK ? K * PX : 1];
    const auto tap_coords = [&](int k, int p, PT dh_, PT dw_, float &h_im, float &w_im) {
        const int t = k < REF ? k : k + 1;
        const int i = t / KW, j = t % KW;
        // modulated_deform_im2col_cuda.cuh:178-189: the tap's base coordinates as exact
        // float sums of small integers (one add per tap instead of an integer add and a
        // convert): the same values as (float)(y - PH + i) and (float)(xb + p - PW + j)
        const float hb = i == 0 ? yb_f : yb_f + (float)i;  // yb_f + 0 == yb_f: never -0
        const float wb = xb_f + (float)(p + j);
        if constexpr (MIX) {
            h_im = fma_mix_lo(dh_, one, hb);
            w_im = fma_mix_lo(dw_, one, wb);
        } else {
            h_im = hb + (float)dh_;
            w_im = wb + (float)dw_;
        }
    };
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const int t = k < REF ? k : k + 1;
        const int i = t / KW, j = t % KW;
        PT ak[PX], tdh[PX], tdw[PX];
        if (PRE) {
#pragma unroll
            for (int p = 0; p < PX; ++p) {
                ak[p] = av[PRE ? k : 0][p];
                tdh[p] = dh[PRE ? k : 0][p];
                tdw[p] = dw[PRE ? k : 0][p];
            }
        } else if constexpr (!MIX) {
            BVec<T, PX>::load(ra, vpix, (unsigned)t * plane_bytes, ak);
            if (OFFSET) {
                const unsigned c = a.off_raw ? k : t;
                BVec<T, PX>::load(ro, vpix, (2 * c) * plane_bytes, tdh);
                BVec<T, PX>::load(ro, vpix, (2 * c + 1) * plane_bytes, tdw);
            }
        }
#pragma unroll
        for (int p = 0; p < PX; ++p) {
            if constexpr (MIX) {  // asum += a as one v_fma_mix_f32 (a * 1 + asum, a read as f16)
                asum[p] = fma_mix_lo(ak[p], one, asum[p]);
            } else {
                asum[p] += ak[p];
            }
            if (!OFFSET) {
                col[k][p] = win[(ly + RY + i - 1) * WW + lx + p + RX + j - 1] * ak[p];
                continue;
            }
            float h_im, w_im;
            tap_coords(k, p, tdh[p], tdw[p], h_im, w_im);
            const bool in = __builtin_bit_cast(unsigned, h_im - lo_h) < kLimH && __builtin_bit_cast(unsigned, w_im - lo_w) < kLimW;
            anyout |= !in;
            if constexpr (TAPMASK) tapout[k * PX + p] = __builtin_amdgcn_ballot_w64(!in);
            float v = 0.f;
            if (in) {
                // mdmcn_im2col_bilinear (.cuh:24-54), in the window: (float)h_low == fh, so
                // h_im - fh is the reference's h_im - (float)h_low (.cuh:35-36).  Scalar f32:
                // the same sequence as v_pk_fma / v_pk_mul pairs measured 2 % slower at C5
                // (profiles/r03/ab_step_packed_vs_scalar_v1.txt; packed f32 issues at more
                // than two scalar slots on gfx950), so this file is built without SLP packing
                const float fh = floorf(h_im), fw = floorf(w_im);
                const float lh = h_im - fh, lw = w_im - fw, hh = 1.f - lh, hw = 1.f - lw;
                const unsigned bo = (unsigned)__builtin_fmaf(fh, (float)(4 * WW), __builtin_fmaf(fw, 4.f, wofs));
                const float w1 = hh * hw, w2 = hh * lw, w3 = lh * hw, w4 = lh * lw;
                if constexpr (PAIR) {
                    // an odd cell's pair is in copy B, one cell lower: + 4 * (WP - 1) bytes
                    const unsigned ba = bo + (bo & 4u) * (unsigned)(WP - 1);
                    const float *s = reinterpret_cast<const float *>(reinterpret_cast<const char *>(win) + ba);
                    const float2 s01 = *reinterpret_cast<const float2 *>(s);
                    const float2 s23 = *reinterpret_cast<const float2 *>(s + WW);
                    v = (w1 * s01.x + w2 * s01.y + w3 * s23.x + w4 * s23.y);
                } else {
                    const float *s = reinterpret_cast<const float *>(reinterpret_cast<const char *>(win) + bo);
                    v = (w1 * s[0] + w2 * s[1] + w3 * s[WW] + w4 * s[WW + 1]);
                }
            }
            col[k][p] = MIX ? __builtin_fmaf(v, (float)ak[p], 0.f) : v * (float)ak[p];  // .cuh:189 col = val * mask
        }
    }
    if (OFFSET && anyout) {  // pass B: the lane's taps outside the window, offsets re-read
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const int t = k < REF ? k : k + 1;
            const int i = t / KW, j = t % KW;
#pragma unroll
            for (int p = 0; p < PX; ++p) {
                if constexpr (TAPMASK) {
                    if (!edge_fix && tapout[k * PX + p] == 0) continue;  // wave-uniform
                }
                const unsigned c = a.off_raw ? k : t;
                float o1[1], a1[1];
                BVec<T, 1>::load(ro, vpix + p * ES, (2 * c) * plane_bytes, o1);
                const float h_im = (float)(y - PH + i) + o1[0];
                BVec<T, 1>::load(ro, vpix + p * ES, (2 * c + 1) * plane_bytes, o1);
                const float w_im = (float)(xb + p - PW + j) + o1[0];
                if (edge_fix && (h_im == -1.f || w_im == -1.f)) {  // invalid (.cuh:180): val = 0
                    if (FIRST) a1[0] = av[PRE ? k : 0][p];
                    else BVec<T, 1>::load(ra, vpix + p * ES, (unsigned)t * plane_bytes, a1);
                    col[k][p] = 0.f * a1[0];
                    continue;
                }
                {  // served by pass A (the same test on the same values)
                    if (__builtin_bit_cast(unsigned, h_im - lo_h) < kLimH && __builtin_bit_cast(unsigned, w_im - lo_w) < kLimW)
                        continue;
                }
                // invalid (.cuh:180, NaN included): the reference's val = 0, already col = 0 * a above
                if (!(h_im > -1.f && w_im > -1.f && h_im < Hf && w_im < Wf)) continue;
                if (FIRST) a1[0] = av[PRE ? k : 0][p];  // normalised in registers above
                else BVec<T, 1>::load(ra, vpix + p * ES, (unsigned)t * plane_bytes, a1);
                const int h_low = (int)floorf(h_im), w_low = (int)floorf(w_im);
                const int h_high = h_low + 1, w_high = w_low + 1;
                const float lh = h_im - (float)h_low, lw = w_im - (float)w_low;
                const float hh = 1.f - lh, hw = 1.f - lw;
                const int r0 = h_low * W, r1 = h_high * W;
                const float v1 = (h_low >= 0 && w_low >= 0)
                                     ? fetch_f<T, FIRST>(rp, rc, rd, has_conf, preserve, clip, (r0 + w_low) * ES) : 0.f;
                const float v2 = (h_low >= 0 && w_high <= W - 1)
                                     ? fetch_f<T, FIRST>(rp, rc, rd, has_conf, preserve, clip, (r0 + w_high) * ES) : 0.f;
                const float v3 = (h_high <= H - 1 && w_low >= 0)
                                     ? fetch_f<T, FIRST>(rp, rc, rd, has_conf, preserve, clip, (r1 + w_low) * ES) : 0.f;
                const float v4 = (h_high <= H - 1 && w_high <= W - 1)
                                     ? fetch_f<T, FIRST>(rp, rc, rd, has_conf, preserve, clip, (r1 + w_high) * ES) : 0.f;
                const float w1 = hh * hw, w2 = hh * lw, w3 = lh * hw, w4 = lh * lw;
                col[k][p] = (w1 * v1 + w2 * v2 + w3 * v3 + w4 * v4) * a1[0];
            }
        }
    }
    float acc[PX];
#pragma unroll
    for (int p = 0; p < PX; ++p) {
        // reference tap: zero offset, integer sample point -> bilinear weights exactly
        // (1, 0, 0, 0): its own cell, unless the window holds a non-finite f — then the
        // reference's four-corner sum (.cuh:52; zero-padded window = its bounds checks)
        const float aref = FIRST ? fref_a[p] : 1.0f - asum[p];
        const float *sr = &win[(ly + RY) * WW + lx + p + RX];
        const float vref = OFFSET && win_nf ? ((1.f * sr[0] + 0.f * sr[1]) + 0.f * sr[WW]) + 0.f * sr[WW + 1] : sr[0];
        const float cref = vref * aref;
        acc[p] = 0.f;
#pragma unroll
        for (int t = 0; t < KK; ++t) acc[p] += t == REF ? cref : col[t < REF ? t : t - 1][p];
    }

    // ---- 5. preserve-input blend (:355-357), clamp (:359-361), final clamp (:375-377)
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
    BVec<T, PX>::store(make_rsrc(static_cast<T *>(a.p_out) + b * HW), vpix, 0u, o);
    if (a.pred_out) BVec<T, PX>::store(make_rsrc(static_cast<T *>(a.pred_out) + b * HW), vpix, 0u, fin);
    if (a.poison) {  // raw bit stores (a float or half conversion would quiet the signalling NaN)
        const rsrc_t rq = make_rsrc(static_cast<T *>(a.poison) + b * HW);
#pragma unroll
        for (int p = 0; p < PX; ++p) {
            if constexpr (sizeof(T) == 4) __builtin_amdgcn_raw_buffer_store_b32(kPoison32, rq, vpix + p * ES, 0u, 0);
            else __builtin_amdgcn_raw_buffer_store_b16(kPoison16, rq, vpix + p * ES, 0u, 0);
        }
    }
}

}  // namespace nlspn
