// Resident propagation: iterations 2..T of the NLSPN loop in ONE launch per image
// group, with every iteration-invariant plane held on chip.
//
// Why: a per-iteration launch (nlspn_step.h) must re-read the invariant planes
// — K normalised affinities, 2K offsets, conf', dep: 27 fp32 planes = 108 of its
// 112 B/px at K=8 — every iteration, so it is HBM-bound at ~6 TB/s however it is
// tiled.  Those planes do not change between iterations (nlspnmodel.py:340-363
// re-uses offset / aff / confidence / dep), and a group of images whose planes fit
// the register files and LDS (C2: all 8 NYU images, 60 MB; C3: 2 of the 4 KITTI
// images) keeps them there:
//
//   * one workgroup per CU owns a RECTANGLE of pixel quads of one image (part
//     j = py * gx + px of a gy x gx grid of row bands x quad-column bands; parts
//     are dealt to XCDs in contiguous runs, so neighbouring parts share one); each
//     thread owns one quad (4 pixels of a row) and holds its tap geometry and dep
//     in VGPRs, its affinities and conf' in LDS, for the whole launch;
//   * the part's f window — every cell any valid tap of the part reads (found once:
//     offsets are invariant), zero outside the image — lives in LDS;
//   * per iteration only the previous depth plane moves: the window cells of
//     p_{t-1} owned by OTHER parts are loaded (hand-off, below), multiplied by conf'
//     into the window, the taps are sampled exactly as prop_step_kernel does (same
//     IEEE sequence: bit-identical), and p_t is stored.
//     Rectangular parts keep that staging to the window's rim: at C2 about a
//     third of the cells a full-width row band would restage.
//
// Hand-off: the data is the flag (the R2 form of cdna_hip_programming.md §6 Guideline 16,
// with a poison value as the "not yet" tag).  Every plane p_t a later iteration reads is
// POISONED — kResPoison32 / kResPoison16, signalling-NaN bit patterns that no arithmetic
// result has (IEEE mode quiets every NaN an instruction returns) — before it is written:
// plane 1 by step 1 (the kernel boundary orders it), plane t + 1 by each part for its own
// quads during iteration t, acknowledged (s_waitcnt vmcnt(0)) before the part stores plane
// t.  A consumer re-loads each cell it stages until it is not the poison.  Why a value that
// is not the poison is this call's p_t: the consumer read the same producer's cells of
// plane t - 1 one iteration earlier (the window and every tap are invariant, so a part
// reads the same cells every iteration) and waited for them, and the producer had made
// plane t's poison visible before it stored those (induction from plane 1).  Stores, per
// 128-B line of a plane (kResL2, round 6): `sc1` (write-through; MI355X_MICROARCH.md
// § inter-workgroup visibility) for an EXPORTED line — one that some part on another XCC
// reads (its published window meets the line) — and plain for every other line, which then
// stays in its XCD's L2 for the same-XCD readers.  Every part decides a line from the same
// published words (the windows and XCC ids of its image's parts), so all the quads of a line
// are stored the same way by whichever parts own them: a line is wholly L2-kept (producers
// and readers on one XCD) or wholly write-through.  The decision is the same for every plane
// of the call, so the induction above holds per line.  Without kResL2 every line is
// exported.  Loads of p: `sc1` (L1 bypassed).  Loads of bytes not written in this launch (conf', invariants) are
// plain.  Every plane is written once per call, so there is no write-after-read hazard, a
// part never waits for a whole neighbour part (only for the cells it stages), and a fast
// part may run ahead of parts that do not feed it.  Image groups run in turn inside one
// launch (ResArgs::ngroups; a part sets up group k + 1 as soon as it has stored its last
// iteration of group k, while other parts still finish group k).
//
// Residency: G = B * gy * gx workgroups, at most one per CU (the dynamic LDS
// request exceeds half a CU's LDS) and G <= CU count, so the whole grid is
// resident (the host serialises resident launches of one device across streams,
// nlspn_capi.hip res_guard).  Every spin is bounded: on timeout a part raises the
// abort word (sync[0]) and the device's host-mapped sticky status word
// (ResArgs::status, read by nlspn_resident_status without a device sync), and every
// part that sees the abort fills its own quads of the planes it has not written
// (and pred) with NaN before it exits: an aborted launch never looks valid.
#pragma once

#include "nlspn_common.h"
#include "nlspn_step.h"

namespace nlspn {

typedef __attribute__((address_space(1))) unsigned gu32;
typedef const __attribute__((address_space(3))) f32x2 ldsf2;  // an LDS float pair by byte address
__device__ __forceinline__ float2 lds_pair(unsigned byte_addr) {
    const f32x2 v = *reinterpret_cast<ldsf2 *>((size_t)byte_addr);
    return make_float2(v[0], v[1]);
}

struct ResArgs {
    const void *conf;   // conf' of this launch's images (planes H*W apart), or null (conf_prop off)
    const void *dep;    // planes H*W apart, or null (preserve off)
    const void *aff;    // normalised affinity, (K+1) planes per item, contiguous (aff_out)
    const void *off;    // offsets, batch stride off_bs: raw 2K planes, or inserted 2(K+1) (flags kResOffInserted)
    void *pred_inter;   // plane (t, b) at t * tstride + b * H * W: iteration t reads t-1, writes t
    void *pred;         // planes H*W apart: max(p_T, 0) (nlspnmodel.py:375-377)
    unsigned *sync;     // [0] abort word, per part a line with its XCC id (+1); zeroed by step 1
    unsigned *status;   // host-mapped sticky abort flag of the device (nlspn_resident_status), or null
    long long off_bs;   // elements
    long long tstride;  // elements between iteration planes (B_section * H * W)
    int B, H, W, T;     // B: images of this launch
    int gy, gx;         // parts per image: gy row bands x gx quad-column bands
    int win_cells;      // LDS cells per copy of the f window: res_win_cells(blockDim.x)
    unsigned epoch;     // tag base of this launch's XCC-id words (k * (T + 1) for image group k)
    unsigned flags;
    unsigned dbg;       // experiments build only (NLSPN_RES_DBG, exp_dbg; 0 and folded away in the
                        // product library): 1 no spin on staged cells, 2 no staging, 4 no taps,
                        // 8 trace: s_memrealtime stamps per part and iteration into `pred` (then
                        // invalid; the host checks it is large enough), 32 part 0 aborts at its first
                        // staging (tests of the error path), 64 no general path (wrong results for
                        // taps outside the window: tests that it is taken)
    // image groups this launch runs in turn (0 or 1: one).  Group g is images
    // g*B .. g*B + B - 1 from the base pointers above: a part starts group g + 1 as soon
    // as it has stored its last iteration of group g, with no launch boundary between the
    // groups.
    int ngroups;
    // The output dict's inserted offsets (nlspnmodel.py:324 `offset`: 2(K+1) planes per item,
    // contiguous), or null (step 1 writes them): this launch copies them from the raw `off`
    // planes, one output plane per iteration, so the copy rides the latency-bound loop instead
    // of step 1's HBM-bound pass (raw offset layout only).
    void *off_out;
    // The forward prologue inside the launch (flags kResFirst, round 5): no step-1 launch.  The
    // setup reads the RAW head outputs — `aff` then holds K raw affinity planes per item at
    // batch stride aff_bs, `conf_raw` the raw confidence, `pinit` pred_init — normalises the
    // affinities itself (_affinity_normalization + _aff_insert, nlspnmodel.py:179-201, 261-269),
    // builds conf' (:328-334) and stores it to `conf` (conf_out, the output dict's confidence and
    // the rim staging's conf' source), and iteration 1 runs as the loop's t = 0 from
    // f0 = p0 * conf' of the raw inputs (:341-348).  The output dict's normalised affinity is
    // written to `aff_out` by the setup.
    const void *pinit;
    const void *conf_raw;
    const float *gamma;
    void *aff_out;
    long long aff_bs;
    int kind;
};

typedef const __attribute__((address_space(4))) ResArgs ResArgsK;  // the kernarg segment's ResArgs

constexpr int kResMaxNT = 768;                  // launch bound (threads per part)
constexpr int kResSMax = 1;                      // staging quads per thread per round
constexpr int kResPre = 2;                       // the prologue's window staging: quads per thread in flight
#ifndef NLSPN_RES_SPIN_SLEEP
#define NLSPN_RES_SPIN_SLEEP 1  // s_sleep between a staging spin's re-loads (A/B builds: 0, 2, 4)
#endif
#ifndef NLSPN_RES_WTRACE
#define NLSPN_RES_WTRACE 0  // trace builds: per-wave stamps too (they cost the loop 16 B/lane of scratch)
#endif
constexpr bool kResWTrace = NLSPN_RES_WTRACE;
constexpr int kResRY = 8, kResRXQ = 2;           // fallback window halo (3x3): rows, quad columns
// the fallback halo of a kh x kw geometry: the 3x3 one plus the taps' wider base reach
__host__ __device__ constexpr int res_ry(int kh) { return kResRY + (kh > 3 ? (kh - 3) / 2 : 0); }
__host__ __device__ constexpr int res_rxq(int kw) { return kResRXQ + (kw > 3 ? ((kw - 3) / 2 + 3) / 4 : 0); }
// pixels per thread of a kh x kw geometry (a quad's 4 pixels as 1, 2 or 4 threads): the tap
// geometry of K x PX tap-pixels lives in registers (2 per tap-pixel + half a packed index), so
// PX shrinks as K grows — 3x3 (K = 8): 4; 1x17 (K = 16): 2; 5x5 (K = 24): 1; 0: not resident
// (7x7, K = 48: 4 x 48 registers of tap geometry alone pass the 168-VGPR cap)
__host__ __device__ constexpr int res_px(int kh, int kw) {
    return (kh == 3 && kw == 3) ? 4 : (kh == 1 && kw == 17) ? 2 : (kh == 5 && kw == 5) ? 1 : 0;
}
// bytes of a thread's LDS rows: the K affinities, 1 - sum, conf', dep of its PX pixels
__host__ __device__ constexpr int res_row_bytes(int K, int px) { return (K + 3) * px * 4; }
constexpr int kResPadX = 4;                      // zero columns either side of the window (keeps 16-B rows)
// The export list (per-line write-through, below): at most kResNC foreign windows per part
// (the parts on another XCC whose windows reach this part's 128-B lines), two words each
constexpr int kResNC = 28;
constexpr int kResCtl = 8 + 2 * kResNC;          // LDS control words ahead of the window
constexpr int kResAS = 11;                       // float4 per thread (3x3): K = 8 affinities, 1 - sum, conf', dep
constexpr int kResLds = 160 * 1024;              // LDS per CU

// LDS cells per copy of the f window for nt threads: what the per-thread rows leave,
// a multiple of 4 (16-B aligned copies), both copies addressable by 16-bit indices.
// (A PITCH build's copies stay within 16-bit byte addresses: at most 8,184 cells.)
__host__ __device__ constexpr int res_win_cells(int nt, int row_bytes = 16 * kResAS, int cap = 32764) {
    return ((kResLds - 4 * kResCtl - row_bytes * nt) / 8 / 4 * 4) < cap
               ? ((kResLds - 4 * kResCtl - row_bytes * nt) / 8 / 4 * 4)
               : cap;
}

// the compile-time window pitch of a fixed-thread-count build (0: the pitch is the window's
// width, a run-time value): 128 cells for 576 threads, whose two window copies span
// 2 * 7,740 cells = 61.9 KB of byte addresses (below 64 KB: 16-bit)
__host__ __device__ constexpr int res_pitch(int ntc) { return ntc == 576 ? 128 : 0; }
// the window cells per copy of a build (threads ntc, 0: nt at run time) and geometry
__host__ __device__ constexpr int res_build_cells(int ntc, int nt, int K, int px) {
    return res_win_cells(ntc ? ntc : nt, res_row_bytes(K, px), res_pitch(ntc) ? 8184 : 32764);
}
static_assert(4 * (kResCtl + 2 * res_win_cells(576)) < 65536, "576-thread window byte addresses need 16 bits");
static_assert(kResCtl % 4 == 0, "the window starts 16-B aligned");

constexpr unsigned kResSpinLimit = 1u << 22;     // ~seconds of polling before giving up
#ifndef NLSPN_RES_NOGP
constexpr bool kResGeneralPath = true;
#else
constexpr bool kResGeneralPath = false;  // experiment only: wrong results for taps outside the window
#endif
constexpr unsigned kSc1 = 16u;                   // buffer-instruction aux bit: sc1 (write-through / L1 bypass)
constexpr unsigned kResOffInserted = 0x100u;      // ResArgs::flags: offsets in the inserted 2(K+1)-plane layout
constexpr unsigned kResL2 = 0x400u;               // ResArgs::flags: same-XCD hand-offs may stay in the XCD's L2
constexpr unsigned kResFirst = 0x800u;            // ResArgs::flags: the prologue and iteration 1 in the launch
// The sync workspace: one 128-B line per word group — [0] the abort word, [1] the count of
// parts that have finished, then per part i (blockIdx) the line kResLine * (1 + i) holding
// (word + 1) its tagged XCC id.  No two parts share a line, so a line is only ever written
// from one XCD.  The words are zero when a launch starts and zero again when it ends: the
// last part to finish (the count) clears them (res_finish), so a plan's launches need no
// clearing pass (the host clears a workspace once, before its first resident launch).
constexpr int kResLine = 32;
// "not yet written" values of the handed-off planes (nlspn_step.h kPoison32 / kPoison16,
// also stored by step 1): signalling NaNs (quiet bit clear), which no arithmetic result is
// (an instruction returns a NaN quieted), so a computed p_t never equals them
constexpr unsigned kResPoison32 = kPoison32;
constexpr unsigned short kResPoison16 = kPoison16;

// q = k / d for 0 <= k < 2^22, d >= 1, by the float reciprocal rd = 1/d plus one
// correction step (the product is within 1 of the quotient at these sizes).
__device__ __forceinline__ int res_div(int k, int d, float rd) {
    int q = (int)((float)k * rd);
    const int r = k - q * d;
    q += r < 0 ? -1 : (r >= d ? 1 : 0);
    return q;
}

// Merges lane spans (rows mn..mx, columns cmn..cmx) of the lanes with `on` into
// ctl[1..4]: a wave reduction first, then one LDS atomic per wave and bound (576
// lanes' atomics on 4 words serialise: 4.7 us of the setup at C2).
__device__ __forceinline__ void res_span_merge(int *ctl, bool on, int mn, int mx, int cmn, int cmx) {
    if (!on) { mn = cmn = 0x7fffffff; mx = cmx = -0x7fffffff; }
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        mn = min(mn, __shfl_xor(mn, d));
        mx = max(mx, __shfl_xor(mx, d));
        cmn = min(cmn, __shfl_xor(cmn, d));
        cmx = max(cmx, __shfl_xor(cmx, d));
    }
    if ((threadIdx.x & 63) == 0 && mn <= mx) {
        atomicMin(&ctl[1], mn); atomicMax(&ctl[2], mx); atomicMin(&ctl[3], cmn); atomicMax(&ctl[4], cmx);
    }
}

// A part's exit, once every wave of it has made its last read of the sync words (the
// caller's barrier): one add to the finished-parts count; the part whose add completes the
// grid zeroes the abort word, the count and every part's XCC-id word for the next launch
// (every other part has made its last read before its own add).  Wave 0 only.
__device__ __forceinline__ void res_finish(gu32 *sync) {
    if (threadIdx.x >= 64) return;
    unsigned done = 0;
    if (threadIdx.x == 0) done = __hip_atomic_fetch_add(&sync[1], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    done = __builtin_amdgcn_readfirstlane(done);
    if (done != gridDim.x - 1) return;
    for (unsigned i = threadIdx.x; i < gridDim.x; i += 64)
        __hip_atomic_store(&sync[kResLine * (1 + i) + 1], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (threadIdx.x < 2) __hip_atomic_store(&sync[threadIdx.x], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// The trace's per-wave stamp pair of iteration t (dbg 8): after every part's five stamps
// per row (T + 1 rows: the setup, then iteration t in row t + 1), 12 pairs per part and row;
// wb = the wave's first thread (uniform); t = -1: row 0 (the wave's HW_ID)
__device__ __forceinline__ unsigned long long *res_wtrace(void *pred, int T, unsigned wb, int t) {
    return reinterpret_cast<unsigned long long *>(pred) + (size_t)gridDim.x * (T + 1) * 5 +
           ((size_t)blockIdx.x * (T + 1) + t + 1) * 24 + 2 * (wb >> 6);
}

// A value as storage type T holds it (fp32: itself; fp16: rounded), back in fp32.
template <typename T> __device__ __forceinline__ float round_to(float v);
template <> __device__ __forceinline__ float round_to<float>(float v) { return v; }
template <> __device__ __forceinline__ float round_to<__half>(float v) { return (float)(_Float16)v; }

template <typename T> struct ResVec;  // 4 contiguous elements <-> float[4], buffer access with cache bits
template <> struct ResVec<float> {
    template <unsigned AUX>
    static __device__ __forceinline__ void load(rsrc_t r, unsigned vo, unsigned so, float (&v)[4]) {
        const f32x4 q = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, vo, so, AUX));
        v[0] = q[0]; v[1] = q[1]; v[2] = q[2]; v[3] = q[3];
    }
    template <unsigned AUX>
    static __device__ __forceinline__ void store(rsrc_t r, unsigned vo, unsigned so, const float (&v)[4]) {
        const f32x4 q = {v[0], v[1], v[2], v[3]};
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, q), r, vo, so, AUX);
    }
    template <unsigned AUX>
    static __device__ __forceinline__ float load1(rsrc_t r, unsigned vo, unsigned so) {
        return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, vo, so, AUX));
    }
    // a handed-off quad: false while any element is the poison (then v is not this call's)
    template <unsigned AUX>
    static __device__ __forceinline__ bool load_p(rsrc_t r, unsigned vo, float (&v)[4]) {
        // (whole-vector casts only: DESIGN.md §3.1, compiler pitfall)
        const u32x4 q = __builtin_amdgcn_raw_buffer_load_b128(r, vo, 0u, AUX);
        const f32x4 f = __builtin_bit_cast(f32x4, q);
        v[0] = f[0]; v[1] = f[1]; v[2] = f[2]; v[3] = f[3];
        return q[0] != kResPoison32 && q[1] != kResPoison32 && q[2] != kResPoison32 && q[3] != kResPoison32;
    }
    template <unsigned AUX>
    static __device__ __forceinline__ float load1_p(rsrc_t r, unsigned vo, bool &ready) {
        const unsigned q = __builtin_amdgcn_raw_buffer_load_b32(r, vo, 0u, AUX);
        ready = q != kResPoison32;
        return __builtin_bit_cast(float, q);
    }
    template <unsigned AUX>
    static __device__ __forceinline__ void poison(rsrc_t r, unsigned vo) {
        // materialised at the store (opaque): hoisted as a loop constant it was spilled
        unsigned p = kResPoison32;
        asm volatile("" : "+v"(p));
        const u32x4 q = {p, p, p, p};
        __builtin_amdgcn_raw_buffer_store_b128(q, r, vo, 0u, AUX);
    }
    // one element (PX = 1: the 5x5 build)
    template <unsigned AUX>
    static __device__ __forceinline__ void store1(rsrc_t r, unsigned vo, unsigned so, float v) {
        __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v), r, vo, so, AUX);
    }
    template <unsigned AUX>
    static __device__ __forceinline__ void poison1(rsrc_t r, unsigned vo) {
        unsigned p = kResPoison32;
        asm volatile("" : "+v"(p));
        __builtin_amdgcn_raw_buffer_store_b32(p, r, vo, 0u, AUX);
    }
};
template <> struct ResVec<__half> {
    template <unsigned AUX>
    static __device__ __forceinline__ void load(rsrc_t r, unsigned vo, unsigned so, float (&v)[4]) {
        const f16x4 q = __builtin_bit_cast(f16x4, __builtin_amdgcn_raw_buffer_load_b64(r, vo, so, AUX));
        v[0] = (float)q[0]; v[1] = (float)q[1]; v[2] = (float)q[2]; v[3] = (float)q[3];
    }
    template <unsigned AUX>
    static __device__ __forceinline__ void store(rsrc_t r, unsigned vo, unsigned so, const float (&v)[4]) {
        const f16x4 q = {(_Float16)v[0], (_Float16)v[1], (_Float16)v[2], (_Float16)v[3]};
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, q), r, vo, so, AUX);
    }
    // one element by a 4-byte load of its aligned dword (the hand-off table of
    // MI355X_MICROARCH.md validates sc1 loads of 4/8/16 bytes, not 2), half selected
    template <unsigned AUX>
    static __device__ __forceinline__ float load1(rsrc_t r, unsigned vo, unsigned so) {
        const unsigned at = vo + so;
        const unsigned w = __builtin_amdgcn_raw_buffer_load_b32(r, at & ~3u, 0u, AUX);
        return (float)__builtin_bit_cast(_Float16, (unsigned short)((at & 2u) ? (w >> 16) : (w & 0xffffu)));
    }
    // the poison tests read the halves' bits (a conversion would quiet the signalling NaN)
    template <unsigned AUX>
    static __device__ __forceinline__ bool load_p(rsrc_t r, unsigned vo, float (&v)[4]) {
        const u32x2 q = __builtin_amdgcn_raw_buffer_load_b64(r, vo, 0u, AUX);
        const f16x4 f = __builtin_bit_cast(f16x4, q);
        v[0] = (float)f[0]; v[1] = (float)f[1]; v[2] = (float)f[2]; v[3] = (float)f[3];
        const unsigned P2 = (unsigned)kResPoison16;
        return (q[0] & 0xffffu) != P2 && (q[0] >> 16) != P2 && (q[1] & 0xffffu) != P2 && (q[1] >> 16) != P2;
    }
    template <unsigned AUX>
    static __device__ __forceinline__ float load1_p(rsrc_t r, unsigned vo, bool &ready) {
        const unsigned w = __builtin_amdgcn_raw_buffer_load_b32(r, vo & ~3u, 0u, AUX);
        const unsigned short h = (unsigned short)((vo & 2u) ? (w >> 16) : (w & 0xffffu));
        ready = h != kResPoison16;
        return (float)__builtin_bit_cast(_Float16, h);
    }
    template <unsigned AUX>
    static __device__ __forceinline__ void poison(rsrc_t r, unsigned vo) {
        unsigned w = (unsigned)kResPoison16 | ((unsigned)kResPoison16 << 16);
        asm volatile("" : "+v"(w));  // (opaque: see the float form)
        const u32x2 q = {w, w};
        __builtin_amdgcn_raw_buffer_store_b64(q, r, vo, 0u, AUX);
    }
    // one element (PX = 1: the 5x5 build)
    template <unsigned AUX>
    static __device__ __forceinline__ void store1(rsrc_t r, unsigned vo, unsigned so, float v) {
        __builtin_amdgcn_raw_buffer_store_b16(__builtin_bit_cast(unsigned short, (_Float16)v), r, vo, so, AUX);
    }
    template <unsigned AUX>
    static __device__ __forceinline__ void poison1(rsrc_t r, unsigned vo) {
        __builtin_amdgcn_raw_buffer_store_b16(kResPoison16, r, vo, 0u, AUX);
    }
};

// A thread's PX pixels (PX = 4: a quad, as ResVec; 2: a pair; 1: a pixel) <-> float[PX].
template <typename T, int PX> struct PixVec {
    template <unsigned AUX>
    static __device__ __forceinline__ void load(rsrc_t r, unsigned vo, unsigned so, float (&v)[PX]) {
        if constexpr (PX == 4) {
            ResVec<T>::template load<AUX>(r, vo, so, v);
        } else if constexpr (PX == 1) {
            if constexpr (sizeof(T) == 4) v[0] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, vo, so, AUX));
            else v[0] = (float)__builtin_bit_cast(_Float16, __builtin_amdgcn_raw_buffer_load_b16(r, vo, so, AUX));
        } else if constexpr (sizeof(T) == 4) {  // fp32 pair
            const f32x2 q = __builtin_bit_cast(f32x2, __builtin_amdgcn_raw_buffer_load_b64(r, vo, so, AUX));
            v[0] = q[0]; v[1] = q[1];
        } else {  // fp16 pair
            const unsigned w = __builtin_amdgcn_raw_buffer_load_b32(r, vo, so, AUX);
            v[0] = (float)__builtin_bit_cast(_Float16, (unsigned short)(w & 0xffffu));
            v[1] = (float)__builtin_bit_cast(_Float16, (unsigned short)(w >> 16));
        }
    }
    template <unsigned AUX>
    static __device__ __forceinline__ void store(rsrc_t r, unsigned vo, unsigned so, const float (&v)[PX]) {
        if constexpr (PX == 4) {
            ResVec<T>::template store<AUX>(r, vo, so, v);
        } else if constexpr (PX == 1) {
            ResVec<T>::template store1<AUX>(r, vo, so, v[0]);
        } else if constexpr (sizeof(T) == 4) {
            const f32x2 q = {v[0], v[1]};
            __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, q), r, vo, so, AUX);
        } else {
            const unsigned w = (unsigned)__builtin_bit_cast(unsigned short, (_Float16)v[0]) |
                               ((unsigned)__builtin_bit_cast(unsigned short, (_Float16)v[1]) << 16);
            __builtin_amdgcn_raw_buffer_store_b32(w, r, vo, so, AUX);
        }
    }
    template <unsigned AUX>
    static __device__ __forceinline__ void poison(rsrc_t r, unsigned vo) {
        if constexpr (PX == 4) {
            ResVec<T>::template poison<AUX>(r, vo);
        } else if constexpr (PX == 1) {
            ResVec<T>::template poison1<AUX>(r, vo);
        } else {  // (opaque: see ResVec<float>::poison)
            unsigned p = sizeof(T) == 4 ? kResPoison32 : ((unsigned)kResPoison16 | ((unsigned)kResPoison16 << 16));
            asm volatile("" : "+v"(p));
            if constexpr (sizeof(T) == 4) __builtin_amdgcn_raw_buffer_store_b64(u32x2{p, p}, r, vo, 0u, AUX);
            else __builtin_amdgcn_raw_buffer_store_b32(p, r, vo, 0u, AUX);
        }
    }
};
// a thread's LDS row: PX floats, naturally aligned
template <int PX> struct RowT;
template <> struct RowT<4> { using type = float4; };
template <> struct RowT<2> { using type = float2; };
template <> struct RowT<1> { using type = float; };
template <int PX> __device__ __forceinline__ void rv_get(const typename RowT<PX>::type &r, float (&v)[PX]) {
    if constexpr (PX == 4) { v[0] = r.x; v[1] = r.y; v[2] = r.z; v[3] = r.w; }
    else if constexpr (PX == 2) { v[0] = r.x; v[1] = r.y; }
    else v[0] = r;
}
template <int PX> __device__ __forceinline__ typename RowT<PX>::type rv_make(const float (&v)[PX]) {
    if constexpr (PX == 4) return make_float4(v[0], v[1], v[2], v[3]);
    else if constexpr (PX == 2) return make_float2(v[0], v[1]);
    else return v[0];
}
// PX cells of f into the window at cell li (li % PX == 0) and its shifted copy (fwinB[i] = f[i + 1])
template <int PX> __device__ __forceinline__ void win_put(float *fwin, float *fwinB, int li, const float (&f)[PX]) {
    if constexpr (PX == 4) {
        *reinterpret_cast<float4 *>(&fwin[li]) = make_float4(f[0], f[1], f[2], f[3]);
        fwinB[li - 1] = f[0];
        *reinterpret_cast<float2 *>(&fwinB[li]) = make_float2(f[1], f[2]);
        fwinB[li + 2] = f[3];
    } else if constexpr (PX == 2) {
        *reinterpret_cast<float2 *>(&fwin[li]) = make_float2(f[0], f[1]);
        fwinB[li - 1] = f[0];
        fwinB[li] = f[1];
    } else {
        fwin[li] = f[0];
        fwinB[li - 1] = f[0];
    }
}

// 3x3 geometry (K = 8, prop_kernel 3, the reference default), raw offset layout.
// MAXNT = launch bound (threads), SMAX = staging quads per thread per round.
// NTC = the thread count as a compile-time constant (0: blockDim.x at run time).
// GROUPS: runs ResArgs::ngroups image groups in turn (false: one; the group loop then
// folds away, and with it the setup spill slots it costs).
// KH x KW: the tap geometry; PX = res_px(KH, KW) pixels per thread (4: a quad per thread).
// PXO: pixels per thread overriding res_px (0: res_px): small latency-bound parts (a B = 1 NYU
// image in 247 parts of 72 quads) split a 3x3 quad over two threads, halving each thread's
// dependency chain of tap-pixel slots.
template <typename T, int KH, int KW, int MAXNT, int SMAX, int NTC, bool GROUPS, bool FIRST, int PXO = 0>
__global__ void __launch_bounds__(MAXNT) prop_resident_kernel(ResArgs a) {
    constexpr int K = KH * KW - 1, REF = K / 2, PH = (KH - 1) / 2, PW = (KW - 1) / 2;
    constexpr int RY = res_ry(KH), RXQ = res_rxq(KW), PADX = kResPadX;
    constexpr int PX = PXO ? PXO : res_px(KH, KW), TPQ = 4 / PX;  // pixels per thread, threads per quad
    static_assert(PX == 1 || PX == 2 || PX == 4, "no resident form for this geometry");
    using RowV = typename RowT<PX>::type;
    constexpr unsigned ES = sizeof(T);
    extern __shared__ __attribute__((aligned(16))) float smem[];
    // [0] abort, [1] / [2] row range, [3] / [4] column range (scratch of the setup)
    int *ctl = reinterpret_cast<int *>(smem);
    // f window twice: fwin[i] and fwinB[i] = fwin[i + 1], so any horizontal pair
    // (s[rx], s[rx+1]) is ONE 8-byte-aligned ds_read_b64 from one of the copies
    // With a compile-time thread count the window size is one too (res_win_cells),
    // so every fwinB access is an immediate offset from its fwin address.
    const int NT = NTC ? NTC : (int)blockDim.x;
    const int WC = NTC ? res_build_cells(NTC, NTC, K, PX) : a.win_cells;
    // PITCH: the window's row pitch as a compile-time constant (576-thread builds: the
    // second footprint row is a ds_read immediate offset, and the window cells are kept as
    // 16-bit byte addresses, so a tap spends one VALU on its address instead of three)
    constexpr int PITCH = res_pitch(NTC);
    const int tid = threadIdx.x, lane = tid & 63;
    float *fwin = smem + kResCtl;                                            // [WH][WW] used of WC
    float *fwinB = fwin + WC;                                                // shifted by 1
    // Per thread, K + 3 rows of PX floats (thread-major, an odd count of 16-B rows at PX = 4,
    // 8-B rows at an odd pair stride at PX = 2, odd dwords at PX = 1: conflict-free reads
    // across lanes): the K affinities, 1 - sum, the own pixels' conf' (1 with conf_prop off)
    // and dep (0 with preserve off) — every one an immediate offset from ONE address register.
    RowV *akl = reinterpret_cast<RowV *>(fwinB + WC) + (size_t)tid * (K + 3);
    constexpr int SM = SMAX;  // staging quads per thread per round

    gu32 *sync = (gu32 *)(a.sync);
    const int ngroups = GROUPS && a.ngroups > 1 ? a.ngroups : 1;
    // ---- image groups in turn: every plane pointer below is offset by the image b
    for (int grp = 0;; ++grp) {  // (exits at its end: without GROUPS the compiler folds it away)
    unsigned bid = blockIdx.x;
    asm volatile("" : "+s"(bid));
    // GROUPS: the arguments are re-read per group through an opaque kernarg-segment
    // pointer, so their loads are not hoisted out of the group loop and held (spilled)
    // across every iteration of every group
    ResArgsK *akp = (ResArgsK *)__builtin_amdgcn_kernarg_segment_ptr();
    if constexpr (GROUPS) asm volatile("" : "+s"(akp));
    const ResArgsK &a = *akp;
    const int H = a.H, W = a.W, W4 = W / 4;
    // Part numbering: logical index L = b * (gy*gx) + j, dealt to the XCDs in contiguous
    // runs (xcd_remap), so the parts of an image — and neighbouring parts — share an
    // XCD where the counts allow (C2: one image per XCD; C3: each image over four XCDs
    // in bands of 32 parts).  Speed only: the placement words are indexed by blockIdx, and
    // a reader maps the parts of its image back (xcd_unmap).
    const int nparts = a.gy * a.gx, G = a.B * nparts;
    // (bid: blockIdx behind an opaque move, so that nothing derived from it is hoisted
    // out of the group loop and held in registers across the groups)
    const int L = xcd_remap((int)bid, G);
    const int bl = L / nparts, j = L - bl * nparts;  // image of the group, part of the image
    const int py = j / a.gx, px = j % a.gx;
    const int r0 = (int)((long long)py * H / a.gy), r1 = (int)((long long)(py + 1) * H / a.gy);    // own rows
    const int c0 = (int)((long long)px * W4 / a.gx), c1 = (int)((long long)(px + 1) * W4 / a.gx);  // own quad cols
    const int nqw = c1 - c0, nownq = (r1 - r0) * nqw, nown = nownq * TPQ;  // own quads; own threads

    const bool has_conf = a.conf != nullptr;
    const bool preserve = (a.flags & kPreserve) != 0;
    const bool clip = (a.flags & kAlwaysClip) != 0;
    const bool off_ins = (a.flags & kResOffInserted) != 0;
    const long long HW = (long long)H * W;
    const unsigned plane_bytes = (unsigned)HW * ES;
    const int b = bl + grp * a.B;

    // ---- own quad and its invariants.  Taps are held as their sample coordinates
    // (h_im, w_im) = (y - PH + i + dh, x - PW + j + dw), the reference's own
    // expression (.cuh:178-179), so the geometry below starts from them.
    // trace (dbg 8): row t = 0 of this part holds the setup stamps
    unsigned long long *trace0 = (exp_dbg(a.dbg) & 8u) ? reinterpret_cast<unsigned long long *>(a.pred) +
                                                   (size_t)blockIdx.x * (a.T + 1) * 5 : nullptr;
    if (trace0 && tid == 0) trace0[0] = __builtin_amdgcn_s_memrealtime();
    // trace: per wave and iteration two more stamps (taps + stores issued, stores drained)
    // after the parts' five, 24 per part and iteration (wave-uniform addresses, res_wtrace);
    // row t = 0 holds each wave's HW_ID
    if (kResWTrace && trace0 && (threadIdx.x & 63) == 0) {
        unsigned hw;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
        res_wtrace(a.pred, a.T, __builtin_amdgcn_readfirstlane(threadIdx.x & ~63u), -1)[0] = hw;
    }
    const int nq_main = nown;
    const bool active = tid < nq_main;
    // Every part publishes, once its setup is done, the XCC it runs on, tagged with the image
    // group (grp + 1, above the 5-bit XCC field; the words start every launch at zero,
    // res_finish), and iteration 1 of the group waits until every part of its image has
    // published a tag of this group or a later one.  Two uses:
    //  * per-line hand-offs (flags kResL2, host: plane layout line-aligned): beside the tag a
    //    part publishes its in-image window (the cells it stages; with the fixed halo, whose
    //    general path reads any cell, the whole image), and a line is exported iff a part on
    //    another XCC has a window meeting it (above).  Placement is read, never assumed;
    //  * the prologue in the launch (kResFirst): a part publishes only after its stores of
    //    conf' and of plane 0's poison are acknowledged, so a consumer that has seen every tag
    //    of its image reads neither a previous call's conf' nor its plane 0 (the sc1 row of
    //    MI355X_MICROARCH.md's hand-off table: sc1 stores, every storing wave's vmcnt(0) and a
    //    workgroup barrier before the tag, sc1 loads behind the poll and a barrier).
    const bool l2try = (a.flags & kResL2) != 0;
    constexpr bool first = FIRST;
    const bool publish = l2try || first;
    unsigned xcc_self = 0;
    const unsigned xtag = (unsigned)(grp + 1) << 5;
    if (publish) {
        unsigned x;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
        xcc_self = (x & 0xfu) + 1u;
    }
    // this part's sync line: word 1 the tag, words 2 + 2 (grp & 1) and 3 + 2 (grp & 1) the
    // window of group grp (two slots: a part publishes group g + 1 while a slower part of its
    // image may still read group g's; it cannot reach group g + 2 before that part has
    // published g + 1, which the t = 1 wait of g + 1 needs)
    gu32 *const myline = &sync[kResLine * (1 + blockIdx.x)];
    const float Hf = (float)H, Wf = (float)W;
    int y = r0, x0 = 4 * c0;
    if (active) {  // quad tid / TPQ of the part (row-major), pixels (tid % TPQ) * PX .. + PX - 1 of it
        const int q = TPQ == 1 ? tid : tid / TPQ, rr = q / nqw;
        y = r0 + rr;
        x0 = 4 * (c0 + q - rr * nqw) + (TPQ == 1 ? 0 : (tid % TPQ) * PX);
    }
    const unsigned vpix = (unsigned)(y * W + x0) * ES;
    float hy[K][PX], hx[K][PX];
    // the quad's affinities, dep and conf (with the prologue in the launch: raw, processed after
    // the geometry pass below, so that pass runs while they stream in)
    float ak[K][PX], dv[PX], cq[PX];
#pragma unroll
    for (int e = 0; e < PX; ++e) cq[e] = 1.f;
    {
        float aref[PX];
        // the normalised (K+1)-plane layout, or with the prologue in the launch the K raw planes
        const rsrc_t ra_ = make_rsrc(static_cast<const T *>(a.aff) + (first ? (long long)b * a.aff_bs : (long long)b * (K + 1) * HW));
        const rsrc_t ro = make_rsrc(static_cast<const T *>(a.off) + (long long)b * a.off_bs);
        // Issue order (loads return in order): the affinities, dep and conf first — the row
        // stores and the prologue's normalisation and conf' then run while the 2K offset planes
        // still stream in — the offsets last (the window pass below waits for them)
#pragma unroll
        for (int k = 0; k < K; ++k)
            PixVec<T, PX>::template load<0>(ra_, vpix, (unsigned)(first || k < REF ? k : k + 1) * plane_bytes, ak[k]);
#pragma unroll
        for (int e = 0; e < PX; ++e) dv[e] = 0.f;
        if (preserve) PixVec<T, PX>::template load<0>(make_rsrc(static_cast<const T *>(a.dep) + b * HW), vpix, 0u, dv);
        if (has_conf)
            PixVec<T, PX>::template load<0>(make_rsrc(static_cast<const T *>(first ? a.conf_raw : a.conf) + b * HW), vpix, 0u, cq);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const int ok = (off_ins && k >= REF) ? k + 1 : k;  // inserted layout: skip the reference tap's planes
            PixVec<T, PX>::template load<0>(ro, vpix, (unsigned)(2 * ok) * plane_bytes, hy[k]);
            PixVec<T, PX>::template load<0>(ro, vpix, (unsigned)(2 * ok + 1) * plane_bytes, hx[k]);
        }
        if (first) {
            // the prologue (step 1's FIRST path, the same IEEE sequence): conf' = (1 - m) conf + m,
            // m = dep > 0 (:328-334), stored (the output dict's confidence, and the conf' other
            // parts stage from); plane 0 poisoned (iteration 1 of the launch reads it from the
            // other parts).  The affinities are normalised below, from the LDS rows.
            if (preserve) {
#pragma unroll
                for (int e = 0; e < PX; ++e) {
                    const float m = dv[e] > 0.f ? 1.f : 0.f;
                    cq[e] = (1.0f - m) * cq[e] + m;
                }
            }
            if (active) {
                if (has_conf) PixVec<T, PX>::template store<kSc1>(make_rsrc(static_cast<T *>(const_cast<void *>(a.conf)) + b * HW), vpix, 0u, cq);
                PixVec<T, PX>::template poison<kSc1>(make_rsrc(static_cast<T *>(a.pred_inter) + b * HW), vpix);
            }
            // conf' as stored (fp16: rounded): the own quad's f_t = p_t * conf' of every later
            // iteration uses it, as the staging's loads of the stored planes do (iteration 1
            // stages f0 from the unrounded value, as step 1 does)
#pragma unroll
            for (int e = 0; e < PX; ++e) cq[e] = round_to<T>(cq[e]);
        }
        if (!first) {
#pragma unroll
            for (int e = 0; e < PX; ++e) {  // reference tap weight, the step kernel's 1 - sum (same order)
                float s = 0.f;
#pragma unroll
                for (int k = 0; k < K; ++k) s += ak[k][e];
                aref[e] = 1.0f - s;
            }
        }
        // the affinities are consumed last in a tap, so they wait in LDS (conflict-
        // free 16-B rows per thread) and leave the registers to the tap coordinates
#pragma unroll
        for (int k = 0; k < K; ++k) akl[k] = rv_make<PX>(ak[k]);
        if (!first) akl[K] = rv_make<PX>(aref);
        akl[K + 1] = rv_make<PX>(cq);
        akl[K + 2] = rv_make<PX>(dv);
    }
    // the prologue: the affinity normalisation with the reference-tap weight 1 - sum
    // (nlspn_common.h normalize_taps, step 1's IEEE sequence), one pixel of the quad at a time
    // from the raw values in the LDS rows (a rolled loop: the 4 x K values of the quad at once
    // cost the GROUPS builds scratch)
    {
        if (first) {
            const float gamma = *a.gamma;
#pragma unroll 1
            for (int e = 0; e < PX; ++e) {
                float *row = reinterpret_cast<float *>(akl) + e;
                float t1[K][1], r1[1];
#pragma unroll
                for (int k = 0; k < K; ++k) t1[k][0] = row[PX * k];
                normalize_taps<K, 1>(t1, r1, a.kind, gamma);
#pragma unroll
                for (int k = 0; k < K; ++k) row[PX * k] = t1[k][0];
                row[PX * K] = r1[0];
            }
            // the output dict's `aff` ((K+1) planes, the normalisation's values: fp16 storage
            // rounds them as step 1 does), streamed now, while the offsets still stream in
            // (measured faster than one plane per iteration in the loop: C2 104.6 vs 105.8,
            // C3 223.8 vs 227.9 us per section, profiles/r05)
            if (active) {
                const rsrc_t rao = make_rsrc(static_cast<T *>(a.aff_out) + (long long)b * (K + 1) * HW);
#pragma unroll
                for (int c = 0; c <= K; ++c) {
                    float q[PX];
                    rv_get<PX>(akl[c == REF ? K : (c < REF ? c : c - 1)], q);
                    PixVec<T, PX>::template store<kNT>(rao, vpix, (unsigned)c * plane_bytes, q);
                }
            }
        }
    }
    if (trace0 && tid == 0) trace0[4] = __builtin_amdgcn_s_memrealtime();  // (the prologue's normalisation done)
    // the own pixels' row k (affinity k < K, K: 1 - sum, K + 1: conf', K + 2: dep)
    const auto aff4 = [&](const int k) -> RowV { return akl[k]; };

    // ---- the window: the rectangle of every cell a valid tap of this part touches
    // (offsets are invariant, so once), when it fits the LDS cells allocated;
    // otherwise the part +- (RY rows, RXQ quads), and the rare taps outside it take
    // the general path.  Columns are whole quads plus PADX zero columns each side.
    // The setup's barriers order LDS only (lds_barrier).
    // The own rectangle plus one row and one column: the reference tap's four-corner
    // footprint (read when the window holds a non-finite f, below).  ctl[6] / ctl[7]: the
    // per-iteration "window holds a non-finite f" flags (by iteration parity).
    if (tid == 0) { ctl[0] = 0; ctl[1] = r0; ctl[2] = r1; ctl[3] = 4 * c0; ctl[4] = 4 * c1; ctl[6] = ctl[7] = 0; }
    lds_barrier();
    if (trace0 && tid == 0) trace0[1] = __builtin_amdgcn_s_memrealtime();
    // The output dict's inserted offsets (ResArgs::off_out: 2(K+1) planes, the reference tap's
    // two planes zero).  The 128-thread build (small parts, C1's 247 of 72 quads: a latency-bound
    // loop, a cheap setup) streams them from the raw offsets here, as they arrive; its loop
    // copy cost it 13 % (216.0 k vs 197.1 k iters/s same box, profiles/r05/ab_offsetup_*.txt).
    // The other builds (large parts: the setup is bandwidth-bound — the setup stores cost C2
    // 8 %, C3 6 %) copy one plane per iteration in the loop (below).
    constexpr bool OFFSETUP = NTC == 128 || PXO != 0;
    if (OFFSETUP && a.off_out && !off_ins && active) {
        const rsrc_t rco = make_rsrc(static_cast<T *>(a.off_out) + (long long)b * 2 * (K + 1) * HW);
        float z[PX];
#pragma unroll
        for (int e = 0; e < PX; ++e) z[e] = 0.f;
#pragma unroll
        for (int c = 0; c < K + 1; ++c) {
            const int k = c < REF ? c : c - 1;
            PixVec<T, PX>::template store<kNT>(rco, vpix, (unsigned)(2 * c) * plane_bytes, c == REF ? z : hy[k]);
            PixVec<T, PX>::template store<kNT>(rco, vpix, (unsigned)(2 * c + 1) * plane_bytes, c == REF ? z : hx[k]);
        }
    }
    {
        // the extremes of the valid taps' coordinates, floored once (floor is monotonic:
        // min floor(h) = floor(min h)); a valid tap's coordinates are finite
        float hmn = __builtin_inff(), hmx = -__builtin_inff(), wmn = __builtin_inff(), wmx = -__builtin_inff();
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const int t = k < REF ? k : k + 1, i = t / KW, jj = t % KW;
#pragma unroll
            for (int e = 0; e < PX; ++e) {  // sample coordinates, .cuh:178-179
                const float h_im = (float)(y - PH + i) + hy[k][e];
                const float w_im = (float)(x0 + e - PW + jj) + hx[k][e];
                hy[k][e] = h_im;
                hx[k][e] = w_im;
                // branch-free: an invalid tap offers the identities (the per-tap branches and
                // the min / max operands' canonicalisation were most of this pass)
                const bool ok = h_im > -1.f && w_im > -1.f && h_im < Hf && w_im < Wf;
                hmn = fminf(hmn, ok ? h_im : __builtin_inff());
                hmx = fmaxf(hmx, ok ? h_im : -__builtin_inff());
                wmn = fminf(wmn, ok ? w_im : __builtin_inff());
                wmx = fmaxf(wmx, ok ? w_im : -__builtin_inff());
            }
        }
        int mn = r0, mx = r1, cmn = 4 * c0, cmx = 4 * c1;
        if (hmn <= hmx) {
            mn = min(mn, (int)floorf(hmn));
            mx = max(mx, (int)floorf(hmx) + 1);
            cmn = min(cmn, (int)floorf(wmn));
            cmx = max(cmx, (int)floorf(wmx) + 1);
        }
        res_span_merge(ctl, active, mn, mx, cmn, cmx);
    }
    lds_barrier();
    int rlo = ctl[1], rhi = ctl[2], wq0 = ctl[3] >> 2, wq1 = ctl[4] >> 2;  // >> 2: floor for negatives too
    if (rhi < rlo + 1) rhi = rlo + 1;  // at least two rows (the zero redirect reads a 2x2 footprint)
    // the dynamic window holds every valid tap's footprint by construction (workgroup-uniform)
    // (PITCH builds: rows of PITCH cells, so the span must also fit the pitch; the host
    // picks a PITCH build only when the fixed halo does, res_pitch_ok)
    const bool dynwin = PITCH ? ((rhi - rlo + 1) * PITCH <= WC && 4 * (wq1 - wq0 + 1) + 2 * PADX <= PITCH)
                              : (rhi - rlo + 1) * (4 * (wq1 - wq0 + 1) + 2 * PADX) <= WC;
    if (!dynwin) {  // too large: fixed halo + general path
        rlo = r0 - RY;
        rhi = r1 - 1 + RY;
        wq0 = c0 - RXQ;
        wq1 = c1 - 1 + RXQ;
    }
    const int WH = rhi - rlo + 1, WWp = 4 * (wq1 - wq0 + 1), WW = PITCH ? PITCH : WWp + 2 * PADX;
    const int ra = max(rlo, 0), rb = min(rhi, H - 1);      // in-image window rows
    const int qa = max(wq0, 0), qb = min(wq1, W4 - 1);     // in-image window quad columns
    const int wqn = qb - qa + 1;
    // the window as published (16-bit fields): the in-image cells this part reads of other
    // parts' planes; the fixed halo's general path reads any cell: the whole image
    const unsigned pw0 = dynwin ? (unsigned)ra | ((unsigned)rb << 16) : ((unsigned)(H - 1) << 16);
    const unsigned pw1 = dynwin ? (unsigned)qa | ((unsigned)qb << 16) : ((unsigned)(W4 - 1) << 16);
    if (l2try && tid == 0) {
        __hip_atomic_store(&myline[2 + 2 * (grp & 1)], pw0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&myline[3 + 2 * (grp & 1)], pw1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    // after a step-1 launch the tag carries the placement and the window: published now (its
    // words acknowledged first); the prologue form publishes after its stores, below
    if (publish && !first && tid == 0) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __hip_atomic_store(&myline[1], xtag | xcc_self, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    lds_barrier();
    for (int i = tid; i < WH * WW; i += NT) fwin[i] = fwinB[i] = 0.f;  // cells outside the image stay 0
    lds_barrier();
    if (trace0 && tid == 0) trace0[2] = __builtin_amdgcn_s_memrealtime();
    // Classify every tap once:
    //  * invalid (outside (-1,H) x (-1,W), or NaN): the reference samples 0.  Its
    //    coordinates are redirected to (rlo, 4*wq0 - PADX), an integer point of the
    //    window's zero padding columns, so the branch-free path reads four zeros with
    //    weights (1,0,0,0): v = +0 exactly, as the reference's val = 0;
    //  * in the LDS window: the branch-free path;
    //  * valid but outside the window (only with the fixed halo): read from global
    //    memory by the general path (has_fb), the same cells every iteration.
    // With the dynamic window no valid tap is outside it, so only the redirect of invalid
    // taps runs then (the whole pass took 4.2 us of the C2 setup, profiles/r04).
    bool has_fb = false;
    if (!dynwin) {
#pragma unroll
        for (int k = 0; k < K; ++k) {
#pragma unroll
            for (int e = 0; e < PX; ++e) {
                const float h_im = hy[k][e], w_im = hx[k][e];
                if (h_im > -1.f && w_im > -1.f && h_im < Hf && w_im < Wf) {
                    const int h_low = (int)floorf(h_im), w_low = (int)floorf(w_im);
                    if (!((unsigned)(h_low - rlo) < (unsigned)(WH - 1) &&
                          (unsigned)(w_low - 4 * wq0) < (unsigned)(WWp - 1)))
                        has_fb = true;
                } else {
                    hy[k][e] = (float)rlo;
                    hx[k][e] = (float)(4 * wq0 - PADX);
                }
            }
        }
        has_fb = has_fb && active;
    } else {
        const float rlof = (float)rlo, zcf = (float)(4 * wq0 - PADX);
#pragma unroll
        for (int k = 0; k < K; ++k) {
#pragma unroll
            for (int e = 0; e < PX; ++e) {  // (branch-free)
                const bool ok = hy[k][e] > -1.f && hx[k][e] > -1.f && hy[k][e] < Hf && hx[k][e] < Wf;
                hy[k][e] = ok ? hy[k][e] : rlof;  // invalid: the zero redirect
                hx[k][e] = ok ? hx[k][e] : zcf;
            }
        }
    }
    if (trace0 && tid == 0) trace0[3] = __builtin_amdgcn_s_memrealtime();
    const bool wave_fb = __ballot(has_fb) != 0;  // wave-uniform: this wave has general-path lanes
    // Every tap's bilinear geometry is iteration-invariant, so it is resolved once:
    // the fractional parts lh = h - floor(h), lw = w - floor(w) (.cuh:35-36, the same
    // values the per-iteration form computes) and the window cell of the footprint's
    // top-left corner as a float index into fwin/fwinB (the copy that makes the
    // horizontal pair 8-byte aligned), two 16-bit indices per register.  An iteration
    // then spends no VALU on floors or addresses.
    float lhv[K][PX], lwv[K][PX];
    constexpr int NSL = K * PX;  // tap-pixel slots s = k PX + e
    unsigned adp[NSL / 2];       // slot s's footprint cell: half s & 1 of adp[s >> 1]
    {
        const float WWf = (float)WW;
        const int lbase = PADX - 4 * wq0 - rlo * WW, bofs = WC - 1;
#pragma unroll
        for (int k = 0; k < K; ++k) {
#pragma unroll
            for (int e = 0; e < PX; ++e) {
                const int sl = k * PX + e;
                if ((sl & 1) == 0) adp[sl >> 1] = 0u;
                const float fh = floorf(hy[k][e]), fw = floorf(hx[k][e]);
                lhv[k][e] = hy[k][e] - fh;
                lwv[k][e] = hx[k][e] - fw;
                // window index (h_low - rlo) * WW + w_low - 4 wq0 + PADX, in exact float
                // arithmetic; out-of-window (general-path) taps are clamped to cell 0 and
                // never read
                int li = (int)(fh * WWf + fw) + lbase;
                li = ((unsigned)li < (unsigned)(WH * WW)) ? li : 0;
                unsigned idx = (li & 1) ? (unsigned)(li + bofs) : (unsigned)li;
                if constexpr (PITCH != 0) idx = 4u * ((unsigned)kResCtl + idx);  // byte address in the LDS
                adp[sl >> 1] |= idx << (16 * (sl & 1));
            }
        }
    }

    // Staging map (iterations t >= 2): the in-image window quads outside the own
    // rectangle — the bands above and below it (full window width), then the
    // columns left and right of it.  Iteration 1 stages the whole in-image window.
    const int ntop = r0 - ra, nband = (ntop + rb - r1 + 1) * wqn;
    const int side = wqn - nqw, left = c0 - qa;
    // wave-uniform: held in SGPRs (as VGPRs they were the loop's one scratch reload)
    const int nall = __builtin_amdgcn_readfirstlane((rb - ra + 1) * wqn), nrest = __builtin_amdgcn_readfirstlane(nall - nownq);
    const float rwqn = 1.0f / (float)wqn, rside = 1.0f / (float)(side > 0 ? side : 1);

    const T *p_all = static_cast<const T *>(a.pred_inter);
    T *p_out_all = static_cast<T *>(a.pred_inter);
    const rsrc_t rcg = make_rsrc(has_conf ? static_cast<const T *>(a.conf) + b * HW : p_all);
    const int lown = (y - rlo) * WW + x0 - 4 * wq0 + PADX;  // window cell of the own quad's first pixel
    // rim quad k (0 <= k < nrest) of the staging map: window quad row and quad column
    const auto rim_quad = [&](int k, int &r, int &c) {
        if (k < nband) {
            const int rr = res_div(k, wqn, rwqn);
            r = rr < ntop ? ra + rr : r1 + rr - ntop;
            c = qa + k - rr * wqn;
        } else {
            const int m = k - nband, rr = res_div(m, side, rside), cc = m - rr * side;
            r = r0 + rr;
            c = cc < left ? qa + cc : c1 + cc - left;
        }
    };
    // ---- the prologue in the launch: iteration 1 (the loop's t = 0) stages the whole in-image
    // window from the raw inputs, f0 = p0 * conf' with p0 = (1 - m) pred_init + m dep
    // [clamped] and the unrounded conf' (step 1's make_f, :328-348), by plain loads: none of
    // these planes is written by the launch.  Up to kResPre quads per thread in flight.
    if (first) {
        const T *pin = static_cast<const T *>(a.pinit) + b * HW;
        const rsrc_t rpi = make_rsrc(pin);
        const rsrc_t rcr = make_rsrc(has_conf ? static_cast<const T *>(a.conf_raw) + b * HW : pin);
        const rsrc_t rdr = make_rsrc(preserve ? static_cast<const T *>(a.dep) + b * HW : pin);
        bool nonfin = false;
        for (int base = tid; base < nall; base += kResPre * NT) {
            float pv[kResPre][4], cv[kResPre][4], dv[kResPre][4];
            int li[kResPre];
#pragma unroll
            for (int s = 0; s < kResPre; ++s) {
                const int k = base + s * NT, rr = res_div(k, wqn, rwqn), r = ra + rr, c = qa + k - rr * wqn;
                li[s] = (r - rlo) * WW + 4 * (c - wq0) + PADX;
                const unsigned q = (unsigned)(r * W + 4 * c) * ES;
#pragma unroll
                for (int e = 0; e < 4; ++e) { cv[s][e] = 1.f; dv[s][e] = 0.f; }
                if (k < nall) {
                    ResVec<T>::template load<0>(rpi, q, 0u, pv[s]);
                    if (has_conf) ResVec<T>::template load<0>(rcr, q, 0u, cv[s]);
                    if (preserve) ResVec<T>::template load<0>(rdr, q, 0u, dv[s]);
                }
            }
#pragma unroll
            for (int s = 0; s < kResPre; ++s) {
                if (base + s * NT >= nall) continue;
                float f[4];
#pragma unroll
                for (int e = 0; e < 4; ++e) f[e] = make_f<true>(pv[s][e], cv[s][e], dv[s][e], has_conf, preserve, clip);
                nonfin |= !__builtin_isfinite((f[0] + f[1]) + (f[2] + f[3]));
                *reinterpret_cast<float4 *>(&fwin[li[s]]) = make_float4(f[0], f[1], f[2], f[3]);
                fwinB[li[s] - 1] = f[0];
                *reinterpret_cast<float2 *>(&fwinB[li[s]]) = make_float2(f[1], f[2]);
                fwinB[li[s] + 2] = f[3];
            }
        }
        if (__builtin_amdgcn_ballot_w64(nonfin) != 0 && lane == 0) ctl[6] = 1;  // iteration 0's flag
        // the prologue's conf' and plane-0 poison stores (and tid 0's window words) acknowledged
        // by every wave, then a barrier, then the part publishes (the hand-off table's sc1 row)
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        lds_barrier();
        if (tid == 0) __hip_atomic_store(&myline[1], xtag | xcc_self, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }

    // Iteration t reads plane t-1 and writes plane t: t = 1 .. T-1 (the section's iterations
    // 2 .. T) after step 1, whose plane 0 is the launch's input (never poisoned: the first
    // iteration stages without waiting); with the prologue in the launch t = 0 .. T-1, t = 0
    // staged above.  The XCC ids are read by the last wave holding quads (any wave would do).
    const int t0 = first ? 0 : 1;
    const int pwave = (nq_main - 1) >> 6;
    // this thread's quad's line is exported (sc1 stores); decided in iteration 1, before
    // that (the prologue form's plane 0 and plane-1 poison) every line is.  The small-part
    // builds export every line: the fp32 128-thread build (read-ahead taps at the 168-VGPR
    // cap) paid a scratch reload in its iteration loop for the per-lane flag, and the split
    // builds (C1: 247 parts over all eight XCDs, most lines read across XCDs anyway) measured
    // 10 % slower with it (55.1 vs 50.1 us per section same process, profiles/r06)
    constexpr bool LINES = !(NTC == 128 || PXO != 0);
    bool ex = true;
    const int wbase = __builtin_amdgcn_readfirstlane(tid & ~63);  // first thread of this wave
    int t_abort = 0;
    for (int t = t0; t < a.T; ++t) {
        // trace rows: 0 the setup, t + 1 iteration t
        unsigned long long *trace = (exp_dbg(a.dbg) & 8u) ? reinterpret_cast<unsigned long long *>(a.pred) +
                                                       ((size_t)blockIdx.x * (a.T + 1) + t + 1) * 5 : nullptr;
        if (trace && tid == 0) trace[0] = __builtin_amdgcn_s_memrealtime();
        const rsrc_t rp = make_rsrc(p_all + (size_t)(t > 0 ? t - 1 : 0) * a.tstride + b * HW);
        // ---- the inserted-offset copy (ResArgs::off_out): output plane t - t0 (a raw plane, or
        // the reference tap's zero plane) loaded here, stored after the staging phase (by then
        // the staging waits have covered the load).  It costs the large builds 5 % (C2) and
        // 9 % (C3) per section against no copy at all (timing builds, profiles/r05/
        // ab_offcopy_cost_*.txt); stored by the setup instead it costs 8 % / 6 % more, and with
        // its load sent straight to LDS (global_load_lds, no registers held) 1 % / 2 % more
        // (ab_offcopy_dma_*.txt): it is traffic beside the hand-offs, not register pressure
        const int cpc = t - t0;
        const bool cpy = !OFFSETUP && a.off_out != nullptr && cpc < 2 * (K + 1);
        const int cptt = cpc >> 1;
        const int cpsrc = cptt == REF ? -1 : 2 * (cptt < REF ? cptt : cptt - 1) + (cpc & 1);
        float cpq[PX];
#pragma unroll
        for (int e = 0; e < PX; ++e) cpq[e] = 0.f;
        if (cpy && cpsrc >= 0) {
            const rsrc_t ro = make_rsrc(static_cast<const T *>(a.off) + (long long)b * a.off_bs);
            if (active) PixVec<T, PX>::template load<0>(ro, vpix, (unsigned)cpsrc * plane_bytes, cpq);
        }
        // ---- iteration 1, the first to read other parts' cells: wait until every part of the
        // image has published this group's tag (or a later group's).  Then the export list: the
        // published windows of the image's parts on ANOTHER XCC that can meet a line holding one
        // of this part's quads (rows r0 - 1 .. r1: a line spans at most two rows; columns within
        // a line of the own ones, or every column for a part at a row's start or end, whose
        // lines wrap), into LDS (ctl[8 ..], ctl[5] their count; -1: every line exported — no
        // per-line mode, a timed-out wait, or more than kResNC such windows).  With the prologue
        // in the launch a timed-out wait aborts (the conf' and plane 0 it guards are unknown).
        constexpr int LQ = 128 / (4 * (int)ES);  // quads per 128-B line
        if (t == 1) {
            if ((tid >> 6) == pwave) {
                bool fail = false, ovf = false;
                int nc = 0;  // (wave-uniform)
                unsigned spins = 0;
                const int er0 = r0 - 1, er1 = r1;
                const bool wrap = c0 == 0 || c1 == W4;
                const int ec0 = wrap ? 0 : c0 - LQ, ec1 = wrap ? W4 - 1 : c1 - 1 + LQ;
                for (int base = 0; publish && base < nparts && !fail; base += 64) {
                    const int jj = base + lane;
                    gu32 *wp = &sync[kResLine * (1 + xcd_unmap(bl * nparts + (jj < nparts ? jj : 0), G)) + 1];
                    unsigned v;
                    for (;;) {
                        v = __hip_atomic_load(wp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        if (__all((v >> 5) >= (xtag >> 5))) break;
                        if (++spins > kResSpinLimit ||
                            ((spins & 15u) == 0u && __hip_atomic_load(&sync[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u)) {
                            fail = true;
                            break;
                        }
                        __builtin_amdgcn_s_sleep(1);
                    }
                    if (l2try && !fail) {  // (the window words were acknowledged before the tag)
                        const unsigned w0 = __hip_atomic_load(wp + 1 + 2 * (grp & 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        const unsigned w1 = __hip_atomic_load(wp + 2 + 2 * (grp & 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        const bool cand = jj < nparts && (v & 31u) != xcc_self && (int)(w0 & 0xffffu) <= er1 &&
                                          (int)(w0 >> 16) >= er0 && (int)(w1 & 0xffffu) <= ec1 && (int)(w1 >> 16) >= ec0;
                        const unsigned long long m = __builtin_amdgcn_ballot_w64(cand);
                        const int at = nc + (int)__builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u));
                        if (cand && at < kResNC) {
                            ctl[8 + 2 * at] = (int)w0;
                            ctl[9 + 2 * at] = (int)w1;
                        }
                        nc += __builtin_popcountll(m);
                        ovf = ovf || nc > kResNC;
                    }
                }
                if (lane == 0) {
                    ctl[5] = (!l2try || fail || ovf) ? -1 : nc;
                    if (fail && first) {
                        ctl[0] = 1;
                        __hip_atomic_store(&sync[0], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        if (a.status) __hip_atomic_store(a.status, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                    }
                }
            }
            lds_barrier();
            // this quad's line: flat quad range [lq, lq + LQ) of the plane (planes start on a line,
            // host), row ya from column ca, wrapping into row ya + 1 when it passes the row's end
            const int nc = __builtin_amdgcn_readfirstlane(ctl[5]);
            if (LINES && nc >= 0) {
                // (the own quad's row and column recomputed from its byte offset: not live across the loop)
                const int pe = (int)(vpix / ES), yq = pe / W, fq = pe >> 2, lq = fq & ~(LQ - 1);
                const int ya = lq < yq * W4 ? yq - 1 : yq, ca = lq - ya * W4, ce = ca + LQ - 1;
                const int ca1 = min(ce, W4 - 1), cb1 = ce - W4;  // cb1 >= 0: columns 0..cb1 of row ya + 1
                bool hit = false;
                for (int i = 0; i < nc; ++i) {
                    const unsigned w0 = (unsigned)ctl[8 + 2 * i], w1 = (unsigned)ctl[9 + 2 * i];
                    const int wr0 = (int)(w0 & 0xffffu), wr1 = (int)(w0 >> 16), wc0 = (int)(w1 & 0xffffu), wc1 = (int)(w1 >> 16);
                    hit = hit || (ya >= wr0 && ya <= wr1 && ca <= wc1 && ca1 >= wc0) ||
                          (cb1 >= 0 && ya + 1 >= wr0 && ya + 1 <= wr1 && wc0 <= cb1);
                }
                ex = hit;
            }
        }
        if (trace && tid == 0) trace[1] = __builtin_amdgcn_s_memrealtime();

        // ---- stage f = p_{t-1} * conf' for the in-image window cells: p by sc1 loads,
        // re-loaded until not the poison (written by other parts in this launch), conf' by
        // plain loads (invariant).  After a launch's first iteration the own quads are in the
        // window already (written back below), so only the other parts' quads are loaded.
        const bool rim = t > t0;
        const bool spin = rim && !(exp_dbg(a.dbg) & 1u);
        // the staging index (= tid) rebuilt per iteration from the wave's base (an SGPR) and
        // the lane id, so no VGPR holds it across the loop (it was spilled and reloaded)
        const int tb = wbase + (int)__builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
        // (the prologue's t = 0: staged from the raw inputs above)
        const int nsq_it = (exp_dbg(a.dbg) & 2u) ? 0 : (rim ? nrest : (first ? 0 : nall));
        bool nonfin = false;  // this thread staged a non-finite f
        for (int base = tb; base < nsq_it; base += SM * NT) {
            float sv[SM][4], cv[SM][4];
            int sl[SM];
            unsigned gq[SM];
            bool ok = true;  // every staged quad of this lane holds this call's values
#pragma unroll
            for (int s = 0; s < SM; ++s) {
                const int k = base + s * NT;
                int r, c;  // window quad: row, quad column
                if (!rim) {
                    const int rr = res_div(k, wqn, rwqn);
                    r = ra + rr;
                    c = qa + k - rr * wqn;
                } else {
                    rim_quad(k, r, c);
                }
                sl[s] = (r - rlo) * WW + 4 * (c - wq0) + PADX;  // window cell, % 4 == 0
                gq[s] = (unsigned)(r * W + 4 * c) * ES;
                if (k < nsq_it) {
                    ok = ResVec<T>::template load_p<kSc1>(rp, gq[s], sv[s]) && ok;
                    // conf': sc1 when this launch wrote it (the prologue's setup, published by the tags)
                    if (has_conf) {
                        if (first) ResVec<T>::template load<kSc1>(rcg, gq[s], 0u, cv[s]);
                        else ResVec<T>::template load<0>(rcg, gq[s], 0u, cv[s]);
                    }
                }
            }
            if (spin) {  // this wave's lanes re-load the quads still poisoned (a bounded spin)
                bool fail = (exp_dbg(a.dbg) & 32u) && L == 0;  // test hook: part 0 of image 0 aborts
                unsigned spins = 0;
                while (!fail && __builtin_amdgcn_ballot_w64(!ok) != 0) {
                    __builtin_amdgcn_s_sleep(NLSPN_RES_SPIN_SLEEP);
                    if (!ok) {
                        ok = true;
#pragma unroll
                        for (int s = 0; s < SM; ++s)
                            if (base + s * NT < nsq_it) ok = ResVec<T>::template load_p<kSc1>(rp, gq[s], sv[s]) && ok;
                    }
                    if (++spins > kResSpinLimit ||
                        ((spins & 15u) == 0u && __hip_atomic_load(&sync[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u))
                        fail = true;
                }
                if (fail) {
                    ctl[0] = 1;
                    __hip_atomic_store(&sync[0], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    if (a.status) __hip_atomic_store(a.status, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                }
            }
#pragma unroll
            for (int s = 0; s < SM; ++s) {
                const int k = base + s * NT;
                if (k < nsq_it) {
                    float4 f = make_float4(sv[s][0], sv[s][1], sv[s][2], sv[s][3]);
                    if (has_conf) {
                        f.x = f.x * cv[s][0]; f.y = f.y * cv[s][1]; f.z = f.z * cv[s][2]; f.w = f.w * cv[s][3];
                    }
                    // a non-finite cell makes the sum non-finite (a finite sum that overflows
                    // only sends the iteration to the exact four-corner form, harmlessly)
                    nonfin |= !__builtin_isfinite((f.x + f.y) + (f.z + f.w));
                    const int li = sl[s];
                    *reinterpret_cast<float4 *>(&fwin[li]) = f;
                    fwinB[li - 1] = f.x;
                    *reinterpret_cast<float2 *>(&fwinB[li]) = make_float2(f.y, f.z);
                    fwinB[li + 2] = f.w;
                }
            }
        }
        if (kResWTrace && trace && lane == 0) res_wtrace(a.pred, a.T, wbase, t)[1] = __builtin_amdgcn_s_memrealtime();
        if (__builtin_amdgcn_ballot_w64(nonfin) != 0 && lane == 0) ctl[6 + (t & 1)] = 1;
        lds_barrier();
        if (trace && tid == 0) trace[2] = __builtin_amdgcn_s_memrealtime();
        if (ctl[0]) {  // aborted (a spin timed out, or another part's abort): below the loop
            t_abort = t;
            break;
        }
        if (cpy) {  // streaming (nt): an output only
            const rsrc_t rco = make_rsrc(static_cast<T *>(a.off_out) + (long long)b * 2 * (K + 1) * HW);
            if (active) PixVec<T, PX>::template store<kNT>(rco, vpix, (unsigned)cpc * plane_bytes, cpq);
            if (t == a.T - 1) {  // a short section: the planes past T - 1, here
                const rsrc_t ro = make_rsrc(static_cast<const T *>(a.off) + (long long)b * a.off_bs);
                for (int c = cpc + 1; c < 2 * (K + 1); ++c) {
                    const int tt = c >> 1, src = tt == REF ? -1 : 2 * (tt < REF ? tt : tt - 1) + (c & 1);
                    float q[PX];
#pragma unroll
                    for (int e = 0; e < PX; ++e) q[e] = 0.f;
                    if (src >= 0) {
                        if (active) PixVec<T, PX>::template load<0>(ro, vpix, (unsigned)src * plane_bytes, q);
                    }
                    if (active) PixVec<T, PX>::template store<kNT>(rco, vpix, (unsigned)c * plane_bytes, q);
                }
            }
        }
        // the window holds a non-finite f (staged now, or an own quad written back after
        // the previous iteration): the reference tap takes the four-corner form below
        const bool refull = __builtin_amdgcn_readfirstlane(ctl[6 + (t & 1)]) != 0;
        T *p_out = p_out_all + (size_t)t * a.tstride + b * HW;
        // plane t + 1 is read by iteration t + 2 (if any): its own quad poisoned now, the
        // store acknowledged before plane t's store below (the hand-off's ordering)
        if (active && t + 2 < a.T) {
            if (ex) PixVec<T, PX>::template poison<kSc1>(make_rsrc(p_out + a.tstride), vpix);
            else PixVec<T, PX>::template poison<0>(make_rsrc(p_out + a.tstride), vpix);
        }

        // ---- taps (prop_step_kernel's arithmetic, accumulated in tap-index order)
        // The tap geometry depends only on the (invariant) coordinates, so the
        // compiler would hoist all 32 taps' weights and addresses out of the loop
        // and spill them; opaque register moves keep them per iteration (no code).
#pragma unroll
        for (int k = 0; k < K; ++k) {
#pragma unroll
            for (int e = 0; e < PX; ++e) asm volatile("" : "+v"(lhv[k][e]), "+v"(lwv[k][e]));
#pragma unroll
            for (int i = k * PX / 2; i < (k + 1) * PX / 2; ++i) asm volatile("" : "+v"(adp[i]));
        }
        float pown[PX];  // p_t of the own pixels, as stored
#pragma unroll
        for (int e = 0; e < PX; ++e) pown[e] = 0.f;
        // The general path's tap sum of one pixel (y, x) (window cell lcell, byte offset gvo):
        // every tap in tap order with the reference tap (weight 1 - sum, the setup's order) at
        // K/2, in the reference's per-corner form where its footprint leaves the window.
        // A corner spin that times out (or sees another part's abort: polled every 16
        // spins) raises the abort like the staging spin's, and the lane stops spinning on
        // later corners (gp_fail); the poison then reaches the sum as a NaN, and the abort
        // fill below the loop covers the later planes.
        bool gp_fail = false;
        // A general-path corner's f at byte offset qo: in the prologue form's iteration 1 from
        // the raw inputs (step 1's pass B, make_f); otherwise p_{t-1}, re-loaded until not the
        // poison (after a step-1 launch its plane 0 never is), times conf'
        const auto gp_corner = [&](const unsigned qo) -> float {
            if (first && t == 0) {
                const float p = ResVec<T>::template load1<0>(make_rsrc(static_cast<const T *>(a.pinit) + b * HW), qo, 0u);
                const float c = has_conf ? ResVec<T>::template load1<0>(make_rsrc(static_cast<const T *>(a.conf_raw) + b * HW), qo, 0u)
                                         : 1.f;
                const float d = preserve ? ResVec<T>::template load1<0>(make_rsrc(static_cast<const T *>(a.dep) + b * HW), qo, 0u)
                                         : 0.f;
                return make_f<true>(p, c, d, has_conf, preserve, clip);
            }
            float pv = 0.f;
            for (unsigned sp = 0;; ++sp) {  // per lane, bounded
                bool rdy;
                pv = ResVec<T>::template load1_p<kSc1>(rp, qo, rdy);
                if (rdy || (!first && t == 1) || gp_fail || (exp_dbg(a.dbg) & 1u)) break;
                if (sp > kResSpinLimit ||
                    ((sp & 15u) == 15u && __hip_atomic_load(&sync[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u)) {
                    gp_fail = true;
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
            }
            return has_conf ? pv * ResVec<T>::template load1<kSc1>(rcg, qo, 0u) : pv;
        };
        const auto gp_raise = [&]() {  // a general-path spin timed out: the abort (rare lanes)
            if (gp_fail) {
                ctl[0] = 1;
                __hip_atomic_store(&sync[0], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (a.status) __hip_atomic_store(a.status, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            }
        };
        if (active && !(exp_dbg(a.dbg) & 4u)) {
            float acc[PX];
#pragma unroll
            for (int e = 0; e < PX; ++e) acc[e] = 0.f;
            // branch-free path: every tap from the LDS window (invalid taps read zeros), in
            // K PX tap-pixel slots s = PX k + e (3x3 quads: 32).  The large builds leave the
            // schedule to the compiler (waits per slot): nine waves per CU already keep the LDS
            // array busy, and its bank-conflict cycles, not the read latency, bound the taps
            // (issuing 1-4 slots ahead measured 3-5 % slower at C2, profiles/r04/ab_pf_r4b.txt).
            // 128-thread and split-quad builds (small parts, e.g. C1's 247 of 72 quads: two
            // waves, the taps one wave's dependency chain) issue slot s + PF's two footprint
            // reads before slot s's arithmetic, PF = 4: C1 +3.9 % same-box
            // (profiles/r04/ab_pf_r4s_*.txt; fp32: the fp16 build spills with it).  Same
            // arithmetic, same order per pixel either way.
            constexpr int PF = ((NTC == 128 || PXO != 0) && ES == 4) ? 4 : 0;
            float2 g01[NSL], g23[NSL];
            RowV akv[K + 1];
            RowV cref;  // the reference tap's own-pixel cells (one-cell form; the four-corner
                        // form is applied after the taps, below)
            auto issue = [&](const int s) {
                const int k = s / PX, e = s % PX;
                if (e == 0) akv[k] = aff4(k);
                if (s == PX * REF) {  // the reference tap's own-pixel cells and weight
                    akv[K] = aff4(K);
                    cref = *reinterpret_cast<const RowV *>(&fwin[lown]);
                }
                const unsigned idx = (s & 1) ? (adp[s >> 1] >> 16) : (adp[s >> 1] & 0xffffu);
                if constexpr (PITCH != 0) {  // an LDS byte address (the dynamic LDS starts at 0)
                    g01[s] = lds_pair(idx);
                    // two ds_read_b64 (one address register, the lower row an immediate offset):
                    // ds_read2st64_b64, what the compiler would merge the pair into, runs at
                    // half the LDS rate (16-lane groups, MI355X_MICROARCH.md LDS table); a
                    // scheduling barrier keeps them apart
                    __builtin_amdgcn_sched_barrier(0);
                    g23[s] = lds_pair(idx + 4u * PITCH);
                } else {
                    g01[s] = *reinterpret_cast<const float2 *>(fwin + idx);
                    g23[s] = *reinterpret_cast<const float2 *>(fwin + idx + WW);
                }
            };
#pragma unroll
            for (int s = 0; s < PF; ++s) issue(s);
#pragma unroll
            for (int s = 0; s < NSL; ++s) {
                if (s + PF < NSL) issue(s + PF);
                if constexpr (PF > 0) __builtin_amdgcn_sched_barrier(0);
                const int k = s / PX, e = s % PX;
                if (PF == 0) issue(s);
                if (s == PX * REF) {  // reference tap (t = K/2): zero offset, weight 1 - sum
                    float ar[PX], cr[PX];
                    rv_get<PX>(akv[K], ar);
                    rv_get<PX>(cref, cr);
#pragma unroll
                    for (int e2 = 0; e2 < PX; ++e2) acc[e2] += cr[e2] * ar[e2];
                }
                float av[PX];
                rv_get<PX>(akv[k], av);
                const float lh = lhv[k][e], lw = lwv[k][e];  // = h - (float)h_low (.cuh:35-36)
                const float hh = 1.f - lh, hw = 1.f - lw;
                const float w1 = hh * hw, w2 = hh * lw, w3 = lh * hw, w4 = lh * lw;
                const float2 s01 = g01[s], s23 = g23[s];
                const float v = (w1 * s01.x + w2 * s01.y + w3 * s23.x + w4 * s23.y);
                acc[e] += v * av[e];  // .cuh:189 col = val * mask, summed in tap order
            }
            // general path (rare; only waves holding a tap outside the window): the
            // reference's per-corner checks, from global memory where needed (the same
            // cells every iteration, re-loaded until not the poison, as the staging's).  It
            // re-reads its offsets and affinities from global memory and runs a rolled tap
            // loop, so it shares no registers with the branch-free path (no spills around it).
            if (kResGeneralPath && wave_fb && has_fb && !(exp_dbg(a.dbg) & 64u)) {
                // the own quad's row and first column, recomputed from its byte offset (not
                // live across the loop)
                const int pe = (int)(vpix / ES), y = pe / W, x0 = pe - y * W;
                {
                    // (the same sum written out, every loop rolled: the pixel, the tap and the
                    // corner; unrolled, this rare path's code cost the 128-thread build's loop
                    // 3 % of C1, profiles/r05/ab_gp_r5.txt)
                    const rsrc_t ro = make_rsrc(static_cast<const T *>(a.off) + (long long)b * a.off_bs);
#pragma unroll 1
                    for (int e = 0; e < PX; ++e) {
                        const float *arow = reinterpret_cast<const float *>(akl) + e;  // row k: arow[PX * k]
                        float s = 0.f;
#pragma unroll 1
                        for (int k = 0; k < K; ++k) {
                            if (k == REF) s += fwin[lown + e] * arow[PX * K];
                            const float av = arow[PX * k];
                            const int tt = k < REF ? k : k + 1, i = tt / KW, jj = tt % KW;
                            const int ok = (off_ins && k >= REF) ? k + 1 : k;
                            const float h_im = (float)(y - PH + i) +
                                               ResVec<T>::template load1<0>(ro, vpix + e * ES, (unsigned)(2 * ok) * plane_bytes);
                            const float w_im = (float)(x0 + e - PW + jj) +
                                               ResVec<T>::template load1<0>(ro, vpix + e * ES, (unsigned)(2 * ok + 1) * plane_bytes);
                            float v = 0.f;
                            if (h_im > -1.f && w_im > -1.f && h_im < Hf && w_im < Wf) {
                                const int h_low = (int)floorf(h_im), w_low = (int)floorf(w_im);
                                const float lh = h_im - (float)h_low, lw = w_im - (float)w_low;
                                const float hh = 1.f - lh, hw = 1.f - lw;
                                const float w1 = hh * hw, w2 = hh * lw, w3 = lh * hw, w4 = lh * lw;
                                if ((unsigned)(h_low - rlo) < (unsigned)(WH - 1) &&
                                    (unsigned)(w_low - 4 * wq0) < (unsigned)(WWp - 1)) {
                                    const float *sp = &fwin[(h_low - rlo) * WW + w_low - 4 * wq0 + PADX];
                                    v = (w1 * sp[0] + w2 * sp[1] + w3 * sp[WW] + w4 * sp[WW + 1]);
                                } else {
                                    // ((w1 c0 + w2 c1) + w3 c2) + w4 c3, the four-term sum's order
#pragma unroll 1
                                    for (int u = 0; u < 4; ++u) {
                                        const int cy = h_low + (u >> 1), cx = w_low + (u & 1);
                                        float c = 0.f;
                                        if (cy >= 0 && cy <= H - 1 && cx >= 0 && cx <= W - 1)
                                            c = gp_corner((unsigned)(cy * W + cx) * ES);
                                        const float wu = u == 0 ? w1 : (u == 1 ? w2 : (u == 2 ? w3 : w4));
                                        v = u == 0 ? wu * c : v + wu * c;
                                    }
                                }
                            }
                            s += v * av;
                        }
#pragma unroll
                        for (int e2 = 0; e2 < PX; ++e2) acc[e2] = e == e2 ? s : acc[e2];
                    }
                }
                gp_raise();
            }
            // the reference tap in the reference's four-corner form (.cuh:37-52: the integer
            // point's weights are exactly (1, 0, 0, 0)) differs from the one-cell form used
            // above only when its right / lower neighbour is non-finite: 0 * inf = NaN, and
            // a NaN term makes the whole tap sum NaN whatever its position (any other
            // difference is the sign of a zero term, which an accumulator starting at +0
            // never shows).  A uniform branch, taken only when the window holds a
            // non-finite f; the window's zero cells outside the image are its bounds checks.
            if (refull) {
                const float *r0p = &fwin[lown], *r1p = r0p + WW;
#pragma unroll
                for (int e = 0; e < PX; ++e)
                    if (!__builtin_isfinite(r0p[e + 1]) || !__builtin_isfinite(r1p[e]) || !__builtin_isfinite(r1p[e + 1]))
                        acc[e] = __builtin_nanf("");
            }
            float o[PX], fin[PX], dv[PX];
            rv_get<PX>(aff4(K + 2), dv);
#pragma unroll
            for (int e = 0; e < PX; ++e) {
                float vv = acc[e];
                if (preserve) {  // :355-357
                    const float m = dv[e] > 0.f ? 1.f : 0.f;
                    vv = (1.0f - m) * vv + m * dv[e];
                }
                if (clip) vv = clamp0(vv);  // :359-361
                o[e] = vv;
                fin[e] = clip ? vv : clamp0(vv);  // :375-377
            }
            // plane t + 1's poison acknowledged first (issued before the taps: no wait left)
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            if (ex) PixVec<T, PX>::template store<kSc1>(make_rsrc(p_out), vpix, 0u, o);  // write-through
            else PixVec<T, PX>::template store<0>(make_rsrc(p_out), vpix, 0u, o);   // kept in the XCD's L2
#pragma unroll
            for (int e = 0; e < PX; ++e) pown[e] = round_to<T>(o[e]);
            if (t == a.T - 1 && !(exp_dbg(a.dbg) & 8u))
                PixVec<T, PX>::template store<0>(make_rsrc(static_cast<T *>(a.pred) + b * HW), vpix, 0u, fin);
        }
        if (trace && tid == 0) trace[3] = __builtin_amdgcn_s_memrealtime();
        if (kResWTrace && trace && lane == 0) res_wtrace(a.pred, a.T, wbase, t)[0] = __builtin_amdgcn_s_memrealtime();
        // ---- every tap of iteration t is done: the window may change
        lds_barrier();
        if (trace && tid == 0) trace[4] = __builtin_amdgcn_s_memrealtime();
        if (tid == 0) ctl[6 + (t & 1)] = 0;  // iteration t's flag, next used by iteration t + 2
        // ---- the own quad's f_t = p_t * conf' straight into the window, as the next
        // staging would load it
        if (t < a.T - 1 && active && !(exp_dbg(a.dbg) & 2u)) {
            float cw[PX], f[PX];
            rv_get<PX>(aff4(K + 1), cw);
#pragma unroll
            for (int e = 0; e < PX; ++e) f[e] = has_conf ? pown[e] * cw[e] : pown[e];
            win_put<PX>(fwin, fwinB, lown, f);
            float fs = f[0];
            if constexpr (PX == 4) fs = (f[0] + f[1]) + (f[2] + f[3]);
            else if constexpr (PX == 2) fs = f[0] + f[1];
            if (!__builtin_isfinite(fs))
                ctl[6 + ((t + 1) & 1)] = 1;  // (benign race: every writer stores 1)
        }
        // fp16 storage with the prologue in the launch: iteration 1 used the normalisation's
        // own values (step 1 does); later iterations use them as stored, as the step launches
        // read them back (rounded to fp16, the reference-tap weight 1 - sum of the rounded ones)
        if constexpr (ES == 2) {
            if (first && t == t0) {
                float s4[PX], v[PX];
#pragma unroll
                for (int e = 0; e < PX; ++e) s4[e] = 0.f;
#pragma unroll
                for (int k = 0; k < K; ++k) {
                    rv_get<PX>(akl[k], v);
#pragma unroll
                    for (int e = 0; e < PX; ++e) {
                        v[e] = round_to<T>(v[e]);
                        s4[e] += v[e];
                    }
                    akl[k] = rv_make<PX>(v);
                }
#pragma unroll
                for (int e = 0; e < PX; ++e) s4[e] = 1.0f - s4[e];
                akl[K] = rv_make<PX>(s4);
            }
        }
    }
    // aborted: NaN in every plane this part has not written (this group's remaining
    // iterations, every later group's), then exit.  Write-through: a consumer spinning on
    // these cells takes the NaN and runs on.  (Out of the loop: its registers would cost
    // the loop scratch.)
    if (t_abort) {
        if (active) {
            float qn[PX];
#pragma unroll
            for (int e = 0; e < PX; ++e) qn[e] = __builtin_nanf("");
            for (int g2 = grp; g2 < ngroups; ++g2) {
                const int b2 = bl + g2 * a.B;
                for (int tt = g2 == grp ? t_abort : t0; tt < a.T; ++tt)
                    PixVec<T, PX>::template store<kSc1>(make_rsrc(p_out_all + (size_t)tt * a.tstride + b2 * HW), vpix, 0u, qn);
                PixVec<T, PX>::template store<kSc1>(make_rsrc(static_cast<T *>(a.pred) + b2 * HW), vpix, 0u, qn);
            }
        }
        lds_barrier();  // (every wave of the part is here: the abort word is read after a barrier)
        res_finish(sync);
        return;
    }
    if (!GROUPS || grp + 1 >= ngroups) break;
    }  // image groups
    lds_barrier();  // every wave has made its last read of the sync words
    res_finish(sync);
}

}  // namespace nlspn
