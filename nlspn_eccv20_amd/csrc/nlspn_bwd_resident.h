// Resident pass 1 of the two-pass backward (nlspn_backward.h bwd_step_kernel<SPLIT>) for
// gfx950: iterations T..1 of dL/dout and the col2im scatter of dL/df_{t-1} in ONE launch,
// the invariant planes on chip.
//
// What it replaces, per iteration: the reference's autograd through nlspnmodel.py:350-361
// and the DCN backward's grad_input scatter (modulated_deform_conv_cuda.cu:124-280,
// col2im .cuh:196-254; NLSPN's DCN weight is all ones, so col = grad_output).  The step form
// re-reads the K normalised affinities, the 2K offsets, conf' and dep every iteration
// (~29 of its ~32 plane accesses per pixel); here a part loads them once into registers.
//
// One workgroup (kBrNT threads) owns a part: a PR x PC rectangle of one image, up to
// kBrPX pixels per thread.  The tap positions (2K floats per pixel) stay in registers, the K
// affinities in LDS (the register file holds ~2,200 pixels' positions per CU, not all 3K
// invariants).  Every part of the launch is co-resident (the host launches at
// most one part per CU and checks the occupancy).  Per iteration t = T..1 a part
//   1. waits until every part of its neighbour set has finished iteration t+1 (one arrival
//      counter per part, cumulative over the iterations);
//   2. forms dL/df_t at its own pixels: its own scatter of iteration t+1, kept in its LDS
//      window as 64-bit fixed point, plus what other parts added to the global dL/df plane,
//      read and zeroed in one memory-side atomic exchange;
//   3. computes dL/dout_t exactly as the step does and stores it for pass 2
//      (bwd_coef_kernel, unchanged), and accumulates dL/dconf' in a register;
//   4. scatters dL/df_{t-1} into its LDS window (fixed point, the step's tile scale rule);
//      2x2 footprints that leave the window add to the global plane with float atomics;
//   5. flushes the window's halo cells (other parts' pixels) with global float atomics and,
//      once every wave's atomics are acknowledged (s_waitcnt vmcnt(0)), adds one to the
//      arrival counter of every neighbour.
// The neighbour set is symmetric and fixed for the launch (the offsets do not change over
// the iterations): in the setup each part marks the parts its taps' corners land in, tells
// each of them (an atomic OR into its adjacency row), and after one grid-wide arrival count
// reads the parts that marked it.  With a symmetric set a part is never more than one
// iteration ahead of a neighbour, so two dL/df planes (ping-pong) suffice: a part scatters
// into plane (t-1)&1 only after each neighbour has consumed that plane's previous contents.
//
// Every access to the dL/df planes inside the launch is a device-scope atomic, which gfx950
// executes at the memory side (MI355X_MICROARCH.md "Global float atomics"): no XCD's L2
// holds a line of them, so no cache state can be stale.  Counters: agent-scope atomic adds,
// polled by one lane with sc1 loads (the hand-off table's first row).
//
// Not bit-reproducible run to run (float atomics), like the step form and the reference's
// col2im; equal to it to float rounding (tests/test_gpu_backward.py).  Every spin is bounded:
// a timed-out wait raises the abort word and the device's sticky status word; every part that
// sees it (the word is global: parts of other images that spin long enough abort too) fills the
// dL/dout planes it has not written, its dL/dconf' and its dL/df_0 cells with NaN before it exits.
#pragma once

#include "nlspn_backward.h"

namespace nlspn {

constexpr int kBrNT = 1024;        // threads per part
constexpr int kBrPX = 3;           // pixels per thread, at most
constexpr int kBrR = 8;            // LDS window halo (the step form's RY = RX = 8)
constexpr int kBrMaxParts = 256;   // parts per launch (one per CU)
constexpr int kBrMaskWords = kBrMaxParts / 32;
constexpr int kBrLine = 32;        // words per 128-B line: every counter on a line of its own
constexpr int kBrMaxCells = 8192;  // LDS window cells (64 KiB of fixed-point sums)
constexpr int kBrLdsBytes = 150 * 1024;  // dynamic LDS: window (8 B per cell) + affinities (32 B per pixel)
constexpr unsigned kBrSpinLimit = 1u << 22;
// sync words: line 0 = {abort, registration count}; line 1 + i = part i's arrival count;
// then one adjacency row (kBrMaskWords) per part.  Zeroed by the host before each launch.
constexpr size_t kBrSyncWords = (size_t)kBrLine * (1 + kBrMaxParts) + (size_t)kBrMaxParts * kBrMaskWords;

struct BwdResArgs {
    const float *pred_inter;  // T planes of N: plane t-1 = p_t
    const float *conf_eff;    // conf' (forward conf_out), or null (conf_prop off)
    const float *dep;         // null unless preserve_input
    const float *aff;         // normalised affinity, (K+1) planes per item
    const float *off;         // raw offsets, 2K planes per item at off_bs
    const float *g_pred;      // dL/dpred or null
    const float *g_inter;     // dL/dpred_inter, T planes of N, or null
    float *gf;                // two planes of N: dL/df ping-pong, zero on entry
    float *g_conf;            // dL/dconf' (the final kernel's accumulator plane), or null
    float *g_off, *g_aff;     // dL/dout_t goes to plane t-1 of g_off (t-1 < 2K), else of g_aff
    long long goff_bs, gaff_bs, off_bs, N;
    unsigned *sync;           // kBrSyncWords, zero on entry
    unsigned *status;         // host-mapped sticky abort word of the device, or null
    int H, W, T;               // (the whole batch in one launch)
    int py, px, PR, PC;       // parts per image py x px, each PR x PC pixels
    int WH, WW;               // LDS window (PR + 2R) x (PC + 2R)
    unsigned flags;           // kPreserve (kAlwaysClip is not taken: the host keeps the step form)
    unsigned dbg;             // experiments build only (exp_dbg; results wrong on purpose): 1 no LDS
                              // scatter, 2 no halo flush, 4 no waits, 8 no exchange read, 16 part 0
                              // aborts at its first wait (the abort path's test)
};

__device__ __forceinline__ unsigned br_load(const unsigned *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// One lane spins until *p >= need (or the abort word is set, or the spin limit passes).
// Returns false on failure, after raising the abort.
__device__ __forceinline__ bool br_wait(unsigned *sync, unsigned *status, const unsigned *p, unsigned need) {
    unsigned spins = 0;
    while (br_load(p) < need) {
        if (++spins > kBrSpinLimit || ((spins & 15u) == 0u && br_load(&sync[0]) != 0u)) {
            __hip_atomic_store(&sync[0], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (status) __hip_atomic_store(status, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            return false;
        }
        __builtin_amdgcn_s_sleep(1);
    }
    return true;
}

// (Two 512-thread parts per CU, each with half the pixels, so that one part's waits overlap the
// other's scatter, measured no faster: C2 0.4566 vs 0.4536 ms per backward,
// profiles/r06/ab_bwd_two_parts_per_cu_*_rejected.json.)
template <int PX>
__global__ void __launch_bounds__(kBrNT, 1) bwd_res_kernel(BwdResArgs a) {
    constexpr int K = 8, REF = 4, NT = kBrNT, R = kBrR;
    extern __shared__ __attribute__((aligned(16))) unsigned long long gacc[];  // WH x WW window, then avl
    float *avl = reinterpret_cast<float *>(gacc + ((a.WH * a.WW + 1) & ~1));  // K affinities per pixel (index i), 32 B each
    __shared__ float redm[NT / 64];
    __shared__ unsigned nbmask[kBrMaskWords];
    __shared__ int nbl[kBrMaxParts];
    __shared__ int ctl[2];  // [0] abort seen, [1] neighbour count

    const int tid = threadIdx.x;
    const int ppi = a.py * a.px;
    const int part = blockIdx.x;
    const int bl = part / ppi, pl = part - bl * ppi;
    const int b = bl;
    const int pr = pl / a.px, pc = pl - pr * a.px;
    const int PR = a.PR, PC = a.PC, WH = a.WH, WW = a.WW, H = a.H, W = a.W;
    const int y0 = pr * PR, x0 = pc * PC, wy0 = y0 - R, wx0 = x0 - R;
    const long long HW = (long long)H * W;
    const bool has_conf = a.conf_eff != nullptr;
    const bool preserve = (a.flags & kPreserve) != 0;
    const float Hf = (float)H, Wf = (float)W;
    unsigned *sync = a.sync;
    unsigned *adj = sync + (size_t)kBrLine * (1 + kBrMaxParts);
    float *gfb[2] = {a.gf + b * HW, a.gf + a.N + b * HW};

    if (tid < kBrMaskWords) nbmask[tid] = 0u;
    if (tid < 2) ctl[tid] = 0;
    for (int i = tid; i < WH * WW; i += NT) gacc[i] = 0ull;

    // ---- the part's pixels and their invariants (for the whole launch)
    const int npx = PR * PC;
    float hs[PX][K], ws[PX][K], ce[PX], pm[PX], gcv[PX], aref[PX], amass[PX];
    int own[PX];  // (ly << 16) | lx, or -1 outside the image / part
    const rsrc_t ra = make_rsrc(a.aff + b * (K + 1) * HW);
    const rsrc_t ro = make_rsrc(a.off + b * a.off_bs);
    const unsigned plane_bytes = (unsigned)HW * 4u;
#pragma unroll
    for (int j = 0; j < PX; ++j) {
        const int i = tid + j * NT;
        const int ly = i / PC, lx = i - (i / PC) * PC;
        const int y = y0 + ly, x = x0 + lx;
        const bool act = i < PR * PC && y < H && x < W;
        own[j] = act ? (ly << 16) | lx : -1;
        const unsigned vpix = (act ? (unsigned)(y * W + x) : 0u) * 4u;
        float asum = 0.f;
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const float v = bld(ra, vpix, (unsigned)(k < REF ? k : k + 1) * plane_bytes);
            if (i < npx) avl[i * K + k] = v;
            asum += v;
            const int t = k < REF ? k : k + 1;
            const int ti = t / 3, tj = t % 3;
            hs[j][k] = (float)(y - 1 + ti) + bld(ro, vpix, (2u * k) * plane_bytes);
            ws[j][k] = (float)(x - 1 + tj) + bld(ro, vpix, (2u * k + 1) * plane_bytes);
        }
        // aref = 1 - sum a_k; the scatter bound |aref| + sum |a_k| (bwd_step_kernel's order)
        aref[j] = 1.0f - asum;
        {
            float m = fabsf(aref[j]);
#pragma unroll
            for (int k = 0; k < K; ++k) m += fabsf(avl[(i < npx ? i : 0) * K + k]);
            amass[j] = m;
        }
        ce[j] = has_conf ? bld(make_rsrc(a.conf_eff + b * HW), vpix, 0u) : 1.f;
        const float dv = preserve ? bld(make_rsrc(a.dep + b * HW), vpix, 0u) : 0.f;
        pm[j] = 1.0f - (dv > 0.f ? 1.f : 0.f);
        gcv[j] = 0.f;
    }
    lds_barrier();

    // ---- neighbour set: the parts (of this image) that the taps' in-image corners land in
    const float rPR = 1.0f / (float)PR, rPC = 1.0f / (float)PC;
#pragma unroll
    for (int j = 0; j < PX; ++j) {
        if (own[j] < 0) continue;
#pragma unroll
        for (int k = 0; k < K; ++k) {
            if (!(hs[j][k] > -1.f && ws[j][k] > -1.f && hs[j][k] < Hf && ws[j][k] < Wf)) continue;
            const int hl = (int)floorf(hs[j][k]), wl = (int)floorf(ws[j][k]);
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                const int cy = hl + (c >> 1), cx = wl + (c & 1);
                if (cy < 0 || cy > H - 1 || cx < 0 || cx > W - 1) continue;
                if (cy >= y0 && cy < y0 + PR && cx >= x0 && cx < x0 + PC) continue;
                int qy = (int)((float)cy * rPR), qx = (int)((float)cx * rPC);
                qy += cy - qy * PR < 0 ? -1 : (cy - qy * PR >= PR ? 1 : 0);
                qx += cx - qx * PC < 0 ? -1 : (cx - qx * PC >= PC ? 1 : 0);
                const int q = qy * a.px + qx;
                if ((unsigned)q < (unsigned)ppi) atomicOr(&nbmask[q >> 5], 1u << (q & 31));
            }
        }
    }
    lds_barrier();
    // tell each marked part (its adjacency row, bit pl), then one grid-wide count
    if (tid < ppi && tid != pl && ((nbmask[tid >> 5] >> (tid & 31)) & 1u))
        __hip_atomic_fetch_or(&adj[(size_t)(bl * ppi + tid) * kBrMaskWords + (pl >> 5)], 1u << (pl & 31),
                              __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
        __hip_atomic_fetch_add(&sync[1], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (!br_wait(sync, a.status, &sync[1], gridDim.x)) ctl[0] = 1;
    }
    __syncthreads();
    if (tid < kBrMaskWords) {
        const unsigned w = __hip_atomic_fetch_or(&adj[(size_t)part * kBrMaskWords + tid], 0u, __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_AGENT);
        nbmask[tid] |= w;
    }
    lds_barrier();
    if (tid < ppi && tid != pl && ((nbmask[tid >> 5] >> (tid & 31)) & 1u)) nbl[atomicAdd(&ctl[1], 1)] = bl * ppi + tid;
    __syncthreads();
    const int nnb = ctl[1];

    // the reference tap's own-cell term go_t * aref of the previous iteration, kept in a register
    // instead of an LDS atomic (its float rounding differs from the fixed-point window's; the
    // last iteration adds it to the window, which it flushes whole)
    float refc[PX];
#pragma unroll
    for (int j = 0; j < PX; ++j) refc[j] = 0.f;
    int sh_prev = 0, t_abort = 0;
    for (int t = a.T; t >= 1 && !t_abort; --t) {
        const bool last = t == a.T;
        // ---- 1. wait for the neighbours' iteration t+1
        if (!last) {
            if (tid == 0 && (exp_dbg(a.dbg) & 16u) && part == 0 && !ctl[0]) {  // test hook: raise the abort
                __hip_atomic_store(&sync[0], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (a.status) __hip_atomic_store(a.status, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                ctl[0] = 1;
            }
            if (tid == 0 && nnb > 0 && !ctl[0] && !(exp_dbg(a.dbg) & 4u))
                if (!br_wait(sync, a.status, &sync[kBrLine * (1 + part)], (unsigned)nnb * (unsigned)(a.T - t))) ctl[0] = 1;
            __syncthreads();
            if (ctl[0]) { t_abort = t; break; }
        }
        // ---- 2./3. dL/df_t at the own pixels, dL/dout_t
        const float *pt_p = a.pred_inter + (size_t)(t - 1) * a.N + b * HW;
        const float *gi_p = a.g_inter ? a.g_inter + (size_t)(t - 1) * a.N + b * HW : nullptr;
        const int jgo = t - 1;
        float *go_p = jgo < 2 * K ? a.g_off + b * a.goff_bs + (size_t)jgo * HW
                                  : a.g_aff + b * a.gaff_bs + (size_t)(jgo - 2 * K) * HW;
        float *gfr_p = gfb[t & 1];
        float go[PX], mass = 0.f;
#pragma unroll
        for (int j = 0; j < PX; ++j) {
            go[j] = 0.f;
            if (own[j] < 0) continue;
            const int ly = own[j] >> 16, lx = own[j] & 0xffff;
            const int cell = (y0 + ly) * W + x0 + lx;
            float gfr = 0.f;
            if (!last) {
                const float mine = ldexpf((float)(long long)gacc[(ly + R) * WW + lx + R], -sh_prev);
                const float others = (exp_dbg(a.dbg) & 8u) ? 0.f
                                     : __hip_atomic_exchange(&gfr_p[cell], 0.f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                gfr = (mine + others) + refc[j];
            }
            const float pt = pt_p[cell];
            float g = has_conf ? gfr * ce[j] : gfr;
            if (gi_p) g += gi_p[cell];
            if (last && a.g_pred) g += pt >= 0.f ? a.g_pred[b * HW + cell] : 0.f;  // pred = clamp(p_T, 0)
            if (has_conf) gcv[j] = gcv[j] + gfr * pt;
            go[j] = preserve ? pm[j] * g : g;
            go_p[cell] = go[j];
            mass += fabsf(go[j]) * amass[j];
        }
        // ---- the part's scatter scale (bwd_step_kernel's rule over the part)
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) mass += __shfl_xor(mass, o, 64);
        if ((tid & 63) == 0) redm[tid >> 6] = mass;
        lds_barrier();  // (also: every own-cell read of the window is done)
        for (int i = tid; i < WH * WW; i += NT) gacc[i] = 0ull;
        float tot = 0.f;
#pragma unroll
        for (int i = 0; i < NT / 64; ++i) tot += redm[i];
        const bool exact = tot < 3.0e38f;
        const int sh = exact && tot > 0.f ? 58 - ilogbf(tot) : 0;
        lds_barrier();

        // (the tap geometry is t-invariant: opaque moves keep the compiler from hoisting every
        // tap's corner weights and cells out of the t loop, which would not fit the registers)
#pragma unroll
        for (int j = 0; j < PX; ++j)
#pragma unroll
            for (int k = 0; k < K; ++k) asm volatile("" : "+v"(hs[j][k]), "+v"(ws[j][k]));
        // ---- 4. scatter dL/df_{t-1}: footprints inside the window into LDS; the rest (outside
        //      the window, or a part whose mass is not finite) marked, then added to the plane
        //      by a second, rarely entered pass (kept out of the common path's registers)
        const rsrc_t rgw = make_rsrc(gfb[(t - 1) & 1]);
        const auto add_win = [&](int c, float v) {
            if (!(exp_dbg(a.dbg) & 1u)) atomicAdd(&gacc[c], (unsigned long long)__float2ll_rn(ldexpf(v, sh)));
        };
        const auto add_gl = [&](int c, float v) {
            __builtin_amdgcn_raw_ptr_buffer_atomic_fadd_f32(v, rgw, (unsigned)c * 4u, 0, 0);
        };
        unsigned slow = 0u;  // bit j * K + k: tap k of pixel j goes to the plane
#pragma unroll
        for (int j = 0; j < PX; ++j) {
            if (own[j] < 0) continue;
            const int ly = own[j] >> 16, lx = own[j] & 0xffff;
            const int i = tid + j * NT;
            // reference tap: integer point, weight 1 (a register until the last iteration)
            refc[j] = 0.f;
            if (!exact) add_gl((y0 + ly) * W + x0 + lx, go[j] * aref[j]);
            else if (t == 1) add_win((ly + R) * WW + lx + R, go[j] * aref[j]);
            else refc[j] = go[j] * aref[j];
            const float4 a0 = reinterpret_cast<const float4 *>(avl)[2 * i], a1 = reinterpret_cast<const float4 *>(avl)[2 * i + 1];
            const float avj[K] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
#pragma unroll
            for (int k = 0; k < K; ++k) {
                const float h = hs[j][k], w = ws[j][k];
                if (h > -1.f && w > -1.f && h < Hf && w < Wf) {
                    const int hl = (int)floorf(h), wl = (int)floorf(w);
                    const bool inwin = (unsigned)(hl - wy0) < (unsigned)(WH - 1) && (unsigned)(wl - wx0) < (unsigned)(WW - 1);
                    if (inwin && exact) {
                        const float lh = h - (float)hl, lw = w - (float)wl, hh = 1.f - lh, hw = 1.f - lw;
                        const float w1 = hh * hw, w2 = hh * lw, w3 = lh * hw, w4 = lh * lw;
                        const float top = go[j] * avj[k];
                        const int c0 = (hl - wy0) * WW + (wl - wx0);
                        add_win(c0, w1 * top);
                        add_win(c0 + 1, w2 * top);
                        add_win(c0 + WW, w3 * top);
                        add_win(c0 + WW + 1, w4 * top);
                    } else {
                        slow |= 1u << (j * K + k);
                    }
                }
            }
        }
        if (__builtin_amdgcn_ballot_w64(slow != 0u)) {
#pragma unroll
            for (int j = 0; j < PX; ++j) {
                const int i = tid + j * NT;
#pragma unroll
                for (int k = 0; k < K; ++k) {
                    if (!((slow >> (j * K + k)) & 1u)) continue;
                    const float h = hs[j][k], w = ws[j][k];
                    const int hl = (int)floorf(h), wl = (int)floorf(w);
                    const float lh = h - (float)hl, lw = w - (float)wl, hh = 1.f - lh, hw = 1.f - lw;
                    const float wts[4] = {hh * hw, hh * lw, lh * hw, lh * lw};
                    const float top = go[j] * avl[i * K + k];
#pragma unroll
                    for (int cnr = 0; cnr < 4; ++cnr) {
                        const int hy = hl + (cnr >> 1), wx = wl + (cnr & 1);
                        if (hy >= 0 && hy <= H - 1 && wx >= 0 && wx <= W - 1) add_gl(hy * W + wx, wts[cnr] * top);
                    }
                }
            }
        }
        lds_barrier();
        // ---- 5. flush the halo (iteration 1: every cell, for the final kernel), then arrive
        if (exact && !(exp_dbg(a.dbg) & 2u)) {
            for (int i = tid; i < WH * WW; i += NT) {
                const int r = i / WW, c = i - (i / WW) * WW;
                const int gy = wy0 + r, gx = wx0 + c;
                const long long q = (long long)gacc[i];
                const bool mine = r >= R && r < R + PR && c >= R && c < R + PC;
                if (q != 0 && (t == 1 || !mine) && gy >= 0 && gy < H && gx >= 0 && gx < W)
                    add_gl(gy * W + gx, ldexpf((float)q, -sh));
            }
        }
        sh_prev = sh;  // (not exact: the window stayed zero, the own cells read the plane alone)
        if (t > 1) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            if (tid < nnb) __hip_atomic_fetch_add(&sync[kBrLine * (1 + nbl[tid])], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    // ---- outputs: dL/dconf'; an aborted part fills the dL/dout planes it did not write with NaN
#pragma unroll
    for (int j = 0; j < PX; ++j) {
        if (own[j] < 0) continue;
        const int cell = (y0 + (own[j] >> 16)) * W + x0 + (own[j] & 0xffff);
        if (has_conf) a.g_conf[b * HW + cell] = t_abort ? __builtin_nanf("") : gcv[j];
        // (and dL/df_0, which the final kernel turns into grad_pred_init: a memory-side store, the
        // plane's other accesses in the launch being atomics)
        if (t_abort) __hip_atomic_store(&gfb[0][cell], __builtin_nanf(""), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        for (int t = t_abort; t >= 1; --t) {
            const int jgo = t - 1;
            float *go_p = jgo < 2 * K ? a.g_off + b * a.goff_bs + (size_t)jgo * HW
                                      : a.g_aff + b * a.gaff_bs + (size_t)(jgo - 2 * K) * HW;
            go_p[cell] = __builtin_nanf("");
        }
    }
}

}  // namespace nlspn
