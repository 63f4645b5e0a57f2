// A/B harness for prop_step_kernel / prologue_kernel variants (diagnostic tool,
// not part of the product).  Generates SURVEY §8d synthetic inputs on the host,
// runs every variant on the same device buffers, checks each variant's output is
// BIT-identical to variant 0, then times the variants in interleaved rounds with
// dispatch-recorded events (hipExtLaunchKernel start/stop), cdna_hip_programming.md §5.4 rule 24.
//
// usage: step_bench [B H W] [reps] [rounds] [sigma]
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#include "../nlspn_eccv20_amd/csrc/nlspn_step.h"
#include "step2_exp.h"

using namespace nlspn;

#define CK(x)                                                                          \
    do {                                                                               \
        hipError_t e = (x);                                                            \
        if (e != hipSuccess) {                                                         \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e)); \
            exit(1);                                                                   \
        }                                                                              \
    } while (0)

struct Variant {
    std::string name;
    const void *fn;
    int TH, TW, PX;
    bool persistent = false;  // grid = CUs x resident workgroups (prop_step2_kernel walks tiles)
};

unsigned grid_of(const Variant &v, int ntiles) {
    if (!v.persistent) return (unsigned)ntiles;
    int dev = 0, cus = 0, occ = 0;
    CK(hipGetDevice(&dev));
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, v.fn, v.TH * v.TW / v.PX, 0));
    return (unsigned)std::min(ntiles, cus * std::max(occ, 1));
}

template <typename T, int KH, int KW, int TH, int TW, int PX, int RY, int RX, int SV, bool PRE>
Variant mk(const char *name) {
    return Variant{name, reinterpret_cast<const void *>(&prop_step_kernel<T, KH, KW, TH, TW, PX, RY, RX, SV, true, PRE, false>),
                   TH, TW, PX};
}

// The pixel-pair kernel (nlspn_step2.h): PX = 2 for the launch shape
template <typename T, int KH, int KW, int TH, int TW, int RY, int RX, int DBG = 0>
Variant mk2(const char *name) {
    return Variant{name, reinterpret_cast<const void *>(&prop_step2_kernel<T, KH, KW, TH, TW, RY, RX, DBG>), TH, TW, 2,
                   true};
}

// Memory-only ceiling: the same per-pixel planes (K aff, 2K offsets, dep, p_in,
// conf) read with the same lane mapping, summed, one plane written — no LDS, no
// gather.  Its time is what this data layout can stream at.
template <int PX>
__global__ void __launch_bounds__(256) stream_ceiling(StepArgs a) {
    const long long HW = (long long)a.H * a.W;
    const long long g = (long long)blockIdx.x * 256 + threadIdx.x;
    if (g * PX >= (long long)a.B * HW) return;
    const long long b = (g * PX) / HW, q = (g * PX) % HW;
    const float *ab = static_cast<const float *>(a.aff) + b * a.aff_bs + q;
    const float *ob = static_cast<const float *>(a.off) + b * a.off_bs + q;
    float acc[PX] = {0}, v[PX];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        Vec<float, PX>::load(ab + (k < 4 ? k : k + 1) * HW, v);
        for (int e = 0; e < PX; ++e) acc[e] += v[e];
        Vec<float, PX>::load(ob + 2 * k * HW, v);
        for (int e = 0; e < PX; ++e) acc[e] += v[e];
        Vec<float, PX>::load(ob + (2 * k + 1) * HW, v);
        for (int e = 0; e < PX; ++e) acc[e] += v[e];
    }
    Vec<float, PX>::load(static_cast<const float *>(a.dep) + b * HW + q, v);
    for (int e = 0; e < PX; ++e) acc[e] += v[e];
    Vec<float, PX>::load(static_cast<const float *>(a.p_in) + b * HW + q, v);
    for (int e = 0; e < PX; ++e) acc[e] += v[e];
    Vec<float, PX>::load(static_cast<const float *>(a.conf) + b * HW + q, v);
    for (int e = 0; e < PX; ++e) acc[e] += v[e];
    Vec<float, PX>::store(static_cast<float *>(a.p_out) + b * HW + q, acc);
}

// Generic memory-only ceiling over the step kernel's exact plane set (K aff, 2K
// offsets, dep, p_in, conf; one plane written), PX pixels per lane, buffer loads.
template <typename T, int K, int PX>
__global__ void __launch_bounds__(256) stream_ceiling_t(StepArgs a) {
    const unsigned HW = (unsigned)a.H * a.W, ES = sizeof(T);
    const long long g = (long long)blockIdx.x * 256 + threadIdx.x;
    if (g * PX >= (long long)a.B * HW) return;
    const unsigned b = (unsigned)((g * PX) / HW), q = (unsigned)((g * PX) % HW);
    const rsrc_t ra = make_rsrc(static_cast<const T *>(a.aff) + b * a.aff_bs);
    const rsrc_t ro = make_rsrc(static_cast<const T *>(a.off) + b * a.off_bs);
    float acc[PX] = {0}, v[PX];
#pragma unroll
    for (int k = 0; k < K; ++k) {
        BVec<T, PX>::load(ra, q * ES, (k < K / 2 ? k : k + 1) * HW * ES, v);
        for (int e = 0; e < PX; ++e) acc[e] += v[e];
        BVec<T, PX>::load(ro, q * ES, 2 * k * HW * ES, v);
        for (int e = 0; e < PX; ++e) acc[e] += v[e];
        BVec<T, PX>::load(ro, q * ES, (2 * k + 1) * HW * ES, v);
        for (int e = 0; e < PX; ++e) acc[e] += v[e];
    }
    BVec<T, PX>::load(make_rsrc(static_cast<const T *>(a.dep) + b * HW), q * ES, 0, v);
    for (int e = 0; e < PX; ++e) acc[e] += v[e];
    BVec<T, PX>::load(make_rsrc(static_cast<const T *>(a.p_in) + b * HW), q * ES, 0, v);
    for (int e = 0; e < PX; ++e) acc[e] += v[e];
    BVec<T, PX>::load(make_rsrc(static_cast<const T *>(a.conf) + b * HW), q * ES, 0, v);
    for (int e = 0; e < PX; ++e) acc[e] += v[e];
    BVec<T, PX>::store(make_rsrc(static_cast<T *>(a.p_out) + b * HW), q * ES, 0, acc);
}

template <typename T> std::vector<T> conv(const std::vector<float> &v);
template <> std::vector<float> conv<float>(const std::vector<float> &v) { return v; }
template <> std::vector<__half> conv<__half>(const std::vector<float> &v) {
    std::vector<__half> o(v.size());
    for (size_t i = 0; i < v.size(); ++i) o[i] = __float2half(v[i]);
    return o;
}

template <typename T, int KH, int KW> std::vector<Variant> variants();
template <> std::vector<Variant> variants<float, 3, 3>() {
    return {
        mk<float, 3, 3, 8, 32, 1, 8, 8, 4, true>("8x32 px1 R8 (product)"),
        mk2<float, 3, 3, 8, 64, 8, 8>("pair 8x64 R8"),
        mk2<float, 3, 3, 8, 32, 8, 8>("pair 8x32 R8 (128t)"),
        mk2<float, 3, 3, 16, 32, 8, 8>("pair 16x32 R8"),
        mk<float, 3, 3, 16, 16, 1, 8, 8, 4, true>("16x16 px1 R8"),
        mk<float, 3, 3, 4, 64, 1, 8, 8, 4, true>("4x64 px1 R8"),
        mk<float, 3, 3, 8, 64, 1, 8, 8, 4, true>("8x64 px1 R8 (512t)"),
        mk<float, 3, 3, 16, 32, 1, 8, 8, 4, true>("16x32 px1 R8 (512t)"),
        mk<float, 3, 3, 4, 32, 1, 8, 8, 4, true>("4x32 px1 R8 (128t)"),
        mk<float, 3, 3, 16, 64, 4, 8, 8, 4, true>("16x64 px4 R8"),
        mk<float, 3, 3, 8, 64, 2, 8, 8, 4, true>("8x64 px2 R8"),
        mk<float, 3, 3, 4, 64, 1, 8, 8, 1, true>("4x64 px1 scalar-stage"),
    };
}
template <> std::vector<Variant> variants<__half, 1, 17>() {
    return {
        mk<__half, 1, 17, 8, 32, 1, 8, 16, 4, true>("8x32 px1 (round 1)"),
        mk2<__half, 1, 17, 8, 64, 8, 16>("pair 8x64 (product)"),
        mk2<__half, 1, 17, 4, 128, 8, 16>("pair 4x128"),
        mk2<__half, 1, 17, 16, 32, 8, 16>("pair 16x32"),
        mk2<__half, 1, 17, 8, 32, 8, 16>("pair 8x32 (128t)"),
        mk2<__half, 1, 17, 8, 128, 8, 16>("pair 8x128 (512t)"),
        mk2<__half, 1, 17, 16, 32, 8, 16, 1>("pair 16x32 DBG nostage"),
        mk2<__half, 1, 17, 16, 32, 8, 16, 2>("pair 16x32 DBG notaps"),
        mk2<__half, 1, 17, 16, 32, 8, 16, 3>("pair 16x32 DBG neither"),
        mk<__half, 1, 17, 16, 16, 1, 8, 16, 4, true>("16x16 px1"),
        mk<__half, 1, 17, 4, 64, 1, 8, 16, 4, true>("4x64 px1"),
        mk<__half, 1, 17, 8, 64, 1, 8, 16, 4, true>("8x64 px1 (512t)"),
        mk<__half, 1, 17, 4, 32, 1, 8, 16, 4, true>("4x32 px1 (128t)"),
        mk<__half, 1, 17, 8, 32, 1, 4, 12, 4, true>("8x32 px1 RY4 RX12"),
        mk<__half, 1, 17, 8, 64, 2, 8, 16, 4, true>("8x64 px2"),
        mk<__half, 1, 17, 4, 64, 2, 8, 16, 4, true>("4x64 px2 (128t)"),
        mk<__half, 1, 17, 16, 32, 2, 8, 16, 4, true>("16x32 px2"),
        mk<__half, 1, 17, 8, 32, 2, 8, 16, 4, true>("8x32 px2 (128t)"),
        mk<__half, 1, 17, 4, 64, 4, 8, 16, 4, true>("4x64 px4 (64t)"),
    };
}

template <typename T, int KH, int KW>
int run(int B, int H, int W, int reps, int rounds, float sigma) {


    constexpr int K = KH * KW - 1;
    constexpr int ES = sizeof(T);
    const long long HW = (long long)H * W, N = (long long)B * HW;
    printf("B=%d H=%d W=%d K=%d sigma=%.1f reps=%d rounds=%d\n", B, H, W, K, sigma, reps, rounds);

    // ---- synthetic inputs: convex |N(0,1)| affinity (TGASS), N(0, sigma^2) offsets
    std::mt19937 rng(7240);
    std::uniform_real_distribution<float> U(0.f, 1.f);
    std::normal_distribution<float> Nd(0.f, 1.f);
    std::vector<float> p(N), conf(N), dep(N), aff((size_t)B * (K + 1) * HW), affraw((size_t)B * K * HW),
        off((size_t)B * 2 * K * HW);
    for (long long i = 0; i < N; ++i) {
        p[i] = 10.f * U(rng);
        dep[i] = U(rng) < 0.0072f ? 10.f * U(rng) : 0.f;
        conf[i] = dep[i] > 0 ? 1.f : U(rng);
    }
    for (auto &v : affraw) v = std::fabs(Nd(rng));
    for (auto &v : off) v = sigma * Nd(rng);
    for (int b = 0; b < B; ++b)
        for (long long q = 0; q < HW; ++q) {
            float t[K], s = 0.f, sum = 0.f;
            for (int k = 0; k < K; ++k) { t[k] = std::tanh(affraw[((size_t)b * K + k) * HW + q]) / (0.5f * K + 1e-8f); s += std::fabs(t[k]); }
            s += 1e-4f;
            if (s < 1.f) s = 1.f;
            for (int k = 0; k < K; ++k) { t[k] /= s; sum += t[k]; }
            for (int c = 0, k = 0; c < K + 1; ++c)
                aff[((size_t)b * (K + 1) + c) * HW + q] = c == K / 2 ? 1.f - sum : t[k++];
        }

    auto up = [](const std::vector<float> &hf) {
        std::vector<T> h = conv<T>(hf);
        T *d;
        CK(hipMalloc(&d, h.size() * ES));
        CK(hipMemcpy(d, h.data(), h.size() * ES, hipMemcpyHostToDevice));
        return d;
    };
    T *dp = up(p), *dc = up(conf), *dd = up(dep), *da = up(aff), *dr = up(affraw), *doff = up(off);
    T *dout, *dscratch;
    CK(hipMalloc(&dout, N * ES));
    CK(hipMalloc(&dscratch, (size_t)N * ES * (6 * K + 12)));

    std::vector<Variant> vs = variants<T, KH, KW>();

    hipStream_t s;
    CK(hipStreamCreate(&s));
    std::vector<T> ref(N), got(N);
    auto args_for = [&](const Variant &v) {
        StepArgs a{dp, dc, dd, da, doff, dout, nullptr, (long long)(K + 1) * HW, (long long)2 * K * HW, B, H, W,
                   (W + v.TW - 1) / v.TW, (H + v.TH - 1) / v.TH, 1, 0x1u};
        return a;
    };
    for (size_t vi = 0; vi < vs.size(); ++vi) {
        StepArgs a = args_for(vs[vi]);
        void *kargs[] = {&a};
        CK(hipMemset(dout, 0, N * ES));
        CK(hipLaunchKernel(vs[vi].fn, dim3(grid_of(vs[vi], B * a.tiles_x * a.tiles_y)), dim3(vs[vi].TH * vs[vi].TW / vs[vi].PX), kargs, 0, s));
        CK(hipStreamSynchronize(s));
        CK(hipMemcpy(vi == 0 ? ref.data() : got.data(), dout, N * ES, hipMemcpyDeviceToHost));
        if (vi > 0) {
            long long bad = 0;
            for (long long i = 0; i < N; ++i) bad += memcmp(&ref[i], &got[i], ES) != 0;
            printf("variant %-24s bit-identical to v0: %s (%lld differ)\n", vs[vi].name.c_str(), bad ? "NO" : "yes", bad);
        }
    }

    {   // host restatement (reference arithmetic, -ffp-contract=off) on every 7th pixel
        auto rnd = [](float x) { return (float)conv<T>(std::vector<float>{x})[0]; };
        auto val_of = [&](const std::vector<float> &hv, long long i) { return rnd(hv[i]); };
        long long bad = 0, checked = 0;
        constexpr int PHh = (KH - 1) / 2, PWw = (KW - 1) / 2, REFk = K / 2;
        for (long long g = 0; g < N; g += 7) {
            const int b = (int)(g / HW), q = (int)(g % HW), yy = q / W, xx = q % W;
            auto f = [&](int hy, int wx) {
                const long long idx = (long long)b * HW + (long long)hy * W + wx;
                return val_of(p, idx) * val_of(conf, idx);
            };
            float asum = 0.f, acc = 0.f, cols[64];
            for (int k = 0; k < K; ++k) {
                const int t = k < REFk ? k : k + 1, i = t / KW, j = t % KW;
                const float ak = val_of(aff, ((long long)b * (K + 1) + t) * HW + q);
                const float oh = val_of(off, ((long long)b * 2 * K + 2 * k) * HW + q);
                const float ow = val_of(off, ((long long)b * 2 * K + 2 * k + 1) * HW + q);
                asum += ak;
                const float h_im = (float)(yy - PHh + i) + oh, w_im = (float)(xx - PWw + j) + ow;
                float v = 0.f;
                if (h_im > -1.f && w_im > -1.f && h_im < (float)H && w_im < (float)W) {
                    const int hl = (int)std::floor(h_im), wl = (int)std::floor(w_im), hh_ = hl + 1, wh = wl + 1;
                    const float lh = h_im - (float)hl, lw = w_im - (float)wl, hh = 1.f - lh, hw = 1.f - lw;
                    const float v1 = (hl >= 0 && wl >= 0) ? f(hl, wl) : 0.f;
                    const float v2 = (hl >= 0 && wh <= W - 1) ? f(hl, wh) : 0.f;
                    const float v3 = (hh_ <= H - 1 && wl >= 0) ? f(hh_, wl) : 0.f;
                    const float v4 = (hh_ <= H - 1 && wh <= W - 1) ? f(hh_, wh) : 0.f;
                    const float w1 = hh * hw, w2 = hh * lw, w3 = lh * hw, w4 = lh * lw;
                    v = (w1 * v1 + w2 * v2 + w3 * v3 + w4 * v4);
                }
                cols[k] = v * ak;
            }
            const float cref = f(yy, xx) * (1.0f - asum);
            for (int t = 0; t < K + 1; ++t) acc += t == REFk ? cref : cols[t < REFk ? t : t - 1];
            const float d = val_of(dep, g), m = d > 0.f ? 1.f : 0.f;
            const float o = rnd((1.0f - m) * acc + m * d);
            float gv;
            if constexpr (sizeof(T) == 4) gv = ref[g]; else gv = __half2float(ref[g]);
            bad += memcmp(&o, &gv, 4) != 0;
            ++checked;
        }
        printf("v0 vs host restatement: %lld of %lld sampled pixels differ%s\n", bad, checked, bad ? "  <-- BUG" : "");
    }

    std::vector<std::vector<float>> mean(vs.size()), mins(vs.size());
    std::vector<hipEvent_t> ev(2 * reps);
    for (auto &evt : ev) CK(hipEventCreate(&evt));
    for (int r = 0; r < rounds; ++r)
        for (size_t vi = 0; vi < vs.size(); ++vi) {
            StepArgs a = args_for(vs[vi]);
            void *kargs[] = {&a};
            for (int i = 0; i < reps; ++i)
                CK(hipExtLaunchKernel(vs[vi].fn, dim3(grid_of(vs[vi], B * a.tiles_x * a.tiles_y)), dim3(vs[vi].TH * vs[vi].TW / vs[vi].PX),
                                      kargs, 0, s, ev[2 * i], ev[2 * i + 1], 0));
            CK(hipStreamSynchronize(s));
            double sum = 0;
            float mn = 1e9f;
            for (int i = 0; i < reps; ++i) {
                float ms;
                CK(hipEventElapsedTime(&ms, ev[2 * i], ev[2 * i + 1]));
                sum += ms;
                mn = std::min(mn, ms);
            }
            mean[vi].push_back((float)(sum / reps));
            mins[vi].push_back(mn);
        }
    const double bytes = (double)ES * (4 + 3 * K) * N;
    printf("%-26s %10s %10s %10s  (%d B/px)\n", "variant", "med_us", "min_us", "GB/s(med)", ES * (4 + 3 * K));
    for (size_t vi = 0; vi < vs.size(); ++vi) {
        auto m = mean[vi];
        std::sort(m.begin(), m.end());
        float med = m[m.size() / 2];
        float mn = *std::min_element(mins[vi].begin(), mins[vi].end());
        printf("%-26s %10.2f %10.2f %10.0f\n", vs[vi].name.c_str(), med * 1e3, mn * 1e3, bytes / (med * 1e-3) / 1e9);
    }

    for (int px : {1, 2, 4}) {
        StepArgs a = args_for(vs[0]);
        void *kargs[] = {&a};
        const void *fn = px == 1 ? reinterpret_cast<const void *>(&stream_ceiling_t<T, K, 1>)
                       : px == 2 ? reinterpret_cast<const void *>(&stream_ceiling_t<T, K, 2>)
                                 : reinterpret_cast<const void *>(&stream_ceiling_t<T, K, 4>);
        unsigned grid = (unsigned)((N / px + 255) / 256);
        std::vector<float> ts;
        for (int r = 0; r < rounds; ++r) {
            for (int i = 0; i < reps; ++i)
                CK(hipExtLaunchKernel(fn, dim3(grid), dim3(256), kargs, 0, s, ev[2 * i], ev[2 * i + 1], 0));
            CK(hipStreamSynchronize(s));
            double sum = 0;
            for (int i = 0; i < reps; ++i) { float ms; CK(hipEventElapsedTime(&ms, ev[2 * i], ev[2 * i + 1])); sum += ms; }
            ts.push_back((float)(sum / reps));
        }
        std::sort(ts.begin(), ts.end());
        printf("stream ceiling px%-8d %10.2f us  (%.0f GB/s)\n", px, ts[ts.size() / 2] * 1e3,
               bytes / (ts[ts.size() / 2] * 1e-3) / 1e9);
    }

    return 0;
}

int main(int argc, char **argv) {
    // usage: step_bench MODE [B H W] [reps] [rounds] [sigma];  MODE = k8f32 | k16f16
    std::string mode = argc >= 2 ? argv[1] : "k8f32";
    int B = 8, H = 228, W = 304, reps = 100, rounds = 5;
    float sigma = 2.0f;
    if (argc >= 5) { B = atoi(argv[2]); H = atoi(argv[3]); W = atoi(argv[4]); }
    if (argc >= 6) reps = atoi(argv[5]);
    if (argc >= 7) rounds = atoi(argv[6]);
    if (argc >= 8) sigma = (float)atof(argv[7]);
    printf("mode=%s\n", mode.c_str());
    if (mode == "k16f16") return run<__half, 1, 17>(B, H, W, reps, rounds, sigma);
    return run<float, 3, 3>(B, H, W, reps, rounds, sigma);
}
