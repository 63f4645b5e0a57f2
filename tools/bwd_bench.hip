// A/B harness for bwd_step_kernel variants (diagnostic tool, not part of the
// product).  One mid-loop backward iteration (t < T, not FIRST) of config C2 by
// default on synthetic inputs (offsets N(0, sigma^2)), g_inter
// non-zero so every pixel scatters.  Times each variant in interleaved rounds
// with dispatch-recorded events (hipExtLaunchKernel), next to a streaming
// ceiling that reads and writes the same planes with no gather or scatter.
// Variants with DIAG != 0 compute wrong gradients on purpose (they drop a part of
// the work to show its cost).
//
// usage: bwd_bench [B H W] [reps] [rounds] [sigma]
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <string>
#include <vector>

#include "../nlspn_eccv20_amd/csrc/nlspn_backward.h"

using namespace nlspn;

#define CHECK_HIP(x)                                                                   \
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
    int TH, TW;
};

template <int TH, int TW, int R, int DIAG, bool SPLIT = false>
Variant mk(const char *name) {
    return Variant{name, reinterpret_cast<const void *>(&bwd_step_kernel<3, 3, TH, TW, R, R, 4, true, false, DIAG, SPLIT>),
                   TH, TW};
}

// The two-pass step's planes streamed (29 reads, 3 writes per pixel), no gather or scatter.
__global__ void __launch_bounds__(256) bwd_split_stream_ceiling(BwdArgs a) {
    const long long HW = (long long)a.H * a.W;
    const long long g = (long long)blockIdx.x * 256 + threadIdx.x;
    if (g >= (long long)a.B * HW) return;
    const long long b = g / HW, q = g % HW;
    constexpr int K = 8;
    float s = a.p_out[g] + a.conf_eff[g] + a.dep[g] + a.gf_read[g] + a.g_inter[g];
    const float gc = a.g_conf[g];
    for (int k = 0; k < K; ++k) s += a.aff[(b * (K + 1) + k) * HW + q];
    for (int k = 0; k < 2 * K; ++k) s += a.off[b * a.off_bs + k * HW + q];
    a.g_conf[g] = gc + s;
    a.gf_read[g] = 0.f;
    a.go_out[g] = s;
}

// Same planes, same per-pixel lane mapping, streamed: 56 plane reads, 27 writes.
__global__ void __launch_bounds__(256) bwd_stream_ceiling(BwdArgs a) {
    const long long HW = (long long)a.H * a.W;
    const long long g = (long long)blockIdx.x * 256 + threadIdx.x;
    if (g >= (long long)a.B * HW) return;
    const long long b = g / HW, q = g % HW;
    constexpr int K = 8;
    float s = a.p_in[g] + a.conf[g] + a.p_out[g] + a.conf_eff[g] + a.dep[g] + a.gf_read[g] + a.g_inter[g];
    float gc = a.g_conf[g];
    for (int k = 0; k < K; ++k) s += a.aff[(b * (K + 1) + k) * HW + q];
    float o[2 * K], ga[K];
    for (int k = 0; k < 2 * K; ++k) o[k] = a.off[b * a.off_bs + k * HW + q] + a.g_off[(b * 2 * K + k) * HW + q];
    for (int k = 0; k < K; ++k) ga[k] = a.g_aff[(b * K + k) * HW + q];
    for (int k = 0; k < 2 * K; ++k) a.g_off[(b * 2 * K + k) * HW + q] = o[k] * s;
    for (int k = 0; k < K; ++k) a.g_aff[(b * K + k) * HW + q] = ga[k] + s;
    a.g_conf[g] = gc + s;
    a.gf_read[g] = 0.f;
    a.gf_write[g] += s;
}

int main(int argc, char **argv) {
    int B = 8, H = 228, W = 304, reps = 50, rounds = 5;
    float sigma = 2.0f;
    if (argc >= 4) { B = atoi(argv[1]); H = atoi(argv[2]); W = atoi(argv[3]); }
    if (argc >= 5) reps = atoi(argv[4]);
    if (argc >= 6) rounds = atoi(argv[5]);
    if (argc >= 7) sigma = (float)atof(argv[6]);
    constexpr int K = 8;
    const size_t N = (size_t)B * H * W;
    std::mt19937 rng(7240);
    std::uniform_real_distribution<float> U(0.f, 1.f);
    std::normal_distribution<float> Nrm(0.f, 1.f);
    auto plane = [&](size_t n, auto gen) { std::vector<float> v(n); for (auto &x : v) x = gen(); return v; };
    auto up = [&](const std::vector<float> &h) {
        float *d;
        CHECK_HIP(hipMalloc(&d, h.size() * 4));
        CHECK_HIP(hipMemcpy(d, h.data(), h.size() * 4, hipMemcpyHostToDevice));
        return d;
    };
    float *p_in = up(plane(N, [&] { return 10 * U(rng); }));
    float *p_out = up(plane(N, [&] { return 10 * U(rng); }));
    float *conf = up(plane(N, [&] { return U(rng); }));
    float *dep = up(plane(N, [&] { return U(rng) < 0.01f ? 10 * U(rng) : 0.f; }));
    float *aff = up(plane(N * (K + 1), [&] { return U(rng) / K; }));
    float *off = up(plane(N * 2 * K, [&] { return sigma * Nrm(rng); }));
    float *g_inter = up(plane(N, [&] { return Nrm(rng); }));
    float *gf_read = up(plane(N, [&] { return Nrm(rng); }));
    float *gf_write = up(plane(N, [] { return 0.f; }));
    float *g_aff = up(plane(N * K, [] { return 0.f; }));
    float *g_off = up(plane(N * 2 * K, [] { return 0.f; }));
    float *g_conf = up(plane(N, [] { return 0.f; }));

    BwdArgs a{};
    a.p_in = p_in; a.p_out = p_out; a.conf = conf; a.conf_eff = conf; a.dep = dep; a.aff = aff; a.off = off;
    a.g_pred = nullptr; a.g_inter = g_inter; a.gf_read = gf_read; a.gf_write = gf_write;
    a.g_aff = g_aff; a.g_off = g_off; a.g_conf = g_conf;
    a.off_bs = 2LL * K * H * W;
    a.B = B; a.H = H; a.W = W;
    a.last = 0;
    a.flags = kPreserve;
    float *go_out = up(plane(N, [] { return 0.f; }));
    a.go_out = go_out;
    a.go_bs = (long long)H * W;

    std::vector<Variant> vs = {
        mk<8, 32, 8, 0>("8x32 R8 (library)"),
        mk<8, 32, 8, 1>("8x32 R8 no-flush"),
        mk<8, 32, 8, 4>("8x32 R8 no-accum-RMW"),
        mk<8, 32, 8, 5>("8x32 R8 no-flush no-RMW"),
        mk<8, 32, 4, 0>("8x32 R4"),
        mk<16, 32, 8, 0>("16x32 R8"),
        mk<8, 64, 8, 0>("8x64 R8"),
        mk<16, 64, 8, 0>("16x64 R8"),
        {"stream ceiling (83 planes)", reinterpret_cast<const void *>(&bwd_stream_ceiling), 0, 0},
        mk<8, 32, 8, 0, true>("SPLIT 8x32 R8 (library)"),
        mk<8, 32, 8, 1, true>("SPLIT no-flush"),
        mk<8, 32, 8, 9, true>("SPLIT no-scatter"),
        mk<8, 32, 8, 16, true>("SPLIT LDS f64 atomics"),
        mk<8, 32, 8, 17, true>("SPLIT LDS f64 atomics no-flush"),
        {"SPLIT stream ceiling (32 planes)", reinterpret_cast<const void *>(&bwd_split_stream_ceiling), 0, 0},
    };
    const double bytes = 83.0 * 4 * N;
    std::vector<std::vector<float>> ms(vs.size());
    hipEvent_t e0, e1;
    CHECK_HIP(hipEventCreate(&e0));
    CHECK_HIP(hipEventCreate(&e1));
    for (int r = 0; r < rounds; ++r) {
        for (size_t v = 0; v < vs.size(); ++v) {
            BwdArgs x = a;
            dim3 grid, block;
            if (vs[v].TH) {
                x.tiles_x = (W + vs[v].TW - 1) / vs[v].TW;
                x.tiles_y = (H + vs[v].TH - 1) / vs[v].TH;
                grid = dim3(B * x.tiles_x * x.tiles_y);
                block = dim3(vs[v].TH * vs[v].TW);
            } else {
                grid = dim3((unsigned)((N + 255) / 256));
                block = dim3(256);
            }
            void *args[] = {&x};
            for (int i = 0; i < reps; ++i) {
                // g_inter keeps every pixel's gradient non-zero although gf_read is consumed
                CHECK_HIP(hipExtLaunchKernel(vs[v].fn, grid, block, args, 0, 0, e0, e1, 0));
                CHECK_HIP(hipEventSynchronize(e1));
                float t = 0.f;
                CHECK_HIP(hipEventElapsedTime(&t, e0, e1));
                if (r > 0 || i >= 5) ms[v].push_back(t);
            }
        }
    }
    printf("B=%d H=%d W=%d sigma=%.1f  (%zu px; 83 planes = %.1f MB)\n", B, H, W, sigma, N, bytes / 1e6);
    for (size_t v = 0; v < vs.size(); ++v) {
        auto &t = ms[v];
        std::sort(t.begin(), t.end());
        const float med = t[t.size() / 2];
        printf("%-30s median %8.2f us  min %8.2f us  (%6.0f GB/s at 83 planes)\n", vs[v].name.c_str(), 1e3f * med,
               1e3f * t[0], bytes / (med * 1e-3) / 1e9);
    }
    return 0;
}
