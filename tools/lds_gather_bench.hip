// LDS bilinear-gather microbenchmark (diagnostic, not product code): the resident
// kernel's tap phase reads each bilinear footprint as two ds_read_b64 (the top and the
// bottom pair of the window stored twice, fwin / fwinB).  Alternative: a "quad image"
// that stores every cell's whole 2x2 footprint (f[y][x], f[y][x+1], f[y+1][x],
// f[y+1][x+1]) so a footprint is ONE ds_read_b128 (4x the window cells).
// Same geometry as C2's parts: 576 threads, each 4 pixels of a row x 8 taps, tap point =
// pixel + 3x3 base + N(0, sigma^2) offsets, 256 blocks (one per CU).
// usage: lds_gather_bench [sigma]   prints ns per launch and per tap-pixel for both forms
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

constexpr int NT = 576, QX = 32, ROWS = 18;   // 18 rows x 32 quads = 576 quads per part
constexpr int PAD = 12, WW = 4 * QX + 2 * PAD, WH = ROWS + 2 * PAD;
constexpr int CELLS = WW * WH;
constexpr int K = 8, E = 4, REPS = 64;

// idx[tid][k][e]: window cell of the footprint's top-left corner
__global__ void __launch_bounds__(NT) gather_b64(const unsigned short *idx, const float *wts, float *out) {
    extern __shared__ float lds[];
    float *fwin = lds, *fwinB = lds + CELLS;
    for (int i = threadIdx.x; i < CELLS; i += NT) { fwin[i] = (float)(i % 97); fwinB[i] = (float)((i + 1) % 97); }
    __syncthreads();
    unsigned id[K][E];
    for (int k = 0; k < K; ++k)
        for (int e = 0; e < E; ++e) id[k][e] = idx[(threadIdx.x * K + k) * E + e];
    const float w = wts[threadIdx.x];
    float acc = 0.f;
    for (int r = 0; r < REPS; ++r) {
#pragma unroll
        for (int k = 0; k < K; ++k)
#pragma unroll
            for (int e = 0; e < E; ++e) {
                const unsigned i = id[k][e];
                const float *base = (i & 1) ? fwinB + (i - 1) : fwin + i;  // 8-byte aligned pair
                const float2 a = *reinterpret_cast<const float2 *>(base);
                const float2 b = *reinterpret_cast<const float2 *>(base + WW);
                acc += w * a.x + a.y * w + b.x * w + b.y;
            }
        asm volatile("" : "+v"(acc));
    }
    out[blockIdx.x * NT + threadIdx.x] = acc;
}

__global__ void __launch_bounds__(NT) gather_b128(const unsigned short *idx, const float *wts, float *out) {
    extern __shared__ float lds[];
    for (int i = threadIdx.x; i < CELLS; i += NT) {
        lds[4 * i + 0] = (float)(i % 97); lds[4 * i + 1] = (float)((i + 1) % 97);
        lds[4 * i + 2] = (float)((i + WW) % 97); lds[4 * i + 3] = (float)((i + WW + 1) % 97);
    }
    __syncthreads();
    unsigned id[K][E];
    for (int k = 0; k < K; ++k)
        for (int e = 0; e < E; ++e) id[k][e] = idx[(threadIdx.x * K + k) * E + e];
    const float w = wts[threadIdx.x];
    float acc = 0.f;
    for (int r = 0; r < REPS; ++r) {
#pragma unroll
        for (int k = 0; k < K; ++k)
#pragma unroll
            for (int e = 0; e < E; ++e) {
                const float4 q = *reinterpret_cast<const float4 *>(lds + 4 * id[k][e]);
                acc += w * q.x + q.y * w + q.z * w + q.w;
            }
        asm volatile("" : "+v"(acc));
    }
    out[blockIdx.x * NT + threadIdx.x] = acc;
}

static float time_kernel(void (*k)(const unsigned short *, const float *, float *), size_t lds,
                         const unsigned short *idx, const float *w, float *out) {
    hipFuncSetAttribute(reinterpret_cast<const void *>(k), hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    for (int i = 0; i < 3; ++i) hipLaunchKernelGGL(k, dim3(256), dim3(NT), lds, 0, idx, w, out);
    hipEventRecord(a);
    const int n = 20;
    for (int i = 0; i < n; ++i) hipLaunchKernelGGL(k, dim3(256), dim3(NT), lds, 0, idx, w, out);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0.f;
    hipEventElapsedTime(&ms, a, b);
    return ms / n;
}

int main(int argc, char **argv) {
    const float sigma = argc > 1 ? (float)atof(argv[1]) : 2.0f;
    std::vector<unsigned short> h(NT * K * E);
    srand(7);
    auto gauss = [] {
        const float u1 = (rand() + 1.f) / (RAND_MAX + 2.f), u2 = (rand() + 1.f) / (RAND_MAX + 2.f);
        return sqrtf(-2.f * logf(u1)) * cosf(6.2831853f * u2);
    };
    for (int t = 0; t < NT; ++t)
        for (int k = 0; k < K; ++k)
            for (int e = 0; e < E; ++e) {
                const int tt = k < K / 2 ? k : k + 1, dy = tt / 3 - 1, dx = tt % 3 - 1;
                const int y = t / QX + PAD, x = 4 * (t % QX) + e + PAD;
                int yy = (int)floorf(y + dy + sigma * gauss()), xx = (int)floorf(x + dx + sigma * gauss());
                yy = yy < 0 ? 0 : (yy > WH - 2 ? WH - 2 : yy);
                xx = xx < 0 ? 0 : (xx > WW - 2 ? WW - 2 : xx);
                h[(t * K + k) * E + e] = (unsigned short)(yy * WW + xx);
            }
    unsigned short *idx;
    float *w, *out;
    hipMalloc(&idx, h.size() * 2);
    hipMalloc(&w, NT * 4);
    hipMalloc(&out, 256 * NT * 4);
    hipMemcpy(idx, h.data(), h.size() * 2, hipMemcpyHostToDevice);
    hipMemset(w, 0, NT * 4);
    const float t64 = time_kernel(gather_b64, 2 * CELLS * 4, idx, w, out);
    const float t128 = time_kernel(gather_b128, 4 * CELLS * 4, idx, w, out);
    const double taps = (double)256 * NT * K * E * REPS;
    printf("sigma %.1f  cells %d  two ds_read_b64: %.3f ms (%.3f ns per CU-tap)  one ds_read_b128: %.3f ms (%.3f ns)\n",
           sigma, CELLS, t64, t64 * 1e6 / (taps / 256), t128, t128 * 1e6 / (taps / 256));
    const double per_iter = (double)NT * K * E;  // tap-pixels of one part per iteration
    printf("per resident iteration (576 quads x 32 tap-pixels): b64 %.3f us, b128 %.3f us\n",
           t64 * 1e3 / REPS * (per_iter / (NT * K * E)), t128 * 1e3 / REPS * (per_iter / (NT * K * E)));
    return 0;
}
