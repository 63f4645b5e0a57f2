// Setup-load microbenchmark (diagnostic, not product code): how fast can the resident
// kernel's setup pull a part's invariant planes when they are NOT the L2-hot outputs of a
// preceding step-1 launch?  C2's shape: 8 NYU images (228 x 304), 32 parts per image, one
// 576-thread workgroup per CU, each thread loading its quad (16 B) of NP planes (27: the
// raw K = 8 affinities, 2K offsets, conf, dep, pred_init).  Compared with a streaming
// kernel (many workgroups, grid-stride) reading the same bytes.  Cache states: "hot" (the
// previous run's reads), "l2cold" (a 48 MB scrub write between runs: evicts the XCD L2s),
// "cold" (a 640 MB scrub: evicts the Infinity Cache too).
// usage: setup_load_bench [planes]     prints microseconds per launch and GB/s
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>

constexpr int B = 8, H = 228, W = 304, W4 = W / 4, GY = 8, GX = 4, NT = 576;

typedef float f32x4 __attribute__((ext_vector_type(4)));

// one part per workgroup: rows [r0, r1) x quad columns [c0, c1) of image b
__global__ void __launch_bounds__(NT) part_loads(const float *planes, int np, float *out) {
    const int part = blockIdx.x, b = part / (GY * GX), j = part % (GY * GX), py = j / GX, px = j % GX;
    const int r0 = py * H / GY, r1 = (py + 1) * H / GY, c0 = px * W4 / GX, c1 = (px + 1) * W4 / GX;
    const int nqw = c1 - c0, nown = (r1 - r0) * nqw;
    const int t = threadIdx.x;
    if (t >= nown) return;
    const int y = r0 + t / nqw, x = 4 * (c0 + t % nqw);
    const size_t HW = (size_t)H * W;
    const float *base = planes + (size_t)b * np * HW + (size_t)y * W + x;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    f32x4 v[32];
#pragma unroll
    for (int p = 0; p < 32; ++p)
        if (p < np) v[p] = *reinterpret_cast<const f32x4 *>(base + p * HW);
#pragma unroll
    for (int p = 0; p < 32; ++p)
        if (p < np) acc += v[p];
    out[(size_t)part * NT + t] = acc[0] + acc[1] + acc[2] + acc[3];
}

__global__ void __launch_bounds__(256) stream_loads(const f32x4 *p, size_t n4, float *out) {
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (size_t)gridDim.x * 256) acc += p[i];
    out[(size_t)blockIdx.x * 256 + threadIdx.x] = acc[0] + acc[1] + acc[2] + acc[3];
}

__global__ void scrub(f32x4 *p, size_t n4, float v) {
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (size_t)gridDim.x * 256)
        p[i] = f32x4{v, v, v, v};
}

int main(int argc, char **argv) {
    const int np = argc > 1 ? atoi(argv[1]) : 27;
    const size_t HW = (size_t)H * W, bytes = (size_t)B * np * HW * 4;
    float *planes, *out;
    f32x4 *junk;
    const size_t jbytes = 640ull << 20;
    hipMalloc(&planes, bytes);
    hipMalloc(&out, (size_t)4096 * 256 * 4);
    hipMalloc(&junk, jbytes);
    hipMemset(planes, 0, bytes);
    hipEvent_t a, e;
    hipEventCreate(&a);
    hipEventCreate(&e);
    const char *states[3] = {"hot", "l2cold", "cold"};
    const size_t scrub_bytes[3] = {0, 48ull << 20, jbytes};
    for (int form = 0; form < 2; ++form) {
        for (int s = 0; s < 3; ++s) {
            std::vector<float> ts;
            for (int r = 0; r < 12; ++r) {
                if (scrub_bytes[s]) hipLaunchKernelGGL(scrub, dim3(2048), dim3(256), 0, 0, junk, scrub_bytes[s] / 16, (float)r);
                hipEventRecord(a);
                if (form == 0) hipLaunchKernelGGL(part_loads, dim3(B * GY * GX), dim3(NT), 0, 0, planes, np, out);
                else hipLaunchKernelGGL(stream_loads, dim3(4096), dim3(256), 0, 0, reinterpret_cast<const f32x4 *>(planes),
                                        bytes / 16, out);
                hipEventRecord(e);
                hipEventSynchronize(e);
                float ms = 0.f;
                hipEventElapsedTime(&ms, a, e);
                if (r >= 2) ts.push_back(ms * 1e3f);
            }
            std::sort(ts.begin(), ts.end());
            const float med = ts[ts.size() / 2];
            printf("%-12s %-7s planes %d  %.1f MB  median %.2f us  min %.2f us  %.2f TB/s\n",
                   form == 0 ? "part_loads" : "stream", states[s], np, bytes / 1e6, med, ts[0], bytes / med / 1e6);
        }
    }
    return 0;
}
