// tools/compat_bench.hip -- A/B timing of the a1 compatibility kernel against
// pure-store baselines with the same and with row-contiguous write patterns
// (what does the N x N write cost by itself?).
// Build: hipcc -O3 --offload-arch=gfx950 -std=c++17 -ffp-contract=off -I pointdsc_amd/csrc \
//        tools/compat_bench.hip -o tools/compat_bench
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>
#include "compat.hip"

using namespace pdsc;
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

// store-only, the production tile pattern (64x64 tile + its transpose, 16 B per lane)
__global__ __launch_bounds__(256) void store_tiles(int N, int ntile, float *M) {
    int t = blockIdx.x, ti = 0;
    while (t >= ntile - ti) { t -= ntile - ti; ++ti; }
    const int tj = ti + t;
    M += (size_t)blockIdx.y * N * N;
    const int cq = threadIdx.x & 15, rq = threadIdx.x >> 4;
    for (int rr = 0; rr < 4; ++rr) {
        const int i = ti * 64 + rq + 16 * rr, j = tj * 64 + cq * 4;
        if (i < N && j + 3 < N) *reinterpret_cast<f32x4 *>(M + (size_t)i * N + j) = f32x4{1, 2, 3, 4};
        const int i2 = tj * 64 + rq + 16 * rr, j2 = ti * 64 + cq * 4;
        if (ti != tj && i2 < N && j2 + 3 < N) *reinterpret_cast<f32x4 *>(M + (size_t)i2 * N + j2) = f32x4{1, 2, 3, 4};
    }
}
// store-only, the packed layout's pattern (four contiguous 4 KiB tiles per 64 x 64 block)
__global__ __launch_bounds__(256) void store_packed(int N, int ntile, float *M) {
    int t = blockIdx.x, ti = 0;
    while (t >= ntile - ti) { t -= ntile - ti; ++ti; }
    const int tj = ti + t, nt32 = mpack_ntile(N);
    M += (size_t)blockIdx.y * mpack_floats(N);
    const int cq = threadIdx.x & 15, rq = threadIdx.x >> 4, tc = 2 * tj + (cq >> 3);
    for (int rr = 0; rr < 4; ++rr) {
        const int r = rq + 16 * rr, tr = 2 * ti + (r >> 5);
        if (tr > tc || tr >= nt32 || tc >= nt32) continue;
#ifdef COMPAT_NT
        __builtin_nontemporal_store(f32x4{1, 2, 3, 4}, reinterpret_cast<f32x4 *>(M + (size_t)mpack_tile(tr, tc, nt32) * 1024 + (r & 31) * 32 + ((cq * 4) & 31)));
#else
        *reinterpret_cast<f32x4 *>(M + (size_t)mpack_tile(tr, tc, nt32) * 1024 + (r & 31) * 32 + ((cq * 4) & 31)) = f32x4{1, 2, 3, 4};
#endif
    }
}
// store-only, whole rows: block = 4 rows, thread = 16 B columns strided
__global__ __launch_bounds__(256) void store_rows(int N, float *M) {
    M += (size_t)blockIdx.y * N * N;
    const int i = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (i >= N) return;
    for (int j = (threadIdx.x & 63) * 4; j + 3 < N; j += 256)
        *reinterpret_cast<f32x4 *>(M + (size_t)i * N + j) = f32x4{1, 2, 3, 4};
}

int main(int argc, char **argv) {
    int B = argc > 1 ? atoi(argv[1]) : 8, N = argc > 2 ? atoi(argv[2]) : 5000, iters = 10;
    const bool dm = argc > 3 && argv[3][0] == '3';  // 3DMatch-like: 30 % inliers under a rigid motion
    std::vector<float> hp((size_t)B * N * 6);
    srand(1);
    for (auto &x : hp) x = 3.0f * (float)rand() / (float)RAND_MAX;
    if (dm) {
        const float c = 0.8660254f, s = 0.5f;  // 30 degrees about z, then a shift
        for (size_t p = 0; p < (size_t)B * N; ++p) {
            if (rand() % 10 >= 3) continue;
            const float *a = &hp[p * 3];
            float *t = &hp[(size_t)B * N * 3 + p * 3];
            t[0] = c * a[0] - s * a[1] + 0.3f + 0.005f * (float)rand() / (float)RAND_MAX;
            t[1] = s * a[0] + c * a[1] - 0.2f + 0.005f * (float)rand() / (float)RAND_MAX;
            t[2] = a[2] + 0.1f + 0.005f * (float)rand() / (float)RAND_MAX;
        }
    }
    float *dp, *dM, *dsd;
    CK(hipMalloc(&dp, hp.size() * 4)); CK(hipMalloc(&dM, (size_t)B * N * N * 4)); CK(hipMalloc(&dsd, 4));
    float sd = 0.1f;
    CK(hipMemcpy(dp, hp.data(), hp.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(dsd, &sd, 4, hipMemcpyHostToDevice));
    const int ntile = (N + 63) / 64, ntri = ntile * (ntile + 1) / 2;
    auto run = [&](int v) {
        if (v == 0) CK(launch_compat(dp, dp + (size_t)B * N * 3, B, N, dsd, dM, 0));
        if (v == 1) hipLaunchKernelGGL(store_tiles, dim3(ntri, B), dim3(256), 0, 0, N, ntile, dM);
        if (v == 2) hipLaunchKernelGGL(store_rows, dim3((N + 3) / 4, B), dim3(256), 0, 0, N, dM);
        if (v == 3) CK(launch_compat_packed(dp, dp + (size_t)B * N * 3, B, N, dsd, dM, 0));
        if (v == 4) hipLaunchKernelGGL(store_packed, dim3(ntri, B), dim3(256), 0, 0, N, ntile, dM);
    };
    const char *names[] = {"compat_kernel", "store-only tiles", "store-only rows", "compat_packed", "store-only packed"};
    const int NV = 5;
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    std::vector<std::vector<float>> t(NV);
    for (int round = 0; round < 5; ++round)
        for (int v = 0; v < NV; ++v) {
            run(v);
            CK(hipEventRecord(e0, 0));
            for (int i = 0; i < iters; ++i) run(v);
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float ms; CK(hipEventElapsedTime(&ms, e0, e1));
            t[v].push_back(ms / iters);
        }
    const double bytes = (double)B * N * N * 4;
    for (int v = 0; v < NV; ++v) {
        std::sort(t[v].begin(), t[v].end());
        printf("%-18s %s B=%d N=%d median %8.1f us  %7.1f GB/s (dense-equivalent)\n", names[v], dm ? "3dm" : "rnd", B, N, t[v][2] * 1e3, bytes / (t[v][2] * 1e-3) / 1e9);
    }
    return 0;
}
