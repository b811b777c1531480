// tools/lds_mode_probe.hip -- does launching a workgroup with > 64 KiB of LDS
// change the speed of later 64-KiB-LDS kernels in the same process?
// (a 4-wave attention instantiation ran 2-4x slower after a
// 128-KiB-LDS instantiation had run.)  Times an LDS-streaming probe kernel at
// 64 KiB before and after one launch at 128 KiB, and the real attention_h3
// kernel (4 waves, 64 KiB) before and after the same.
// Build: hipcc -O3 --offload-arch=gfx950 -std=c++17 -ffp-contract=off -I pointdsc_amd/csrc \
//        tools/lds_mode_probe.hip -o tools/lds_mode_probe
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "attention_h3.hpp"

using namespace pdsc;

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

// Each workgroup streams its LDS allocation `rounds` times (ds_write + ds_read of 16 B per lane).
__global__ __launch_bounds__(256) void probe_kernel(int lds_bytes, int rounds, float *out) {
    extern __shared__ __attribute__((aligned(16))) float sm[];
    const int n4 = lds_bytes / 16;
    f32x4 acc = {0, 0, 0, 0};
    for (int r = 0; r < rounds; ++r) {
        for (int i = threadIdx.x; i < n4; i += 256)
            reinterpret_cast<f32x4 *>(sm)[i] = f32x4{(float)i, (float)r, 1.0f, 2.0f};
        __syncthreads();
        for (int i = threadIdx.x; i < n4; i += 256) acc += reinterpret_cast<const f32x4 *>(sm)[(i * 7) % n4];
        __syncthreads();
    }
    if (acc[0] == 12345.0f) out[blockIdx.x] = acc[1];
}

static float time_probe(int lds, int grid, hipStream_t s, float *out) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    hipLaunchKernelGGL(probe_kernel, dim3(grid), dim3(256), lds, s, lds, 64, out);
    CK(hipEventRecord(a, s));
    for (int i = 0; i < 5; ++i) hipLaunchKernelGGL(probe_kernel, dim3(grid), dim3(256), lds, s, lds, 64, out);
    CK(hipEventRecord(b, s));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    return ms / 5;
}

int main() {
    hipStream_t s;
    CK(hipStreamCreate(&s));
    CK(hipFuncSetAttribute((const void *)probe_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    float *out;
    CK(hipMalloc(&out, 1 << 20));
    // attention inputs: B pairs x N, zero Q/K/V (timing only), packed M of zeros
    const int B = 8, N = 5000;
    AttnGridH3 g = attention_h3_grid<4>(B, N, 512);
    const size_t per = (size_t)B * g.Npad * 2 * CH;
    _Float16 *qkv;
    CK(hipMalloc(&qkv, 3 * per * sizeof(_Float16)));
    CK(hipMemset(qkv, 0, 3 * per * sizeof(_Float16)));
    const size_t mfl = (size_t)B * mpack_floats(N);
    float *M, *op, *ml;
    CK(hipMalloc(&M, mfl * 4));
    CK(hipMemset(M, 0, mfl * 4));
    CK(hipMalloc(&op, (size_t)B * g.nsplit * g.Npad * CH * 4));
    CK(hipMalloc(&ml, (size_t)B * g.nsplit * g.Npad * 2 * 4));
    const int G = g.B * g.nqb * g.nsplit;
    auto time_attn = [&]() {
        hipEvent_t a, b;
        CK(hipEventCreate(&a));
        CK(hipEventCreate(&b));
        hipLaunchKernelGGL((attention_h3_kernel<4, true, true>), dim3(G), dim3(256), attention_h3_lds_bytes<4>(), s,
                           qkv, qkv + per, qkv + 2 * per, M, g, op, ml);
        CK(hipEventRecord(a, s));
        for (int i = 0; i < 5; ++i)
            hipLaunchKernelGGL((attention_h3_kernel<4, true, true>), dim3(G), dim3(256), attention_h3_lds_bytes<4>(),
                               s, qkv, qkv + per, qkv + 2 * per, M, g, op, ml);
        CK(hipEventRecord(b, s));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        return ms / 5;
    };
    const int grid = 2048;
    printf("probe 64K before: %.3f ms   attention(4 waves, 64K) before: %.3f ms\n", time_probe(64 * 1024, grid, s, out),
           time_attn());
    printf("one probe launch at 128K: %.3f ms\n", time_probe(128 * 1024, grid, s, out));
    printf("probe 64K after:  %.3f ms   attention(4 waves, 64K) after:  %.3f ms\n", time_probe(64 * 1024, grid, s, out),
           time_attn());
    printf("probe 32K after:  %.3f ms\n", time_probe(32 * 1024, grid, s, out));
    return 0;
}
