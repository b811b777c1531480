// tools/att_h3_bench.hip -- timing of the production attention_h3_kernel
// (packed M, XCD mapping) at the headline shape, for A/B builds of
// attention_h3.hpp (diagnostics; the numbers that count come from bench.py).
// Build: hipcc -O3 --offload-arch=gfx950 -std=c++17 -ffp-contract=off -I pointdsc_amd/csrc \
//        [-D...] tools/att_h3_bench.hip -o /tmp/att_h3_bench
// Run:   att_h3_bench [B=128] [N=1000] [reps=20]
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "attention_h3.hpp"

using namespace pdsc;
#ifndef NWV
#define NWV 4  // waves (x 32 queries) per workgroup
#endif

#define CK(x)                                                                       \
    do {                                                                            \
        hipError_t e_ = (x);                                                        \
        if (e_ != hipSuccess) {                                                     \
            printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__);        \
            exit(1);                                                                \
        }                                                                           \
    } while (0)

__global__ void fill_h(_Float16 *p, size_t n, unsigned seed, float scale) {
    const size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (i >= n) return;
    unsigned x = (unsigned)i * 2654435761u ^ seed;
    x ^= x >> 13;
    x *= 0x5bd1e995u;
    x ^= x >> 15;
    p[i] = (_Float16)(((x & 0xffff) / 65536.0f - 0.5f) * scale);
}
__global__ void fill_f(float *p, size_t n, unsigned seed) {
    const size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (i >= n) return;
    unsigned x = (unsigned)i * 2654435761u ^ seed;
    x ^= x >> 13;
    x *= 0x5bd1e995u;
    x ^= x >> 15;
    p[i] = (x & 0xffff) / 65536.0f;
}

int main(int argc, char **argv) {
    const int B = argc > 1 ? atoi(argv[1]) : 128, N = argc > 2 ? atoi(argv[2]) : 1000;
    const int reps = argc > 3 ? atoi(argv[3]) : 20;
    const AttnGridH3 g = attention_h3_grid<NWV>(B, N, 512);
    const size_t rows = (size_t)B * g.Npad * CH * 2, mper = mpack_floats(N);
    _Float16 *Q, *K, *V;
    float *M, *vexp, *op, *ml;
    CK(hipMalloc(&Q, rows * 2));
    CK(hipMalloc(&K, rows * 2));
    CK(hipMalloc(&V, rows * 2));
    CK(hipMalloc(&M, (size_t)B * mper * 4));
    CK(hipMalloc(&vexp, (size_t)B * (g.Npad / 32) * 4));
    CK(hipMalloc(&op, (size_t)B * g.nsplit * g.Npad * CH * 4));
    CK(hipMalloc(&ml, (size_t)B * g.nsplit * g.Npad * 2 * 4));
    hipLaunchKernelGGL(fill_h, dim3((rows + 255) / 256), dim3(256), 0, 0, Q, rows, 1u, 0.2f);
    hipLaunchKernelGGL(fill_h, dim3((rows + 255) / 256), dim3(256), 0, 0, K, rows, 2u, 0.2f);
    hipLaunchKernelGGL(fill_h, dim3((rows + 255) / 256), dim3(256), 0, 0, V, rows, 3u, 1.0f);
    hipLaunchKernelGGL(fill_f, dim3((B * mper + 255) / 256), dim3(256), 0, 0, M, (size_t)B * mper, 4u);
    CK(hipMemset(vexp, 0, (size_t)B * (g.Npad / 32) * 4));
    const size_t lds = attention_h3_lds_bytes<NWV>();
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    auto launch = [&] {
        hipLaunchKernelGGL((attention_h3_kernel<NWV, true, true>), dim3(g.B * g.nqb * g.nsplit), dim3(NWV * 64), lds, 0, Q,
                           K, V, vexp, M, g, op, ml);
    };
    for (int i = 0; i < 3; ++i) launch();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(a));
    for (int i = 0; i < reps; ++i) launch();
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    const double us = ms * 1e3 / reps, flop = 4.0 * B * (double)N * N * CH;
    std::vector<float> h(16);
    CK(hipMemcpy(h.data(), ml, 16 * 4, hipMemcpyDeviceToHost));
    printf("B=%d N=%d nsplit=%d grid=%d: %.2f us/launch, %.1f TFLOP/s (%.3f of 833.3)  ml[0..1]=%g %g\n", B, N, g.nsplit,
           g.B * g.nqb * g.nsplit, us, flop / us * 1e-6, flop / us * 1e-6 / 833.3, h[0], h[1]);
    return 0;
}
