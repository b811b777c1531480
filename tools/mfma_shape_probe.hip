// tools/mfma_shape_probe.hip -- f16 MFMA throughput by shape under the chip's
// load clock (diagnostic; MI355X_MICROARCH.md 'DVFS give-back' item 7 measured
// it for bf16): every CU runs 4 waves (one per SIMD, or 8 = two per SIMD), each
// a long loop of v_mfma_f32_32x32x16_f16 or v_mfma_f32_16x16x32_f16 on random
// fp16 operands re-read from LDS every step (as the attention reads K/V
// fragments; 32x32x16: 2 x 2 fragments -> 4 MFMAs, 16x16x32: 4 x 4 -> 16, the
// same LDS bytes per FLOP), independent accumulators.  Prints the
// wall TFLOP/s of back-to-back launches (~2 s each) and the in-kernel clock
// (s_memtime / s_memrealtime x 100 MHz).
// Build: hipcc -O3 --offload-arch=gfx950 -std=c++17 tools/mfma_shape_probe.hip -o tools/mfma_shape_probe
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <vector>
#include <algorithm>
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

// SHAPE 0: 32x32x16 (16384 MACs per instruction), 1: 16x16x32 (8192)
template <int SHAPE>
__global__ __launch_bounds__(512) void probe(const f16x8 *in, float *out, unsigned long long *clk, int iters) {
    __shared__ __attribute__((aligned(16))) f16x8 lds[1024];  // 16 KiB of random fp16
    for (int i = threadIdx.x; i < 1024; i += blockDim.x) lds[i] = in[(blockIdx.x * 1024 + i) % 65536];
    __syncthreads();
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    if constexpr (SHAPE == 0) {
        f32x16 c0 = {}, c1 = {}, c2 = {}, c3 = {};
        for (int it = 0; it < iters; ++it) {
            const int base = ((it * 8 + wave) & 15) * 64;
            const f16x8 a0 = lds[base + lane], b0 = lds[(base + 64 * 3 + lane) & 1023];
            const f16x8 a1 = lds[(base + 64 * 5 + lane) & 1023], b1 = lds[(base + 64 * 7 + lane) & 1023];
            c0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a0, b0, c0, 0, 0, 0);
            c1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a1, b0, c1, 0, 0, 0);
            c2 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a0, b1, c2, 0, 0, 0);
            c3 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a1, b1, c3, 0, 0, 0);
        }
        float s = 0.0f;
        for (int r = 0; r < 16; ++r) s += c0[r] + c1[r] + c2[r] + c3[r];
        out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    } else {
        f32x4 c[16] = {};
        for (int it = 0; it < iters; ++it) {
            const int base = ((it * 8 + wave) & 15) * 64;
            f16x8 a[4], b[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                a[j] = lds[(base + 64 * (2 * j) + lane) & 1023];
                b[j] = lds[(base + 64 * (2 * j + 1) + lane) & 1023];
            }
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    c[4 * i + j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[i], b[j], c[4 * i + j], 0, 0, 0);
        }
        float s = 0.0f;
        for (int j = 0; j < 16; ++j) s += c[j][0] + c[j][1] + c[j][2] + c[j][3];
        out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0) {
        clk[2 * blockIdx.x] = t1 - t0;
        clk[2 * blockIdx.x + 1] = r1 - r0;
    }
}

int main() {
    const int WG = 256, iters = 20000;
    std::vector<_Float16> h(65536 * 8);
    unsigned x = 12345u;
    for (auto &v : h) {
        x = x * 1664525u + 1013904223u;
        v = (_Float16)(((x >> 9) & 0xffff) / 32768.0f - 1.0f);
    }
    f16x8 *d;
    float *o;
    unsigned long long *c;
    CK(hipMalloc(&d, h.size() * 2));
    CK(hipMalloc(&o, WG * 512 * 4));
    CK(hipMalloc(&c, WG * 2 * 8));
    CK(hipMemcpy(d, h.data(), h.size() * 2, hipMemcpyHostToDevice));
    for (int waves : {4, 8})
        for (int shape = 0; shape < 2; ++shape) {
            auto launch = [&] {
                if (shape == 0)
                    hipLaunchKernelGGL(probe<0>, dim3(WG), dim3(64 * waves), 0, 0, d, o, c, iters);
                else
                    hipLaunchKernelGGL(probe<1>, dim3(WG), dim3(64 * waves), 0, 0, d, o, c, iters);
            };
            launch();
            CK(hipDeviceSynchronize());
            int n = 0;
            const auto t0 = std::chrono::steady_clock::now();
            double el = 0;
            while (el < 2.0) {
                launch();
                ++n;
                if (n % 8 == 0) {
                    CK(hipDeviceSynchronize());
                    el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
                }
            }
            CK(hipDeviceSynchronize());
            el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
            std::vector<unsigned long long> hc(WG * 2);
            CK(hipMemcpy(hc.data(), c, hc.size() * 8, hipMemcpyDeviceToHost));
            std::vector<double> ghz;
            for (int i = 0; i < WG; ++i) ghz.push_back((double)hc[2 * i] / (double)hc[2 * i + 1] * 0.1);
            std::sort(ghz.begin(), ghz.end());
            // MACs per iteration and wave: 4 x 32x32x16 = 65536, 16 x 16x16x32 = 131072
            const double flop = 2.0 * (shape == 0 ? 65536.0 : 131072.0) * iters * waves * WG * n;
            printf("waves/CU %d shape %s: %.1f TFLOP/s (fp16 dense), in-kernel clock median %.2f GHz, %d launches\n",
                   waves, shape == 0 ? "32x32x16" : "16x16x32", flop / el * 1e-12, ghz[WG / 2], n);
            fflush(stdout);
        }
    return 0;
}
