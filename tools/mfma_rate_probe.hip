// tools/mfma_rate_probe.hip -- cycles per v_mfma_f32_32x32x16_f16 for the operand
// placements attention_w64 uses (diagnostic): one 256-thread workgroup per CU,
// each wave a chain of asm MFMAs, s_memtime around the loop.
// Build: hipcc -O3 --offload-arch=gfx950 tools/mfma_rate_probe.hip -o tools/mfma_rate_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <algorithm>
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

// PV region as attention_w64 issues it: V fragments from LDS two fragments ahead
template <int WITH_FMA>
__global__ __launch_bounds__(256, 1) void probe_lds(const f16x8 *in, float *out, unsigned long long *cyc, int iters) {
    asm volatile("" ::: "a0", "a255");
    __shared__ __attribute__((aligned(16))) char lds[32768];
    for (int i = threadIdx.x; i < 2048; i += 256) reinterpret_cast<f16x8 *>(lds)[i] = in[i & 511];
    __syncthreads();
    const int lane = threadIdx.x & 63;
    f16x8 p = in[threadIdx.x], q = in[threadIdx.x + 256];
    float x = (float)threadIdx.x, y = 1.0001f;
    f16x8 vf[3][2];
    auto vread = [&](int i, f16x8(&f)[2]) {
        f[0] = *reinterpret_cast<const f16x8 *>(lds + 16384 + (2 * i) * 1024 + 16 * lane);
        f[1] = *reinterpret_cast<const f16x8 *>(lds + 16384 + (2 * i + 1) * 1024 + 16 * lane);
    };
    const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int it = 0; it < iters; ++it) {
        vread(0, vf[0]);
        vread(1, vf[1]);
#pragma unroll
        for (int k = 0; k < 24; ++k) {
            const int i = k / 3, m = k % 3;
            if (m == 0 && i + 2 < 8) vread(i + 2, vf[(i + 2) % 3]);
            const f16x8(&f)[2] = vf[i % 3];
            if (m == 0)
                asm volatile("v_mfma_f32_32x32x16_f16 a[0:15], %0, %1, a[0:15]" ::"v"(f[0]), "v"(p));
            else if (m == 1)
                asm volatile("v_mfma_f32_32x32x16_f16 a[0:15], %0, %1, a[0:15]" ::"v"(f[1]), "v"(q));
            else
                asm volatile("v_mfma_f32_32x32x16_f16 a[0:15], %0, %1, a[0:15]" ::"v"(f[0]), "v"(q));
            if (WITH_FMA) asm volatile("v_fma_f32 %0, %0, %1, %1" : "+v"(x) : "v"(y));
            __builtin_amdgcn_sched_barrier(0);
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    asm volatile("s_nop 15\n s_nop 15");
    float r;
    asm volatile("v_accvgpr_read_b32 %0, a5" : "=v"(r));
    out[blockIdx.x * 256 + threadIdx.x] = r + x;
    if (threadIdx.x % 64 == 0) {
        cyc[blockIdx.x * 4 + threadIdx.x / 64] = t1 - t0;
        cyc[4096 + blockIdx.x * 4 + threadIdx.x / 64] = r1 - r0;
    }
}

template <int MODE, int NT = 256>
__global__ __launch_bounds__(NT, 1) void probe(const f16x8 *in, float *out, unsigned long long *cyc, int iters) {
    asm volatile("" ::: "a0", "a255");
    f16x8 a = in[threadIdx.x], b = in[threadIdx.x + 256];
    f32x16 acc = {};
    float x = (float)threadIdx.x, y = 1.0001f, z = 0.5f;
    f16x8 dsv;
    const unsigned dsa = (threadIdx.x & 63) * 16;
    __shared__ char lds_[65536];
    if (threadIdx.x == 0) lds_[0] = 0;
    asm volatile("v_accvgpr_write_b32 a128, 0\n v_accvgpr_write_b32 a129, 0\n v_accvgpr_write_b32 a130, 0\n v_accvgpr_write_b32 a131, 0");
    const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int k = 0; k < 24; ++k) {
            if (MODE == 0)  // D, C in AGPR; A, B in VGPR (PV)
                asm volatile("v_mfma_f32_32x32x16_f16 a[0:15], %0, %1, a[0:15]" ::"v"(a), "v"(b));
            else if (MODE == 1)  // D, C in VGPR; B in AGPR (QK)
                asm volatile("v_mfma_f32_32x32x16_f16 %0, %1, a[128:131], %0" : "+v"(acc) : "v"(a));
            else if (MODE == 2)  // builtin, compiler's choice
                acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, acc, 0, 0, 0);
            else if (MODE == 3) {  // PV + one fma filler
                asm volatile("v_mfma_f32_32x32x16_f16 a[0:15], %0, %1, a[0:15]" ::"v"(a), "v"(b));
                asm volatile("v_fma_f32 %0, %0, %1, %1" : "+v"(x) : "v"(y));
            } else if (MODE == 4) {  // PV + exp + add + 3 split VALU
                asm volatile("v_mfma_f32_32x32x16_f16 a[0:15], %0, %1, a[0:15]" ::"v"(a), "v"(b));
                asm volatile("v_exp_f32 %0, %0\n v_add_f32 %0, %0, %1\n v_cvt_pk_f16_f32 %1, %0, %0\n v_fma_mixlo_f16 %1, %0, 1.0, -%1 op_sel_hi:[0,0,1]\n v_fma_mixhi_f16 %1, %0, 1.0, -%1 op_sel:[0,0,1] op_sel_hi:[0,0,1]" : "+v"(x), "+v"(y));
            } else if (MODE == 5) {  // PV + ds_read-ish filler: 2 VALU
                asm volatile("v_mfma_f32_32x32x16_f16 a[0:15], %0, %1, a[0:15]" ::"v"(a), "v"(b));
                asm volatile("v_fma_f32 %0, %0, %1, %1\n v_fma_f32 %0, %0, %1, %1\n v_fma_f32 %0, %0, %1, %1" : "+v"(x) : "v"(y));
            } else if (MODE == 6) {  // PV + one exp
                asm volatile("v_mfma_f32_32x32x16_f16 a[0:15], %0, %1, a[0:15]" ::"v"(a), "v"(b));
                asm volatile("v_exp_f32 %0, %0" : "+v"(x));
            } else if (MODE == 7) {  // PV + 4 independent fma
                asm volatile("v_mfma_f32_32x32x16_f16 a[0:15], %0, %1, a[0:15]" ::"v"(a), "v"(b));
                asm volatile("v_fma_f32 %0, %0, %2, %2\n v_fma_f32 %1, %1, %2, %2\n v_fma_f32 %0, %0, %2, %2\n v_fma_f32 %1, %1, %2, %2" : "+v"(x), "+v"(z) : "v"(y));
            } else if (MODE == 8) {  // PV + 8 independent fma
                asm volatile("v_mfma_f32_32x32x16_f16 a[0:15], %0, %1, a[0:15]" ::"v"(a), "v"(b));
                asm volatile("v_fma_f32 %0, %0, %2, %2\n v_fma_f32 %1, %1, %2, %2\n v_fma_f32 %0, %0, %2, %2\n v_fma_f32 %1, %1, %2, %2\n"
                             "v_fma_f32 %0, %0, %2, %2\n v_fma_f32 %1, %1, %2, %2\n v_fma_f32 %0, %0, %2, %2\n v_fma_f32 %1, %1, %2, %2" : "+v"(x), "+v"(z) : "v"(y));
            } else if (MODE == 9) {  // PV + 2 independent exp
                asm volatile("v_mfma_f32_32x32x16_f16 a[0:15], %0, %1, a[0:15]" ::"v"(a), "v"(b));
                asm volatile("v_exp_f32 %0, %0\n v_exp_f32 %1, %1" : "+v"(x), "+v"(z));
            } else if (MODE == 10) {  // PV + 16 independent fma
                asm volatile("v_mfma_f32_32x32x16_f16 a[0:15], %0, %1, a[0:15]" ::"v"(a), "v"(b));
#pragma unroll
                for (int u = 0; u < 4; ++u)
                asm volatile("v_fma_f32 %0, %0, %2, %2\n v_fma_f32 %1, %1, %2, %2\n v_fma_f32 %0, %0, %2, %2\n v_fma_f32 %1, %1, %2, %2" : "+v"(x), "+v"(z) : "v"(y));
            } else if (MODE == 11) {  // PV + 2 ds_read_b128 (independent, no wait)
                asm volatile("v_mfma_f32_32x32x16_f16 a[0:15], %0, %1, a[0:15]" ::"v"(a), "v"(b));
                asm volatile("ds_read_b128 %0, %1\n ds_read_b128 %0, %1 offset:1024" : "=v"(dsv) : "v"(dsa));
            }
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    asm volatile("s_nop 15\n s_nop 15");
    float r;
    asm volatile("v_accvgpr_read_b32 %0, a5" : "=v"(r));
    asm volatile("s_waitcnt lgkmcnt(0)");
    out[blockIdx.x * NT + threadIdx.x] = r + acc[3] + x + y + z + (float)dsv[0];
    if (threadIdx.x % 64 == 0 && threadIdx.x < 256) {
        cyc[blockIdx.x * 4 + threadIdx.x / 64] = t1 - t0;
        cyc[4096 + blockIdx.x * 4 + threadIdx.x / 64] = r1 - r0;
    }
}

int main() {
    const int G = 256, iters = 20000;
    f16x8 *in;
    float *out;
    unsigned long long *cyc;
    hipMalloc(&in, 512 * 16);
    {
        std::vector<unsigned short> h(512 * 8);
        unsigned x = 12345;
        for (auto &v : h) {
            x = x * 1664525u + 1013904223u;
            v = (unsigned short)(0x3000 + ((x >> 8) & 0x0fff)) ^ ((x >> 31) << 15);  // random f16 in +-[0.125, 1)
        }
        hipMemcpy(in, h.data(), h.size() * 2, hipMemcpyHostToDevice);
    }
    hipMalloc(&out, G * 512 * 4);
    hipMalloc(&cyc, 8192 * 8);
    std::vector<unsigned long long> h(8192);
    auto run = [&](auto k, const char *name, int nt = 256) {
        for (int r = 0; r < 2; ++r) hipLaunchKernelGGL(k, dim3(G), dim3(nt), 0, 0, in, out, cyc, iters);
        hipDeviceSynchronize();
        hipMemcpy(h.data(), cyc, h.size() * 8, hipMemcpyDeviceToHost);
        std::vector<unsigned long long> s(h.begin(), h.begin() + G * 4);
        std::vector<double> clk;
        for (int i = 0; i < G * 4; ++i)
            if (h[4096 + i]) clk.push_back((double)h[i] / h[4096 + i] * 0.1);
        std::sort(s.begin(), s.end());
        std::sort(clk.begin(), clk.end());
        printf("%-40s %.2f cycles per MFMA (median), clock %.2f GHz\n", name, (double)s[s.size() / 2] / (iters * 24.0),
               clk.empty() ? 0.0 : clk[clk.size() / 2]);
    };
    run(probe<0>, "PV: acc AGPR, A/B VGPR");
    run(probe<1>, "QK: acc VGPR, B AGPR");
    run(probe<2>, "builtin");
    run(probe<3>, "PV + 1 fma");
    run(probe<4>, "PV + exp add cvt mix mix");
    run(probe<5>, "PV + 3 dependent fma");
    run(probe<6>, "PV + 1 exp");
    run(probe<9>, "PV + 2 independent exp");
    run(probe<7>, "PV + 4 independent fma");
    run(probe<8>, "PV + 8 independent fma");
    run(probe<10>, "PV + 16 independent fma");
    run(probe<11>, "PV + 2 ds_read_b128");
    run(probe<0, 512>, "2 waves/SIMD: PV (per wave)", 512);
    run(probe<4, 512>, "2 waves/SIMD: PV + exp add cvt mix mix", 512);
    run(probe<8, 512>, "2 waves/SIMD: PV + 8 independent fma", 512);
    run(probe_lds<0>, "PV, V from LDS 2 frags ahead");
    run(probe_lds<1>, "PV, V from LDS + 1 fma");
    return 0;
}
