// MFMA accumulation rounding probe: one wave chains n v_mfma_f32_32x32x16_f16
// into one accumulator (C = A B + C) and, separately, forms each step's A B in a
// zeroed accumulator and adds it on the VALU (round-to-nearest fp32).  Both
// against the exact sum (fp64 on the host; every product is exact).  A linear
// growth of the chained error with n (a signed bias) means the accumulator
// rounds other than to nearest.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <random>
#include <vector>

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

__global__ void probe(const _Float16 *A, int n, float *chained, float *valu) {
    const int lane = threadIdx.x;
    f32x16 acc = {}, tot = {};
    f16x8 b;
    for (int i = 0; i < 8; ++i) b[i] = (_Float16)1.0f;
    for (int s = 0; s < n; ++s) {
        f16x8 a = *reinterpret_cast<const f16x8 *>(A + ((size_t)s * 64 + lane) * 8);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, acc, 0, 0, 0);
        f32x16 z = {};
        z = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, z, 0, 0, 0);
        for (int r = 0; r < 16; ++r) tot[r] += z[r];
    }
    for (int r = 0; r < 16; ++r) {
        chained[lane * 16 + r] = acc[r];
        valu[lane * 16 + r] = tot[r];
    }
}

int main() {
    const int NS[] = {8, 64, 512, 4096};
    std::mt19937 rng(5);
    std::uniform_real_distribution<float> U(0.0f, 1.0f);
    for (int n : NS) {
        std::vector<_Float16> A((size_t)n * 64 * 8);
        for (auto &x : A) x = (_Float16)U(rng);
        _Float16 *dA;
        float *dc, *dv;
        hipMalloc(&dA, A.size() * 2);
        hipMalloc(&dc, 1024 * 4);
        hipMalloc(&dv, 1024 * 4);
        hipMemcpy(dA, A.data(), A.size() * 2, hipMemcpyHostToDevice);
        hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, dA, n, dc, dv);
        std::vector<float> c(1024), v(1024);
        hipMemcpy(c.data(), dc, 4096, hipMemcpyDeviceToHost);
        hipMemcpy(v.data(), dv, 4096, hipMemcpyDeviceToHost);
        // acc element (lane, r): row i = 8 (r / 4) + 4 (lane / 32) ... ; with B = ones every
        // column j is the same: C[i][j] = sum_s sum_k A_s[i][k].  A operand: lane (i = lane % 32,
        // k-group lane / 32) holds A[i][8 (lane/32) .. +7].  Row of acc (lane, r):
        // 8 (r / 4) + 4 (lane / 32) + r % 4.
        std::vector<double> ex(32, 0.0);
        for (int s = 0; s < n; ++s)
            for (int l = 0; l < 64; ++l)
                for (int e = 0; e < 8; ++e) ex[l % 32] += (double)(float)A[((size_t)s * 64 + l) * 8 + e];
        double bc = 0, bv = 0, mc = 0, mv = 0;
        for (int l = 0; l < 64; ++l)
            for (int r = 0; r < 16; ++r) {
                const int row = 8 * (r / 4) + 4 * (l / 32) + r % 4;
                const double dcx = (c[l * 16 + r] - ex[row]) / ex[row], dvx = (v[l * 16 + r] - ex[row]) / ex[row];
                bc += dcx / 1024;
                bv += dvx / 1024;
                mc = fmax(mc, fabs(dcx));
                mv = fmax(mv, fabs(dvx));
            }
        printf("n=%5d  chained: mean rel err %+.3e max %.3e | valu-summed: mean %+.3e max %.3e  (eps %.3e)\n", n, bc,
               mc, bv, mv, 5.96e-8);
        hipFree(dA);
        hipFree(dc);
        hipFree(dv);
    }
    return 0;
}
