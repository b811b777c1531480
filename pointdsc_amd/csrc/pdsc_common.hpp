// pdsc_common.hpp -- device helpers shared by the gfx950 kernels of libpdsc.
//
// Numerics contract: the library is compiled with -ffp-contract=off, so every
// a*b+c in this code is two roundings unless written as __builtin_fmaf; sqrtf
// and '/' are the correctly-rounded IEEE forms (hipcc's default
// -fhip-fp32-correctly-rounded-divide-sqrt), matching torch-CPU fp32.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define PDSC_DEV __device__ __forceinline__

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

namespace pdsc {

constexpr int WAVE = 64;

// v_mfma_f32_32x32x2_f32: D(32x32) += A(32x2) B(2x32), exact f32 fma chain.
// lane l supplies A[l&31][l>>5] and B[l>>5][l&31]; D register r of lane l
// holds D[acc_row(r, l>>5)][l&31].
PDSC_DEV f32x16 mfma32(float a, float b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}
PDSC_DEV constexpr int acc_row(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }

PDSC_DEV f32x16 zero16() {
    f32x16 z;
#pragma unroll
    for (int i = 0; i < 16; ++i) z[i] = 0.0f;
    return z;
}

// torch.norm(p_i - p_j, dim=-1) as torch-CPU evaluates it for a 3-vector
// (models/PointDSC.py:151-152); bit-exact, see oracle/exact.c.
PDSC_DEV float pdist3(float ax, float ay, float az, float bx, float by, float bz) {
    const float dx = ax - bx, dy = ay - by, dz = az - bz;
    return sqrtf(__builtin_fmaf(dz, dz, __builtin_fmaf(dy, dy, dx * dx)));
}

// |v| for a residual vector, same evaluation order as pdist3.
PDSC_DEV float norm3(float dx, float dy, float dz) {
    return sqrtf(__builtin_fmaf(dz, dz, __builtin_fmaf(dy, dy, dx * dx)));
}

template <typename T> PDSC_DEV T wave_sum(T v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
}
PDSC_DEV float wave_max(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o));
    return v;
}

// Rigid transform applied to one point, as utils/SE3.py:43-57 /
// models/PointDSC.py:325 compute it (R @ p + t, no fma), and the residual norm.
PDSC_DEV float residual(const float *T, float x, float y, float z, float tx, float ty, float tz) {
    const float px = (T[0] * x + T[1] * y) + T[2] * z + T[3];
    const float py = (T[4] * x + T[5] * y) + T[6] * z + T[7];
    const float pz = (T[8] * x + T[9] * y) + T[10] * z + T[11];
    return norm3(px - tx, py - ty, pz - tz);
}

// ---------------------------------------------------------------------------
// 3x3 weighted-Kabsch rotation in fp64 (replaces torch.svd(H.cpu()) of
// models/common.py:36-41).  R = V diag(1,1,det(V U^T)) U^T with H = U S V^T.
// The result is independent of the SVD's sign choices: with u3 = u1 x u2,
// R = v1 u1^T + v2 u2^T + det(V) v3 u3^T.
// ---------------------------------------------------------------------------
PDSC_DEV void jacobi_eig3(double A[3][3], double V[3][3]) {
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) V[i][j] = (i == j) ? 1.0 : 0.0;
    for (int sweep = 0; sweep < 12; ++sweep) {
        const double off = A[0][1] * A[0][1] + A[0][2] * A[0][2] + A[1][2] * A[1][2];
        const double dia = A[0][0] * A[0][0] + A[1][1] * A[1][1] + A[2][2] * A[2][2];
        if (off <= 1e-30 * dia || off == 0.0) break;
        for (int p = 0; p < 2; ++p) {
            for (int q = p + 1; q < 3; ++q) {
                const double apq = A[p][q];
                if (apq == 0.0) continue;
                const double theta = (A[q][q] - A[p][p]) / (2.0 * apq);
                const double t = (theta >= 0 ? 1.0 : -1.0) / (fabs(theta) + sqrt(theta * theta + 1.0));
                const double c = 1.0 / sqrt(t * t + 1.0), s = t * c;
                for (int k = 0; k < 3; ++k) {  // A = J^T A J
                    const double akp = A[k][p], akq = A[k][q];
                    A[k][p] = c * akp - s * akq;
                    A[k][q] = s * akp + c * akq;
                }
                for (int k = 0; k < 3; ++k) {
                    const double apk = A[p][k], aqk = A[q][k];
                    A[p][k] = c * apk - s * aqk;
                    A[q][k] = s * apk + c * aqk;
                }
                for (int k = 0; k < 3; ++k) {
                    const double vkp = V[k][p], vkq = V[k][q];
                    V[k][p] = c * vkp - s * vkq;
                    V[k][q] = s * vkp + c * vkq;
                }
            }
        }
    }
}

PDSC_DEV void cross3(const double *a, const double *b, double *c) {
    c[0] = a[1] * b[2] - a[2] * b[1];
    c[1] = a[2] * b[0] - a[0] * b[2];
    c[2] = a[0] * b[1] - a[1] * b[0];
}

PDSC_DEV double normalize3(double *a) {
    const double n = sqrt(a[0] * a[0] + a[1] * a[1] + a[2] * a[2]);
    if (n > 0) { a[0] /= n; a[1] /= n; a[2] /= n; }
    return n;
}

// Any unit vector orthogonal to a (deterministic).
PDSC_DEV void orthogonal3(const double *a, double *o) {
    const double e[3][3] = {{1, 0, 0}, {0, 1, 0}, {0, 0, 1}};
    int best = 0;
    double bm = fabs(a[0]);
    if (fabs(a[1]) < bm) { best = 1; bm = fabs(a[1]); }
    if (fabs(a[2]) < bm) { best = 2; }
    cross3(a, e[best], o);
    normalize3(o);
}

// H (row-major 3x3, H[i][j] = sum w Am_i Bm_j) -> R (row-major, fp64).
PDSC_DEV void kabsch_rotation(const double H[9], double R[9]) {
    double A[3][3], V[3][3];
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) {
            double s = 0;
            for (int k = 0; k < 3; ++k) s += H[k * 3 + i] * H[k * 3 + j];  // H^T H
            A[i][j] = s;
        }
    jacobi_eig3(A, V);
    // sort eigenpairs descending
    int ord[3] = {0, 1, 2};
    double lam[3] = {A[0][0], A[1][1], A[2][2]};
    for (int i = 0; i < 2; ++i)
        for (int j = 0; j < 2 - i; ++j)
            if (lam[ord[j]] < lam[ord[j + 1]]) { int t = ord[j]; ord[j] = ord[j + 1]; ord[j + 1] = t; }
    double v[3][3], u[3][3];  // v[i] = i-th right singular vector
    for (int i = 0; i < 3; ++i)
        for (int k = 0; k < 3; ++k) v[i][k] = V[k][ord[i]];
    double scale = 0;
    for (int i = 0; i < 9; ++i) scale = fmax(scale, fabs(H[i]));
    if (!(scale > 0)) {  // H == 0: LAPACK returns U = V = I -> R = I
        for (int i = 0; i < 9; ++i) R[i] = (i % 4 == 0) ? 1.0 : 0.0;
        return;
    }
    for (int i = 0; i < 2; ++i)
        for (int r = 0; r < 3; ++r) u[i][r] = H[r * 3 + 0] * v[i][0] + H[r * 3 + 1] * v[i][1] + H[r * 3 + 2] * v[i][2];
    const double n0 = normalize3(u[0]);
    if (!(n0 > 1e-300)) orthogonal3(v[0], u[0]);
    // Gram-Schmidt u1 against u0 for robustness
    double d01 = u[1][0] * u[0][0] + u[1][1] * u[0][1] + u[1][2] * u[0][2];
    for (int r = 0; r < 3; ++r) u[1][r] -= d01 * u[0][r];
    const double n1 = normalize3(u[1]);
    if (!(n1 > 1e-12 * n0)) orthogonal3(u[0], u[1]);
    cross3(u[0], u[1], u[2]);
    double c12[3];
    cross3(v[1], v[2], c12);
    const double detV = v[0][0] * c12[0] + v[0][1] * c12[1] + v[0][2] * c12[2];
    const double d = detV < 0 ? -1.0 : 1.0;
    for (int a = 0; a < 3; ++a)
        for (int b = 0; b < 3; ++b)
            R[a * 3 + b] = v[0][a] * u[0][b] + v[1][a] * u[1][b] + d * v[2][a] * u[2][b];
}

}  // namespace pdsc
