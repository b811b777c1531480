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
typedef float f32x2 __attribute__((ext_vector_type(2)));
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

// The squared norm under pdist3's sqrtf (models/PointDSC.py:151-152 order).
PDSC_DEV float sqdist3(float ax, float ay, float az, float bx, float by, float bz) {
    const float dx = ax - bx, dy = ay - by, dz = az - bz;
    return __builtin_fmaf(dz, dz, __builtin_fmaf(dy, dy, dx * dx));
}

// Comparisons against a correctly rounded square root without taking it:
// sqrtf is monotone, so for the smallest float t with sqrtf(t) >= R,
//   sqrtf(x) >= R  <=>  x >= t      and      sqrtf(x) < R  <=>  x < t
// for every x (NaN included: both sides false).  Host-side, IEEE sqrtf.
inline float sqrt_ge_threshold(float R) {
    if (R != R) return R;            // NaN: every comparison false, as with sqrtf(x) >= NaN
    if (R <= 0.0f) return 0.0f;      // sqrtf(x) >= R for every x >= 0
    float t = R * R;
    while (t > 0.0f && sqrtf(__builtin_nextafterf(t, 0.0f)) >= R) t = __builtin_nextafterf(t, 0.0f);
    while (sqrtf(t) < R) t = __builtin_nextafterf(t, __builtin_inff());
    return t;
}

// Correctly rounded sqrtf for x == 0, +inf or x >= 2^-96 (the caller takes
// the library sqrtf when a wave holds a smaller positive x): v_sqrt_f32 is
// within 1 ulp, and the neighbour whose fma residual shows it closer replaces
// it -- the same correction hipcc's -fhip-fp32-correctly-rounded-divide-sqrt
// emits, minus the denormal rescaling and class fix-ups this domain needs not.
PDSC_DEV float cr_sqrt(float x) {
    const float s = __builtin_amdgcn_sqrtf(x);
    const float dn = __uint_as_float(__float_as_uint(s) - 1u), up = __uint_as_float(__float_as_uint(s) + 1u);
    const float rdn = __builtin_fmaf(-dn, s, x), rup = __builtin_fmaf(-up, s, x);
    float r = rdn <= 0.0f ? dn : s;
    r = rup > 0.0f ? up : r;
    return x == 0.0f ? x : r;
}

// Correctly rounded x / d given rcp = RN(1/d) (Markstein: q = RN(x rcp) is
// within 1 ulp, the fma remainder is exact, and one fma correction rounds
// to RN(x / d); x, d normal and no overflow -- d = sigma_d^2 > 0).
PDSC_DEV float cr_div(float x, float d, float rcp) {
    const float q = x * rcp;
    const float r = __builtin_fmaf(-q, d, x);
    return __builtin_fmaf(r, rcp, q);
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
// Sum over the 64 lanes without an LDS round trip: DPP butterflies inside each
// row of 16 (quad swaps, half-row and row mirrors), then gfx950's
// v_permlane16_swap / v_permlane32_swap across rows; every lane ends with the
// same bits (each step adds two equal-by-symmetry partial sums).  A different
// summation order from wave_sum's xor butterfly.
PDSC_DEV float wave_sum_dpp(float x) {
    x += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), 0xB1, 0xF, 0xF, false));
    x += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), 0x4E, 0xF, 0xF, false));
    x += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), 0x141, 0xF, 0xF, false));
    x += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), 0x140, 0xF, 0xF, false));
    const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    x = __uint_as_float(r[0]) + __uint_as_float(r[1]);
    const auto q = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    return __uint_as_float(q[0]) + __uint_as_float(q[1]);
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
// residual()^2 before its sqrtf: residual(...) < tau  <=>  residual_sq(...) < sqrt_ge_threshold(tau)
PDSC_DEV float residual_sq(const float *T, float x, float y, float z, float tx, float ty, float tz) {
    const float px = (T[0] * x + T[1] * y) + T[2] * z + T[3];
    const float py = (T[4] * x + T[5] * y) + T[6] * z + T[7];
    const float pz = (T[8] * x + T[9] * y) + T[10] * z + T[11];
    const float dx = px - tx, dy = py - ty, dz = pz - tz;
    return __builtin_fmaf(dz, dz, __builtin_fmaf(dy, dy, dx * dx));
}

// ---------------------------------------------------------------------------
// 3x3 weighted-Kabsch rotation in fp64 (replaces torch.svd(H.cpu()) of
// models/common.py:36-41).  R = V diag(1,1,det(V U^T)) U^T with H = U S V^T.
// The result is independent of the SVD's sign choices: with u3 = u1 x u2,
// R = v1 u1^T + v2 u2^T + det(V) v3 u3^T.
// Written with named scalars only (no runtime-indexed arrays -> no scratch),
// so it runs SIMD-parallel when every lane solves its own H.
// ---------------------------------------------------------------------------
struct D3 {
    double x, y, z;
};
PDSC_DEV D3 d3(double x, double y, double z) { return D3{x, y, z}; }
PDSC_DEV double dot3(const D3 &a, const D3 &b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
PDSC_DEV D3 cross3(const D3 &a, const D3 &b) {
    return D3{a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x};
}
PDSC_DEV double normalize3(D3 &a) {
    const double n = sqrt(dot3(a, a));
    if (n > 0) {
        const double inv = 1.0 / n;
        a.x *= inv;
        a.y *= inv;
        a.z *= inv;
    }
    return n;
}
PDSC_DEV D3 orthogonal3(const D3 &a) {  // a unit vector orthogonal to a (deterministic)
    const double ax = fabs(a.x), ay = fabs(a.y), az = fabs(a.z);
    D3 e = (ax <= ay && ax <= az) ? d3(1, 0, 0) : (ay <= az ? d3(0, 1, 0) : d3(0, 0, 1));
    D3 o = cross3(a, e);
    normalize3(o);
    return o;
}

// One Jacobi rotation zeroing a_pq of a symmetric 3x3 (r = the third index);
// vp, vq = eigenvector columns p and q.
PDSC_DEV void jrot(double &app, double &aqq, double &apq, double &arp, double &arq, D3 &vp, D3 &vq) {
    if (apq == 0.0) return;
    const double theta = (aqq - app) / (2.0 * apq);
    const double t = (theta >= 0 ? 1.0 : -1.0) / (fabs(theta) + sqrt(theta * theta + 1.0));
    const double c = 1.0 / sqrt(t * t + 1.0), s = t * c;
    app -= t * apq;
    aqq += t * apq;
    apq = 0.0;
    const double rp = arp, rq = arq;
    arp = c * rp - s * rq;
    arq = s * rp + c * rq;
    const D3 p0 = vp, q0 = vq;
    vp = d3(c * p0.x - s * q0.x, c * p0.y - s * q0.y, c * p0.z - s * q0.z);
    vq = d3(s * p0.x + c * q0.x, s * p0.y + c * q0.y, s * p0.z + c * q0.z);
}

PDSC_DEV void cswap(double &la, double &lb, D3 &va, D3 &vb) {  // order (la, va) >= (lb, vb)
    if (la < lb) {
        const double t = la;
        la = lb;
        lb = t;
        const D3 tv = va;
        va = vb;
        vb = tv;
    }
}

// H row-major (H[i][j] = sum w Am_i Bm_j) -> R row-major.
PDSC_DEV void kabsch_rotation(const double H[9], double R[9]) {
    // A = H^T H (symmetric)
    double a00 = H[0] * H[0] + H[3] * H[3] + H[6] * H[6];
    double a11 = H[1] * H[1] + H[4] * H[4] + H[7] * H[7];
    double a22 = H[2] * H[2] + H[5] * H[5] + H[8] * H[8];
    double a01 = H[0] * H[1] + H[3] * H[4] + H[6] * H[7];
    double a02 = H[0] * H[2] + H[3] * H[5] + H[6] * H[8];
    double a12 = H[1] * H[2] + H[4] * H[5] + H[7] * H[8];
    D3 v0 = d3(1, 0, 0), v1 = d3(0, 1, 0), v2 = d3(0, 0, 1);  // eigenvector columns
    for (int sweep = 0; sweep < 10; ++sweep) {
        const double off = a01 * a01 + a02 * a02 + a12 * a12;
        const double dia = a00 * a00 + a11 * a11 + a22 * a22;
        // off-diagonal below ~1e-13 of the diagonal: far beyond the fp32 result's needs
        if (off <= 1e-26 * dia || off == 0.0) break;
        jrot(a00, a11, a01, a02, a12, v0, v1);  // (p,q,r) = (0,1,2)
        jrot(a00, a22, a02, a01, a12, v0, v2);  // (0,2,1)
        jrot(a11, a22, a12, a01, a02, v1, v2);  // (1,2,0)
    }
    cswap(a00, a11, v0, v1);
    cswap(a00, a22, v0, v2);
    cswap(a11, a22, v1, v2);
    double scale = 0;
    for (int i = 0; i < 9; ++i) scale = fmax(scale, fabs(H[i]));
    if (!(scale > 0)) {  // H == 0: LAPACK returns U = V = I -> R = I
        for (int i = 0; i < 9; ++i) R[i] = (i % 4 == 0) ? 1.0 : 0.0;
        return;
    }
    D3 u0 = d3(H[0] * v0.x + H[1] * v0.y + H[2] * v0.z, H[3] * v0.x + H[4] * v0.y + H[5] * v0.z,
               H[6] * v0.x + H[7] * v0.y + H[8] * v0.z);
    D3 u1 = d3(H[0] * v1.x + H[1] * v1.y + H[2] * v1.z, H[3] * v1.x + H[4] * v1.y + H[5] * v1.z,
               H[6] * v1.x + H[7] * v1.y + H[8] * v1.z);
    const double n0 = normalize3(u0);
    if (!(n0 > 1e-300)) u0 = orthogonal3(v0);
    const double d01 = dot3(u1, u0);  // Gram-Schmidt u1 against u0 for robustness
    u1 = d3(u1.x - d01 * u0.x, u1.y - d01 * u0.y, u1.z - d01 * u0.z);
    const double n1 = normalize3(u1);
    if (!(n1 > 1e-12 * n0)) u1 = orthogonal3(u0);
    const D3 u2 = cross3(u0, u1);
    const double d = dot3(v0, cross3(v1, v2)) < 0 ? -1.0 : 1.0;  // det(V); det(U) = +1
    R[0] = v0.x * u0.x + v1.x * u1.x + d * v2.x * u2.x;
    R[1] = v0.x * u0.y + v1.x * u1.y + d * v2.x * u2.y;
    R[2] = v0.x * u0.z + v1.x * u1.z + d * v2.x * u2.z;
    R[3] = v0.y * u0.x + v1.y * u1.x + d * v2.y * u2.x;
    R[4] = v0.y * u0.y + v1.y * u1.y + d * v2.y * u2.y;
    R[5] = v0.y * u0.z + v1.y * u1.z + d * v2.y * u2.z;
    R[6] = v0.z * u0.x + v1.z * u1.x + d * v2.z * u2.x;
    R[7] = v0.z * u0.y + v1.z * u1.y + d * v2.z * u2.y;
    R[8] = v0.z * u0.z + v1.z * u1.z + d * v2.z * u2.z;
}

}  // namespace pdsc
