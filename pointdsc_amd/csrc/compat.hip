// compat.hip -- a1: the N x N spatial-compatibility matrix.
//
// Replaces models/PointDSC.py:150-153:
//   src_dist = norm(s_i - s_j); M = clamp(1 - (src_dist - norm(t_i - t_j))^2 / sigma_d^2, min=0)
// Bit-exact with torch-CPU fp32 (pdist3 = sqrtf(fma(dz,dz,fma(dy,dy,dx*dx)))).
//
// Roofline: HBM-write bound, 4 N^2 bytes per pair out, 24 N in.  M is
// symmetric bit-for-bit (squares of negated differences are identical), so
// each workgroup computes one 64x64 tile of the upper triangle once and
// writes it twice: directly, and transposed through LDS.  Each element costs
// two correctly-rounded sqrtf and one correctly-rounded division (~40 VALU
// ops), so computing each pair once halves the VALU work that would otherwise
// sit right at the write roofline.  Stores are 16 B per lane.
#include "pdsc_internal.hpp"

namespace pdsc {

constexpr int CT = 64;  // tile edge

__global__ __launch_bounds__(256) void compat_kernel(const float *__restrict__ src,
                                                     const float *__restrict__ tgt, int N,
                                                     int ntile, const float *__restrict__ sigma_d_ptr,
                                                     float *__restrict__ M) {
    __shared__ float tileT[CT][CT + 1];
    __shared__ float pts[4][CT][3];  // row src, row tgt, col src, col tgt
    // linear upper-triangular tile index -> (ti, tj), ti <= tj
    int t = blockIdx.x, ti = 0;
    while (t >= ntile - ti) { t -= ntile - ti; ++ti; }
    const int tj = ti + t;
    const int b = blockIdx.y;
    const float sd = sigma_d_ptr[0];
    const float s2 = sd * sd;
    src += (size_t)b * N * 3;
    tgt += (size_t)b * N * 3;
    M += (size_t)b * N * N;
    const int tid = threadIdx.x;
    const int i0 = ti * CT, j0 = tj * CT;
    for (int e = tid; e < CT * 3; e += 256) {
        const int p = e / 3, c = e % 3;
        pts[0][p][c] = (i0 + p < N) ? src[(size_t)(i0 + p) * 3 + c] : 0.f;
        pts[1][p][c] = (i0 + p < N) ? tgt[(size_t)(i0 + p) * 3 + c] : 0.f;
        pts[2][p][c] = (j0 + p < N) ? src[(size_t)(j0 + p) * 3 + c] : 0.f;
        pts[3][p][c] = (j0 + p < N) ? tgt[(size_t)(j0 + p) * 3 + c] : 0.f;
    }
    __syncthreads();
    // thread -> 4 consecutive columns (cq*4..+3) of 4 rows (rq, rq+16, rq+32, rq+48)
    const int cq = tid & 15, rq = tid >> 4;
    const bool vec = (N & 3) == 0;
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) {
        const int r = rq + 16 * rr;
        const int i = i0 + r;
        const float six = pts[0][r][0], siy = pts[0][r][1], siz = pts[0][r][2];
        const float tix = pts[1][r][0], tiy = pts[1][r][1], tiz = pts[1][r][2];
        float out[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int c = cq * 4 + q;
            const float ds = pdist3(six, siy, siz, pts[2][c][0], pts[2][c][1], pts[2][c][2]);
            const float dt = pdist3(tix, tiy, tiz, pts[3][c][0], pts[3][c][1], pts[3][c][2]);
            const float d = ds - dt;
            const float m = 1.0f - (d * d) / s2;
            out[q] = m > 0.0f ? m : 0.0f;
            tileT[c][r] = out[q];
        }
        if (i < N) {
            const int j = j0 + cq * 4;
            float *dst = M + (size_t)i * N + j;
            if (vec && j + 3 < N) {
                *reinterpret_cast<f32x4 *>(dst) = f32x4{out[0], out[1], out[2], out[3]};
            } else {
                for (int q = 0; q < 4; ++q)
                    if (j + q < N) dst[q] = out[q];
            }
        }
    }
    if (ti == tj) return;  // diagonal tile: the transpose is itself
    __syncthreads();
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) {
        const int r = rq + 16 * rr;  // row of the transposed tile = column of the tile
        const int i = j0 + r;
        if (i >= N) continue;
        const int j = i0 + cq * 4;
        float *dst = M + (size_t)i * N + j;
        const float o0 = tileT[r][cq * 4], o1 = tileT[r][cq * 4 + 1], o2 = tileT[r][cq * 4 + 2],
                    o3 = tileT[r][cq * 4 + 3];
        if (vec && j + 3 < N) {
            *reinterpret_cast<f32x4 *>(dst) = f32x4{o0, o1, o2, o3};
        } else {
            const float o[4] = {o0, o1, o2, o3};
            for (int q = 0; q < 4; ++q)
                if (j + q < N) dst[q] = o[q];
        }
    }
}

hipError_t launch_compat(const float *src, const float *tgt, int B, int N, const float *sigma_d,
                         float *M, hipStream_t stream) {
    const int ntile = (N + CT - 1) / CT;
    const int ntri = ntile * (ntile + 1) / 2;
    hipLaunchKernelGGL(compat_kernel, dim3(ntri, B), dim3(256), 0, stream, src, tgt, N, ntile,
                       sigma_d, M);
    return hipGetLastError();
}

}  // namespace pdsc
