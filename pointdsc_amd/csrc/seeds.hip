// seeds.hip -- a5: radius NMS + top-S seed ranking.
//
// Replaces models/PointDSC.py:199-217 (pick_seeds, bs = 1 per pair):
//   is_local_max_i = AND_j ( c_i >= c_j  OR  |s_i - s_j| >= R )
//   seeds = argsort(c * is_local_max, descending)[:S]
// The distance is recomputed from xyz bit-exactly as a1 computes src_dist, so
// no N x N matrix is read.  torch's argsort orders ties arbitrarily; here ties
// are broken by ascending index (rank_i = #{s_j > s_i} + #{j < i : s_j == s_i}),
// which is deterministic and equals torch's order whenever scores are distinct.
// Both kernels are O(N^2) compare loops over LDS-staged tiles (VALU bound, a
// few microseconds at N = 5000).
#include "pdsc_internal.hpp"

namespace pdsc {

// A workgroup owns 64 rows i (lane = i) and sweeps all j in 256-point LDS
// tiles; its four waves take disjoint quarters of each tile, so a pair of
// N = 1000 runs on 16 workgroups instead of 4.  Partial results meet in LDS.
constexpr int SQ = 64;  // rows per workgroup

__global__ __launch_bounds__(256) void local_max_kernel(const float *__restrict__ src,
                                                        const float *__restrict__ conf, int Nstr,
                                                        float R2, float *__restrict__ lm, Ragged rg) {
    __shared__ f32x4 tile[256];
    __shared__ int part[4][SQ];
    const int b = blockIdx.y, tid = threadIdx.x, q = tid >> 6, il = tid & 63;
    const int i = blockIdx.x * SQ + il;
    const int N = rg.n(b, Nstr);  // this pair's points; Nstr: the row stride
    if (blockIdx.x * SQ >= N) return;  // workgroup-uniform
    src += (size_t)b * Nstr * 3;
    conf += (size_t)b * Nstr;
    float xi = 0, yi = 0, zi = 0, ci = 0;
    if (i < N) {
        xi = src[3 * i];
        yi = src[3 * i + 1];
        zi = src[3 * i + 2];
        ci = conf[i];
    }
    bool ok = true;
    for (int j0 = 0; j0 < N; j0 += 256) {
        __syncthreads();
        const int j = j0 + tid;
        // padding points never violate: conf -inf
        tile[tid] = (j < N) ? f32x4{src[3 * j], src[3 * j + 1], src[3 * j + 2], conf[j]}
                            : f32x4{0.0f, 0.0f, 0.0f, -INFINITY};
        __syncthreads();
        // violation: c_i < c_j and !(|s_i - s_j| >= R), the latter as !(x >= R2) on the
        // squared norm (sqrt_ge_threshold: exact, no sqrtf, branch-free)
        bool bad = false;
#pragma unroll 8
        for (int jj = q * 64; jj < q * 64 + 64; ++jj) {
            const f32x4 pj = tile[jj];
            const float x = sqdist3(xi, yi, zi, pj[0], pj[1], pj[2]);
            bad |= (ci < pj[3]) & !(x >= R2);
        }
        if (bad) ok = false;
    }
    part[q][il] = ok;
    __syncthreads();
    if (q == 0 && i < N) lm[(size_t)b * Nstr + i] = (part[0][il] & part[1][il] & part[2][il] & part[3][il]) ? 1.0f : 0.0f;
}

__global__ __launch_bounds__(256) void seed_rank_kernel(const float *__restrict__ conf,
                                                        const float *__restrict__ lm, int Nstr, int Sstr,
                                                        int *__restrict__ seeds, Ragged rg) {
    __shared__ float ss[256];
    __shared__ int part[4][SQ];
    const int b = blockIdx.y, tid = threadIdx.x, q = tid >> 6, il = tid & 63;
    const int i = blockIdx.x * SQ + il;
    // this pair's points and seeds; Nstr, Sstr: the strides of conf / lm and seeds
    const int N = rg.n(b, Nstr), S = rg.s(b, Sstr);
    if (blockIdx.x * SQ >= N) return;  // workgroup-uniform
    conf += (size_t)b * Nstr;
    lm += (size_t)b * Nstr;
    const float si = (i < N) ? conf[i] * lm[i] : 0.0f;  // scores * is_local_max (:217)
    int rank = 0;
    for (int j0 = 0; j0 < N; j0 += 256) {
        __syncthreads();
        ss[tid] = (j0 + tid < N) ? conf[j0 + tid] * lm[j0 + tid] : -INFINITY;
        __syncthreads();
#pragma unroll 8
        for (int jj = q * 64; jj < q * 64 + 64; ++jj) {
            const float sj = ss[jj];
            rank += (sj > si) || (sj == si && j0 + jj < i);
        }
    }
    part[q][il] = rank;
    __syncthreads();
    if (q == 0 && i < N) {
        rank = part[0][il] + part[1][il] + part[2][il] + part[3][il];
        if (rank < S) seeds[(size_t)b * Sstr + rank] = i;
    }
}

hipError_t launch_local_max(const float *src, const float *conf, int B, int N, float radius,
                            float *lm, hipStream_t s, Ragged rg) {
    hipLaunchKernelGGL(local_max_kernel, dim3((N + SQ - 1) / SQ, B), dim3(256), 0, s, src, conf, N,
                       sqrt_ge_threshold(radius), lm, rg);
    return hipGetLastError();
}

hipError_t launch_seed_rank(const float *conf, const float *lm, int B, int N, int S, int *seeds,
                            hipStream_t s, Ragged rg) {
    hipLaunchKernelGGL(seed_rank_kernel, dim3((N + SQ - 1) / SQ, B), dim3(256), 0, s, conf, lm, N, S,
                       seeds, rg);
    return hipGetLastError();
}

}  // namespace pdsc
