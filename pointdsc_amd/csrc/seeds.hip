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

// A workgroup owns SQ rows i (thread (slice, il): row il) and sweeps all j in
// 1024-point LDS tiles (one tile for N <= 1024: one global-load round trip);
// its 256 / SQ slices take disjoint parts of each tile, and the partial
// results meet in LDS.  SQ = 64 for batches; SQ = 16 when the batch has fewer
// than 512 row blocks of 64 (a single N = 1000 pair: 63 workgroups instead of
// 16, each thread 64 compares instead of 256).
constexpr int SEED_TILE = 1024;

template <int SQ>
__global__ __launch_bounds__(256) void local_max_kernel(const float *__restrict__ src,
                                                        const float *__restrict__ conf, int Nstr,
                                                        float R2, float *__restrict__ lm, Ragged rg) {
    constexpr int NSL = 256 / SQ, PER = SEED_TILE / NSL;  // slices, points per slice and tile
    __shared__ f32x4 tile[SEED_TILE];
    __shared__ int part[NSL][SQ];
    const int b = blockIdx.y, tid = threadIdx.x, sl = tid / SQ, il = tid % SQ;
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
    for (int j0 = 0; j0 < N; j0 += SEED_TILE) {
        __syncthreads();
#pragma unroll
        for (int e = 0; e < SEED_TILE / 256; ++e) {
            const int t = tid + 256 * e, j = j0 + t;
            // padding points never violate: conf -inf
            tile[t] = (j < N) ? f32x4{src[3 * j], src[3 * j + 1], src[3 * j + 2], conf[j]}
                              : f32x4{0.0f, 0.0f, 0.0f, -INFINITY};
        }
        __syncthreads();
        // violation: c_i < c_j and !(|s_i - s_j| >= R), the latter as !(x >= R2) on the
        // squared norm (sqrt_ge_threshold: exact, no sqrtf, branch-free)
        bool bad = false;
        const int jn = min(PER, max(N - j0 - sl * PER, 0));  // slice-uniform: skip the padded tail
#pragma unroll 8
        for (int jj = sl * PER; jj < sl * PER + jn; ++jj) {
            const f32x4 pj = tile[jj];
            const float x = sqdist3(xi, yi, zi, pj[0], pj[1], pj[2]);
            bad |= (ci < pj[3]) & !(x >= R2);
        }
        if (bad) ok = false;
    }
    part[sl][il] = ok;
    __syncthreads();
    if (sl == 0 && i < N) {
        int all = 1;
#pragma unroll
        for (int q = 0; q < NSL; ++q) all &= part[q][il];
        lm[(size_t)b * Nstr + i] = all ? 1.0f : 0.0f;
    }
}

template <int SQ>
__global__ __launch_bounds__(256) void seed_rank_kernel(const float *__restrict__ conf,
                                                        const float *__restrict__ lm, int Nstr, int Sstr,
                                                        int *__restrict__ seeds, Ragged rg) {
    constexpr int NSL = 256 / SQ, PER = SEED_TILE / NSL;
    __shared__ float ss[SEED_TILE];
    __shared__ int part[NSL][SQ];
    const int b = blockIdx.y, tid = threadIdx.x, sl = tid / SQ, il = tid % SQ;
    const int i = blockIdx.x * SQ + il;
    // this pair's points and seeds; Nstr, Sstr: the strides of conf / lm and seeds
    const int N = rg.n(b, Nstr), S = rg.s(b, Sstr);
    if (blockIdx.x * SQ >= N) return;  // workgroup-uniform
    conf += (size_t)b * Nstr;
    lm += (size_t)b * Nstr;
    const float si = (i < N) ? conf[i] * lm[i] : 0.0f;  // scores * is_local_max (:217)
    int rank = 0;
    for (int j0 = 0; j0 < N; j0 += SEED_TILE) {
        __syncthreads();
#pragma unroll
        for (int e = 0; e < SEED_TILE / 256; ++e) {
            const int t = tid + 256 * e;
            ss[t] = (j0 + t < N) ? conf[j0 + t] * lm[j0 + t] : -INFINITY;
        }
        __syncthreads();
        const int jn = min(PER, max(N - j0 - sl * PER, 0));
#pragma unroll 8
        for (int jj = sl * PER; jj < sl * PER + jn; ++jj) {
            const float sj = ss[jj];
            rank += (sj > si) || (sj == si && j0 + jj < i);
        }
    }
    part[sl][il] = rank;
    __syncthreads();
    if (sl == 0 && i < N) {
        rank = 0;
#pragma unroll
        for (int q = 0; q < NSL; ++q) rank += part[q][il];
        if (rank < S) seeds[(size_t)b * Sstr + rank] = i;
    }
}

static bool seed_small(int B, int N) { return (long)B * ((N + 63) / 64) < 512; }

hipError_t launch_local_max(const float *src, const float *conf, int B, int N, float radius,
                            float *lm, hipStream_t s, Ragged rg) {
    if (seed_small(B, N))
        hipLaunchKernelGGL(local_max_kernel<16>, dim3((N + 15) / 16, B), dim3(256), 0, s, src, conf, N,
                           sqrt_ge_threshold(radius), lm, rg);
    else
        hipLaunchKernelGGL(local_max_kernel<64>, dim3((N + 63) / 64, B), dim3(256), 0, s, src, conf, N,
                           sqrt_ge_threshold(radius), lm, rg);
    return hipGetLastError();
}

hipError_t launch_seed_rank(const float *conf, const float *lm, int B, int N, int S, int *seeds,
                            hipStream_t s, Ragged rg) {
    if (seed_small(B, N))
        hipLaunchKernelGGL(seed_rank_kernel<16>, dim3((N + 15) / 16, B), dim3(256), 0, s, conf, lm, N, S, seeds, rg);
    else
        hipLaunchKernelGGL(seed_rank_kernel<64>, dim3((N + 63) / 64, B), dim3(256), 0, s, conf, lm, N, S, seeds, rg);
    return hipGetLastError();
}

}  // namespace pdsc
