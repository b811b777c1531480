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

__global__ __launch_bounds__(256) void local_max_kernel(const float *__restrict__ src,
                                                        const float *__restrict__ conf, int N,
                                                        float R, float *__restrict__ lm) {
    __shared__ float sx[256], sy[256], sz[256], sc[256];
    const int b = blockIdx.y, tid = threadIdx.x, i = blockIdx.x * 256 + tid;
    src += (size_t)b * N * 3;
    conf += (size_t)b * N;
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
        if (j < N) {
            sx[tid] = src[3 * j];
            sy[tid] = src[3 * j + 1];
            sz[tid] = src[3 * j + 2];
            sc[tid] = conf[j];
        }
        __syncthreads();
        const int cnt = min(256, N - j0);
        for (int jj = 0; jj < cnt; ++jj) {
            if (ci < sc[jj]) {  // relation false unless the pair is out of radius
                const float d = pdist3(xi, yi, zi, sx[jj], sy[jj], sz[jj]);
                if (!(d >= R)) ok = false;
            }
        }
    }
    if (i < N) lm[(size_t)b * N + i] = ok ? 1.0f : 0.0f;
}

__global__ __launch_bounds__(256) void seed_rank_kernel(const float *__restrict__ conf,
                                                        const float *__restrict__ lm, int N, int S,
                                                        int *__restrict__ seeds) {
    __shared__ float ss[256];
    const int b = blockIdx.y, tid = threadIdx.x, i = blockIdx.x * 256 + tid;
    conf += (size_t)b * N;
    lm += (size_t)b * N;
    const float si = (i < N) ? conf[i] * lm[i] : 0.0f;  // scores * is_local_max (:217)
    int rank = 0;
    for (int j0 = 0; j0 < N; j0 += 256) {
        __syncthreads();
        if (j0 + tid < N) ss[tid] = conf[j0 + tid] * lm[j0 + tid];
        __syncthreads();
        const int cnt = min(256, N - j0);
        for (int jj = 0; jj < cnt; ++jj) {
            const float sj = ss[jj];
            rank += (sj > si) || (sj == si && j0 + jj < i);
        }
    }
    if (i < N && rank < S) seeds[(size_t)b * S + rank] = i;
}

hipError_t launch_local_max(const float *src, const float *conf, int B, int N, float radius,
                            float *lm, hipStream_t s) {
    hipLaunchKernelGGL(local_max_kernel, dim3((N + 255) / 256, B), dim3(256), 0, s, src, conf, N,
                       radius, lm);
    return hipGetLastError();
}

hipError_t launch_seed_rank(const float *conf, const float *lm, int B, int N, int S, int *seeds,
                            hipStream_t s) {
    hipLaunchKernelGGL(seed_rank_kernel, dim3((N + 255) / 256, B), dim3(256), 0, s, conf, lm, N, S,
                       seeds);
    return hipGetLastError();
}

}  // namespace pdsc
