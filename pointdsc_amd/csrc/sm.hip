// sm.hip -- SURVEY 8(f) row 3: the spectral-matching baseline SM of
// baseline_scripts/baseline_3DMatch.py:19-53 (Leordeanu & Hebert), the
// reference's N x N power-iteration method, on the same machinery:
//
//   M_ij = max(0, 4.5 - (|c_j - c_i|_src - |c_j - c_i|_tgt)^2 / 2 / sigma^2),
//          sigma = inlier_threshold / 3, diag 0            (:20-36, c = corr_pos)
//   v <- 1; 10 x { v <- M v; v <- v / (|v| + 1e-6) }      (:39-43)
//   labels = top int(N * top_ratio) of v (descending)      (:46-48)
//   trans = rigid_transform_3d(src, tgt, v * labels)       (:51)
//
//   sm_compat    dense M (4 N^2 B written once), 64 x 64 tiles, 16-B stores
//   sm_matvec    one wave per row, 16-B loads: HBM/MALL-bound, 4 N^2 B per iterate
//   sm_normalize one workgroup: fixed-order sum of squares, scale
//   sm_select    one workgroup: the S-th largest key by bitwise bisection,
//                ties to the lower index (the reference's argsort orders ties
//                arbitrarily), labels and Kabsch weights
#include "pdsc_internal.hpp"

namespace pdsc {

constexpr int SM_T = 64;

__global__ __launch_bounds__(256) void sm_compat_kernel(const float *__restrict__ corr, int N, float sig2,
                                                        float *__restrict__ M) {
    __shared__ float ci[SM_T][6], cj[SM_T][6];
    const int i0 = blockIdx.y * SM_T, j0 = blockIdx.x * SM_T, tid = threadIdx.x;
    for (int e = tid; e < SM_T * 6; e += 256) {
        const int p = e / 6, c = e % 6;
        ci[p][c] = i0 + p < N ? corr[(size_t)(i0 + p) * 6 + c] : 0.0f;
        cj[p][c] = j0 + p < N ? corr[(size_t)(j0 + p) * 6 + c] : 0.0f;
    }
    __syncthreads();
    const int cq = tid & 15, rq = tid >> 4;
    const bool vec = (N & 3) == 0;
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) {
        const int r = rq + 16 * rr, i = i0 + r;
        if (i >= N) continue;
        float out[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int c = cq * 4 + q;
            // diff[i][j] = corr[j] - corr[i]; torch.sum(d ** 2, -1) ** 0.5 (:21)
            float dx = cj[c][0] - ci[r][0], dy = cj[c][1] - ci[r][1], dz = cj[c][2] - ci[r][2];
            const float ds = sqrtf((dx * dx + dy * dy) + dz * dz);
            dx = cj[c][3] - ci[r][3];
            dy = cj[c][4] - ci[r][4];
            dz = cj[c][5] - ci[r][5];
            const float dt = sqrtf((dx * dx + dy * dy) + dz * dz);
            const float m = ds - dt;
            const float v = 4.5f - ((m * m) / 2.0f) / sig2;  // :35
            out[q] = (i == j0 + c) ? 0.0f : fmaxf(v, 0.0f);  // :36
        }
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

// y = M v: one wave per row; lane l sums elements l*4 + 256 t (16-B loads),
// then a butterfly reduction.
__global__ __launch_bounds__(256) void sm_matvec_kernel(const float *__restrict__ M, const float *__restrict__ v,
                                                        int N, float *__restrict__ y) {
    const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (row >= N) return;
    const float *mr = M + (size_t)row * N;
    float acc = 0.0f;
    if ((N & 3) == 0) {
        for (int j = 4 * lane; j < N; j += 256) {
            const f32x4 m = *reinterpret_cast<const f32x4 *>(mr + j);
            const f32x4 x = *reinterpret_cast<const f32x4 *>(v + j);
            acc = __builtin_fmaf(m[0], x[0], acc);
            acc = __builtin_fmaf(m[1], x[1], acc);
            acc = __builtin_fmaf(m[2], x[2], acc);
            acc = __builtin_fmaf(m[3], x[3], acc);
        }
    } else {
        for (int j = lane; j < N; j += 64) acc = __builtin_fmaf(mr[j], v[j], acc);
    }
    acc = wave_sum(acc);
    if (lane == 0) y[row] = acc;
}

// v = y / (|y| + 1e-6) (:42), one 1024-thread workgroup, fixed reduction order
__global__ __launch_bounds__(1024) void sm_normalize_kernel(const float *__restrict__ y, int N,
                                                            float *__restrict__ v) {
    __shared__ float part[16];
    const int tid = threadIdx.x;
    float ss = 0.0f;
    for (int j = tid; j < N; j += 1024) ss = __builtin_fmaf(y[j], y[j], ss);
    ss = wave_sum(ss);
    if ((tid & 63) == 0) part[tid >> 6] = ss;
    __syncthreads();
    float tot = 0.0f;
    for (int w = 0; w < 16; ++w) tot += part[w];
    const float den = sqrtf(tot) + 1e-6f;
    for (int j = tid; j < N; j += 1024) v[j] = y[j] / den;
}

__global__ void sm_fill_kernel(float *v, int N, float x) {
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j < N) v[j] = x;
}

// labels = the S largest entries of v (ties to the lower index); w = v * labels
__global__ __launch_bounds__(1024) void sm_select_kernel(const float *__restrict__ v, int N, int S,
                                                         float *__restrict__ labels, float *__restrict__ w) {
    __shared__ int cnt[16];
    __shared__ int wbase[16];
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    auto key = [](float f) -> uint32_t {  // order-preserving, +-0 equal
        if (f == 0.0f) f = 0.0f;
        const uint32_t u = __float_as_uint(f);
        return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
    };
    auto block_count = [&](uint32_t thr, bool strict) -> int {  // # keys > thr (strict) or >= thr
        int c = 0;
        for (int j = tid; j < N; j += 1024) {
            const uint32_t u = key(v[j]);
            c += strict ? (u > thr) : (u >= thr);
        }
        c = wave_sum(c);
        __syncthreads();
        if (lane == 0) cnt[wave] = c;
        __syncthreads();
        int t = 0;
        for (int q = 0; q < 16; ++q) t += cnt[q];
        return t;
    };
    // largest t with #(key >= t) >= S: the S-th largest key
    uint32_t t = 0;
    if (S > 0) {
        for (int bit = 31; bit >= 0; --bit) {
            const uint32_t cand = t | (1u << bit);
            if (block_count(cand, false) >= S) t = cand;
        }
    }
    const int greater = S > 0 ? block_count(t, true) : 0;
    const int need_eq = S - greater;  // keys equal to t, taken in index order
    int running = 0;
    for (int base = 0; base < N; base += 1024) {
        const int j = base + tid;
        uint32_t u = 0;
        bool eq = false, gt = false;
        if (j < N) {
            u = key(v[j]);
            gt = S > 0 && u > t;
            eq = S > 0 && u == t;
        }
        const unsigned long long m = __ballot(eq);
        __syncthreads();
        if (lane == 0) wbase[wave] = __popcll(m);
        __syncthreads();
        int before = 0, tot = 0;
        for (int q = 0; q < 16; ++q) {
            before += q < wave ? wbase[q] : 0;
            tot += wbase[q];
        }
        const int r = running + before + __popcll(m & ((1ull << lane) - 1ull));
        if (j < N) {
            const bool sel = gt || (eq && r < need_eq);
            labels[j] = sel ? 1.0f : 0.0f;
            w[j] = v[j] * (sel ? 1.0f : 0.0f);  // leading_eig * pred_labels (:51)
        }
        running += tot;
    }
}

hipError_t launch_sm(const float *corr, const float *src, const float *tgt, int N, float sig2, int S, int iters,
                     float *M, float *v, float *y, float *w, float *labels, float *trans, hipStream_t s) {
    const int nt = (N + SM_T - 1) / SM_T;
    hipLaunchKernelGGL(sm_compat_kernel, dim3(nt, nt), dim3(256), 0, s, corr, N, sig2, M);
    HIP_RET(hipGetLastError());
    hipLaunchKernelGGL(sm_fill_kernel, dim3((N + 255) / 256), dim3(256), 0, s, v, N, 1.0f);  // :39
    for (int it = 0; it < iters; ++it) {
        hipLaunchKernelGGL(sm_matvec_kernel, dim3((N + 3) / 4), dim3(256), 0, s, M, v, N, y);
        hipLaunchKernelGGL(sm_normalize_kernel, dim3(1), dim3(1024), 0, s, y, N, v);
    }
    hipLaunchKernelGGL(sm_select_kernel, dim3(1), dim3(1024), 0, s, v, N, S, labels, w);
    HIP_RET(hipGetLastError());
    return launch_rigid(src, tgt, w, 1, N, trans, s);
}

hipError_t launch_sm_matvec(const float *M, const float *v, int N, float *y, hipStream_t s) {
    hipLaunchKernelGGL(sm_matvec_kernel, dim3((N + 3) / 4), dim3(256), 0, s, M, v, N, y);
    return hipGetLastError();
}

}  // namespace pdsc
