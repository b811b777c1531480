// corr.hip -- SURVEY 8(f) row 1: correspondence construction, the step that
// feeds the hot path (datasets/ThreeDMatch.py:277-308, datasets/KITTI.py:85-99,
// demo_registration.py:101-108):
//
//   distance = sqrt(2 - 2 src_desc @ tgt_desc^T + 1e-6)       (fp32)
//   source_idx = argmin_j distance[i, j]; target_idx = argmin_i distance[i, j]
//   mutual: keep i with target_idx[source_idx[i]] == i, in ascending i
//   labels = |gt_trans(src) - tgt| < inlier_threshold;  corr_pos = [src, tgt] - mean
//
//   nn_argmin      64 x 64 distance tiles (fp32 FMA chains from LDS), per-tile
//                  row / column minima folded into 64-bit (key, index) words
//                  with atomicMin, so ties resolve to the first index like
//                  numpy.argmin; the Ns x Nt matrix never reaches HBM
//   corr_select    one workgroup: mutual test + ordered compaction (np.where order)
//   corr_gather    one workgroup: keypoint gather, the reference's sequential
//                  fp32 column mean, centring, ground-truth labels (fp64)
#include "pdsc_internal.hpp"

namespace pdsc {

constexpr int NN_T = 64;     // tile edge
constexpr int NN_DMAX = 64;  // descriptor width limit (FCGF 32, FPFH 33)

// order-preserving float -> uint; NaN -> 0 (numpy.argmin returns the first NaN)
PDSC_DEV uint32_t nn_key(float f) {
    if (f != f) return 0u;
    if (f == 0.0f) f = 0.0f;
    const uint32_t u = __float_as_uint(f);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

PDSC_DEV unsigned long long umin64(unsigned long long a, unsigned long long b) { return a < b ? a : b; }

PDSC_DEV unsigned long long shfl_xor64(unsigned long long v, int m) {
    const int lo = __shfl_xor((int)(uint32_t)v, m), hi = __shfl_xor((int)(uint32_t)(v >> 32), m);
    return ((unsigned long long)(uint32_t)hi << 32) | (uint32_t)lo;
}

__global__ __launch_bounds__(256) void nn_argmin_kernel(const float *__restrict__ A, const float *__restrict__ Bd,
                                                        int Na, int Nb, int D, unsigned long long *__restrict__ rowkey,
                                                        unsigned long long *__restrict__ colkey) {
    __shared__ __attribute__((aligned(16))) float sa[NN_DMAX][NN_T + 4];  // sa[k][row]
    __shared__ __attribute__((aligned(16))) float sb[NN_DMAX][NN_T + 4];  // sb[k][col]
    const int i0 = blockIdx.y * NN_T, j0 = blockIdx.x * NN_T;
    const int tid = threadIdx.x;
    for (int e = tid; e < NN_T * D; e += 256) {
        const int r = e / D, k = e % D;
        sa[k][r] = (i0 + r < Na) ? A[(size_t)(i0 + r) * D + k] : 0.0f;
        sb[k][r] = (j0 + r < Nb) ? Bd[(size_t)(j0 + r) * D + k] : 0.0f;
    }
    __syncthreads();
    const int tx = tid & 15, ty = tid >> 4;  // columns 4tx..+3, rows 4ty..+3
    float acc[4][4] = {};
    for (int k = 0; k < D; ++k) {
        const f32x4 a = *reinterpret_cast<const f32x4 *>(&sa[k][4 * ty]);
        const f32x4 b = *reinterpret_cast<const f32x4 *>(&sb[k][4 * tx]);
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int c = 0; c < 4; ++c) acc[r][c] = __builtin_fmaf(a[r], b[c], acc[r][c]);
    }
    const float eps = 1e-6f;  // numpy: float32 array + python float -> float32 add
    unsigned long long rbest[4], cbest[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) rbest[q] = cbest[q] = ~0ull;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int i = i0 + 4 * ty + r;
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            const int j = j0 + 4 * tx + c;
            if (i < Na && j < Nb) {
                const float d = sqrtf((2.0f - 2.0f * acc[r][c]) + eps);
                const unsigned long long key = (unsigned long long)nn_key(d) << 32;
                rbest[r] = umin64(rbest[r], key | (uint32_t)j);
                cbest[c] = umin64(cbest[c], key | (uint32_t)i);
            }
        }
    }
    // rows: the 16 threads sharing ty are 16 consecutive lanes
#pragma unroll
    for (int r = 0; r < 4; ++r) {
#pragma unroll
        for (int m = 8; m > 0; m >>= 1) rbest[r] = umin64(rbest[r], shfl_xor64(rbest[r], m));
        const int i = i0 + 4 * ty + r;
        if (tx == 0 && i < Na && rbest[r] != ~0ull) atomicMin(rowkey + i, rbest[r]);
    }
    // columns: lanes tx, tx+16, tx+32, tx+48 of a wave share tx
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        cbest[c] = umin64(cbest[c], shfl_xor64(cbest[c], 16));
        cbest[c] = umin64(cbest[c], shfl_xor64(cbest[c], 32));
        const int j = j0 + 4 * tx + c;
        if ((tid & 63) < 16 && j < Nb && cbest[c] != ~0ull) atomicMin(colkey + j, cbest[c]);
    }
}

hipError_t launch_nn_argmin(const float *A, const float *B, int Na, int Nb, int D, unsigned long long *rowkey,
                            unsigned long long *colkey, hipStream_t s) {
    if (D < 1 || D > NN_DMAX) return hipErrorInvalidValue;
    HIP_RET(hipMemsetAsync(rowkey, 0xff, (size_t)Na * sizeof(unsigned long long), s));
    HIP_RET(hipMemsetAsync(colkey, 0xff, (size_t)Nb * sizeof(unsigned long long), s));
    hipLaunchKernelGGL(nn_argmin_kernel, dim3((Nb + NN_T - 1) / NN_T, (Na + NN_T - 1) / NN_T), dim3(256), 0, s, A,
                       B, Na, Nb, D, rowkey, colkey);
    return hipGetLastError();
}

// One 1024-thread workgroup: exclusive scan of the keep flags, 1024 at a time.
__global__ __launch_bounds__(1024) void corr_select_kernel(const unsigned long long *__restrict__ rowkey,
                                                           const unsigned long long *__restrict__ colkey, int Na,
                                                           int mutual, int *__restrict__ corr,
                                                           int *__restrict__ count) {
    __shared__ int wsum[16];
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    int running = 0;
    for (int base = 0; base < Na; base += 1024) {
        const int i = base + tid;
        int nn = 0;
        bool keep = false;
        if (i < Na) {
            nn = (int)(uint32_t)rowkey[i];
            keep = !mutual || (int)(uint32_t)colkey[nn] == i;
        }
        const unsigned long long m = __ballot(keep);
        if (lane == 0) wsum[wave] = __popcll(m);
        __syncthreads();
        int before = 0, total = 0;
        for (int w = 0; w < 16; ++w) {
            before += w < wave ? wsum[w] : 0;
            total += wsum[w];
        }
        if (keep) {
            const int pos = running + before + __popcll(m & ((1ull << lane) - 1ull));
            corr[2 * pos] = i;
            corr[2 * pos + 1] = nn;
        }
        running += total;
        __syncthreads();
    }
    if (tid == 0) count[0] = running;
}

// gather + centring + labels for the `count` correspondences (one workgroup).
// The column mean restates numpy's float32 axis-0 reduction: a sequential fp32
// sum in row order, divided in float64 and rounded (numpy _mean, out=float32).
__global__ __launch_bounds__(1024) void corr_gather_kernel(const float *__restrict__ src_xyz,
                                                           const float *__restrict__ tgt_xyz,
                                                           const int *__restrict__ corr, const int *__restrict__ count,
                                                           const double *__restrict__ gt, double thr,
                                                           float *__restrict__ corr_pos, float *__restrict__ src_out,
                                                           float *__restrict__ tgt_out, float *__restrict__ labels) {
    __shared__ float mean[6];
    const int n = count[0], tid = threadIdx.x;
    for (int p = tid; p < n; p += 1024) {
        const int i = corr[2 * p], j = corr[2 * p + 1];
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            src_out[3 * p + c] = src_xyz[3 * (size_t)i + c];
            tgt_out[3 * p + c] = tgt_xyz[3 * (size_t)j + c];
        }
        if (labels) {
            const double x = src_xyz[3 * (size_t)i], y = src_xyz[3 * (size_t)i + 1], z = src_xyz[3 * (size_t)i + 2];
            const double wx = (gt[0] * x + gt[1] * y) + gt[2] * z + gt[3];
            const double wy = (gt[4] * x + gt[5] * y) + gt[6] * z + gt[7];
            const double wz = (gt[8] * x + gt[9] * y) + gt[10] * z + gt[11];
            const double dx = wx - tgt_xyz[3 * (size_t)j], dy = wy - tgt_xyz[3 * (size_t)j + 1],
                         dz = wz - tgt_xyz[3 * (size_t)j + 2];
            labels[p] = sqrt((dx * dx + dy * dy) + dz * dz) < thr ? 1.0f : 0.0f;
        }
    }
    __threadfence_block();
    __syncthreads();  // src_out / tgt_out complete (global writes of this workgroup)
    if (tid < 6) {
        const float *col = tid < 3 ? src_out + tid : tgt_out + (tid - 3);
        float sum = 0.0f;
        for (int p = 0; p < n; ++p) sum += col[3 * p];
        mean[tid] = n > 0 ? (float)((double)sum / (double)n) : 0.0f;
    }
    __syncthreads();
    for (int p = tid; p < n; p += 1024) {
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            corr_pos[6 * p + c] = src_out[3 * p + c] - mean[c];
            corr_pos[6 * p + 3 + c] = tgt_out[3 * p + c] - mean[3 + c];
        }
    }
}

hipError_t launch_corr_build(const unsigned long long *rowkey, const unsigned long long *colkey,
                             const float *src_xyz, const float *tgt_xyz, int Na, int mutual, const double *gt,
                             double thr, int *corr, int *count, float *corr_pos, float *src_out, float *tgt_out,
                             float *labels, hipStream_t s) {
    hipLaunchKernelGGL(corr_select_kernel, dim3(1), dim3(1024), 0, s, rowkey, colkey, Na, mutual, corr, count);
    HIP_RET(hipGetLastError());
    hipLaunchKernelGGL(corr_gather_kernel, dim3(1), dim3(1024), 0, s, src_xyz, tgt_xyz, corr, count, gt, thr,
                       corr_pos, src_out, tgt_out, labels);
    return hipGetLastError();
}

}  // namespace pdsc
