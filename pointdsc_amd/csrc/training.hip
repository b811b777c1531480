// training.hip -- SURVEY 8(f) row 3, second half: the training-mode forward's
// feature-similarity matrix and the spectral-matching loss (forward only).
//
//   feat_sim   M_ij = clamp(1 - (1 - f_i . f_j) / sigma^2, 0, 1), M_ii = 0
//              (models/PointDSC.py:158-163) for B pairs; the dot products on the
//              fp16 matrix cores with the 3-product split of the normed split
//              copy (H3) or on exact fp32 MFMA (F32)
//   sm_loss    SpectralMatchingLoss (libs/loss.py:115-139), balanced or MSE, in
//              fp64 partial sums: one workgroup per (pair, 64-row strip), then a
//              fixed-order per-pair reduction
#include "attention_h3.hpp"

namespace pdsc {

// A workgroup = 4 waves = one 64 x 64 tile of M (wave (wi, wj): rows 64 by + 32 wi,
// columns 64 bx + 32 wj); accumulator register r of lane (h, l32) is
// (row i0 + acc_row(r, h), column j0 + l32): each store writes 128 B of a row.
template <bool F32>
__global__ __launch_bounds__(256) void feat_sim_kernel(const void *__restrict__ feats, int N,
                                                       const float *__restrict__ sigma_p, float *__restrict__ M) {
    const int b = blockIdx.z, wave = threadIdx.x >> 6, lane = threadIdx.x & 63, h = lane >> 5, l32 = lane & 31;
    const int i0 = blockIdx.y * 64 + 32 * (wave >> 1), j0 = blockIdx.x * 64 + 32 * (wave & 1);
    if (i0 >= N || j0 >= N) return;  // wave-uniform, no barriers
    const int ra = min(i0 + l32, N - 1), rb = min(j0 + l32, N - 1);
    f32x16 acc = zero16();
    if constexpr (F32) {
        const float *F = static_cast<const float *>(feats) + (size_t)b * N * CH;
        const float *pa = F + (size_t)ra * CH + 4 * h, *pb = F + (size_t)rb * CH + 4 * h;
#pragma unroll 4
        for (int j = 0; j < CH / 8; ++j) {
            const f32x4 av = *reinterpret_cast<const f32x4 *>(pa + 8 * j), bv = *reinterpret_cast<const f32x4 *>(pb + 8 * j);
#pragma unroll
            for (int e = 0; e < 4; ++e) acc = mfma32(av[e], bv[e], acc);
        }
    } else {
        const _Float16 *F = static_cast<const _Float16 *>(feats) + (size_t)b * N * 2 * CH;
        const _Float16 *pa = F + (size_t)ra * 2 * CH + 8 * h, *pb = F + (size_t)rb * 2 * CH + 8 * h;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const f16x8 ah = *reinterpret_cast<const f16x8 *>(pa + 16 * j);
            const f16x8 al = *reinterpret_cast<const f16x8 *>(pa + CH + 16 * j);
            const f16x8 bh = *reinterpret_cast<const f16x8 *>(pb + 16 * j);
            const f16x8 bl = *reinterpret_cast<const f16x8 *>(pb + CH + 16 * j);
            acc = mfma_h3(ah, al, bh, bl, acc);
        }
    }
    const float sig = sigma_p[0];
    const float sig2 = sig * sig;  // self.sigma ** 2 (a tensor: fp32)
    const int j = j0 + l32;
    if (j >= N) return;
    float *Mb = M + (size_t)b * N * N;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const int i = i0 + acc_row(r, h);
        if (i >= N) continue;
        const float m = fminf(fmaxf(1.0f - (1.0f - acc[r]) / sig2, 0.0f), 1.0f);  // clamp(min=0, max=1)
        Mb[(size_t)i * N + j] = (i == j) ? 0.0f : m;                             // diagonal := 0
    }
}

hipError_t launch_feat_sim(const void *feats, bool f32, int B, int N, const float *sigma, float *M, hipStream_t s) {
    const dim3 grid((N + 63) / 64, (N + 63) / 64, B);
    if (f32)
        hipLaunchKernelGGL(feat_sim_kernel<true>, grid, dim3(256), 0, s, feats, N, sigma, M);
    else
        hipLaunchKernelGGL(feat_sim_kernel<false>, grid, dim3(256), 0, s, feats, N, sigma, M);
    return hipGetLastError();
}

// Per (pair, 64-row strip): sum over its rows of [sum gt (M-1)^2, sum gt, sum (1-gt) M^2]
// (balanced) or sum (M - gt)^2 (MSE, slot 0), gt_ij = (l_i + l_j == 2) and 0 on
// the diagonal (:126-129), in fp64 (wave sums, then the workgroup's 4 waves).
constexpr int SML_ROWS = 64;

__global__ __launch_bounds__(256) void sm_loss_partial_kernel(const float *__restrict__ M,
                                                              const float *__restrict__ labels, int N,
                                                              double *__restrict__ part) {
    __shared__ double red[4][3];
    const int b = blockIdx.y, strip = blockIdx.x, tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const float *Mb = M + (size_t)b * N * N, *lb = labels + (size_t)b * N;
    double sp = 0.0, np = 0.0, sn = 0.0, mse = 0.0;
    for (int i = strip * SML_ROWS + wave; i < min(N, (strip + 1) * SML_ROWS); i += 4) {
        const bool li = lb[i] == 1.0f;
        for (int j = lane; j < N; j += 64) {
            const double m = Mb[(size_t)i * N + j];
            const bool g = li && (lb[j] == 1.0f) && (i != j);  // (gt_i + gt_j) == 2, fill_diagonal_(0)
            if (g) {
                sp += (m - 1.0) * (m - 1.0);
                np += 1.0;
                mse += (m - 1.0) * (m - 1.0);
            } else {
                sn += m * m;
                mse += m * m;
            }
        }
    }
    sp = wave_sum(sp);
    np = wave_sum(np);
    sn = wave_sum(sn);
    mse = wave_sum(mse);
    if (lane == 0) {
        red[wave][0] = sp;
        red[wave][1] = np;
        red[wave][2] = sn;
    }
    __syncthreads();
    if (tid == 0) {
        double a = 0, c = 0, d = 0;
        for (int w = 0; w < 4; ++w) {
            a += red[w][0];
            c += red[w][1];
            d += red[w][2];
        }
        double *o = part + ((size_t)b * gridDim.x + strip) * 4;
        o[0] = a;
        o[1] = c;
        o[2] = d;
    }
    __syncthreads();
    if (lane == 0) red[wave][0] = mse;
    __syncthreads();
    if (tid == 0) part[((size_t)b * gridDim.x + strip) * 4 + 3] = red[0][0] + red[1][0] + red[2][0] + red[3][0];
}

// loss = mean_b(0.5 sum gt (M-1)^2 / (relu(sum gt - 1) + 1) + 0.5 sum (1-gt) M^2 /
// (relu(sum (1-gt) - 1) + 1)) (balanced, :131-134), else mean((M - gt)^2) (:136)
__global__ void sm_loss_final_kernel(const double *__restrict__ part, int B, int N, int nstrip, int balanced,
                                     float *__restrict__ loss) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    double total = 0.0, mse = 0.0;
    for (int b = 0; b < B; ++b) {
        double sp = 0, np = 0, sn = 0;
        for (int s = 0; s < nstrip; ++s) {
            const double *o = part + ((size_t)b * nstrip + s) * 4;
            sp += o[0];
            np += o[1];
            sn += o[2];
            mse += o[3];
        }
        const double nn = (double)N * N - np;  // sum (1 - gt): the diagonal counts as negative
        total += 0.5 * sp / (fmax(np - 1.0, 0.0) + 1.0) + 0.5 * sn / (fmax(nn - 1.0, 0.0) + 1.0);
    }
    loss[0] = balanced ? (float)(total / B) : (float)(mse / ((double)B * N * N));
}

size_t sm_loss_partial_doubles(int B, int N) { return (size_t)B * ((N + SML_ROWS - 1) / SML_ROWS) * 4; }

hipError_t launch_sm_loss(const float *M, const float *labels, int B, int N, int balanced, double *part, float *loss,
                          hipStream_t s) {
    const int nstrip = (N + SML_ROWS - 1) / SML_ROWS;
    hipLaunchKernelGGL(sm_loss_partial_kernel, dim3(nstrip, B), dim3(256), 0, s, M, labels, N, part);
    hipLaunchKernelGGL(sm_loss_final_kernel, dim3(1), dim3(64), 0, s, part, B, N, nstrip, balanced, loss);
    return hipGetLastError();
}

}  // namespace pdsc
