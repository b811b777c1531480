// nsm.hip -- a6-a11: Neural Spectral Matching, hypothesis verification and
// post-refinement.
//
//   knn_dist     a6  seed rows of 2 - 2 F F^T (v_mfma_f32_32x32x2_f32), [B][S][N]
//   knn_select   a6  topk(k+1, smallest)[1:] per seed row: 4-pass 8-bit radix
//                    select + ordered tie resolution (ascending index)
//   nsm_power    a7-a8  gather k neighbours, k x k feature*spatial consistency,
//                    all num_iterations power iterates + per-iterate allclose flags
//   nsm_finish   a8  pair-global early exit t* = first iterate where every seed
//                    is allclose (torch.allclose over the whole batch, :354)
//   hypotheses   a9-a10  weighted Kabsch per seed (fp64 3x3 SVD on device) +
//                    inlier count over all N correspondences
//   select_best  a10 first argmax of fitness, labels of the best hypothesis
//   post_refine  a11 <= 20 device-side IRLS refits, one workgroup per pair
#include "pdsc_internal.hpp"

namespace pdsc {

// ------------------------------------------------------------------ a6 kNN
// dist[b][s][j] = 2 - 2 * <normed[seed_s], normed[j]>   (models/common.py:58-60)
__global__ __launch_bounds__(256) void knn_dist_kernel(const float *__restrict__ normed,
                                                       const int *__restrict__ seeds, int N, int S,
                                                       float *__restrict__ dist) {
    const int b = blockIdx.z, tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int h = lane >> 5, l32 = lane & 31;
    const int s0 = blockIdx.y * 32, j0 = blockIdx.x * 128 + wave * 32;
    const float *F = normed + (size_t)b * N * CH;
    const int sidx = s0 + l32;
    const int seed = (sidx < S) ? seeds[(size_t)b * S + sidx] : -1;
    float af[64];
    {
        const f32x4 *src4 = reinterpret_cast<const f32x4 *>(F + (size_t)max(seed, 0) * CH + h * 64);
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            f32x4 t = src4[i];
            if (seed < 0) t = f32x4{0, 0, 0, 0};
            af[4 * i] = t[0];
            af[4 * i + 1] = t[1];
            af[4 * i + 2] = t[2];
            af[4 * i + 3] = t[3];
        }
    }
    const int j = j0 + l32;
    const f32x4 *bp = reinterpret_cast<const f32x4 *>(F + (size_t)min(j, N - 1) * CH + h * 64);
    f32x16 acc = zero16();
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        const f32x4 bv = bp[i];
        acc = mfma32(af[4 * i], bv[0], acc);
        acc = mfma32(af[4 * i + 1], bv[1], acc);
        acc = mfma32(af[4 * i + 2], bv[2], acc);
        acc = mfma32(af[4 * i + 3], bv[3], acc);
    }
    if (j < N) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int s = s0 + acc_row(r, h);
            if (s < S) dist[((size_t)b * S + s) * N + j] = 2.0f - 2.0f * acc[r];
        }
    }
}

hipError_t launch_knn_dist(const float *normed, const int *seeds, int B, int N, int S, float *dist,
                           hipStream_t s) {
    hipLaunchKernelGGL(knn_dist_kernel, dim3((N + 127) / 128, (S + 31) / 32, B), dim3(256), 0, s,
                       normed, seeds, N, S, dist);
    return hipGetLastError();
}

// order-preserving float -> uint key (+0 and -0 share a key, like float ==)
PDSC_DEV uint32_t fkey(float f) {
    if (f == 0.0f) f = 0.0f;
    const uint32_t u = __float_as_uint(f);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

constexpr int SEL_MAX = 256;  // k + 1 <= SEL_MAX

// topk(k+1, smallest) of one seed row, sorted (key asc, index asc), first dropped.
__global__ __launch_bounds__(256) void knn_select_kernel(const float *__restrict__ dist, int N, int S,
                                                         int k, int *__restrict__ knn) {
    __shared__ uint32_t hist[256];
    __shared__ uint32_t sel_bin, sel_need;
    __shared__ uint32_t cnt_less[256], cnt_eq[256];
    __shared__ uint32_t lkey[SEL_MAX];
    __shared__ int lidx[SEL_MAX];
    const int b = blockIdx.y, s = blockIdx.x, tid = threadIdx.x;
    const float *row = dist + ((size_t)b * S + s) * N;
    const int want = k + 1;
    uint32_t need = want, prefix = 0, mask = 0;
    for (int pass = 0; pass < 4; ++pass) {
        const int shift = 24 - 8 * pass;
        hist[tid] = 0;
        __syncthreads();
        for (int j = tid; j < N; j += 256) {
            const uint32_t u = fkey(row[j]);
            if ((u & mask) == prefix) atomicAdd(&hist[(u >> shift) & 255u], 1u);
        }
        __syncthreads();
        if (tid < 64) {
            uint32_t c[4], tot = 0;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                c[e] = hist[4 * tid + e];
                tot += c[e];
            }
            uint32_t incl = tot;  // inclusive scan over lanes
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const uint32_t y = __shfl_up(incl, o);
                if (tid >= o) incl += y;
            }
            uint32_t base = incl - tot;
            if (base < need && need <= incl) {
                uint32_t cum = base;
                for (int e = 0; e < 4; ++e) {
                    if (cum + c[e] >= need) {
                        sel_bin = 4 * tid + e;
                        sel_need = need - cum;
                        break;
                    }
                    cum += c[e];
                }
            }
        }
        __syncthreads();
        prefix |= sel_bin << shift;
        mask |= 255u << shift;
        need = sel_need;
        __syncthreads();
    }
    // prefix = threshold key T; take all keys < T and the `need` lowest-index keys == T.
    const int chunk = (N + 255) / 256;
    const int jb = tid * chunk, je = min(N, jb + chunk);
    uint32_t nl = 0, ne = 0;
    for (int j = jb; j < je; ++j) {
        const uint32_t u = fkey(row[j]);
        nl += u < prefix;
        ne += u == prefix;
    }
    cnt_less[tid] = nl;
    cnt_eq[tid] = ne;
    __syncthreads();
    if (tid == 0) {  // exclusive scans (256 entries)
        uint32_t a = 0, e = 0;
        for (int t = 0; t < 256; ++t) {
            const uint32_t x = cnt_less[t], y = cnt_eq[t];
            cnt_less[t] = a;
            cnt_eq[t] = e;
            a += x;
            e += y;
        }
    }
    __syncthreads();
    uint32_t pl = cnt_less[tid], pe = cnt_eq[tid];
    const uint32_t nless = want - need;
    for (int j = jb; j < je; ++j) {
        const uint32_t u = fkey(row[j]);
        if (u < prefix) {
            if (pl < (uint32_t)want) {
                lkey[pl] = u;
                lidx[pl] = j;
            }
            ++pl;
        } else if (u == prefix) {
            if (pe < need) {
                lkey[nless + pe] = u;
                lidx[nless + pe] = j;
            }
            ++pe;
        }
    }
    __syncthreads();
    if (tid < want) {
        const uint32_t ku = lkey[tid];
        const int ki = lidx[tid];
        int rank = 0;
        for (int m = 0; m < want; ++m) {
            const uint32_t mu = lkey[m];
            rank += (mu < ku) || (mu == ku && lidx[m] < ki);
        }
        if (rank > 0) knn[((size_t)b * S + s) * k + rank - 1] = ki;  // drop position 0 (:68)
    }
}

hipError_t launch_knn_select(const float *dist, int B, int N, int S, int k, int *knn, hipStream_t s) {
    hipLaunchKernelGGL(knn_select_kernel, dim3(S, B), dim3(256), 0, s, dist, N, S, k, knn);
    return hipGetLastError();
}

// -------------------------------------------------------------- a7-a8 NSM
constexpr int KMAX = 64;
constexpr int FSTR = CH + 4;

// One workgroup per (seed, pair).  hist[b][s][t][a] = iterate t+1, lane a.
// Bit t of the seed's flag word = allclose(v_{t+1}, v_t); AND-ed into pair_mask[b].
__global__ __launch_bounds__(256) void nsm_power_kernel(const float *__restrict__ normed,
                                                        const float *__restrict__ src,
                                                        const float *__restrict__ tgt,
                                                        const int *__restrict__ knn, int N, int S,
                                                        int k, int T, const float *__restrict__ sigma_p,
                                                        const float *__restrict__ sigma_d_p,
                                                        float *__restrict__ hist,
                                                        unsigned *__restrict__ pair_mask) {
    __shared__ __attribute__((aligned(16))) float F[KMAX * FSTR];
    __shared__ float P[KMAX][6];
    __shared__ float Tm[KMAX][KMAX + 1];
    __shared__ float vbuf[KMAX];
    __shared__ int nidx[KMAX];
    const int b = blockIdx.y, s = blockIdx.x, tid = threadIdx.x;
    const float sig = sigma_p[0], sd = sigma_d_p[0];
    const float sig2 = sig * sig, sd2 = sd * sd;
    if (tid < k) nidx[tid] = min(max(knn[((size_t)b * S + s) * k + tid], 0), N - 1);
    __syncthreads();
    const float *Fb = normed + (size_t)b * N * CH;
    for (int e = tid; e < k * (CH / 4); e += 256) {
        const int a = e / (CH / 4), c4 = e % (CH / 4);
        *reinterpret_cast<f32x4 *>(&F[a * FSTR + 4 * c4]) =
            *reinterpret_cast<const f32x4 *>(Fb + (size_t)nidx[a] * CH + 4 * c4);
    }
    for (int e = tid; e < k * 6; e += 256) {
        const int a = e / 6, c = e % 6;
        const float *base = (c < 3 ? src : tgt) + ((size_t)b * N + nidx[a]) * 3;
        P[a][c] = base[c % 3];
    }
    __syncthreads();
    // local consistency (models/PointDSC.py:257-278)
    for (int e = tid; e < k * k; e += 256) {
        const int a = e / k, c = e % k;
        float val = 0.0f;
        if (a != c) {
            const f32x4 *fa = reinterpret_cast<const f32x4 *>(&F[a * FSTR]);
            const f32x4 *fc = reinterpret_cast<const f32x4 *>(&F[c * FSTR]);
            f32x4 acc = {0, 0, 0, 0};
#pragma unroll 8
            for (int i = 0; i < CH / 4; ++i) {
                const f32x4 x = fa[i], y = fc[i];
                acc[0] = __builtin_fmaf(x[0], y[0], acc[0]);
                acc[1] = __builtin_fmaf(x[1], y[1], acc[1]);
                acc[2] = __builtin_fmaf(x[2], y[2], acc[2]);
                acc[3] = __builtin_fmaf(x[3], y[3], acc[3]);
            }
            const float dot = (acc[0] + acc[1]) + (acc[2] + acc[3]);
            const float fm = fmaxf(1.0f - (1.0f - dot) / sig2, 0.0f);
            float dx = P[a][0] - P[c][0], dy = P[a][1] - P[c][1], dz = P[a][2] - P[c][2];
            const float ds = sqrtf((dx * dx + dy * dy) + dz * dz);
            dx = P[a][3] - P[c][3];
            dy = P[a][4] - P[c][4];
            dz = P[a][5] - P[c][5];
            const float dt = sqrtf((dx * dx + dy * dy) + dz * dz);
            const float dd = ds - dt;
            const float sm = fmaxf(1.0f - (dd * dd) / sd2, 0.0f);
            val = fm * sm;
        }
        Tm[a][c] = val;
    }
    if (tid < KMAX) vbuf[tid] = 1.0f;
    __syncthreads();
    // power iteration (models/PointDSC.py:347-358), all T iterates, in wave 0
    if (tid < 64) {
        const int a = tid;
        float v = (a < k) ? 1.0f : 0.0f;
        unsigned flags = 0;
        float *hb = hist + ((size_t)b * S + s) * T * k;
        for (int t = 0; t < T; ++t) {
            float nv = 0.0f;
            if (a < k) {
                for (int c = 0; c < k; ++c) nv = __builtin_fmaf(Tm[a][c], vbuf[c], nv);
            }
            const float nrm = sqrtf(wave_sum(nv * nv));
            nv = nv / (nrm + 1e-6f);
            const bool close = (a >= k) || (fabsf(nv - v) <= 1e-8f + 1e-5f * fabsf(v));
            if (__all(close)) flags |= 1u << t;
            if (a < k) hb[(size_t)t * k + a] = nv;
            v = nv;
            __builtin_amdgcn_wave_barrier();
            if (a < KMAX) vbuf[a] = nv;
            __builtin_amdgcn_wave_barrier();
        }
        if (a == 0) atomicAnd(&pair_mask[b], flags);
    }
}

hipError_t launch_nsm_power(const float *normed, const float *src, const float *tgt, const int *knn,
                            int B, int N, int S, int k, int T, const float *sigma,
                            const float *sigma_d, float *hist, unsigned *pair_mask, hipStream_t s) {
    hipLaunchKernelGGL(nsm_power_kernel, dim3(S, B), dim3(256), 0, s, normed, src, tgt, knn, N, S, k,
                       T, sigma, sigma_d, hist, pair_mask);
    return hipGetLastError();
}

// w = v_{t*} / (sum v_{t*} + 1e-6)  (models/PointDSC.py:280-282)
__global__ __launch_bounds__(64) void nsm_finish_kernel(const float *__restrict__ hist,
                                                        const unsigned *__restrict__ pair_mask, int S,
                                                        int k, int T, float *__restrict__ weights,
                                                        int *__restrict__ iters_used) {
    const int b = blockIdx.y, s = blockIdx.x, a = threadIdx.x;
    const unsigned m = pair_mask[b] & ((T >= 32) ? 0xffffffffu : ((1u << T) - 1u));
    const int tstar = m ? (__ffs(m)) : T;  // 1-based iterate index
    float v = 1.0f;
    if (tstar > 0 && a < k) v = hist[(((size_t)b * S + s) * T + (tstar - 1)) * k + a];
    if (a >= k) v = 0.0f;
    const float sum = wave_sum(v);
    if (a < k) weights[((size_t)b * S + s) * k + a] = v / (sum + 1e-6f);
    if (s == 0 && a == 0 && iters_used) iters_used[b] = tstar;
}

hipError_t launch_nsm_finish(const float *hist, const unsigned *pair_mask, int B, int S, int k, int T,
                             float *weights, int *iters_used, hipStream_t s) {
    hipLaunchKernelGGL(nsm_finish_kernel, dim3(S, B), dim3(64), 0, s, hist, pair_mask, S, k, T,
                       weights, iters_used);
    return hipGetLastError();
}

// ------------------------------------------------------------ a9 Kabsch
// Finish a weighted Kabsch from its sums: centroids already formed, H given.
// t = c_B - R c_A in fp32 as models/common.py:42 computes it.
PDSC_DEV void kabsch_finish(const float H[9], const float cA[3], const float cB[3], float *T) {
    double Hd[9], Rd[9];
    for (int i = 0; i < 9; ++i) Hd[i] = H[i];
    kabsch_rotation(Hd, Rd);
    float R[9];
    for (int i = 0; i < 9; ++i) R[i] = (float)Rd[i];
    for (int r = 0; r < 3; ++r) {
        T[4 * r + 0] = R[3 * r + 0];
        T[4 * r + 1] = R[3 * r + 1];
        T[4 * r + 2] = R[3 * r + 2];
        T[4 * r + 3] = cB[r] - ((R[3 * r] * cA[0] + R[3 * r + 1] * cA[1]) + R[3 * r + 2] * cA[2]);
    }
    T[12] = 0.0f;
    T[13] = 0.0f;
    T[14] = 0.0f;
    T[15] = 1.0f;
}

// Hypothesis per seed: Kabsch on its k neighbours (wave 0), then count inliers
// over all N correspondences (all waves).  models/PointDSC.py:287-328.
__global__ __launch_bounds__(256) void hypotheses_kernel(const float *__restrict__ src,
                                                         const float *__restrict__ tgt,
                                                         const int *__restrict__ knn,
                                                         const float *__restrict__ weights, int N,
                                                         int S, int k, float tau,
                                                         float *__restrict__ seed_trans,
                                                         int *__restrict__ counts) {
    __shared__ float Ts[16];
    __shared__ int wcnt[4];
    const int b = blockIdx.y, s = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const float *sb = src + (size_t)b * N * 3, *tb = tgt + (size_t)b * N * 3;
    if (wave == 0) {
        float w = 0, ax = 0, ay = 0, az = 0, bx = 0, by = 0, bz = 0;
        if (lane < k) {
            const int j = min(max(knn[((size_t)b * S + s) * k + lane], 0), N - 1);
            w = weights[((size_t)b * S + s) * k + lane];
            ax = sb[3 * j];
            ay = sb[3 * j + 1];
            az = sb[3 * j + 2];
            bx = tb[3 * j];
            by = tb[3 * j + 1];
            bz = tb[3 * j + 2];
        }
        const float den = wave_sum(w) + 1e-6f;
        const float cA[3] = {wave_sum(ax * w) / den, wave_sum(ay * w) / den, wave_sum(az * w) / den};
        const float cB[3] = {wave_sum(bx * w) / den, wave_sum(by * w) / den, wave_sum(bz * w) / den};
        const float am[3] = {ax - cA[0], ay - cA[1], az - cA[2]};
        const float bm[3] = {bx - cB[0], by - cB[1], bz - cB[2]};
        float H[9];
#pragma unroll
        for (int i = 0; i < 3; ++i)
#pragma unroll
            for (int jj = 0; jj < 3; ++jj) H[3 * i + jj] = wave_sum((am[i] * w) * bm[jj]);
        if (lane == 0) {
            float T[16];
            kabsch_finish(H, cA, cB, T);
            for (int e = 0; e < 16; ++e) {
                Ts[e] = T[e];
                seed_trans[((size_t)b * S + s) * 16 + e] = T[e];
            }
        }
    }
    __syncthreads();
    float T[12];
#pragma unroll
    for (int e = 0; e < 12; ++e) T[e] = Ts[e];
    int c = 0;
    for (int n = tid; n < N; n += 256) {
        const float L2 = residual(T, sb[3 * n], sb[3 * n + 1], sb[3 * n + 2], tb[3 * n], tb[3 * n + 1],
                                  tb[3 * n + 2]);
        c += L2 < tau;
    }
    c = wave_sum(c);
    if (lane == 0) wcnt[wave] = c;
    __syncthreads();
    if (tid == 0) counts[(size_t)b * S + s] = wcnt[0] + wcnt[1] + wcnt[2] + wcnt[3];
}

hipError_t launch_hypotheses(const float *src, const float *tgt, const int *knn, const float *weights,
                             int B, int N, int S, int k, float tau, float *seed_trans, int *counts,
                             hipStream_t s) {
    hipLaunchKernelGGL(hypotheses_kernel, dim3(S, B), dim3(256), 0, s, src, tgt, knn, weights, N, S, k,
                       tau, seed_trans, counts);
    return hipGetLastError();
}

// ------------------------------------------------------------- a10 best
__global__ __launch_bounds__(256) void select_best_kernel(const float *__restrict__ src,
                                                          const float *__restrict__ tgt,
                                                          const float *__restrict__ seed_trans,
                                                          const int *__restrict__ counts, int N, int S,
                                                          float tau, float *__restrict__ fitness,
                                                          int *__restrict__ best_out,
                                                          float *__restrict__ trans,
                                                          float *__restrict__ labels) {
    __shared__ int wbest[4], wcnt[4];
    __shared__ float Ts[16];
    const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    int bc = -1, bi = 0x7fffffff;
    for (int s = tid; s < S; s += 256) {
        const int c = counts[(size_t)b * S + s];
        if (fitness) fitness[(size_t)b * S + s] = (float)c / (float)N;  // torch.mean of 0/1
        if (c > bc) { bc = c; bi = s; }  // strided ascending s: first max kept
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const int oc = __shfl_xor(bc, o), oi = __shfl_xor(bi, o);
        if (oc > bc || (oc == bc && oi < bi)) { bc = oc; bi = oi; }
    }
    if (lane == 0) { wcnt[wave] = bc; wbest[wave] = bi; }
    __syncthreads();
    if (tid == 0) {
        int c = wcnt[0], i = wbest[0];
        for (int w = 1; w < 4; ++w)
            if (wcnt[w] > c || (wcnt[w] == c && wbest[w] < i)) { c = wcnt[w]; i = wbest[w]; }
        wbest[0] = i;
        if (best_out) best_out[b] = i;
    }
    __syncthreads();
    const int best = wbest[0];
    if (tid < 16) {
        Ts[tid] = seed_trans[((size_t)b * S + best) * 16 + tid];
        trans[(size_t)b * 16 + tid] = Ts[tid];
    }
    __syncthreads();
    float T[12];
#pragma unroll
    for (int e = 0; e < 12; ++e) T[e] = Ts[e];
    const float *sb = src + (size_t)b * N * 3, *tb = tgt + (size_t)b * N * 3;
    for (int n = tid; n < N; n += 256) {
        const float L2 = residual(T, sb[3 * n], sb[3 * n + 1], sb[3 * n + 2], tb[3 * n], tb[3 * n + 1],
                                  tb[3 * n + 2]);
        labels[(size_t)b * N + n] = (L2 < tau) ? 1.0f : 0.0f;
    }
}

hipError_t launch_select_best(const float *src, const float *tgt, const float *seed_trans,
                              const int *counts, int B, int N, int S, float tau, float *fitness,
                              int *best, float *trans, float *labels, hipStream_t s) {
    hipLaunchKernelGGL(select_best_kernel, dim3(B), dim3(256), 0, s, src, tgt, seed_trans, counts, N, S,
                       tau, fitness, best, trans, labels);
    return hipGetLastError();
}

// --------------------------------------------------- block-wide Kabsch
constexpr int RB = 1024;  // threads per refinement / rigid workgroup
constexpr int RW = RB / 64;

template <int NV>
PDSC_DEV void block_sum(float (&v)[NV], float (*red)[NV], int tid) {
#pragma unroll
    for (int i = 0; i < NV; ++i) v[i] = wave_sum(v[i]);
    const int lane = tid & 63, wave = tid >> 6;
    if (lane == 0)
#pragma unroll
        for (int i = 0; i < NV; ++i) red[wave][i] = v[i];
    __syncthreads();
#pragma unroll
    for (int i = 0; i < NV; ++i) {
        float a = 0.0f;
        for (int w = 0; w < RW; ++w) a += red[w][i];
        v[i] = a;
    }
    __syncthreads();
}

// rigid_transform_3d on (A, B, w) rows [0, n) (models/common.py:7-45).
// wfun(i) returns the weight of row i (0 drops it).
template <typename WF>
PDSC_DEV void block_rigid(const float *__restrict__ A, const float *__restrict__ Bp, int n, WF wfun,
                          float *Tout, float (*red)[9], int tid) {
    float s7[7] = {0, 0, 0, 0, 0, 0, 0};
    for (int i = tid; i < n; i += RB) {
        const float w = wfun(i);
        s7[0] += w;
        s7[1] += A[3 * i] * w;
        s7[2] += A[3 * i + 1] * w;
        s7[3] += A[3 * i + 2] * w;
        s7[4] += Bp[3 * i] * w;
        s7[5] += Bp[3 * i + 1] * w;
        s7[6] += Bp[3 * i + 2] * w;
    }
    block_sum<7>(s7, reinterpret_cast<float (*)[7]>(red), tid);
    const float den = s7[0] + 1e-6f;
    const float cA[3] = {s7[1] / den, s7[2] / den, s7[3] / den};
    const float cB[3] = {s7[4] / den, s7[5] / den, s7[6] / den};
    float H[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
    for (int i = tid; i < n; i += RB) {
        const float w = wfun(i);
        if (w == 0.0f) continue;
        const float am[3] = {A[3 * i] - cA[0], A[3 * i + 1] - cA[1], A[3 * i + 2] - cA[2]};
        const float bm[3] = {Bp[3 * i] - cB[0], Bp[3 * i + 1] - cB[1], Bp[3 * i + 2] - cB[2]};
#pragma unroll
        for (int r = 0; r < 3; ++r)
#pragma unroll
            for (int c = 0; c < 3; ++c) H[3 * r + c] += (am[r] * w) * bm[c];
    }
    block_sum<9>(H, red, tid);
    if (tid == 0) kabsch_finish(H, cA, cB, Tout);
    __syncthreads();
}

// ---------------------------------------------------- a11 post-refinement
__global__ __launch_bounds__(RB) void post_refine_kernel(float *__restrict__ trans,
                                                         const float *__restrict__ src,
                                                         const float *__restrict__ tgt, int N,
                                                         float thr) {
    __shared__ float red[RW][9];
    __shared__ float Ts[16];
    const int b = blockIdx.x, tid = threadIdx.x;
    const float *sb = src + (size_t)b * N * 3, *tb = tgt + (size_t)b * N * 3;
    if (tid < 16) Ts[tid] = trans[(size_t)b * 16 + tid];
    __syncthreads();
    int prev = 0;
    for (int it = 0; it < 20; ++it) {
        float T[12];
#pragma unroll
        for (int e = 0; e < 12; ++e) T[e] = Ts[e];
        float c1[1] = {0.0f};
        for (int n = tid; n < N; n += RB) {
            const float L2 = residual(T, sb[3 * n], sb[3 * n + 1], sb[3 * n + 2], tb[3 * n], tb[3 * n + 1],
                                      tb[3 * n + 2]);
            c1[0] += (L2 < thr) ? 1.0f : 0.0f;
        }
        block_sum<1>(c1, reinterpret_cast<float (*)[1]>(red), tid);
        const int cnt = (int)c1[0];
        if (cnt == prev) break;  // abs(int(inlier_num - previous_inlier_num)) < 1 (:426)
        prev = cnt;
        auto wfun = [&](int n) -> float {
            const float L2 = residual(T, sb[3 * n], sb[3 * n + 1], sb[3 * n + 2], tb[3 * n], tb[3 * n + 1],
                                      tb[3 * n + 2]);
            if (!(L2 < thr)) return 0.0f;
            const float r = L2 / thr;
            return 1.0f / (1.0f + r * r);  // 1/(1 + (L2/thr)^2) (:435)
        };
        float Tn[16];
        block_rigid(sb, tb, N, wfun, Tn, red, tid);
        if (tid == 0)
            for (int e = 0; e < 16; ++e) Ts[e] = Tn[e];
        __syncthreads();
    }
    if (tid < 16) trans[(size_t)b * 16 + tid] = Ts[tid];
}

hipError_t launch_post_refine(float *trans, const float *src, const float *tgt, int B, int N, float thr,
                              hipStream_t s) {
    hipLaunchKernelGGL(post_refine_kernel, dim3(B), dim3(RB), 0, s, trans, src, tgt, N, thr);
    return hipGetLastError();
}

__global__ __launch_bounds__(RB) void rigid_kernel(const float *__restrict__ A, const float *__restrict__ Bp,
                                                   const float *__restrict__ w, int n,
                                                   float *__restrict__ trans) {
    __shared__ float red[RW][9];
    __shared__ float Ts[16];
    const int b = blockIdx.x, tid = threadIdx.x;
    const float *Ab = A + (size_t)b * n * 3, *Bb = Bp + (size_t)b * n * 3;
    const float *wb = w ? w + (size_t)b * n : nullptr;
    auto wfun = [&](int i) -> float {
        if (!wb) return 1.0f;
        const float x = wb[i];
        return x < 0.0f ? 0.0f : x;  // weights[weights < weight_threshold(=0)] = 0 (:20)
    };
    float T[16];
    block_rigid(Ab, Bb, n, wfun, T, red, tid);
    if (tid == 0)
        for (int e = 0; e < 16; ++e) Ts[e] = T[e];
    __syncthreads();
    if (tid < 16) trans[(size_t)b * 16 + tid] = Ts[tid];
}

hipError_t launch_rigid(const float *A, const float *Bp, const float *w, int nb, int n, float *trans,
                        hipStream_t s) {
    hipLaunchKernelGGL(rigid_kernel, dim3(nb), dim3(RB), 0, s, A, Bp, w, n, trans);
    return hipGetLastError();
}

}  // namespace pdsc
