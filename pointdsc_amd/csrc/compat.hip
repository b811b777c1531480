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
#include <algorithm>
#include <type_traits>
#include <vector>

#include "pdsc_internal.hpp"

namespace pdsc {

constexpr int CT = 64;  // tile edge (dense kernel)

// Rows of 4 columns per lane that compat_n evaluates in one call (the packed
// kernel's 4 rows in 4 / COMPAT_RP calls).  Build knob for A/B: -DCOMPAT_RP=1|2|4.
#ifndef COMPAT_RP
#define COMPAT_RP 1
#endif
// Per-wave LDS scratch of compat_n<E> (E elements per lane): a queue of the
// elements that need the exact evaluation and the wave's E x 64 outputs
// (group-major: out[g][4 lane + e], so each lane's 16-B read is conflict-free).
template <int E> struct CompatScratch {
    float qx[64 * E], qt[64 * E], out[64 * E];
    unsigned qs[64 * E];  // 32-bit: the same byte offset as qx / qt (no separate address)
};

// M for E (row, column) pairs of this lane, given their squared distances.
// M is 0 whenever |sqrt(xs) - sqrt(xt)| >= sigma_d, and
//   |sqrt(xs) - sqrt(xt)| = |xs - xt| / (sqrt(xs) + sqrt(xt)) >= |xs - xt| / sqrt(2 (xs + xt)),
// so (xs - xt)^2 > 2 s2 (xs + xt) (1 + 2^-10) proves M = 0 without a square
// root (the 2^-10 slack covers the fp32 evaluation of both sides; the guard
// xs + xt <= 2^20 s2 keeps the rounding of the correctly rounded square roots,
// <= 2^-24 (sqrt(xs) + sqrt(xt)), below that slack).  Only the other elements
// -- typically a fifth to a third -- are compacted into an LDS queue (ballot
// order) and evaluated exactly, 64 per pass, so the ~40-op correctly rounded
// sqrtf/sqrtf/'/' chain runs on full waves of useful work.
template <int E>
PDSC_DEV void compat_n(const float (&xs)[E], const float (&xt)[E], float s2, float rs2, bool s2ok, float kzero,
                       float gmax, CompatScratch<E> &sc, int lane, float (&out)[E]) {
#pragma unroll
    for (int g = 0; g < E / 4; ++g)
        *reinterpret_cast<f32x4 *>(&sc.out[256 * g + 4 * lane]) = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
    int cnt = 0;
#pragma unroll
    for (int q = 0; q < E; ++q) {
        const float dxt = xs[q] - xt[q], sum = xs[q] + xt[q];
        // zero = (dxt^2 > kzero sum) && (sum <= gmax); NaN, xs = xt = 0 -> exact path.
        // The queue mask as the OR of the two compares' own lane masks (a ballot
        // of the combined bool widens it to a VGPR and compares it again: 2 VALU
        // per element), the lane's rank among the queued lanes by v_mbcnt (2 VALU,
        // instead of and + bcnt x 2)
        const bool nz0 = !(dxt * dxt > kzero * sum), nz1 = !(sum <= gmax);
        const unsigned long long m = __builtin_amdgcn_ballot_w64(nz0) | __builtin_amdgcn_ballot_w64(nz1);
        if (nz0 || nz1) {
            const int pos = cnt + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                                                 __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
            sc.qx[pos] = xs[q];
            sc.qt[pos] = xt[q];
            sc.qs[pos] = (unsigned)(256 * (q >> 2) + 4 * lane + (q & 3));
        }
        cnt += __popcll(m);
    }
    __builtin_amdgcn_wave_barrier();
    for (int c0 = 0; c0 < cnt; c0 += 64) {  // wave-uniform
        const int e = c0 + lane;
        const bool act = e < cnt;
        const float x = act ? sc.qx[e] : 1.0f, t = act ? sc.qt[e] : 1.0f;
        const bool tiny = (x != 0.0f && !(x >= 0x1p-96f)) || (t != 0.0f && !(t >= 0x1p-96f));
        float m;
        if (s2ok && !__any(tiny)) {
            const float d = cr_sqrt(x) - cr_sqrt(t);
            m = 1.0f - cr_div(d * d, s2, rs2);
        } else {  // library sqrtf and '/' (correctly rounded in every case)
            const float d = sqrtf(x) - sqrtf(t);
            m = 1.0f - (d * d) / s2;
        }
        if (act) sc.out[sc.qs[e]] = m > 0.0f ? m : 0.0f;
    }
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int g = 0; g < E / 4; ++g) {
        const f32x4 o = *reinterpret_cast<const f32x4 *>(&sc.out[256 * g + 4 * lane]);
#pragma unroll
        for (int q = 0; q < 4; ++q) out[4 * g + q] = o[q];
    }
    __builtin_amdgcn_wave_barrier();  // the next call rewrites sc
}

__global__ __launch_bounds__(256) void compat_kernel(const float *__restrict__ src,
                                                     const float *__restrict__ tgt, int Nstr,
                                                     int ntile, const float *__restrict__ sigma_d_ptr,
                                                     float *__restrict__ M, Ragged rg) {
    __shared__ float tileT[CT][CT + 1];
    __shared__ float pts[4][CT][3];  // row src, row tgt, col src, col tgt
    // linear upper-triangular tile index -> (ti, tj), ti <= tj
    int t = blockIdx.x, ti = 0;
    while (t >= ntile - ti) { t -= ntile - ti; ++ti; }
    const int tj = ti + t;
    const int b = blockIdx.y;
    // N: this pair's correspondences (rows / columns past it are not written);
    // Nstr: the row stride of the batch's buffers
    const int N = rg.n(b, Nstr);
    if (tj * CT >= N) return;  // workgroup-uniform
    const float sd = sigma_d_ptr[0];
    const float s2 = sd * sd;
    const float rs2 = 1.0f / s2;  // correctly rounded (the library division)
    // fast path: every squared distance of the tile is 0 or >= 2^-96 and s2 is a normal
    // number with a normal reciprocal (checked per element below, wave-uniformly)
    const bool s2ok = s2 >= 1.17549435e-38f && s2 < 1e30f && rs2 >= 1.17549435e-38f;
    src += (size_t)b * Nstr * 3;
    tgt += (size_t)b * Nstr * 3;
    M += (size_t)b * Nstr * Nstr;
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
    const bool vec = (Nstr & 3) == 0;
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) {
        const int r = rq + 16 * rr;
        const int i = i0 + r;
        const float six = pts[0][r][0], siy = pts[0][r][1], siz = pts[0][r][2];
        const float tix = pts[1][r][0], tiy = pts[1][r][1], tiz = pts[1][r][2];
        float out[4];
        float xs[4], xt[4];
        bool tiny = false;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int c = cq * 4 + q;
            xs[q] = sqdist3(six, siy, siz, pts[2][c][0], pts[2][c][1], pts[2][c][2]);
            xt[q] = sqdist3(tix, tiy, tiz, pts[3][c][0], pts[3][c][1], pts[3][c][2]);
            tiny |= (xs[q] != 0.0f && !(xs[q] >= 0x1p-96f)) || (xt[q] != 0.0f && !(xt[q] >= 0x1p-96f));
        }
        if (s2ok && !__any(tiny)) {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const float d = cr_sqrt(xs[q]) - cr_sqrt(xt[q]);
                const float m = 1.0f - cr_div(d * d, s2, rs2);
                out[q] = m > 0.0f ? m : 0.0f;
            }
        } else {  // library sqrtf and '/' (correctly rounded in every case)
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const float d = sqrtf(xs[q]) - sqrtf(xt[q]);
                const float m = 1.0f - (d * d) / s2;
                out[q] = m > 0.0f ? m : 0.0f;
            }
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) tileT[cq * 4 + q][r] = out[q];
        if (i < N) {
            const int j = j0 + cq * 4;
            float *dst = M + (size_t)i * Nstr + j;
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
        float *dst = M + (size_t)i * Nstr + j;
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

// The forward's M: symmetric-packed 32 x 32 tiles (pdsc_internal.hpp,
// mpack_tile), each one contiguous 4 KiB block -- half the bytes of the dense
// matrix, and each block exactly the 32 keys x 32 queries an attention wave
// reads per step (in either orientation).  A workgroup computes a 64 x 64
// upper-triangle block (ti <= tj) like the dense kernel and stores its four
// 32 x 32 tiles (three on the diagonal: the lower one is the transpose of the
// upper).  (The dense, twice-written form above costs 2x the bytes in 256-B
// segments strided by 4N B: ~2.9 TB/s at N = 5000 against ~5.3 TB/s for
// contiguous stores, tools/compat_bench.hip.)  Entries past N are written as 0.
__global__ __launch_bounds__(256) void compat_packed_kernel(const float *__restrict__ src,
                                                            const float *__restrict__ tgt, int Nstr, int ntile,
                                                            const float *__restrict__ sigma_d_ptr,
                                                            float *__restrict__ Mp, Ragged rg) {
    __shared__ float pts[4][CT][3];  // row src, row tgt, col src, col tgt
    constexpr int RP = COMPAT_RP, E = 4 * RP;  // rows per compat_n call, elements per lane
    __shared__ CompatScratch<E> scr[4];
    int t = blockIdx.x, ti = 0;
    while (t >= ntile - ti) { t -= ntile - ti; ++ti; }
    const int tj = ti + t;
    const int b = blockIdx.y;
    // N: this pair's correspondences; Nstr: the batch's stride (the packed layout
    // is that of Nstr for every pair).  Blocks whose rows all lie past N are
    // never read: every tile an attention wave of this pair reads has its
    // smaller tile index below ceil(N / 32).
    const int N = rg.n(b, Nstr);
    if (ti * CT >= N) return;  // workgroup-uniform
    const float sd = sigma_d_ptr[0];
    const float s2 = sd * sd;
    const float rs2 = 1.0f / s2;
    const bool s2ok = s2 >= 1.17549435e-38f && s2 < 1e30f && rs2 >= 1.17549435e-38f;
    const float kzero = 2.0f * s2 * (1.0f + 0x1p-10f), gmax = 0x1p20f * s2;  // compat_n's zero test
    src += (size_t)b * Nstr * 3;
    tgt += (size_t)b * Nstr * 3;
    const int nt32 = mpack_ntile(Nstr);
    float *Mb = Mp + (size_t)b * mpack_floats(Nstr);
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int i0 = ti * CT, j0 = tj * CT;
    for (int e = tid; e < CT * 3; e += 256) {
        const int p = e / 3, c = e % 3;
        pts[0][p][c] = (i0 + p < N) ? src[(size_t)(i0 + p) * 3 + c] : 0.f;
        pts[1][p][c] = (i0 + p < N) ? tgt[(size_t)(i0 + p) * 3 + c] : 0.f;
        pts[2][p][c] = (j0 + p < N) ? src[(size_t)(j0 + p) * 3 + c] : 0.f;
        pts[3][p][c] = (j0 + p < N) ? tgt[(size_t)(j0 + p) * 3 + c] : 0.f;
    }
    __syncthreads();
    const int cq = tid & 15, rq = tid >> 4;
    const int tc = 2 * tj + (cq >> 3);  // the 32-tile column of this thread's 4 columns
    float cs[4][3], ct[4][3];  // this thread's 4 columns, the same for every row below
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            cs[q][k] = pts[2][cq * 4 + q][k];
            ct[q][k] = pts[3][cq * 4 + q][k];
        }
    // EDGE: a diagonal block or one that reaches past N (per-element masking);
    // every other block (all but ~2 / ntile of them) runs without the masks
    auto rows = [&](auto edge_tag) {
        constexpr bool EDGE = decltype(edge_tag)::value;
#pragma unroll
        for (int r0 = 0; r0 < 4; r0 += RP) {
            // rows rq + 16 rr, rr = r0 .. r0 + RP - 1.  Elements below the diagonal
            // (diagonal blocks) or past N are not stored: their distances are set to
            // pass compat_n's zero test, so they never queue for the exact path.
            bool skip[RP], any = false;
            float xs[E], xt[E], out[E];
#pragma unroll
            for (int u = 0; u < RP; ++u) {
                const int r = rq + 16 * (r0 + u), tr = 2 * ti + (r >> 5);
                skip[u] = EDGE && (tr > tc || tr >= nt32 || tc >= nt32);
                any |= !skip[u];
                const float six = pts[0][r][0], siy = pts[0][r][1], siz = pts[0][r][2];
                const float tix = pts[1][r][0], tiy = pts[1][r][1], tiz = pts[1][r][2];
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    xs[4 * u + q] = sqdist3(six, siy, siz, cs[q][0], cs[q][1], cs[q][2]);
                    xt[4 * u + q] = sqdist3(tix, tiy, tiz, ct[q][0], ct[q][1], ct[q][2]);
                    if (EDGE && (skip[u] || i0 + r >= N || j0 + cq * 4 + q >= N)) {
                        xs[4 * u + q] = 4.0f * s2;
                        xt[4 * u + q] = 0.0f;
                    }
                }
            }
            if (EDGE && !__any(any)) continue;  // wave-uniform
            compat_n<E>(xs, xt, s2, rs2, s2ok, kzero, gmax, scr[wave], lane, out);
#pragma unroll
            for (int u = 0; u < RP; ++u) {
                if (skip[u]) continue;
                const int r = rq + 16 * (r0 + u), tr = 2 * ti + (r >> 5);
                float o[4];
#pragma unroll
                for (int q = 0; q < 4; ++q)
                    o[q] = (EDGE && (i0 + r >= N || j0 + cq * 4 + q >= N)) ? 0.0f : out[4 * u + q];
                float *tile = Mb + (size_t)mpack_tile(tr, tc, nt32) * (MPACK_T * MPACK_T);
                *reinterpret_cast<f32x4 *>(tile + (r & 31) * MPACK_T + ((cq * 4) & 31)) = f32x4{o[0], o[1], o[2], o[3]};
            }
        }
    };
    if (ti < tj && j0 + CT <= N)  // workgroup-uniform
        rows(std::false_type{});
    else
        rows(std::true_type{});
}

hipError_t launch_compat_packed(const float *src, const float *tgt, int B, int N, const float *sigma_d,
                                float *Mp, hipStream_t stream, Ragged rg) {
    const int ntile = (N + CT - 1) / CT;  // 64-point compute blocks
    const int ntri = ntile * (ntile + 1) / 2;
    hipLaunchKernelGGL(compat_packed_kernel, dim3(ntri, B), dim3(256), 0, stream, src, tgt, N, ntile, sigma_d, Mp, rg);
    return hipGetLastError();
}

hipError_t launch_compat(const float *src, const float *tgt, int B, int N, const float *sigma_d,
                         float *M, hipStream_t stream, Ragged rg) {
    const int ntile = (N + CT - 1) / CT;
    const int ntri = ntile * (ntile + 1) / 2;
    hipLaunchKernelGGL(compat_kernel, dim3(ntri, B), dim3(256), 0, stream, src, tgt, N, ntile,
                       sigma_d, M, rg);
    return hipGetLastError();
}

// counts -> nv, sv (one launch per RAGGED_CHUNK pairs, the counts as a kernel argument)
struct RaggedChunk {
    int32_t n[RAGGED_CHUNK];
};
__global__ void ragged_setup_kernel(RaggedChunk c, int nb, double ratio, int *__restrict__ nv, int *__restrict__ sv) {
    const int i = threadIdx.x;
    if (i >= nb) return;
    nv[i] = c.n[i];
    sv[i] = (int)((double)c.n[i] * ratio);  // int(num_corr * self.ratio) (models/PointDSC.py:174)
}

hipError_t launch_ragged_setup(const int32_t *counts, int B, double ratio, int *nv, int *sv, hipStream_t s) {
    for (int b0 = 0; b0 < B; b0 += RAGGED_CHUNK) {
        RaggedChunk c{};
        const int nb = std::min(RAGGED_CHUNK, B - b0);
        for (int i = 0; i < nb; ++i) c.n[i] = counts[b0 + i];
        hipLaunchKernelGGL(ragged_setup_kernel, dim3(1), dim3(RAGGED_CHUNK), 0, s, c, nb, ratio, nv + b0, sv + b0);
        HIP_RET(hipGetLastError());
    }
    return hipSuccess;
}

__global__ void ragged_order_kernel(RaggedChunk c, int nb, int *__restrict__ po) {
    const int i = threadIdx.x;
    if (i < nb) po[i] = c.n[i];
}

hipError_t launch_ragged_order(const int32_t *counts, int B, int *po, hipStream_t s) {
    std::vector<int> rank(B), order(B), next(8), end(8);
    for (int b = 0; b < B; ++b) rank[b] = b;
    std::stable_sort(rank.begin(), rank.end(), [&](int a, int b) { return counts[a] > counts[b]; });
    // the slot ranges of the 8 XCDs (attention_h3_block: consecutive workgroup
    // ids round-robin over the XCDs, each XCD's logical ids contiguous)
    for (int x = 0; x < 8; ++x) {
        next[x] = (int)((long)B * x / 8);
        end[x] = (int)((long)B * (x + 1) / 8);
    }
    std::vector<double> load(8, 0.0);
    for (int r = 0; r < B; ++r) {
        int best = -1;
        for (int x = 0; x < 8; ++x)
            if (next[x] < end[x] && (best < 0 || load[x] < load[best])) best = x;
        order[next[best]++] = rank[r];
        load[best] += (double)counts[rank[r]] * counts[rank[r]];
    }
    for (int b0 = 0; b0 < B; b0 += RAGGED_CHUNK) {
        RaggedChunk c{};
        const int nb = std::min(RAGGED_CHUNK, B - b0);
        for (int i = 0; i < nb; ++i) c.n[i] = order[b0 + i];
        hipLaunchKernelGGL(ragged_order_kernel, dim3(1), dim3(RAGGED_CHUNK), 0, s, c, nb, po + b0);
        HIP_RET(hipGetLastError());
    }
    return hipSuccess;
}

}  // namespace pdsc
