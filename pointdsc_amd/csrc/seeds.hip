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
#include <algorithm>
#include <cstdlib>

#include "pdsc_internal.hpp"

namespace pdsc {

// A workgroup owns SQ rows i (thread (slice, il): row il) and sweeps all j in
// 1024-point LDS tiles (one tile for N <= 1024: one global-load round trip);
// its 256 / SQ slices take disjoint parts of each tile, and the partial
// results meet in LDS.  SQ = 64 for batches; SQ = 16 when the batch has fewer
// than 1024 row blocks of 64 (a single N = 1000 pair: 63 workgroups instead of
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

// The same NMS with RPT rows per thread (rows blockIdx.x SQ RPT + r SQ + il):
// each LDS point feeds RPT compares (the one-row kernel above reads 16 B of LDS
// per compare and measured LDS-bound: packing its arithmetic cut VALU 8 -> 5.25
// per compare at unchanged time), and row pairs share packed fp32 arithmetic
// (v_pk_add / v_pk_mul / v_pk_fma_f32 against the point splat, the same
// per-component rounding as sqdist3).
template <int SQ, int RPT>
__global__ __launch_bounds__(256) void local_max_rows_kernel(const float *__restrict__ src,
                                                             const float *__restrict__ conf, int Nstr, float R2,
                                                             float *__restrict__ lm, Ragged rg) {
    static_assert(RPT % 2 == 0, "row pairs");
    constexpr int NSL = 256 / SQ, PER = SEED_TILE / NSL, NP = RPT / 2;
    __shared__ f32x4 tile[SEED_TILE];
    __shared__ unsigned char part[NSL][SQ * RPT];
    const int b = blockIdx.y, tid = threadIdx.x, sl = tid / SQ, il = tid % SQ;
    const int i0 = blockIdx.x * SQ * RPT + il;
    const int N = rg.n(b, Nstr);  // this pair's points; Nstr: the row stride
    if (blockIdx.x * SQ * RPT >= N) return;  // workgroup-uniform
    src += (size_t)b * Nstr * 3;
    conf += (size_t)b * Nstr;
    f32x2 xi[NP], yi[NP], zi[NP];
    float ci[RPT];
#pragma unroll
    for (int r = 0; r < RPT; ++r) {
        const int i = i0 + r * SQ;
        const bool in = i < N;
        const float x = in ? src[3 * i] : 0.0f, y = in ? src[3 * i + 1] : 0.0f, z = in ? src[3 * i + 2] : 0.0f;
        xi[r / 2][r & 1] = x;
        yi[r / 2][r & 1] = y;
        zi[r / 2][r & 1] = z;
        ci[r] = in ? conf[i] : 0.0f;
    }
    bool ok[RPT];
#pragma unroll
    for (int r = 0; r < RPT; ++r) ok[r] = true;
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
        bool bad[RPT];
#pragma unroll
        for (int r = 0; r < RPT; ++r) bad[r] = false;
        // the padded tail skipped per wave: lane 0's slice (the wave's lowest) has the
        // most points; the higher slices' extra points are other slices' points or
        // padding (conf -inf), both harmless to an OR of violations, and a
        // wave-uniform trip count keeps the loop scalar and unrolled
        const int jn = __builtin_amdgcn_readfirstlane(min(PER, max(N - j0 - sl * PER, 0)));
        const f32x4 *ts = tile + sl * PER;
#pragma unroll 4
        for (int t = 0; t < jn; ++t) {
            const f32x4 pj = ts[t];
            const f32x2 xj = {pj[0], pj[0]}, yj = {pj[1], pj[1]}, zj = {pj[2], pj[2]};
#pragma unroll
            for (int q = 0; q < NP; ++q) {
                const f32x2 dx = xi[q] - xj, dy = yi[q] - yj, dz = zi[q] - zj;
                const f32x2 x = __builtin_elementwise_fma(dz, dz, __builtin_elementwise_fma(dy, dy, dx * dx));
                bad[2 * q] |= (ci[2 * q] < pj[3]) & !(x[0] >= R2);
                bad[2 * q + 1] |= (ci[2 * q + 1] < pj[3]) & !(x[1] >= R2);
            }
        }
#pragma unroll
        for (int r = 0; r < RPT; ++r)
            if (bad[r]) ok[r] = false;
    }
#pragma unroll
    for (int r = 0; r < RPT; ++r) part[sl][r * SQ + il] = ok[r];
    __syncthreads();
    if (sl == 0) {
#pragma unroll
        for (int r = 0; r < RPT; ++r) {
            const int i = i0 + r * SQ;
            if (i >= N) continue;
            int all = 1;
#pragma unroll
            for (int q = 0; q < NSL; ++q) all &= part[q][r * SQ + il];
            lm[(size_t)b * Nstr + i] = all ? 1.0f : 0.0f;
        }
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
            rank += (int)((sj > si) | ((sj == si) & (j0 + jj < i)));  // bitwise: no branch per compare
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

// ------------------------------------------------------------------ sorted forms
// Both O(N^2) compare kernels above have an O(N log^2 N + N w) form for pairs of
// up to SORT_MAX points, one workgroup of 1024 threads per pair (per pair and
// 1024-row chunk for the NMS): a bitonic sort of 64-bit keys in LDS.
//   seed ranking: keys (descending score, ascending index) -- the top S of the
//   sorted list IS the rank order above, bit for bit (-0 is keyed as +0, so the
//   two tie as they compare equal);
//   NMS: keys (ascending x, index); row i compares only the points whose x lies
//   within 1.0625 sqrt(R2) of its own (found by binary search).  Any j farther
//   than that has |fl(x_i - x_j)| >= 1.0625 sqrt(R2) (1 - 2^-24), so its
//   squared distance -- a sum of non-negative terms, rounding monotone -- is
//   >= 1.12 R2 >= R2: the excluded compares are exactly the ones that cannot
//   violate.  A pair with a non-finite coordinate (NaN distances count as
//   within the radius) or a non-finite / NaN window scans every j.
constexpr int SORT_MAX = 8192;     // seed ranking: 64-bit keys, 64 KiB
constexpr int NMS_SORT_MAX = 5120;  // NMS: keys + sorted points (x, y, z, conf), 144 KiB
constexpr int SORT_NT = 1024;

PDSC_DEV void bitonic_sort_u64(unsigned long long *k, int P, int tid) {
    for (int size = 2; size <= P; size <<= 1)
        for (int stride = size >> 1; stride > 0; stride >>= 1) {
            __syncthreads();
            for (int t = tid; t < P / 2; t += SORT_NT) {
                const int i = 2 * t - (t & (stride - 1)), j = i + stride;  // the t-th pair at this stride
                const unsigned long long a = k[i], b = k[j];
                if ((a > b) == ((i & size) == 0)) {
                    k[i] = b;
                    k[j] = a;
                }
            }
        }
    __syncthreads();
}

// order-preserving uint32 of a float (ascending); -0 keyed as +0
PDSC_DEV uint32_t float_key(float f) {
    const uint32_t u = __float_as_uint(f == 0.0f ? 0.0f : f);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

// float_key's inverse (-0 comes back as +0, which compares equal to it; NaN bits kept)
PDSC_DEV float key_float(uint32_t k) { return __uint_as_float((k & 0x80000000u) ? (k & 0x7fffffffu) : ~k); }

PDSC_DEV int pow2_at_least(int n) {
    int P = 64;
    while (P < n) P <<= 1;
    return P;
}

__global__ __launch_bounds__(SORT_NT) void seed_rank_sort_kernel(const float *__restrict__ conf,
                                                                 const float *__restrict__ lm, int Nstr, int Sstr,
                                                                 int *__restrict__ seeds, Ragged rg) {
    extern __shared__ unsigned long long skeys[];
    const int b = blockIdx.x, tid = threadIdx.x;
    const int N = rg.n(b, Nstr), S = rg.s(b, Sstr);
    const int P = pow2_at_least(N);
    conf += (size_t)b * Nstr;
    lm += (size_t)b * Nstr;
    for (int i = tid; i < P; i += SORT_NT)
        skeys[i] = i < N ? ((unsigned long long)~float_key(conf[i] * lm[i]) << 32) | (unsigned)i  // (:217)
                         : ~0ull;
    bitonic_sort_u64(skeys, P, tid);
    for (int r = tid; r < S; r += SORT_NT) seeds[(size_t)b * Sstr + r] = (int)(unsigned)skeys[r];
}

// ------------------------------------------------------------------ select form
// The seed ranking of seed_rank_kernel in O(N + A^2) per pair, one 1024-thread
// workgroup per pair:
//  1. radix-select tau = the key of the S-th largest score (order-preserving
//     keys of conf * lm, -0 keyed as +0, 8-bit digits in LDS histograms whose
//     atomics are aggregated per wave for the wave's most common digit: most
//     scores are the zero of a point that is no local maximum);
//  2. the A < S candidates with key > tau are ranked among themselves -- every
//     j that outranks one (a larger score, or an equal one at a lower index) is
//     itself a candidate -- their keys and indices packed contiguously (one 8-B
//     broadcast read per compare), each candidate's count split over NT / A
//     threads that meet in an LDS sum;
//  3. places A .. S-1 are the first S - A points with key == tau in index order
//     (an ordered compaction: per-thread index ranges + a workgroup scan).
// rank_i = #{j : k_j > k_i} + #{j < i : k_j == k_i}, exactly seed_rank_kernel's
// count, bit for bit.  A > SEL_CMAX or a NaN score (whose compare ranks differ
// from any order): every row is ranked against all N instead, the compare
// kernel's loop.
constexpr int SEL_NT = 1024, SEL_CMAX = 2048;

__host__ __device__ constexpr size_t sel_lds(int N) { return (size_t)((N + 1) & ~1) * 4 + (size_t)SEL_CMAX * 12; }

// SPLIT: step 2 is left to seed_cand_rank_kernel (many workgroups per pair): the
// candidates go to `scratch` (per pair at b Sstr Nstr words: keys [Sstr], indices
// [Sstr], A) instead.
template <bool SPLIT>
__global__ __launch_bounds__(SEL_NT) void seed_select_kernel(const float *__restrict__ conf,
                                                             const float *__restrict__ lm, int Nstr, int Sstr,
                                                             int *__restrict__ seeds, uint32_t *__restrict__ scratch,
                                                             Ragged rg) {
    extern __shared__ __attribute__((aligned(16))) uint32_t selk[];  // [N] keys | [SEL_CMAX] (key, index) | [SEL_CMAX] ranks
    __shared__ int hist[256];
    __shared__ int wtot[SEL_NT / 64];
    __shared__ int sh_digit, sh_need, sh_cnt, sh_nan;
    const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int N = rg.n(b, Nstr), S = rg.s(b, Sstr);
    if (S < 1 || N < 1) return;  // workgroup-uniform: no seed to place (seed_cand_rank_kernel leaves too)
    if (SPLIT) scratch += (size_t)b * Sstr * Nstr;
    uint2 *cand = reinterpret_cast<uint2 *>(selk + ((Nstr + 1) & ~1));
    int *crank = reinterpret_cast<int *>(cand + SEL_CMAX);
    conf += (size_t)b * Nstr;
    lm += (size_t)b * Nstr;
    seeds += (size_t)b * Sstr;
    if (tid == 0) {
        sh_nan = 0;
        sh_cnt = 0;
    }
    __syncthreads();
    int nan = 0;
    for (int i = tid; i < N; i += SEL_NT) {
        const float sc = conf[i] * lm[i];  // (:217)
        nan |= sc != sc;
        selk[i] = float_key(sc);
    }
    if (nan) atomicOr(&sh_nan, 1);
    // radix select of the S-th largest key, most significant digit first
    uint32_t prefix = 0, mask = 0;
    int need = min(S, N);
    for (int shift = 24; shift >= 0; shift -= 8) {
        if (tid < 256) hist[tid] = 0;
        __syncthreads();
        for (int i = tid; i < N; i += SEL_NT) {
            const uint32_t k = selk[i];
            const bool in = (k & mask) == prefix;
            const int d = (int)((k >> shift) & 255u);
            const unsigned long long act = __ballot(in);
            if (act) {
                const int lead = __ffsll((long long)act) - 1;
                const int d0 = __shfl(d, lead);
                const unsigned long long same = __ballot(in && d == d0);
                if (lane == lead) atomicAdd(&hist[d0], __popcll(same));
                else if (in && d != d0) atomicAdd(&hist[d], 1);
            }
        }
        __syncthreads();
        if (tid < 64) {  // wave 0: the digit holding the need-th largest, scanning down
            int acc = 0, d = -1;
            for (int g = 3; g >= 0 && d < 0; --g) {
                const int bin = 64 * g + tid, c = hist[bin];
                // suffix sums from bin 64 g + 63 down to this lane's bin
                int suf = c;
#pragma unroll
                for (int o = 1; o < 64; o <<= 1) {
                    const int v = __shfl_down(suf, o);
                    if (tid + o < 64) suf += v;
                }
                const bool hit = acc + suf >= need && acc + suf - c < need;
                const unsigned long long m = __ballot(hit);
                if (m) {
                    const int l = __ffsll((long long)m) - 1;
                    const int above = __shfl(acc + suf - c, l);
                    d = 64 * g + l;
                    if (tid == 0) {
                        sh_digit = d;
                        sh_need = need - above;
                    }
                }
                acc += __shfl(suf, 0);
            }
        }
        __syncthreads();
        prefix |= (uint32_t)sh_digit << shift;
        mask |= 255u << shift;
        need = sh_need;
    }
    // tau = prefix; need = how many of the points with key == tau are seeds
    // candidates: key > tau, in any order
    for (int i = tid; i < N; i += SEL_NT)
        if (selk[i] > prefix) {
            const int p = atomicAdd(&sh_cnt, 1);
            if (p < SEL_CMAX) {
                cand[p] = uint2{selk[i], (uint32_t)i};
                crank[p] = 0;
            }
        }
    __syncthreads();
    const int A = sh_cnt;
    if (sh_nan || A > SEL_CMAX) {  // workgroup-uniform: the compare ranking of every row
        if (SPLIT && tid == 0) scratch[2 * Sstr] = 0;  // nothing for seed_cand_rank_kernel
        for (int i = tid; i < N; i += SEL_NT) {
            const float si = key_float(selk[i]);
            int rank = 0;
            for (int j = 0; j < N; ++j) {
                const float sj = key_float(selk[j]);
                rank += (int)((sj > si) | ((sj == si) & (j < i)));
            }
            if (rank < S) seeds[rank] = i;
        }
        return;
    }
    // places A .. A + need - 1: the first `need` points with key == tau, by index
    {
        const int chunk = (N + SEL_NT - 1) / SEL_NT, i0 = tid * chunk, i1 = min(N, i0 + chunk);
        int c = 0;
        for (int i = i0; i < i1; ++i) c += selk[i] == prefix;
        int inc = c;  // inclusive scan over the wave, then over the waves
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int v = __shfl_up(inc, o);
            if (lane >= o) inc += v;
        }
        if (lane == 63) wtot[wave] = inc;
        __syncthreads();
        int pos = A + inc - c;
        for (int w = 0; w < wave; ++w) pos += wtot[w];
        for (int i = i0; i < i1 && pos < A + need; ++i)
            if (selk[i] == prefix) seeds[pos++] = i;
    }
    if (SPLIT) {
        for (int q = tid; q < A; q += SEL_NT) {
            scratch[q] = cand[q].x;
            scratch[Sstr + q] = cand[q].y;
        }
        if (tid == 0) scratch[2 * Sstr] = (uint32_t)A;
        return;
    }
    // places 0 .. A - 1: candidate q's count over the r-slice `part` of P slices
    const int P = A > 0 ? max(1, SEL_NT / A) : 1, len = A > 0 ? (A + P - 1) / P : 0;
    for (int t = tid; t < A * P; t += SEL_NT) {
        const int q = t % A, part = t / A;
        const uint2 ci = cand[q];
        int rank = 0;
        const int r1 = min(A, (part + 1) * len);
#pragma unroll 4
        for (int r = part * len; r < r1; ++r) {
            const uint2 cj = cand[r];
            rank += (int)((cj.x > ci.x) | ((cj.x == ci.x) & (cj.y < ci.y)));
        }
        if (P == 1) crank[q] = rank;
        else if (rank) atomicAdd(&crank[q], rank);
    }
    __syncthreads();
    for (int q = tid; q < A; q += SEL_NT) seeds[crank[q]] = (int)cand[q].y;
}

// Step 2 of the split select: workgroup (x, b) ranks pair b's candidates
// 64 x .. 64 x + 63 against all A of them (four threads per candidate, each a
// quarter of the A compares, summed in LDS) -- A^2 compares over A / 64
// workgroups instead of one.
constexpr int SEL_RQ = 64;

__global__ __launch_bounds__(256) void seed_cand_rank_kernel(const uint32_t *__restrict__ scratch, int Nstr,
                                                             int Sstr, int *__restrict__ seeds, Ragged rg) {
    __shared__ uint2 c[SEL_CMAX];
    __shared__ int part[4][SEL_RQ];
    const int b = blockIdx.y, tid = threadIdx.x;
    const int N = rg.n(b, Nstr), S = rg.s(b, Sstr);
    if (S < 1 || N < 1) return;  // workgroup-uniform (seed_select_kernel wrote nothing)
    scratch += (size_t)b * Sstr * Nstr;
    const int A = (int)scratch[2 * Sstr], q0 = blockIdx.x * SEL_RQ;
    if (q0 >= A) return;  // workgroup-uniform
    for (int r = tid; r < A; r += 256) c[r] = uint2{scratch[r], scratch[Sstr + r]};
    __syncthreads();
    const int q = q0 + (tid & (SEL_RQ - 1)), p = tid / SEL_RQ, len = (A + 3) / 4;
    int rank = 0;
    if (q < A) {
        const uint2 ci = c[q];
        const int r1 = min(A, (p + 1) * len);
#pragma unroll 4
        for (int r = p * len; r < r1; ++r) {
            const uint2 cj = c[r];
            rank += (int)((cj.x > ci.x) | ((cj.x == ci.x) & (cj.y < ci.y)));
        }
    }
    part[p][tid & (SEL_RQ - 1)] = rank;
    __syncthreads();
    if (tid < SEL_RQ && q < A)
        seeds[(size_t)b * Sstr + part[0][tid] + part[1][tid] + part[2][tid] + part[3][tid]] = (int)c[q].y;
}

__global__ __launch_bounds__(SORT_NT) void local_max_sort_kernel(const float *__restrict__ src,
                                                                 const float *__restrict__ conf, int Nstr, float R2,
                                                                 float *__restrict__ lm, Ragged rg) {
    extern __shared__ unsigned long long skeys[];
    const int b = blockIdx.y, tid = threadIdx.x;
    const int N = rg.n(b, Nstr);
    if (blockIdx.x * SORT_NT >= N) return;  // workgroup-uniform (ragged pairs)
    const int P = pow2_at_least(N);
    f32x4 *sp = reinterpret_cast<f32x4 *>(skeys + P);  // points in ascending-x order: (x, y, z, conf)
    src += (size_t)b * Nstr * 3;
    conf += (size_t)b * Nstr;
    int bad = 0;
    for (int i = tid; i < P; i += SORT_NT) {
        if (i < N) {
            const float x = src[3 * i], y = src[3 * i + 1], z = src[3 * i + 2];
            bad |= !(__builtin_isfinite(x) && __builtin_isfinite(y) && __builtin_isfinite(z));
            skeys[i] = ((unsigned long long)float_key(x) << 32) | (unsigned)i;
        } else {
            skeys[i] = ~0ull;
        }
    }
    bad = __syncthreads_or(bad);
    bitonic_sort_u64(skeys, P, tid);
    for (int q = tid; q < N; q += SORT_NT) {
        const int i = (int)(unsigned)skeys[q];
        sp[q] = f32x4{src[3 * i], src[3 * i + 1], src[3 * i + 2], conf[i]};
    }
    __syncthreads();
    const int q = blockIdx.x * SORT_NT + tid;  // this thread's row, in sorted order
    if (q >= N) return;
    const f32x4 pi = sp[q];
    const double W = 1.0625 * sqrt((double)R2);
    int lo = 0, hi = N;  // the window [lo, hi) of sorted positions (everything when it cannot be trusted)
    if (!bad && W <= 1e300) {
        const double xl = (double)pi[0] - W, xh = (double)pi[0] + W;
        int a = 0, c = q;  // first position with x >= xl
        while (a < c) {
            const int m = (a + c) >> 1;
            if ((double)sp[m][0] >= xl) c = m; else a = m + 1;
        }
        lo = a;
        a = q + 1;
        c = N;  // first position with x > xh
        while (a < c) {
            const int m = (a + c) >> 1;
            if ((double)sp[m][0] > xh) c = m; else a = m + 1;
        }
        hi = a;
    }
    // violation: c_i < c_j and !(|s_i - s_j| >= R) -- the compare of local_max_kernel
    bool viol = false;
    for (int j = lo; j < hi; ++j) {
        const f32x4 pj = sp[j];
        const float x = sqdist3(pi[0], pi[1], pi[2], pj[0], pj[1], pj[2]);
        viol |= (pi[3] < pj[3]) & !(x >= R2);
    }
    lm[(size_t)b * Nstr + (int)(unsigned)skeys[q]] = viol ? 0.0f : 1.0f;
}

// The 16-row kernels below 1024 blocks of 64 rows (r04: 8 x 5000, 632 blocks:
// seed_rank 49 vs 61 us at 4x the waves, local_max equal; 128 x 1000 keeps 64).
// A/B knob PDSC_SEED_BLOCKS (measurement only) moves the bound.
static bool seed_small(int B, int N) {
    static const long lim = [] {
        const char *e = getenv("PDSC_SEED_BLOCKS");
        return e ? atol(e) : 1024L;
    }();
    return (long)B * ((N + 63) / 64) < lim;
}

// The sorted forms are opt-in (A/B knob PDSC_SEED_SORT=1, measurement only):
// r04 measured them slower than the compare kernels at every bench shape --
// 8 x 5000 forward 4.60 vs 4.51 ms, one N = 1000 pair 0.467 vs 0.441 ms, equal
// at 128 x 1000 -- one 1024-thread workgroup per pair sorts 1024-8192 keys in
// 55-91 barrier-separated steps, against the compare kernels' hundreds of
// workgroups.
static bool seed_sort_on() {
    static const bool on = [] {
        const char *e = getenv("PDSC_SEED_SORT");
        return e && e[0] == '1';
    }();
    return on;
}
static size_t sort_lds(int N) { return (size_t)std::max(64, 1 << (32 - __builtin_clz((unsigned)std::max(N - 1, 1)))) * 8; }

// rows per thread of the NMS compare kernel: 2 (local_max_rows_kernel<16, 2>)
// for batches on the 16-row blocks, else 1 (local_max_kernel) (r06: 8 x 5000
// forward -15 / -24 us on two boxes and local_max 70.8 -> 60.3 us, but the
// 64-row blocks slower with two rows -- 128 x 1000 31.4 -> 37.2 us, the ragged
// bench 52 -> 72 us, r06j vs r06k profiles -- and one pair +2 us at N = 1000,
// +5-10 us at N = 5000: profiles/r06_ab_lm*.log); A/B knob PDSC_LM_RPT=1|2|4
// at every batch size (measurement only, the same bits)
static int lm_rpt(int B, int N) {
    static const int r = [] {
        const char *e = getenv("PDSC_LM_RPT");
        return e ? atoi(e) : 0;
    }();
    return r ? r : (B > 1 && seed_small(B, N) ? 2 : 1);
}

hipError_t launch_local_max(const float *src, const float *conf, int B, int N, float radius,
                            float *lm, hipStream_t s, Ragged rg) {
    if (seed_sort_on() && N <= NMS_SORT_MAX) {
        const size_t lds = sort_lds(N) + (size_t)N * sizeof(f32x4);
        hipLaunchKernelGGL(local_max_sort_kernel, dim3((N + SORT_NT - 1) / SORT_NT, B), dim3(SORT_NT), lds, s, src, conf,
                           N, sqrt_ge_threshold(radius), lm, rg);
    } else if (lm_rpt(B, N) == 4) {
        if (seed_small(B, N))
            hipLaunchKernelGGL((local_max_rows_kernel<16, 4>), dim3((N + 63) / 64, B), dim3(256), 0, s, src, conf, N,
                               sqrt_ge_threshold(radius), lm, rg);
        else
            hipLaunchKernelGGL((local_max_rows_kernel<64, 4>), dim3((N + 255) / 256, B), dim3(256), 0, s, src, conf,
                               N, sqrt_ge_threshold(radius), lm, rg);
    } else if (lm_rpt(B, N) == 2) {
        if (seed_small(B, N))
            hipLaunchKernelGGL((local_max_rows_kernel<16, 2>), dim3((N + 31) / 32, B), dim3(256), 0, s, src, conf, N,
                               sqrt_ge_threshold(radius), lm, rg);
        else
            hipLaunchKernelGGL((local_max_rows_kernel<64, 2>), dim3((N + 127) / 128, B), dim3(256), 0, s, src, conf,
                               N, sqrt_ge_threshold(radius), lm, rg);
    } else if (seed_small(B, N))
        hipLaunchKernelGGL(local_max_kernel<16>, dim3((N + 15) / 16, B), dim3(256), 0, s, src, conf, N,
                           sqrt_ge_threshold(radius), lm, rg);
    else
        hipLaunchKernelGGL(local_max_kernel<64>, dim3((N + 63) / 64, B), dim3(256), 0, s, src, conf, N,
                           sqrt_ge_threshold(radius), lm, rg);
    return hipGetLastError();
}

// The select form (seed_select_kernel) where the compare kernels' B N^2 work is
// large (>= 1e8 compares: 128 x 1000, 8 x 5000) and its keys and candidates fit
// the workgroup's LDS; split in two launches (seed_cand_rank_kernel: the A^2
// candidate compares over many workgroups) from S > 256 when the caller has
// scratch.  Measured (rocprofv3, one box): 128 x 1000 13.2 us vs 15.8 for the
// first select form (256 threads, every compare through an index) and ~26 for
// seed_rank_kernel<64>; one N = 1000 pair 9.5 vs 5.4 (seed_rank_kernel<16>).
// A/B knob PDSC_SEED_SELECT (measurement only): 0 never, 1 at every batch size.
static bool seed_select_on(int B, int N) {
    static const int mode = [] {
        const char *e = getenv("PDSC_SEED_SELECT");
        return e ? atoi(e) : 2;
    }();
    if (mode == 0 || sel_lds(N) > 64 * 1024) return false;
    return mode == 1 || (double)B * N * N >= 1e8;
}

hipError_t launch_seed_rank(const float *conf, const float *lm, int B, int N, int S, int *seeds,
                            hipStream_t s, Ragged rg, uint32_t *scratch) {
    if (seed_select_on(B, N) && !seed_sort_on()) {
        // scratch per pair: 2 S + 1 <= S N words
        static const bool split_off = [] {  // A/B knob PDSC_SEL_SPLIT=0 (measurement only)
            const char *e = getenv("PDSC_SEL_SPLIT");
            return e && e[0] == '0';
        }();
        if (scratch && S > 256 && N >= 3 && !split_off) {
            hipLaunchKernelGGL(seed_select_kernel<true>, dim3(B), dim3(SEL_NT), sel_lds(N), s, conf, lm, N, S, seeds,
                               scratch, rg);
            hipLaunchKernelGGL(seed_cand_rank_kernel, dim3(SEL_CMAX / SEL_RQ, B), dim3(256), 0, s, scratch, N, S,
                               seeds, rg);
        } else {
            hipLaunchKernelGGL(seed_select_kernel<false>, dim3(B), dim3(SEL_NT), sel_lds(N), s, conf, lm, N, S, seeds,
                               nullptr, rg);
        }
    } else if (seed_sort_on() && N <= SORT_MAX)
        hipLaunchKernelGGL(seed_rank_sort_kernel, dim3(B), dim3(SORT_NT), sort_lds(N), s, conf, lm, N, S, seeds, rg);
    else if (seed_small(B, N))
        hipLaunchKernelGGL(seed_rank_kernel<16>, dim3((N + 15) / 16, B), dim3(256), 0, s, conf, lm, N, S, seeds, rg);
    else
        hipLaunchKernelGGL(seed_rank_kernel<64>, dim3((N + 63) / 64, B), dim3(256), 0, s, conf, lm, N, S, seeds, rg);
    return hipGetLastError();
}

}  // namespace pdsc
