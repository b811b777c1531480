// nsm.hip -- a6-a11: Neural Spectral Matching, hypothesis verification and
// post-refinement.
//
//   knn_dist     a6  seed rows of 2 - 2 F F^T (3-product fp16 MFMA), [B][S][N]
//   knn_select   a6  topk(k+1, smallest)[1:] per seed row (one wave per seed,
//                    row in registers): lane-minimum threshold + compaction +
//                    (key, index) ranking; radix-select fallback
//   nsm_seed     a7-a8  one wave per seed: k x k feature Gram on the fp16
//                    matrix cores (3-product split), T = F o S in LDS, then all
//                    num_iterations power iterates + per-iterate allclose flags
//   nsm_finish   a8  pair- or batch-global early exit t* = first iterate where every seed
//                    is allclose (torch.allclose over the whole batch, :354)
//   hypotheses   a9-a10  weighted Kabsch per seed (fp64 3x3 SVD on device) +
//                    inlier count over all N correspondences
//   select_best  a10 first argmax of fitness, labels of the best hypothesis
//   post_refine  a11 <= 20 device-side IRLS refits, one workgroup per pair
#include "attention_h3.hpp"

namespace pdsc {

// NSM A/B build knob: 1 (default) the T build on packed fp32 (source, target)
// pairs and the power iterate's norm through the wave-uniform cr_sqrt; 0 the
// scalar T build and sqrtf (the same bits either way)
#ifndef NSM_PK_TBUILD
#define NSM_PK_TBUILD 1
#endif

// ------------------------------------------------------------------ a6 kNN
// dist[b][s][j] = 2 - 2 * <normed[seed_s], normed[j]>   (models/common.py:58-60)
// on the fp16 matrix cores with the 3-product split of attention_h3.hpp
// (|error| <= 2^-21 on a distance in [0, 4], i.e. fp32-equivalent): ns is the
// split copy of normed, [B][N][2][128] fp16 in qk_pos order (pw_last writes it).
// A workgroup = 4 waves = 4 tiles of 32 seeds (lane <-> seed fragment, held in
// registers for the whole launch) sweeping KNN_KPB tiles of 32 keys; each key
// tile (32 rows x 512 B of split features, contiguous in HBM) is copied once
// into LDS (16-B chunks XOR-swizzled by row: conflict-free fragment reads) and
// feeds all four waves, so a wave-tile of 24 MFMAs costs ~4 KB of L2 traffic
// instead of 24 KB.  lane <-> key in the accumulator (register r is seed row
// acc_row(r, h)): each store instruction writes 128 contiguous bytes.
constexpr int KNN_KPB = 5;

// order-preserving float -> uint key (+0 and -0 share a key, like float ==).
// The kNN distance rows are stored as these keys (knn_select ranks keys; the
// distances themselves are never read back).
PDSC_DEV uint32_t fkey(float f) {
    if (f == 0.0f) f = 0.0f;
    const uint32_t u = __float_as_uint(f);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

__global__ __launch_bounds__(256, 4) void knn_dist_kernel(const _Float16 *__restrict__ ns,
                                                       const int *__restrict__ seeds, int Nstr, int Sstr,
                                                       int kpb, float *__restrict__ dist, Ragged rg) {
    __shared__ f16x8 Bt[32 * 32];
    uint32_t *dkey = reinterpret_cast<uint32_t *>(dist);
    const int b = blockIdx.z, tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int h = lane >> 5, l32 = lane & 31;
    // this pair's keys and seeds; Nstr, Sstr: the batch's strides (rows [b][s] of
    // dist are Nstr long)
    const int N = rg.n(b, Nstr), S = rg.s(b, Sstr);
    if (blockIdx.y * 128 >= S || blockIdx.x * kpb * 32 >= N) return;  // workgroup-uniform
    const int s0 = (blockIdx.y * 4 + wave) * 32;
    const bool active = s0 < S;  // wave-uniform; every wave joins the barriers
    const _Float16 *F = ns + (size_t)b * Nstr * 2 * CH;
    const int sidx = s0 + l32;
    f16x8 ah[8], al[8];
    if (active) {
        const int seed = (sidx < S) ? seeds[(size_t)b * Sstr + sidx] : 0;
        const char *row = reinterpret_cast<const char *>(F + (size_t)min(max(seed, 0), N - 1) * 2 * CH);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            ah[j] = *reinterpret_cast<const f16x8 *>(row + 16 * (2 * j + h));
            al[j] = *reinterpret_cast<const f16x8 *>(row + 2 * CH + 16 * (2 * j + h));
        }
    }
    const int nkt = (N + 31) / 32;
    const int t0 = blockIdx.x * kpb, t1 = min(t0 + kpb, nkt);
    // the wave's 32 seed rows through a buffer resource: rows past S fall outside
    // it (their stores are dropped), row r's offset is an SGPR operand
    const uint32_t rowb = (uint32_t)Nstr * 4u;
    const __amdgpu_buffer_rsrc_t rd =
        h3_rsrc(dkey + ((size_t)b * Sstr + min(s0, S)) * Nstr, (uint32_t)max(min(32, S - s0), 0) * rowb);
    // key tile t+1 is loaded into registers while tile t computes and stores
    f16x8 stage[4];
    auto load_tile = [&](int t) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int e = tid + 256 * q, r = e >> 5, c = e & 31;
            stage[q] = reinterpret_cast<const f16x8 *>(F + (size_t)min(t * 32 + r, N - 1) * 2 * CH)[c];
        }
    };
    if (t0 < t1) load_tile(t0);
    for (int t = t0; t < t1; ++t) {
        const int j0 = t * 32;
        __syncthreads();  // the previous tile's readers are done
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int e = tid + 256 * q, r = e >> 5, c = e & 31;
            Bt[r * 32 + (c & 16) + ((c & 15) ^ (r & 15))] = stage[q];
        }
        __syncthreads();
        if (t + 1 < t1) load_tile(t + 1);
        if (!active) continue;
        const int j = j0 + l32;
        f32x16 acc = zero16();
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int cc = (2 * i + h) ^ (l32 & 15);
            acc = mfma_h3(ah[i], al[i], Bt[l32 * 32 + cc], Bt[l32 * 32 + 16 + cc], acc);
        }
        if (j < N) {
            const uint32_t vo = 4u * j + (uint32_t)(4 * h) * rowb;
#pragma unroll
            for (int r = 0; r < 16; ++r)
                __builtin_amdgcn_raw_buffer_store_b32(fkey(2.0f - 2.0f * acc[r]), rd, vo,
                                                      (uint32_t)((r & 3) + 8 * (r >> 2)) * rowb, 0);
        }
    }
}

hipError_t launch_knn_dist(const _Float16 *ns, const int *seeds, int B, int N, int S, float *dist,
                           hipStream_t s, Ragged rg) {
    const int nkt = (N + 31) / 32;
    // key tiles per workgroup: KNN_KPB, or 1 when that leaves fewer than 256
    // workgroups (a single N = 1000 pair: 32 instead of 7)
    const long wg5 = (long)((nkt + KNN_KPB - 1) / KNN_KPB) * ((S + 127) / 128) * B;
    const int kpb = wg5 >= 256 ? KNN_KPB : 1;
    hipLaunchKernelGGL(knn_dist_kernel, dim3((nkt + kpb - 1) / kpb, (S + 127) / 128, B), dim3(256), 0, s,
                       ns, seeds, N, S, kpb, dist, rg);
    return hipGetLastError();
}

// PDSC_PRECISION_F32: the same seed rows of 2 - 2 F F^T on exact fp32 MFMA
// (32x32x2), straight from the fp32 normed rows [B][N][128].  A wave owns 32
// seeds (its 64 fp32 fragment values per lane held for the launch) and sweeps
// KNN_KPB key tiles, each key fragment read from L2 as 16-B pieces; k-step
// 4j + e of lane (h, .) is channel 8j + 4h + e for both operands.
__global__ __launch_bounds__(256) void knn_dist_f32_kernel(const float *__restrict__ normed,
                                                           const int *__restrict__ seeds, int Nstr, int Sstr,
                                                           float *__restrict__ dist, Ragged rg) {
    uint32_t *dkey = reinterpret_cast<uint32_t *>(dist);
    const int b = blockIdx.z, tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int h = lane >> 5, l32 = lane & 31;
    const int N = rg.n(b, Nstr), S = rg.s(b, Sstr);  // this pair's keys and seeds
    const int s0 = (blockIdx.y * 4 + wave) * 32;
    if (s0 >= S) return;  // wave-uniform; no barriers
    const float *F = normed + (size_t)b * Nstr * CH;
    const int sidx = s0 + l32;
    const int seed = (sidx < S) ? seeds[(size_t)b * Sstr + sidx] : 0;
    const float *srow = F + (size_t)min(max(seed, 0), N - 1) * CH + 4 * h;
    f32x4 a[CH / 8];
#pragma unroll
    for (int j = 0; j < CH / 8; ++j) a[j] = *reinterpret_cast<const f32x4 *>(srow + 8 * j);
    const int nkt = (N + 31) / 32;
    const int t0 = blockIdx.x * KNN_KPB, t1 = min(t0 + KNN_KPB, nkt);
    for (int t = t0; t < t1; ++t) {
        const int j = t * 32 + l32;
        const float *krow = F + (size_t)min(j, N - 1) * CH + 4 * h;
        f32x16 acc = zero16();
#pragma unroll
        for (int jj = 0; jj < CH / 8; ++jj) {
            const f32x4 bv = *reinterpret_cast<const f32x4 *>(krow + 8 * jj);
#pragma unroll
            for (int e = 0; e < 4; ++e) acc = mfma32(a[jj][e], bv[e], acc);
        }
        if (j < N) {
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int sr = s0 + acc_row(r, h);
                if (sr < S) dkey[((size_t)b * Sstr + sr) * Nstr + j] = fkey(2.0f - 2.0f * acc[r]);
            }
        }
    }
}

hipError_t launch_knn_dist_f32(const float *normed, const int *seeds, int B, int N, int S, float *dist,
                               hipStream_t s, Ragged rg) {
    const int nkt = (N + 31) / 32;
    hipLaunchKernelGGL(knn_dist_f32_kernel, dim3((nkt + KNN_KPB - 1) / KNN_KPB, (S + 127) / 128, B), dim3(256), 0,
                       s, normed, seeds, N, S, dist, rg);
    return hipGetLastError();
}

// fp32 rows [rows][128] -> [rows][2][128] fp16 hi/lo in qk_pos order (standalone API)
__global__ void split_rows_kernel(const float *__restrict__ x, size_t rows, _Float16 *__restrict__ out) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= rows * CH) return;
    const size_t row = i / CH;
    const int c = (int)(i % CH);
    _Float16 hi, lo;
    split_h(x[i], hi, lo);
    out[(size_t)row * 2 * CH + qk_pos(c)] = hi;
    out[(size_t)row * 2 * CH + CH + qk_pos(c)] = lo;
}

hipError_t launch_split_rows(const float *x, size_t rows, _Float16 *out, hipStream_t s) {
    const size_t n = rows * CH;
    hipLaunchKernelGGL(split_rows_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, x, rows, out);
    return hipGetLastError();
}

// topk(k+1, smallest) of one seed row, one WAVE per seed (4 per workgroup).
// The row's keys live in registers (R per lane, R*64 >= N; R = 0: re-read
// from memory each pass, any N).  Radix select on the order-preserving keys:
// starting at the highest bit where the row's min and max keys differ (the
// common prefix carries no information -- distances in [0, 4] share their top
// byte, and an 8-bit digit there would put every key in one histogram bin),
// 8-bit digits are histogrammed in LDS until the bin holding the (k+1)-th
// smallest key is taken whole, holds <= KNN_BINCAP keys, or the key is
// resolved.  One ordered pass then collects every key below that bin (ballot
// + popcount compaction) and either the bin's keys (ranked by (key, index) to
// pick the `need` smallest -- usually after ONE histogram pass) or its first
// `need` keys in index order; the k+1 candidates are ranked by (key, index)
// and the first is dropped positionally (models/common.py:68).
// Rows to R = 80 keep 4 waves per SIMD (<= 128 VGPRs; the register fallback
// alone would take 142 at R = 80, and 8 x 5000's 4000 row waves would need two
// rounds of 3: r06, profiles/r06_ab_knn_wpe.log).
constexpr int KNN_BINCAP = 64;
constexpr int KNN_FASTCAP = 128;

#ifdef KNN_DIAG
// Diagnostic build only (-DKNN_DIAG): per launch, how many seed rows took each
// path: [0] bitonic fast path, [1] readlane ranking, [2] radix fallback,
// [3] fallback histogram passes, [4] fallback rows resolved through a small bin.
static __device__ unsigned g_knn_paths[8];
#define KNN_COUNT(i, v) do { if (lane == 0) atomicAdd(&g_knn_paths[i], (unsigned)(v)); } while (0)
extern "C" int pdsc_diag_knn_paths(unsigned *host, int reset) {
    if (hipMemcpyFromSymbol(host, HIP_SYMBOL(g_knn_paths), sizeof(g_knn_paths), 0, hipMemcpyDeviceToHost) != hipSuccess)
        return -1;
    static const unsigned zero[8] = {};
    return reset && hipMemcpyToSymbol(HIP_SYMBOL(g_knn_paths), zero, sizeof(zero), 0, hipMemcpyHostToDevice) != hipSuccess
               ? -1 : 0;
}
#else
#define KNN_COUNT(i, v) do { } while (0)
#endif

template <int R>
__global__ __launch_bounds__(256, R <= 80 ? 4 : 1) void knn_select_kernel(const float *__restrict__ dist, int Nstr, int Sstr,
                                                         int k, int *__restrict__ knn, Ragged rg, int bitonic) {
    __shared__ uint32_t hist[4][256];
    __shared__ uint32_t ckey[4][64];
    __shared__ int cidx[4][64];
    __shared__ uint32_t bkey[4][KNN_BINCAP];
    __shared__ int bidx[4][KNN_BINCAP];
    __shared__ uint32_t fkeyb[4][KNN_FASTCAP];
    __shared__ int fidxb[4][KNN_FASTCAP];
    const int b = blockIdx.y, wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int s = blockIdx.x * (blockDim.x >> 6) + wave;
    // this pair's keys and seeds; Nstr, Sstr: the batch's strides
    const int N = rg.n(b, Nstr), S = rg.s(b, Sstr);
    if (s >= S) return;  // wave-uniform; no workgroup barriers below
    const uint32_t *row = reinterpret_cast<const uint32_t *>(dist) + ((size_t)b * Sstr + s) * Nstr;  // fkey keys
    const uint32_t want = k + 1;
    // Fast path (no atomics): tau0 = the want-th smallest of the 64 per-lane
    // minima bounds the want-th smallest key from above (at least `want` keys are
    // <= tau0), so every key of the answer is <= tau0.  For iid keys about
    // 1.3 * want keys qualify; they are compacted (in any order) and ranked by
    // (key, index).  R > 0: the row is held in registers, lane l owning keys
    // 256 i + 4 l + e (16-B loads); R = 0: re-read from memory.  More than
    // KNN_FASTCAP qualifying keys (heavy ties, adversarial orders) falls through
    // to the radix select below.
    constexpr int NR = R > 0 ? R : 1;
    uint32_t key[NR];  // R > 0: the row in registers (fast path and radix fallback)
    {
        if constexpr (R > 0) {
            if ((Nstr & 3) == 0) {  // rows 16-B aligned (wave-uniform)
                // buffer loads over the row's first round_up(N, 4) keys (lane offset
                // in one VGPR, the key block's offset in the SGPR operand; blocks
                // past them return 0 without a fetch), branch-free, so all R/4
                // loads are in flight together and no per-load 64-bit addresses
                // stay live (97 vs 178 VGPRs at R = 80); keys past N selected away
                const __amdgpu_buffer_rsrc_t rr = h3_rsrc(row, (uint32_t)((N + 3) & ~3) * 4u);
#pragma unroll
                for (int i4 = 0; i4 < R / 4; ++i4) {
                    const u32x4 v = __builtin_bit_cast(
                        u32x4, __builtin_amdgcn_raw_buffer_load_b128(rr, 16u * lane, 1024u * i4, 0));
#pragma unroll
                    for (int e = 0; e < 4; ++e) key[4 * i4 + e] = 256 * i4 + 4 * lane + e < N ? v[e] : 0xffffffffu;
                }
            } else {
                // exec-masked dword loads (measured faster here than branch-free
                // buffer or clamped loads: 134 vs 150 / 145 us at 128 x 1289)
#pragma unroll
                for (int i = 0; i < R; ++i) {
                    const int j = 256 * (i >> 2) + 4 * lane + (i & 3);
                    key[i] = j < N ? row[j] : 0xffffffffu;
                }
            }
        }
    }
    if (want <= 64) {
        const int NI = R > 0 ? R : (N + 63) / 64;
        // index of this lane's i-th key
        auto J = [&](int i) -> int { return R > 0 ? 256 * (i >> 2) + 4 * lane + (i & 3) : lane + 64 * i; };
        auto K = [&](int i) -> uint32_t {
            if constexpr (R > 0) {
                return key[i];
            } else {
                const int j = lane + 64 * i;
                return j < N ? row[j] : 0xffffffffu;
            }
        };
        // Long rows (R >= 32: N > 2048) also keep each lane's second-smallest key:
        // the threshold then comes from 128 values, about half as many keys pass it
        // (clustered rows of a trained network: fewer rows overflow the fast path
        // into the radix select; r06).  Still at least `want` keys <= tau0 (a lane's
        // two values are two of its keys), so the same rows result.
        constexpr bool TWO = R >= 32;
        uint32_t lmin = 0xffffffffu, lmin2 = 0xffffffffu;
#pragma unroll
        for (int i = 0; i < NI; ++i)
            if (R > 0 || J(i) < N) {  // R > 0: keys past N are ~0u
                const uint32_t x = K(i);
                if constexpr (TWO) lmin2 = min(lmin2, max(lmin, x));
                lmin = min(lmin, x);
            }
        // tau0 = the want-th smallest lane minimum (TWO: of the 128 lane minima and
        // second minima): the smallest value v with #{lanes: lmin <= v} (+ #{lanes:
        // lmin2 <= v}) >= want, built bit by bit from the top (one compare + ballot
        // + scalar popcount per bit instead of 64 readlanes)
        uint32_t tau0 = 0;
        for (int bit = 31; bit >= 0; --bit) {
            const uint32_t probe = tau0 | ((1u << bit) - 1u);  // this bit 0, all lower bits 1
            uint32_t cnt = (uint32_t)__popcll(__ballot(lmin <= probe));
            if constexpr (TWO) cnt += (uint32_t)__popcll(__ballot(lmin2 <= probe));
            if (cnt < want) tau0 |= 1u << bit;
        }
        const unsigned long long below = (1ull << lane) - 1ull;
        // the key indices recomputed from an opaque base: otherwise the compiler
        // keeps the R load-time indices live across the threshold search
        int lb = R > 0 ? 4 * lane : lane;
        asm volatile("" : "+v"(lb));
        uint32_t c = 0;
#pragma unroll
        for (int i = 0; i < NI; ++i) {
            const int j = R > 0 ? 256 * (i >> 2) + lb + (i & 3) : lb + 64 * i;
            const uint32_t u = K(i);
            const bool q = j < N && u <= tau0;
            const unsigned long long m = __ballot(q);
            if (m) {
                if (q) {
                    const uint32_t pos = c + __popcll(m & below);
                    if (pos < KNN_FASTCAP) {
                        fkeyb[wave][pos] = u;
                        fidxb[wave][pos] = j;
                    }
                }
                c += __popcll(m);
            }
        }
        if (bitonic && c <= 64) {  // wave-uniform
            // the c <= 64 candidates sorted by (key, index) across the wave (a
            // 21-stage bitonic network of lane-pair exchanges): lane r then holds
            // rank r, the same order the compare ranking below computes
            __builtin_amdgcn_wave_barrier();
            uint32_t kk = lane < (int)c ? fkeyb[wave][lane] : 0xffffffffu;
            int ii = lane < (int)c ? fidxb[wave][lane] : 0x7fffffff;
#pragma unroll
            for (int size = 2; size <= 64; size <<= 1)
#pragma unroll
                for (int stride = size >> 1; stride > 0; stride >>= 1) {
                    const uint32_t ok = (uint32_t)__shfl_xor((int)kk, stride);
                    const int oi = __shfl_xor(ii, stride);
                    const bool other_less = (ok < kk) | ((ok == kk) & (oi < ii));
                    // the lower lane of an ascending pair (or the upper of a descending one) keeps the smaller
                    const bool keep_small = ((lane & stride) == 0) == ((lane & size) == 0);
                    if (keep_small == other_less) {
                        kk = ok;
                        ii = oi;
                    }
                }
            int *out = knn + ((size_t)b * Sstr + s) * k;
            if (lane > 0 && lane < (int)want && lane < (int)c) out[lane - 1] = ii;  // drop position 0 (:68)
            KNN_COUNT(0, 1);
            return;
        }
        if (c <= KNN_FASTCAP) {
            __builtin_amdgcn_wave_barrier();
            const int e0 = lane, e1 = lane + 64;
            const uint32_t k0 = e0 < (int)c ? fkeyb[wave][e0] : 0xffffffffu;
            const int i0 = e0 < (int)c ? fidxb[wave][e0] : 0x7fffffff;
            const uint32_t k1 = e1 < (int)c ? fkeyb[wave][e1] : 0xffffffffu;
            const int i1 = e1 < (int)c ? fidxb[wave][e1] : 0x7fffffff;
            // ranks by (key, index): candidate m broadcast from lane m % 64 by
            // v_readlane (no LDS round trip per candidate)
            uint32_t r0 = 0, r1 = 0;
            for (int m = 0; m < min((int)c, 64); ++m) {
                const uint32_t mu = __builtin_amdgcn_readlane(k0, m);
                const int mi = __builtin_amdgcn_readlane(i0, m);
                r0 += (mu < k0) || (mu == k0 && mi < i0);
                r1 += (mu < k1) || (mu == k1 && mi < i1);
            }
            for (int m = 64; m < (int)c; ++m) {
                const uint32_t mu = __builtin_amdgcn_readlane(k1, m - 64);
                const int mi = __builtin_amdgcn_readlane(i1, m - 64);
                r0 += (mu < k0) || (mu == k0 && mi < i0);
                r1 += (mu < k1) || (mu == k1 && mi < i1);
            }
            int *out = knn + ((size_t)b * Sstr + s) * k;
            if (e0 < (int)c && r0 > 0 && r0 < want) out[r0 - 1] = i0;  // drop position 0 (:68)
            if (e1 < (int)c && r1 > 0 && r1 < want) out[r1 - 1] = i1;
            KNN_COUNT(1, 1);
            return;
        }
    }
    KNN_COUNT(2, 1);
    if constexpr (R > 0) {
        // Radix fallback on the row held in registers (r06: the memory form below
        // re-reads the row from L2 in every histogram pass, one dependent load per
        // atomic; the single N = 5000 pair's clustered rows took 90 us in it).
        // Lane l holds keys 256 b + 4 l + e (block b = i / 4, e = i % 4, ~0u past N):
        // counting passes do not care about order, and the collection pass ranks
        // a block's keys in index order from its four ballots.  The same selection
        // as the memory form, so the same kNN rows.
        uint32_t kmin = 0xffffffffu, kmax = 0u;
#pragma unroll
        for (int i = 0; i < R; ++i) {
            const bool valid = 256 * (i >> 2) + 4 * lane + (i & 3) < N;
            if (valid) {
                kmin = min(kmin, key[i]);
                kmax = max(kmax, key[i]);
            }
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            kmin = min(kmin, (uint32_t)__shfl_xor((int)kmin, o));
            kmax = max(kmax, (uint32_t)__shfl_xor((int)kmax, o));
        }
        uint32_t *hb = hist[wave];
        uint32_t need = want, prefix = kmin, mask = 0xffffffffu, bin_cnt = want;
        bool small_bin = false;
        if (kmin != kmax) {
            const int top = 31 - __clz((int)(kmin ^ kmax));
            mask = top == 31 ? 0u : ~((2u << top) - 1u);
            prefix = kmin & mask;
            for (int hi = top; hi >= 0; hi -= 8) {
                const int lo = max(hi - 7, 0);
                const uint32_t dm = (2u << (hi - lo)) - 1u;
                KNN_COUNT(3, 1);
#pragma unroll
                for (int e = 0; e < 4; ++e) hb[lane + 64 * e] = 0;
                __builtin_amdgcn_wave_barrier();
#pragma unroll
                for (int i = 0; i < R; ++i) {
                    const uint32_t u = key[i];
                    if (256 * (i >> 2) + 4 * lane + (i & 3) < N && (u & mask) == prefix)
                        atomicAdd(&hb[(u >> lo) & dm], 1u);
                    if ((i & 3) == 3) __builtin_amdgcn_sched_barrier(0);
                }
                __builtin_amdgcn_wave_barrier();
                uint32_t c[4], tot = 0;
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    c[e] = hb[4 * lane + e];
                    tot += c[e];
                }
                uint32_t incl = tot;
#pragma unroll
                for (int o = 1; o < 64; o <<= 1) {
                    const uint32_t y = __shfl_up(incl, o);
                    if (lane >= o) incl += y;
                }
                const uint32_t base = incl - tot;
                uint32_t my_bin = 0, my_need = 0, my_cnt = 0;
                const bool hit = base < need && need <= incl;
                if (hit) {
                    uint32_t cum = base;
                    bool done = false;
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        if (!done && cum + c[e] >= need) {
                            my_bin = 4 * lane + e;
                            my_need = need - cum;
                            my_cnt = c[e];
                            done = true;
                        }
                        cum += c[e];
                    }
                }
                const int src_lane = __ffsll((unsigned long long)__ballot(hit)) - 1;
                const uint32_t bin = __shfl(my_bin, src_lane);
                const uint32_t cnt = __shfl(my_cnt, src_lane);
                need = __shfl(my_need, src_lane);
                prefix |= bin << lo;
                mask |= dm << lo;
                bin_cnt = cnt;
                if (cnt == need) break;
                if (cnt <= KNN_BINCAP) {
                    small_bin = true;
                    break;
                }
            }
        }
        const uint32_t nless = want - need;
        const unsigned long long below = (1ull << lane) - 1ull;
        uint32_t pl = 0, pe = 0;
#pragma unroll
        for (int i4 = 0; i4 < R / 4; ++i4) {
            bool less[4], eq[4];
            unsigned long long lm[4], em[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const uint32_t u = key[4 * i4 + e], um = u & mask;
                const bool valid = 256 * i4 + 4 * lane + e < N;
                less[e] = valid && um < prefix;
                eq[e] = valid && um == prefix;
                lm[e] = __ballot(less[e]);
                em[e] = __ballot(eq[e]);
            }
            // index-order rank inside the block: every key of the lanes below, then
            // this lane's keys before e
            uint32_t lb = 0, eb = 0;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                lb += __popcll(lm[e] & below);
                eb += __popcll(em[e] & below);
            }
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int j = 256 * i4 + 4 * lane + e;
                const uint32_t u = key[4 * i4 + e];
                if (less[e]) {
                    const uint32_t pos = pl + lb;
                    if (pos < want) {
                        ckey[wave][pos] = u;
                        cidx[wave][pos] = j;
                    }
                }
                if (eq[e]) {
                    const uint32_t r = pe + eb;
                    if (small_bin) {
                        bkey[wave][r] = u;
                        bidx[wave][r] = j;
                    } else if (r < need) {
                        ckey[wave][nless + r] = u;
                        cidx[wave][nless + r] = j;
                    }
                }
                lb += less[e];
                eb += eq[e];
            }
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                pl += __popcll(lm[e]);
                pe += __popcll(em[e]);
            }
            __builtin_amdgcn_sched_barrier(0);  // one block's ballots live at a time
        }
        __builtin_amdgcn_wave_barrier();
        if (small_bin) KNN_COUNT(4, 1);
        if (small_bin) {
            for (int e = lane; e < (int)bin_cnt; e += 64) {
                const uint32_t ku = bkey[wave][e];
                const int ki = bidx[wave][e];
                uint32_t rank = 0;
                for (int m = 0; m < (int)bin_cnt; ++m) {
                    const uint32_t mu = bkey[wave][m];
                    rank += (mu < ku) || (mu == ku && bidx[wave][m] < ki);
                }
                if (rank < need) {
                    ckey[wave][nless + rank] = ku;
                    cidx[wave][nless + rank] = ki;
                }
            }
            __builtin_amdgcn_wave_barrier();
        }
        if (lane < (int)want) {
            const uint32_t ku = ckey[wave][lane];
            const int ki = cidx[wave][lane];
            int rank = 0;
            for (int m = 0; m < (int)want; ++m) {
                const uint32_t mu = ckey[wave][m];
                rank += (mu < ku) || (mu == ku && cidx[wave][m] < ki);
            }
            if (rank > 0) knn[((size_t)b * Sstr + s) * k + rank - 1] = ki;  // drop position 0 (:68)
        }
        return;
    }
    // Radix fallback, keys re-read from memory (lane l owns keys l + 64 i, so a
    // ballot over lanes visits keys in index order).
    const int NI = (N + 63) / 64;
    auto K = [&](int i) -> uint32_t {
        const int j = lane + 64 * i;
        return j < N ? row[j] : 0xffffffffu;
    };
    uint32_t kmin = 0xffffffffu, kmax = 0u;
    for (int i = 0; i < NI; ++i) {
        if (lane + 64 * i < N) {
            const uint32_t u = K(i);
            kmin = min(kmin, u);
            kmax = max(kmax, u);
        }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        kmin = min(kmin, (uint32_t)__shfl_xor((int)kmin, o));
        kmax = max(kmax, (uint32_t)__shfl_xor((int)kmax, o));
    }
    uint32_t *hb = hist[wave];
    uint32_t need = want, prefix = kmin, mask = 0xffffffffu, bin_cnt = want;
    bool small_bin = false;  // the bin holding the (k+1)-th key has <= KNN_BINCAP keys: rank them directly
    if (kmin != kmax) {
        const int top = 31 - __clz((int)(kmin ^ kmax));  // highest differing bit
        mask = top == 31 ? 0u : ~((2u << top) - 1u);
        prefix = kmin & mask;
        for (int hi = top; hi >= 0; hi -= 8) {
            const int lo = max(hi - 7, 0);
            const uint32_t dm = (2u << (hi - lo)) - 1u;  // digit = bits [lo, hi]
            KNN_COUNT(3, 1);
#pragma unroll
            for (int e = 0; e < 4; ++e) hb[lane + 64 * e] = 0;
            __builtin_amdgcn_wave_barrier();
            for (int i = 0; i < NI; ++i) {
                const uint32_t u = K(i);
                if (lane + 64 * i < N && (u & mask) == prefix) atomicAdd(&hb[(u >> lo) & dm], 1u);
            }
            __builtin_amdgcn_wave_barrier();
            uint32_t c[4], tot = 0;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                c[e] = hb[4 * lane + e];
                tot += c[e];
            }
            uint32_t incl = tot;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const uint32_t y = __shfl_up(incl, o);
                if (lane >= o) incl += y;
            }
            const uint32_t base = incl - tot;
            uint32_t my_bin = 0, my_need = 0, my_cnt = 0;
            const bool hit = base < need && need <= incl;
            if (hit) {
                uint32_t cum = base;
                bool done = false;
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    if (!done && cum + c[e] >= need) {
                        my_bin = 4 * lane + e;
                        my_need = need - cum;
                        my_cnt = c[e];
                        done = true;
                    }
                    cum += c[e];
                }
            }
            const int src_lane = __ffsll((unsigned long long)__ballot(hit)) - 1;
            const uint32_t bin = __shfl(my_bin, src_lane);
            const uint32_t cnt = __shfl(my_cnt, src_lane);
            need = __shfl(my_need, src_lane);
            prefix |= bin << lo;
            mask |= dm << lo;
            bin_cnt = cnt;
            if (cnt == need) break;  // the whole bin is taken: no need to resolve further
            if (cnt <= KNN_BINCAP) {
                small_bin = true;
                break;
            }
        }
    }
    // take every key with (u & mask) < prefix and the first `need` keys with (u & mask) == prefix
    const uint32_t nless = want - need;
    const unsigned long long below = (1ull << lane) - 1ull;
    uint32_t pl = 0, pe = 0;
    for (int i = 0; i < NI; ++i) {
        const int j = lane + 64 * i;
        const uint32_t u = K(i);
        const uint32_t um = u & mask;
        const bool valid = j < N;
        const bool less = valid && um < prefix, eq = valid && um == prefix;
        const unsigned long long lm = __ballot(less), em = __ballot(eq);
        if (less) {
            const uint32_t pos = pl + __popcll(lm & below);
            if (pos < want) {
                ckey[wave][pos] = u;
                cidx[wave][pos] = j;
            }
        }
        if (eq) {
            const uint32_t r = pe + __popcll(em & below);
            if (small_bin) {  // every key of the bin, ranked below
                bkey[wave][r] = u;
                bidx[wave][r] = j;
            } else if (r < need) {
                ckey[wave][nless + r] = u;
                cidx[wave][nless + r] = j;
            }
        }
        pl += __popcll(lm);
        pe += __popcll(em);
    }
    __builtin_amdgcn_wave_barrier();
    if (small_bin) KNN_COUNT(4, 1);
    if (small_bin) {  // the `need` smallest (key, index) of the bin's bin_cnt keys
        for (int e = lane; e < (int)bin_cnt; e += 64) {
            const uint32_t ku = bkey[wave][e];
            const int ki = bidx[wave][e];
            uint32_t rank = 0;
            for (int m = 0; m < (int)bin_cnt; ++m) {
                const uint32_t mu = bkey[wave][m];
                rank += (mu < ku) || (mu == ku && bidx[wave][m] < ki);
            }
            if (rank < need) {
                ckey[wave][nless + rank] = ku;
                cidx[wave][nless + rank] = ki;
            }
        }
        __builtin_amdgcn_wave_barrier();
    }
    if (lane < (int)want) {
        const uint32_t ku = ckey[wave][lane];
        const int ki = cidx[wave][lane];
        int rank = 0;
        for (int m = 0; m < (int)want; ++m) {
            const uint32_t mu = ckey[wave][m];
            rank += (mu < ku) || (mu == ku && cidx[wave][m] < ki);
        }
        if (rank > 0) knn[((size_t)b * Sstr + s) * k + rank - 1] = ki;  // drop position 0 (:68)
    }
}

// Waves (= seeds) per workgroup of the one-wave-per-seed kernels (knn_select,
// nsm_seed, kabsch_sums; none has a workgroup barrier): 4, unless that leaves
// fewer than 2 workgroups per CU (a single N = 5000 pair has 500 seeds = 125
// four-wave workgroups for 256 CUs), then 1 so the seeds spread over all CUs.
static int seed_wpb(int B, int S) {
    static const int force = [] {  // A/B knob PDSC_SEED_WPB=1|2|4 (measurement only)
        const char *e = getenv("PDSC_SEED_WPB");
        const int w = e ? atoi(e) : 0;
        return (w == 1 || w == 2 || w == 4) ? w : 0;
    }();
    if (force) return force;
    return (long)B * ((S + 3) / 4) < 512 ? 1 : 4;
}

hipError_t launch_knn_select(const float *dist, int B, int N, int S, int k, int *knn, hipStream_t s,
                             Ragged rg) {
    const int wpb = seed_wpb(B, S);
    const dim3 grid((S + wpb - 1) / wpb, B), block(64 * wpb);
    const int R = (N + 63) / 64;
    // the fast path's <= 64 candidates ranked by a wave bitonic sort (128 x 1000:
    // 36.5 vs 40.1 us per launch; 8 x 5000 and one pair equal); A/B knob
    // PDSC_KNN_BITONIC=0: the readlane compare ranking (measurement only)
    static const int bit = [] {
        const char *e = getenv("PDSC_KNN_BITONIC");
        return e ? atoi(e) : 1;
    }();
    if (R <= 16)
        hipLaunchKernelGGL(knn_select_kernel<16>, grid, block, 0, s, dist, N, S, k, knn, rg, bit);
    else if (R <= 32)
        hipLaunchKernelGGL(knn_select_kernel<32>, grid, block, 0, s, dist, N, S, k, knn, rg, bit);
    else if (R <= 48)
        hipLaunchKernelGGL(knn_select_kernel<48>, grid, block, 0, s, dist, N, S, k, knn, rg, bit);
    else if (R <= 64)
        hipLaunchKernelGGL(knn_select_kernel<64>, grid, block, 0, s, dist, N, S, k, knn, rg, bit);
    else if (R <= 80)
        hipLaunchKernelGGL(knn_select_kernel<80>, grid, block, 0, s, dist, N, S, k, knn, rg, bit);
    else if (R <= 96)
        hipLaunchKernelGGL(knn_select_kernel<96>, grid, block, 0, s, dist, N, S, k, knn, rg, bit);
    else if (R <= 128)
        hipLaunchKernelGGL(knn_select_kernel<128>, grid, block, 0, s, dist, N, S, k, knn, rg, bit);
    else
        hipLaunchKernelGGL(knn_select_kernel<0>, grid, block, 0, s, dist, N, S, k, knn, rg, bit);
    return hipGetLastError();
}

// -------------------------------------------------------------- a7-a8 NSM
constexpr int KMAX = 64;

// Power iteration of one seed's k x k matrix (models/PointDSC.py:347-358), one
// wave: lane a holds row a of T in registers, v is broadcast from LDS 4 entries
// at a time.  hist[t][a] = iterate t+1; returns bit t = allclose(v_{t+1}, v_t).
// KC: k rounded up to a multiple of 16 (columns past k are zero, their FMAs
// exact no-ops), so k = 40 runs 48-long rows instead of KMAX = 64.
// T's rows in LDS: stride tstride (a multiple of 4), columns k .. KC-1 zero, so
// every row is KC / 4 unconditional 16-B reads (rows past k read as zero rows).
template <int KC>
PDSC_DEV unsigned power_iterate(const float *trow_lds, int tstride, int k, int T, float *vbuf, float *hb, int a) {
    float trow[KC];
    const float *tr = trow_lds + min(a, k - 1) * tstride;
#pragma unroll
    for (int c = 0; c < KC; c += 4) {
        const f32x4 t4 = *reinterpret_cast<const f32x4 *>(tr + c);
#pragma unroll
        for (int e = 0; e < 4; ++e) trow[c + e] = a < k ? t4[e] : 0.0f;
    }
    vbuf[a] = 1.0f;
    float v = (a < k) ? 1.0f : 0.0f;
    unsigned flags = 0;
    __builtin_amdgcn_wave_barrier();
    for (int t = 0; t < T; ++t) {
        // four partial sums as two packed pairs: v_pk_fma_f32, two lanes' worth of
        // fma per instruction, the same arithmetic per component
        f32x2 acc01 = {0.0f, 0.0f}, acc23 = {0.0f, 0.0f};
#pragma unroll
        for (int c = 0; c < KC; c += 4) {
            const f32x4 vv = *reinterpret_cast<const f32x4 *>(&vbuf[c]);
            acc01 = __builtin_elementwise_fma(f32x2{trow[c], trow[c + 1]}, f32x2{vv[0], vv[1]}, acc01);
            acc23 = __builtin_elementwise_fma(f32x2{trow[c + 2], trow[c + 3]}, f32x2{vv[2], vv[3]}, acc23);
        }
        float nv = (acc01[0] + acc01[1]) + (acc23[0] + acc23[1]);   // (T v)_a  (bmm, :352)
        // no LDS round trip per iterate; every lane holds the same sum, so the
        // square root branches wave-uniformly: the fma-corrected cr_sqrt (the
        // same correctly rounded value) where it is exact, sqrtf below 2^-96
#if NSM_PK_TBUILD
        const float ss = __builtin_bit_cast(
            float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, wave_sum_dpp(nv * nv))));
        const float nrm = ss >= 0x1p-96f ? cr_sqrt(ss) : sqrtf(ss);
#else
        const float nrm = sqrtf(wave_sum_dpp(nv * nv));
#endif
        nv = nv / (nrm + 1e-6f);                              // :353
        const bool close = (a >= k) || (fabsf(nv - v) <= 1e-8f + 1e-5f * fabsf(v));  // allclose (:354)
        if (__all(close)) flags |= 1u << t;
        if (a < k) hb[(size_t)t * k + a] = nv;
        v = nv;
        __builtin_amdgcn_wave_barrier();
        vbuf[a] = nv;
        __builtin_amdgcn_wave_barrier();
    }
    return flags;
}

// nsm_seed_kernel: one WAVE per (seed, pair), 4 seeds per workgroup.  The
// k x k feature Gram matrix of the seed's neighbourhood comes from the fp16
// matrix cores with the 3-product split (attention_h3.hpp), its operands read
// straight from the split normed copy ns [B][N][2][128] (the same bytes the
// seed kNN reads) into registers: tiles (0,0), (0,1), (1,1) of 32 x 32 for
// k <= 64.  T = F o S (diag 0, :257-278) goes to the wave's slice of LDS, each
// unordered pair evaluated once and mirrored (T exactly symmetric), then the
// same wave runs the power iteration.  No workgroup barriers: waves are
// independent.
constexpr int NSM_PSTR = 8;  // floats per neighbour in the LDS coordinate table
// cr_sqrt / cr_div (pdsc_common.hpp) on two lanes' worth of operands: the
// fma corrections as v_pk_fma_f32, the same operations per component.
PDSC_DEV f32x2 cr_sqrt2(f32x2 x) {
    const f32x2 s = {__builtin_amdgcn_sqrtf(x[0]), __builtin_amdgcn_sqrtf(x[1])};
    const f32x2 dn = {__uint_as_float(__float_as_uint(s[0]) - 1u), __uint_as_float(__float_as_uint(s[1]) - 1u)};
    const f32x2 up = {__uint_as_float(__float_as_uint(s[0]) + 1u), __uint_as_float(__float_as_uint(s[1]) + 1u)};
    const f32x2 rdn = __builtin_elementwise_fma(-dn, s, x), rup = __builtin_elementwise_fma(-up, s, x);
    f32x2 r;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        float v = rdn[i] <= 0.0f ? dn[i] : s[i];
        v = rup[i] > 0.0f ? up[i] : v;
        r[i] = x[i] == 0.0f ? x[i] : v;
    }
    return r;
}
PDSC_DEV f32x2 cr_div2(f32x2 x, f32x2 d, f32x2 rcp) {
    const f32x2 q = x * rcp;
    const f32x2 r = __builtin_elementwise_fma(-q, d, x);
    return __builtin_elementwise_fma(r, rcp, q);
}
// LDS row stride of T for KC-padded rows: 16-B aligned, 13 (KC + 4) / 4 mod 16
// distinct 16-B banks groups over 16 consecutive rows (conflict-free ds_read_b128)
__host__ __device__ constexpr int nsm_tstride(int kc) { return kc + 4; }
// The unordered pairs a < c < KMAX in c-major order (pair p = c (c - 1) / 2 + a,
// packed a | c << 8): the first k (k - 1) / 2 entries are exactly the pairs of
// a k-neighbourhood, for every k -- one table load per pair instead of a
// square-root index decode.
struct NsmPairs {
    unsigned short v[KMAX * (KMAX - 1) / 2];
};
constexpr NsmPairs make_nsm_pairs() {
    NsmPairs t{};
    int p = 0;
    for (int c = 1; c < KMAX; ++c)
        for (int a = 0; a < c; ++a) t.v[p++] = (unsigned short)(a | (c << 8));
    return t;
}
static __constant__ const NsmPairs g_nsm_pairs = make_nsm_pairs();

#ifdef ATT_STAMPS
// Diagnostic build: stamps of 64 evenly spaced workgroups' waves (tools/nsm_stamps.py).
PDSC_DEV unsigned long long *nsm_stamp_ptr(int wave) {
    const int wg = blockIdx.y * gridDim.x + blockIdx.x, str = max(1, (int)(gridDim.x * gridDim.y) / ST_WGS);
    return (wg % str == 0 && wg / str < ST_WGS && wave < 4) ? g_att_stamps + ((wg / str) * 4 + wave) * ST_PER_WAVE
                                                            : nullptr;
}
#define NSM_STAMP(i) ATT_STAMP(nstp, i)
#else
#define NSM_STAMP(i) \
    do {             \
    } while (0)
#endif

// F32 (PDSC_PRECISION_F32): the Gram tiles on exact fp32 MFMA from the fp32
// normed rows (`feats` = normed [B][N][128]); H3: `feats` = the split copy.
template <bool F32, int KC>
__global__ __launch_bounds__(256, 4) void nsm_seed_kernel(const void *__restrict__ feats,
                                                       const float *__restrict__ src,
                                                       const float *__restrict__ tgt,
                                                       const int *__restrict__ knn, int N, int S, int k, int T,
                                                       const float *__restrict__ sigma_p,
                                                       const float *__restrict__ sigma_d_p,
                                                       float *__restrict__ hist, unsigned *__restrict__ seed_flags,
                                                       Ragged rg) {
    extern __shared__ __attribute__((aligned(16))) float nsm_sdyn[];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, h = lane >> 5, l32 = lane & 31;
    const int b = blockIdx.y, s = blockIdx.x * (blockDim.x >> 6) + wave;
    if (s >= rg.s(b, S)) return;  // wave-uniform (a ragged pair's own seed count; S, N: the strides)
#ifdef ATT_STAMPS
    unsigned long long *nstp = nsm_stamp_ptr(wave);
    ATT_RSTAMP(nstp, 16);
    NSM_STAMP(0);
#endif
    const int tls = nsm_tstride(KC);
    float *Tl = nsm_sdyn + (size_t)wave * (k * tls + k * NSM_PSTR + 64);
    float *P = Tl + k * tls;  // [k][NSM_PSTR]: src xyz, tgt xyz
    float *vb = P + k * NSM_PSTR;
    const float sig = sigma_p[0], sd = sigma_d_p[0];
    const float sig2 = sig * sig, sd2 = sd * sd;
    const float rsig2 = 1.0f / sig2, rsd2 = 1.0f / sd2;
    const int *kr = knn + ((size_t)b * S + s) * k;
    const int idx = min(max(kr[lane < k ? lane : 0], 0), N - 1);
    NSM_STAMP(1);
    // the neighbour's coordinates: loaded now (every lane's idx is a valid row),
    // written to LDS once the Gram gathers are in flight, so the two gathers'
    // latencies overlap
    const float *ps = src + ((size_t)b * N + idx) * 3, *pt = tgt + ((size_t)b * N + idx) * 3;
    const float p0 = ps[0], p1 = ps[1], p2 = ps[2], p3 = pt[0], p4 = pt[1], p5 = pt[2];
    auto store_p = [&] {
        if (lane < k) {
#if NSM_PK_TBUILD
            // (src, tgt) interleaved per axis: the T build's packed fp32 pairs
            *reinterpret_cast<f32x4 *>(P + lane * NSM_PSTR) = f32x4{p0, p3, p1, p4};
            *reinterpret_cast<f32x4 *>(P + lane * NSM_PSTR + 4) = f32x4{p2, p5, 0.0f, 0.0f};
#else
            *reinterpret_cast<f32x4 *>(P + lane * NSM_PSTR) = f32x4{p0, p1, p2, p3};
            *reinterpret_cast<f32x4 *>(P + lane * NSM_PSTR + 4) = f32x4{p4, p5, 0.0f, 0.0f};
#endif
        }
        NSM_STAMP(2);
    };
    // Gram operands streamed one 16-input k-step at a time (16 VGPRs in
    // flight instead of both whole 32-row fragments): the wave fits in 128
    // VGPRs, 4 waves per SIMD to hide the row gathers.  Accumulation order per
    // tile is unchanged (k-steps ascending).
    const int nt = (k + 31) / 32;
    f32x16 G00 = zero16(), G01 = zero16(), G11 = zero16();
    if constexpr (F32) {
        store_p();
        const float *F = static_cast<const float *>(feats) + (size_t)b * N * CH;
        const float *r0 = F + (size_t)__shfl(idx, l32) * CH + 4 * h;
        const float *r1 = F + (size_t)__shfl(idx, 32 + l32) * CH + 4 * h;
#pragma unroll 4
        for (int j = 0; j < CH / 8; ++j) {
            const f32x4 av = *reinterpret_cast<const f32x4 *>(r0 + 8 * j);
#pragma unroll
            for (int e = 0; e < 4; ++e) G00 = mfma32(av[e], av[e], G00);
            if (nt > 1) {
                const f32x4 bv = *reinterpret_cast<const f32x4 *>(r1 + 8 * j);
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    G01 = mfma32(av[e], bv[e], G01);
                    G11 = mfma32(bv[e], bv[e], G11);
                }
            }
        }
    } else {
        // rows past k are never read back (the T triangle takes a < c < k): their
        // lanes point outside the buffer resource, so those loads return zero
        // without a gather (k = 40: 40 of 64 rows).  Branch-free buffer loads:
        // every k-step's fragments can be in flight together (exec-masked loads
        // in branches were issued one k-step at a time, 16 serial gathers).
        const __amdgpu_buffer_rsrc_t rF =
            h3_rsrc(static_cast<const _Float16 *>(feats) + (size_t)b * N * 2 * CH, (uint32_t)N * 4u * CH);
        const uint32_t oob = 0x80000000u;
        const uint32_t o0 = l32 < k ? (uint32_t)__shfl(idx, l32) * 4u * CH + 16u * h : oob;
        const uint32_t o1 = 32 + l32 < k ? (uint32_t)__shfl(idx, 32 + l32) * 4u * CH + 16u * h : oob;
        auto ld = [&](uint32_t o, int off) {
            return __builtin_bit_cast(f16x8, __builtin_amdgcn_raw_buffer_load_b128(rF, o, (uint32_t)off, 0));
        };
        // k-step j's four fragments are issued NSM_GLA steps ahead of its MFMAs
        // (the empty asm keeps the scheduler from sinking them to their uses)
        constexpr int NSM_GLA = 3;
        f16x8 fr[8][4];
        auto issue = [&](int j) {
            fr[j][0] = ld(o0, 32 * j);
            fr[j][1] = ld(o0, 2 * CH + 32 * j);
            if (nt > 1) {
                fr[j][2] = ld(o1, 32 * j);
                fr[j][3] = ld(o1, 2 * CH + 32 * j);
            }
        };
#pragma unroll
        for (int j = 0; j < NSM_GLA; ++j) issue(j);
        store_p();
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            if (j + NSM_GLA < 8) issue(j + NSM_GLA);
            asm volatile("" ::: "memory");
            G00 = mfma_h3(fr[j][0], fr[j][1], fr[j][0], fr[j][1], G00);
            if (nt > 1) {
                G01 = mfma_h3(fr[j][0], fr[j][1], fr[j][2], fr[j][3], G01);
                G11 = mfma_h3(fr[j][2], fr[j][3], fr[j][2], fr[j][3], G11);
            }
        }
    }
    // The Gram tiles' strict upper triangle (a < c < k) to LDS, then T = F o S
    // evaluated once per unordered pair with the pairs dealt evenly over the
    // 64 lanes (triangular index p -> (a, c)): ceil(k(k-1)/128) passes instead
    // of 16 per Gram tile with most lanes masked off.  Each pair is read and
    // overwritten in place by the one lane that owns it, then mirrored.
    auto gstore = [&](const f32x16 &G, int ta, int tb) {
        const int c = 32 * tb + l32;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int a = 32 * ta + acc_row(r, h);
            if (a < c && c < k) Tl[a * tls + c] = G[r];
        }
    };
    gstore(G00, 0, 0);
    if (nt > 1) {
        gstore(G01, 0, 1);
        gstore(G11, 1, 1);
    }
    NSM_STAMP(3);
    if (lane < k) Tl[lane * tls + lane] = 0.0f;  // diag 0 (:278)
    for (int a0 = 0; a0 < k; a0 += 4) {  // pad columns k .. KC-1 (KC - k < 16): 4 rows x 16 columns per pass
        const int a = a0 + (lane >> 4), c = k + (lane & 15);
        if (a < k && c < KC) Tl[a * tls + c] = 0.0f;
    }
    __builtin_amdgcn_wave_barrier();  // P and the Gram triangle visible to the wave
    const int npair = k * (k - 1) / 2;
    // the pair table entry of the next pass is loaded one pass ahead (a global
    // load per pass otherwise exposes its whole latency, 13 passes at k = 40)
    unsigned pc_next = g_nsm_pairs.v[min(lane, npair - 1)];
    for (int p = lane; p < npair; p += 64) {
        const unsigned pc = pc_next;
        pc_next = g_nsm_pairs.v[min(p + 64, npair - 1)];
        const int a = (int)(pc & 255u), c = (int)(pc >> 8);
        const float g = Tl[a * tls + c];
        const f32x4 pa0 = *reinterpret_cast<const f32x4 *>(P + a * NSM_PSTR);
        const f32x4 pa1 = *reinterpret_cast<const f32x4 *>(P + a * NSM_PSTR + 4);
        const f32x4 pc0 = *reinterpret_cast<const f32x4 *>(P + c * NSM_PSTR);
        const f32x4 pc1 = *reinterpret_cast<const f32x4 *>(P + c * NSM_PSTR + 4);
        // correctly rounded '/' and sqrtf through their fma-corrected forms
        // (pdsc_common.hpp; exact for normal operands, within 1 ulp below 2^-96).
        // (r04: the hardware square root and a reciprocal multiply in the H3 build,
        // -22 VALU per pair, flipped one borderline pair of the recall-parity
        // proxy -- test_recall_parity_synthetic -- so both modes keep these.)
#if NSM_PK_TBUILD
        // the source and target halves as packed fp32 pairs (v_pk_add / mul /
        // fma_f32): per component the same operations in the same order as the
        // scalar form below, so the same bits
        const f32x2 dx = f32x2{pa0[0], pa0[1]} - f32x2{pc0[0], pc0[1]};
        const f32x2 dy = f32x2{pa0[2], pa0[3]} - f32x2{pc0[2], pc0[3]};
        const f32x2 dz = f32x2{pa1[0], pa1[1]} - f32x2{pc1[0], pc1[1]};
        const f32x2 d2 = (dx * dx + dy * dy) + dz * dz;                       // :268 (src, tgt)
        const f32x2 st = cr_sqrt2(d2);
        const float dd = st[0] - st[1];
        // (1 - g) / sigma^2 and dd^2 / sigma_d^2 as one packed correctly rounded division
        const f32x2 qd = cr_div2(f32x2{1.0f - g, dd * dd}, f32x2{sig2, sd2}, f32x2{rsig2, rsd2});
        const f32x2 om = f32x2{1.0f, 1.0f} - qd;
        const float val = fmaxf(om[0], 0.0f) * fmaxf(om[1], 0.0f);            // :259, :270, :277
#else
        const float fm = fmaxf(1.0f - cr_div(1.0f - g, sig2, rsig2), 0.0f);  // :259
        float dx = pa0[0] - pc0[0], dy = pa0[1] - pc0[1], dz = pa0[2] - pc0[2];
        const float ds = cr_sqrt((dx * dx + dy * dy) + dz * dz);    // :268
        dx = pa0[3] - pc0[3];
        dy = pa1[0] - pc1[0];
        dz = pa1[1] - pc1[1];
        const float dt = cr_sqrt((dx * dx + dy * dy) + dz * dz);
        const float dd = ds - dt;
        const float sm = fmaxf(1.0f - cr_div(dd * dd, sd2, rsd2), 0.0f);     // :270
        const float val = fm * sm;                                            // :277
#endif
        Tl[a * tls + c] = val;
        Tl[c * tls + a] = val;
    }
    __builtin_amdgcn_wave_barrier();
    NSM_STAMP(4);
    const unsigned flags = power_iterate<KC>(Tl, tls, k, T, vb, hist + ((size_t)b * S + s) * T * k, lane);
    NSM_STAMP(5);
#ifdef ATT_STAMPS
    ATT_RSTAMP(nstp, 17);
#endif
    // this seed's allclose bits; nsm_finish ANDs a pair's seeds (a per-pair
    // atomicAnd here serialised S atomics per address: 30-60 us of the launch)
    if (lane == 0) seed_flags[(size_t)b * S + s] = flags;
}

size_t nsm_seed_lds_bytes(int k, int wpb) {
    const int kc = (k + 15) / 16 * 16;
    return (size_t)wpb * (k * nsm_tstride(kc) + k * NSM_PSTR + 64) * sizeof(float);
}

hipError_t launch_nsm_seed(const void *feats, bool f32, const float *src, const float *tgt, const int *knn, int B,
                           int N, int S, int k, int T, const float *sigma, const float *sigma_d, float *hist,
                           unsigned *seed_flags, hipStream_t s, Ragged rg) {
    if (k < 1 || k > KMAX) return hipErrorInvalidValue;
    const int wpb = seed_wpb(B, S);
    const dim3 grid((S + wpb - 1) / wpb, B), block(64 * wpb);
    const size_t lds = nsm_seed_lds_bytes(k, wpb);
#define NSM_LAUNCH(F, KC)                                                                                     \
    hipLaunchKernelGGL((nsm_seed_kernel<F, KC>), grid, block, lds, s, feats, src, tgt, knn, N, S, k, T, sigma, \
                       sigma_d, hist, seed_flags, rg)
    const int kc = (k + 15) / 16;
    if (f32) {
        if (kc == 1) NSM_LAUNCH(true, 16); else if (kc == 2) NSM_LAUNCH(true, 32);
        else if (kc == 3) NSM_LAUNCH(true, 48); else NSM_LAUNCH(true, 64);
    } else {
        if (kc == 1) NSM_LAUNCH(false, 16); else if (kc == 2) NSM_LAUNCH(false, 32);
        else if (kc == 3) NSM_LAUNCH(false, 48); else NSM_LAUNCH(false, 64);
    }
#undef NSM_LAUNCH
    return hipGetLastError();
}

// w = v_{t*} / (sum v_{t*} + 1e-6)  (models/PointDSC.py:280-282)
// The first iterate t* (1-based; T when none) at which every one of the nq
// seeds' allclose bits from q0 on is set: torch.allclose over the iterate the
// reference compares at once (:354).  Wave-uniform.
PDSC_DEV int nsm_tstar(const unsigned *__restrict__ seed_flags, size_t q0, size_t nq, int T, int lane) {
    unsigned all = 0xffffffffu;
    if (T > 0)
        for (size_t q = lane; q < nq; q += 64) all &= seed_flags[q0 + q];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) all &= (unsigned)__shfl_xor((int)all, o);
    const unsigned m = all & ((T >= 32) ? 0xffffffffu : ((1u << T) - 1u));
    return m ? (__ffs(m)) : T;
}
// This lane's normalised weight of seed row `row` (= b * S + s) from its
// iterate t* (lanes >= k: 0).
PDSC_DEV float nsm_weight(const float *__restrict__ hist, size_t row, int tstar, int k, int T, int lane) {
    float v = 1.0f;
    if (tstar > 0 && lane < k) v = hist[(row * T + (tstar - 1)) * k + lane];
    if (lane >= k) v = 0.0f;
    const float sum = wave_sum(v);
    return lane < k ? v / (sum + 1e-6f) : 0.0f;
}

__global__ __launch_bounds__(64) void nsm_finish_kernel(const float *__restrict__ hist,
                                                        const unsigned *__restrict__ seed_flags, int S,
                                                        int k, int T, int batch_global, float *__restrict__ weights,
                                                        int *__restrict__ iters_used, Ragged rg) {
    const int b = blockIdx.y, s = blockIdx.x, a = threadIdx.x;
    const int Sb = rg.s(b, S);  // this pair's seeds (a ragged batch); S: the stride
    if (s >= Sb) return;
    // the allclose bits ANDed over the seeds torch.allclose sees at once (:354):
    // the pair's S seeds (a bs = 1 testing forward) or, batch_global, all
    // gridDim.y * S seeds of the call (the training forward's [bs * S, k] iterate)
    // (ragged batches run per pair: pdsc_forward_testing_ragged is B bs = 1 forwards)
    const size_t q0 = batch_global ? 0 : (size_t)b * S, nq = batch_global ? (size_t)gridDim.y * S : (size_t)Sb;
    const int tstar = nsm_tstar(seed_flags, q0, nq, T, a);  // 1-based iterate index
    const float w = nsm_weight(hist, (size_t)b * S + s, tstar, k, T, a);
    if (a < k) weights[((size_t)b * S + s) * k + a] = w;
    if (s == 0 && a == 0 && iters_used) iters_used[b] = tstar;
}

hipError_t launch_nsm_finish(const float *hist, const unsigned *seed_flags, int B, int S, int k, int T,
                             bool batch_global, float *weights, int *iters_used, hipStream_t s, Ragged rg) {
    if (batch_global && rg.sv) return hipErrorInvalidValue;
    hipLaunchKernelGGL(nsm_finish_kernel, dim3(S, B), dim3(64), 0, s, hist, seed_flags, S, k, T, (int)batch_global,
                       weights, iters_used, rg);
    return hipGetLastError();
}

// ------------------------------------------------------------ a9 Kabsch
// Hypotheses (models/PointDSC.py:287-328) in three SIMD-friendly steps:
//  1. kabsch_sums   one wave per seed: weighted centroids and H (wave reductions)
//  2. kabsch_solve  one LANE per seed: fp64 3x3 rotation + t (64 solves per wave)
//  3. count_inliers one workgroup per HS seeds: every correspondence's residual
//                   under all HS hypotheses (src/tgt read once per HS seeds)
constexpr int HSUM = 15;  // H[9], cA[3], cB[3]
constexpr int HS = 8;     // seeds per count_inliers workgroup

PDSC_DEV void kabsch_finish(const float H[9], const float cA[3], const float cB[3], float *T);

// for (n = tid; n < N; n += NT) body(n, src row n, tgt row n) with RU rows'
// loads issued together: the pair's rows come from L2, and a loop that loads
// and consumes one row per trip waits a full round trip per row (r06 stamps of
// best_refine at N = 5000: 6.7 us per pass of 20 rows per thread).  body runs
// in the same n order, so sums accumulate in the same order: the same bits.
// A/B build knob: -DROWS_RU=1 consumes each row as it is loaded (measurement only)
#ifndef ROWS_RU
#define ROWS_RU 8
#endif
template <int NT, int RU = ROWS_RU, typename F>
PDSC_DEV void for_rows(const float *__restrict__ sb, const float *__restrict__ tb, int N, int tid, F body) {
    for (int n0 = tid; n0 < N; n0 += RU * NT) {
        float a[RU][3], c[RU][3];
#pragma unroll
        for (int u = 0; u < RU; ++u) {
            const int n = min(n0 + u * NT, N - 1);  // (clamped: an in-range row, not consumed)
#pragma unroll
            for (int e = 0; e < 3; ++e) {
                a[u][e] = sb[3 * n + e];
                c[u][e] = tb[3 * n + e];
            }
        }
#pragma unroll
        for (int u = 0; u < RU; ++u)
            if (n0 + u * NT < N) body(n0 + u * NT, a[u], c[u]);
    }
}

// SOLVE (small batches, kabsch_small): lane 0 of the seed's wave also finishes
// the Kabsch solve (kabsch_finish on the same 15 sums kabsch_solve_kernel would
// read back: the same bits) and writes trans -- one launch instead of two.
// FIN (the testing forward): the seed's NSM weights are finished here, as
// nsm_finish_kernel computes them (nsm_tstar over the pair's seeds, nsm_weight;
// the same bits), and written to `weights` -- one launch fewer per forward.
// COUNT (with SOLVE, small batches): the seed's wave then counts the inliers of
// its own hypothesis over the pair's correspondences (count_inliers_kernel's
// test, residual_sq < tau2, the same integer) -- one launch fewer.
template <bool SOLVE, bool FIN = false, bool COUNT = false>
__global__ __launch_bounds__(256) void kabsch_sums_kernel(const float *__restrict__ src,
                                                          const float *__restrict__ tgt,
                                                          const int *__restrict__ knn,
                                                          const float *__restrict__ weights, int N,
                                                          int S, int k, float *__restrict__ sums, Ragged rg,
                                                          float *__restrict__ trans, const float *__restrict__ hist = nullptr,
                                                          const unsigned *__restrict__ seed_flags = nullptr, int T = 0,
                                                          float *__restrict__ wout = nullptr, float tau2 = 0.0f,
                                                          int *__restrict__ counts = nullptr) {
    const int b = blockIdx.y, lane = threadIdx.x & 63;
    const int s = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    const int Sb = rg.s(b, S);
    if (s >= Sb) return;  // (N, S: the strides; knn entries lie below this pair's count)
    const float *sb = src + (size_t)b * N * 3, *tb = tgt + (size_t)b * N * 3;
    float w = 0, ax = 0, ay = 0, az = 0, bx = 0, by = 0, bz = 0;
    float wf = 0.0f;
    if constexpr (FIN) {
        const int tstar = nsm_tstar(seed_flags, (size_t)b * S, (size_t)Sb, T, lane);
        wf = nsm_weight(hist, (size_t)b * S + s, tstar, k, T, lane);
        if (lane < k) wout[((size_t)b * S + s) * k + lane] = wf;
    }
    if (lane < k) {
        const int j = min(max(knn[((size_t)b * S + s) * k + lane], 0), N - 1);
        w = FIN ? wf : weights[((size_t)b * S + s) * k + lane];
        ax = sb[3 * j];
        ay = sb[3 * j + 1];
        az = sb[3 * j + 2];
        bx = tb[3 * j];
        by = tb[3 * j + 1];
        bz = tb[3 * j + 2];
    }
    // centroid = sum(A * w) / (sum(w) + 1e-6)  (models/common.py:24-25)
    const float den = wave_sum(w) + 1e-6f;
    const float cA0 = wave_sum(ax * w) / den, cA1 = wave_sum(ay * w) / den, cA2 = wave_sum(az * w) / den;
    const float cB0 = wave_sum(bx * w) / den, cB1 = wave_sum(by * w) / den, cB2 = wave_sum(bz * w) / den;
    const float am[3] = {ax - cA0, ay - cA1, az - cA2};
    const float bm[3] = {bx - cB0, by - cB1, bz - cB2};
    float out = 0.0f;  // lane e < 15 keeps sums[e]
    float Hs[9];       // (every lane holds every wave sum)
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int jj = 0; jj < 3; ++jj) {
            const float h = wave_sum((am[i] * w) * bm[jj]);  // H = Am^T diag(w) Bm (:33)
            Hs[3 * i + jj] = h;
            if (lane == 3 * i + jj) out = h;
        }
    if constexpr (SOLVE) {
        float T[16];
        if (lane == 0) {
            const float cA[3] = {cA0, cA1, cA2}, cB[3] = {cB0, cB1, cB2};
            kabsch_finish(Hs, cA, cB, T);
#pragma unroll
            for (int e = 0; e < 16; ++e) trans[((size_t)b * S + s) * 16 + e] = T[e];
        }
        if constexpr (COUNT) {
            // lane 0's pose to every lane, then the pair's correspondences 64 at a time
            float Tb[12];
#pragma unroll
            for (int e = 0; e < 12; ++e) Tb[e] = __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, T[e])));
            const int n = rg.n(b, N);
            int c = 0;
            for_rows<64>(sb, tb, n, lane, [&](int, const float (&p)[3], const float (&q)[3]) {
                c += residual_sq(Tb, p[0], p[1], p[2], q[0], q[1], q[2]) < tau2;  // L2 < tau (:327-328)
            });
            c = wave_sum(c);
            if (lane == 0) counts[(size_t)b * S + s] = c;
        }
        return;
    }
    if (lane == 9) out = cA0;
    if (lane == 10) out = cA1;
    if (lane == 11) out = cA2;
    if (lane == 12) out = cB0;
    if (lane == 13) out = cB1;
    if (lane == 14) out = cB2;
    if (lane < HSUM) sums[((size_t)b * S + s) * HSUM + lane] = out;
}

// Finish a weighted Kabsch from its sums: t = c_B - R c_A in fp32 as
// models/common.py:42 computes it; T row-major 4x4.
PDSC_DEV void kabsch_finish(const float H[9], const float cA[3], const float cB[3], float *T) {
    double Hd[9], Rd[9];
#pragma unroll
    for (int i = 0; i < 9; ++i) Hd[i] = H[i];
    kabsch_rotation(Hd, Rd);
    float R[9];
#pragma unroll
    for (int i = 0; i < 9; ++i) R[i] = (float)Rd[i];
#pragma unroll
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

__global__ __launch_bounds__(64) void kabsch_solve_kernel(const float *__restrict__ sums, int n, int S,
                                                          float *__restrict__ trans, Ragged rg) {
    const int i = blockIdx.x * 64 + threadIdx.x;
    if (i >= n || i % S >= rg.s(i / S, S)) return;  // (a ragged pair's seeds end early)
    const float *p = sums + (size_t)i * HSUM;
    float H[9], cA[3], cB[3], T[16];
#pragma unroll
    for (int e = 0; e < 9; ++e) H[e] = p[e];
#pragma unroll
    for (int e = 0; e < 3; ++e) {
        cA[e] = p[9 + e];
        cB[e] = p[12 + e];
    }
    kabsch_finish(H, cA, cB, T);
#pragma unroll
    for (int e = 0; e < 16; ++e) trans[(size_t)i * 16 + e] = T[e];
}

__global__ __launch_bounds__(256) void count_inliers_kernel(const float *__restrict__ src,
                                                            const float *__restrict__ tgt,
                                                            const float *__restrict__ seed_trans,
                                                            int Nstr, int S, float tau2,
                                                            int *__restrict__ counts, Ragged rg) {
    __shared__ float Ts[HS][12];
    __shared__ int wc[4][HS];
    const int b = blockIdx.y, s0 = blockIdx.x * HS, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int N = rg.n(b, Nstr);  // this pair's correspondences; Nstr, S: the strides
    if (s0 >= rg.s(b, S)) return;  // workgroup-uniform
    const int ns = min(HS, rg.s(b, S) - s0);
    if (tid < HS * 12) {
        const int q = tid / 12, e = tid % 12;
        Ts[q][e] = (q < ns) ? seed_trans[((size_t)b * S + s0 + q) * 16 + e] : 0.0f;
    }
    __syncthreads();
    const float *sb = src + (size_t)b * Nstr * 3, *tb = tgt + (size_t)b * Nstr * 3;
    int c[HS];
#pragma unroll
    for (int q = 0; q < HS; ++q) c[q] = 0;
    for (int n = tid; n < N; n += 256) {
        const float x = sb[3 * n], y = sb[3 * n + 1], z = sb[3 * n + 2];
        const float tx = tb[3 * n], ty = tb[3 * n + 1], tz = tb[3 * n + 2];
#pragma unroll
        for (int q = 0; q < HS; ++q) c[q] += residual_sq(Ts[q], x, y, z, tx, ty, tz) < tau2;  // L2 < tau (:327-328)
    }
#pragma unroll
    for (int q = 0; q < HS; ++q) {
        const int v = wave_sum(c[q]);
        if (lane == 0) wc[wave][q] = v;
    }
    __syncthreads();
    if (tid < ns) counts[(size_t)b * S + s0 + tid] = wc[0][tid] + wc[1][tid] + wc[2][tid] + wc[3][tid];
}

// One solve per seed wave (kabsch_sums_kernel<true>) while the batch has at
// most 1024 seeds (a single pair: 100); past that the solve kernel's 64 seeds
// per wave keep the fp64 work off a lane-per-wave schedule.  A/B knob
// PDSC_KABSCH_FUSED=0 (measurement only; the same bits either way).
static bool kabsch_small(int n) {
    static const bool off = [] {
        const char *e = getenv("PDSC_KABSCH_FUSED");
        return e && e[0] == '0';
    }();
    return !off && n <= 1024;
}

hipError_t launch_hypotheses(const float *src, const float *tgt, const int *knn, const float *weights,
                             int B, int N, int S, int k, float tau, float *seed_trans, int *counts,
                             float *sums, hipStream_t s, Ragged rg, const float *hist, const unsigned *seed_flags,
                             int T, float *wout) {
    const int wpb = seed_wpb(B, S);
    const int n = B * S;
    const dim3 grid((S + wpb - 1) / wpb, B), block(64 * wpb);
    const bool fin = hist != nullptr;
    const float tau2 = sqrt_ge_threshold(tau);
    if (kabsch_small(n)) {
        // the inlier count in the same launch (count_inliers_kernel's integers)
        if (fin)
            hipLaunchKernelGGL((kabsch_sums_kernel<true, true, true>), grid, block, 0, s, src, tgt, knn, weights, N, S,
                               k, sums, rg, seed_trans, hist, seed_flags, T, wout, tau2, counts);
        else
            hipLaunchKernelGGL((kabsch_sums_kernel<true, false, true>), grid, block, 0, s, src, tgt, knn, weights, N, S,
                               k, sums, rg, seed_trans, nullptr, nullptr, 0, nullptr, tau2, counts);
        return hipGetLastError();
    } else {
        if (fin)
            hipLaunchKernelGGL((kabsch_sums_kernel<false, true>), grid, block, 0, s, src, tgt, knn, weights, N, S, k,
                               sums, rg, seed_trans, hist, seed_flags, T, wout);
        else
            hipLaunchKernelGGL((kabsch_sums_kernel<false>), grid, block, 0, s, src, tgt, knn, weights, N, S, k, sums,
                               rg, seed_trans, nullptr, nullptr, 0, nullptr);
        hipLaunchKernelGGL(kabsch_solve_kernel, dim3((n + 63) / 64), dim3(64), 0, s, sums, n, S, seed_trans, rg);
    }
    hipLaunchKernelGGL(count_inliers_kernel, dim3((S + HS - 1) / HS, B), dim3(256), 0, s, src, tgt,
                       seed_trans, N, S, tau2, counts, rg);
    return hipGetLastError();
}

// ------------------------------------------------------------- a10 best
// One 256-thread workgroup per pair: the range guard, the first argmax of the
// inlier counts, the best hypothesis into Ts (LDS) and trans, its labels.
// Returns false for a pair the range guard flagged (workgroup-uniform).
PDSC_DEV bool select_best_wg(const float *__restrict__ src, const float *__restrict__ tgt,
                             const float *__restrict__ seed_trans, const int *__restrict__ counts, int Nstr, int Sstr,
                             float tau, float *__restrict__ fitness, int *__restrict__ best_out,
                             float *__restrict__ trans, float *__restrict__ labels, const Ragged &rg,
                             const float *__restrict__ conf, int *__restrict__ range, int *wbest, int *wcnt, float *Ts) {
    const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int N = rg.n(b, Nstr), S = rg.s(b, Sstr);  // this pair's sizes; Nstr, Sstr: the strides
    if (conf) {
        // the fp16 range guard (pdsc.h, PDSC_ERR_RANGE): an activation that left
        // fp16's range in a 3xfp16 contraction turns into NaN (inf hi, -inf lo),
        // which the encoder's NaN-propagating ReLUs carry into every logit
        int bad = 0;
        const float *cb = conf + (size_t)b * Nstr;
        for (int n0 = tid; n0 < N; n0 += 8 * 256) {  // 8 loads in flight per thread
            float v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) v[u] = cb[min(n0 + 256 * u, N - 1)];
#pragma unroll
            for (int u = 0; u < 8; ++u) bad |= !__builtin_isfinite(v[u]);
        }
        bad = __syncthreads_or(bad);
        if (range && tid == 0) range[b] = bad;
        if (bad) {
            if (tid < 16) trans[(size_t)b * 16 + tid] = __builtin_nanf("");
            for (int n = tid; n < Nstr; n += 256) labels[(size_t)b * Nstr + n] = 0.0f;
            return false;  // workgroup-uniform
        }
    }
    int bc = -1, bi = 0x7fffffff;
    for (int s = tid; s < S; s += 256) {
        const int c = counts[(size_t)b * Sstr + s];
        if (fitness) fitness[(size_t)b * Sstr + s] = (float)c / (float)N;  // torch.mean of 0/1
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
        Ts[tid] = seed_trans[((size_t)b * Sstr + best) * 16 + tid];
        trans[(size_t)b * 16 + tid] = Ts[tid];
    }
    __syncthreads();
    float T[12];
#pragma unroll
    for (int e = 0; e < 12; ++e) T[e] = Ts[e];
    const float *sb = src + (size_t)b * Nstr * 3, *tb = tgt + (size_t)b * Nstr * 3;
    for_rows<256>(sb, tb, N, tid, [&](int n, const float (&a)[3], const float (&c)[3]) {
        const float L2 = residual(T, a[0], a[1], a[2], c[0], c[1], c[2]);
        labels[(size_t)b * Nstr + n] = (L2 < tau) ? 1.0f : 0.0f;
    });
    for (int n = N + tid; n < Nstr; n += 256) labels[(size_t)b * Nstr + n] = 0.0f;  // a ragged pair's padding
    return true;
}

__global__ __launch_bounds__(256) void select_best_kernel(const float *__restrict__ src,
                                                          const float *__restrict__ tgt,
                                                          const float *__restrict__ seed_trans,
                                                          const int *__restrict__ counts, int Nstr, int Sstr,
                                                          float tau, float *__restrict__ fitness,
                                                          int *__restrict__ best_out,
                                                          float *__restrict__ trans,
                                                          float *__restrict__ labels, Ragged rg,
                                                          const float *__restrict__ conf, int *__restrict__ range) {
    __shared__ int wbest[4], wcnt[4];
    __shared__ float Ts[16];
    select_best_wg(src, tgt, seed_trans, counts, Nstr, Sstr, tau, fitness, best_out, trans, labels, rg, conf, range,
                   wbest, wcnt, Ts);
}

hipError_t launch_select_best(const float *src, const float *tgt, const float *seed_trans,
                              const int *counts, int B, int N, int S, float tau, float *fitness,
                              int *best, float *trans, float *labels, hipStream_t s, Ragged rg, const float *conf,
                              int *range) {
    hipLaunchKernelGGL(select_best_kernel, dim3(B), dim3(256), 0, s, src, tgt, seed_trans, counts, N, S,
                       tau, fitness, best, trans, labels, rg, conf, range);
    return hipGetLastError();
}

// --------------------------------------------------- block-wide Kabsch
constexpr int RB = 256;  // threads per refinement / rigid workgroup (register room for the fp64 SVD)
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

template <typename WF>
PDSC_DEV void block_rigid_h(const float *__restrict__ A, const float *__restrict__ Bp, int n, WF wfun,
                            const float (&s7)[7], float *Tout, float (*red)[9], int tid);

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
    block_rigid_h(A, Bp, n, wfun, s7, Tout, red, tid);
}

// block_rigid's second half: the centroids from the block-summed weight and
// weighted coordinate sums s7 = (sum w, sum w A, sum w B), then H and the solve.
template <typename WF>
PDSC_DEV void block_rigid_h(const float *__restrict__ A, const float *__restrict__ Bp, int n, WF wfun,
                            const float (&s7)[7], float *Tout, float (*red)[9], int tid) {
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
// Diagnostic build only (-DATT_STAMPS, tools/refine_stamps.py): pair 0's
// workgroup stamps s_memrealtime into the stamp buffer's last wave slot at the
// refinement's phase ends (BR_ST(i): 0 start, 1 select done, 2 + 3 it + {0, 1,
// 2}: iteration it's count pass, H pass, solve; 98 the iterations run, 99 end).
#ifdef ATT_STAMPS
#define BR_ST(i)                                                                                         \
    do {                                                                                                 \
        if (blockIdx.x == 0 && threadIdx.x == 0 && (i) < ST_PER_WAVE)                                   \
            g_att_stamps[(ST_WGS * 4 - 1) * ST_PER_WAVE + (i)] = __builtin_amdgcn_s_memrealtime();        \
    } while (0)
#else
#define BR_ST(i) \
    do {         \
    } while (0)
#endif
// The refinement of pair blockIdx.x from the pose in Ts (LDS, every thread's
// view current), written to trans[b] at the end.
PDSC_DEV void post_refine_wg(float *Ts, float *__restrict__ trans, const float *__restrict__ src,
                             const float *__restrict__ tgt, int Nstr, float thr, const Ragged &rg, float (*red)[9]) {
    const int b = blockIdx.x, tid = threadIdx.x;
    const int N = rg.n(b, Nstr);  // this pair's correspondences; Nstr: the stride
    const float *sb = src + (size_t)b * Nstr * 3, *tb = tgt + (size_t)b * Nstr * 3;
    int prev = 0;
    for (int it = 0; it < 20; ++it) {
        float T[12];
#pragma unroll
        for (int e = 0; e < 12; ++e) T[e] = Ts[e];
        auto weight = [&](const float (&pa)[3], const float (&pb)[3]) -> float {
            const float L2 = residual(T, pa[0], pa[1], pa[2], pb[0], pb[1], pb[2]);
            const float r = L2 / thr;
            const float wv = 1.0f / (1.0f + r * r);  // 1/(1 + (L2/thr)^2) (:435)
            return L2 < thr ? wv : 0.0f;
        };
        // one pass: the inlier count (:423-426) and block_rigid's weighted sums of
        // the same T (the next iterate's weights), in block_rigid's order
        float c8[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        for_rows<RB>(sb, tb, N, tid, [&](int, const float (&pa)[3], const float (&pb)[3]) {
            const float ax = pa[0], ay = pa[1], az = pa[2];
            const float bx = pb[0], by = pb[1], bz = pb[2];
            const float L2 = residual(T, ax, ay, az, bx, by, bz);
            // branch-free (the weight evaluated for every row, kept where L2 < thr):
            // the rows of a trip are independent chains the scheduler interleaves
            const bool in = L2 < thr;
            const float r = L2 / thr;
            const float wv = 1.0f / (1.0f + r * r);
            const float w = in ? wv : 0.0f;
            c8[7] += in ? 1.0f : 0.0f;
            c8[0] += w;
            c8[1] += ax * w;
            c8[2] += ay * w;
            c8[3] += az * w;
            c8[4] += bx * w;
            c8[5] += by * w;
            c8[6] += bz * w;
        });
        block_sum<8>(c8, reinterpret_cast<float (*)[8]>(red), tid);
        BR_ST(2 + 3 * it);
#ifdef ATT_STAMPS
        if (blockIdx.x == 0 && tid == 0) g_att_stamps[(ST_WGS * 4 - 1) * ST_PER_WAVE + 98] = it + 1;
#endif
        const int cnt = (int)c8[7];
        if (cnt == prev) break;  // abs(int(inlier_num - previous_inlier_num)) < 1 (:426)
        prev = cnt;
        const float s7[7] = {c8[0], c8[1], c8[2], c8[3], c8[4], c8[5], c8[6]};
        float Tn[16];
        {   // block_rigid_h(sb, tb, N, wfun, s7, Tn, red, tid) with the rows loaded RU at a time
            const float den = s7[0] + 1e-6f;
            const float cA[3] = {s7[1] / den, s7[2] / den, s7[3] / den};
            const float cB[3] = {s7[4] / den, s7[5] / den, s7[6] / den};
            float H[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
            for_rows<RB>(sb, tb, N, tid, [&](int, const float (&pa)[3], const float (&pb)[3]) {
                // a zero weight adds (am 0) bm = +-0 to H, which leaves it as skipping the
                // row did (H starts at +0 and x + -0 = x, +0 + -0 = +0): branch-free
                const float w = weight(pa, pb);
                const float am[3] = {pa[0] - cA[0], pa[1] - cA[1], pa[2] - cA[2]};
                const float bm[3] = {pb[0] - cB[0], pb[1] - cB[1], pb[2] - cB[2]};
#pragma unroll
                for (int r = 0; r < 3; ++r)
#pragma unroll
                    for (int c = 0; c < 3; ++c) H[3 * r + c] += (am[r] * w) * bm[c];
            });
            block_sum<9>(H, red, tid);
            BR_ST(3 + 3 * it);
            if (tid == 0) kabsch_finish(H, cA, cB, Tn);
            __syncthreads();
        }
        if (tid == 0)
            for (int e = 0; e < 16; ++e) Ts[e] = Tn[e];
        __syncthreads();
        BR_ST(4 + 3 * it);
    }
    BR_ST(99);
    if (tid < 16) trans[(size_t)b * 16 + tid] = Ts[tid];
}

__global__ __launch_bounds__(RB) void post_refine_kernel(float *__restrict__ trans,
                                                         const float *__restrict__ src,
                                                         const float *__restrict__ tgt, int Nstr,
                                                         float thr, Ragged rg, const int *__restrict__ range) {
    __shared__ float red[RW][9];
    __shared__ float Ts[16];
    const int b = blockIdx.x, tid = threadIdx.x;
    if (range && range[b]) return;  // a pair the range guard flagged keeps its NaN pose (workgroup-uniform)
    if (tid < 16) Ts[tid] = trans[(size_t)b * 16 + tid];
    __syncthreads();
    post_refine_wg(Ts, trans, src, tgt, Nstr, thr, rg, red);
}

// select_best + post_refine of one pair in one launch (the testing forward):
// the same two workgroup bodies back to back, the best pose handed over in LDS.
static_assert(RB == 256, "select_best_wg runs 256 threads");
__global__ __launch_bounds__(RB) void best_refine_kernel(const float *__restrict__ src, const float *__restrict__ tgt,
                                                         const float *__restrict__ seed_trans,
                                                         const int *__restrict__ counts, int Nstr, int Sstr,
                                                         float tau, float thr, float *__restrict__ trans,
                                                         float *__restrict__ labels, Ragged rg,
                                                         const float *__restrict__ conf, int *__restrict__ range) {
    __shared__ int wbest[4], wcnt[4];
    __shared__ float Ts[16];
    __shared__ float red[RW][9];
    BR_ST(0);
    if (!select_best_wg(src, tgt, seed_trans, counts, Nstr, Sstr, tau, nullptr, nullptr, trans, labels, rg, conf, range,
                        wbest, wcnt, Ts))
        return;  // (workgroup-uniform) the range guard's NaN pose stays
    BR_ST(1);
    post_refine_wg(Ts, trans, src, tgt, Nstr, thr, rg, red);
}

hipError_t launch_best_refine(const float *src, const float *tgt, const float *seed_trans, const int *counts, int B,
                              int N, int S, float tau, float thr, float *trans, float *labels, hipStream_t s,
                              Ragged rg, const float *conf, int *range) {
    hipLaunchKernelGGL(best_refine_kernel, dim3(B), dim3(RB), 0, s, src, tgt, seed_trans, counts, N, S, tau, thr, trans,
                       labels, rg, conf, range);
    return hipGetLastError();
}

hipError_t launch_post_refine(float *trans, const float *src, const float *tgt, int B, int N, float thr,
                              hipStream_t s, Ragged rg, const int *range) {
    hipLaunchKernelGGL(post_refine_kernel, dim3(B), dim3(RB), 0, s, trans, src, tgt, N, thr, rg, range);
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

#ifdef ATT_STAMPS
extern "C" int pdsc_diag_nsm_stamps(void *host, size_t bytes) {
    const size_t n = std::min(bytes, sizeof(g_att_stamps));
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_att_stamps), n, 0, hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}
extern "C" int pdsc_diag_nsm_stamps_clear() {
    static unsigned long long zero[ST_WGS * 4 * ST_PER_WAVE];
    return hipMemcpyToSymbol(HIP_SYMBOL(g_att_stamps), zero, sizeof(zero), 0, hipMemcpyHostToDevice) == hipSuccess ? 0
                                                                                                             : -1;
}
#endif

}  // namespace pdsc
