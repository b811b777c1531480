// pdsc_internal.hpp -- launchers and packed-weight layout shared by the
// translation units of libpdsc (not part of the C ABI).
#pragma once
#include <string>
#include "pdsc_common.hpp"
#include "../../include/pdsc.h"

namespace pdsc {

constexpr int CH = 128;       // num_channels implemented by the MFMA kernels
constexpr int CH2 = CH / 2;   // fc_message hidden width (models/PointDSC.py:12-20)
constexpr int CLS = 32;       // classifier hidden width (models/PointDSC.py:107-113)
constexpr int QB = 128;       // queries per attention workgroup (4 waves x 32)
constexpr int KT = 32;        // keys per attention tile
constexpr int PT = 64;        // points per pointwise workgroup

inline int round_up(int x, int m) { return (x + m - 1) / m * m; }

// ---- symmetric-packed M (the forward's a1 output) -------------------------
// M is symmetric bit-for-bit, so the forward stores only its upper-triangle
// MPACK_T x MPACK_T tiles, each contiguous and row-major, enumerated row by
// row: tile (ti, tj), ti <= tj, at index ti*nt - ti*(ti-1)/2 + (tj - ti),
// nt = ceil(N / MPACK_T).  M[i][j] for i > j lives transposed in tile (tj, ti).
constexpr int MPACK_T = 32;  // = the attention's per-wave 32 keys x 32 queries block
__host__ __device__ inline int mpack_ntile(int N) { return (N + MPACK_T - 1) / MPACK_T; }
__host__ __device__ inline size_t mpack_floats(int N) {
    const size_t nt = mpack_ntile(N);
    return nt * (nt + 1) / 2 * MPACK_T * MPACK_T;
}
__host__ __device__ inline int mpack_tile(int ti, int tj, int nt) { return ti * nt - ti * (ti - 1) / 2 + (tj - ti); }
inline size_t align_bytes(size_t x) { return (x + 255) & ~size_t(255); }

// fp16 planes per packed 1x1-conv weight (3xfp16 mode): 2 = hi + mid (22
// significant bits, products wh.xh + wh.xl + wm.xh: 3 MFMAs, as the attention's);
// 3 = hi + mid + lo (every fp32 weight exactly, 4 MFMAs; the r01-r03 format,
// kept as a build option for A/B: -DPDSC_W_PLANES=3).  r04 measured both on the
// goldens (tools/emulate_conv.py): the same error class, inside the fp32
// realisations' noise.
#ifndef PDSC_W_PLANES
#define PDSC_W_PLANES 2
#endif
constexpr int W_PLANES = PDSC_W_PLANES;
static_assert(W_PLANES == 2 || W_PLANES == 3, "weight planes");

// Weight blocks: block (t, ks) = 32 outputs x one 16-input k-step, planes
// hi / mid (/ lo) of 64 lanes x 8 halfs (1 KiB) each, blocks t-major.
// Element (o, c) of plane p sits at w3_index(o, c, in) + 512 p (halfs), with
// lane (h, n), n = o % 32, holding positions 8h .. 8h+7 of the k-step in
// qk_pos order (bits 2 and 3 of c % 16 swapped).
constexpr int W3_BLOCK = W_PLANES * 512;  // halfs per block
__host__ __device__ inline size_t w3_index(int o, int c, int in) {
    const int t = o >> 5, n = o & 31, ks = c >> 4, q = c & 15;
    const int pos = (q & ~12) | ((q & 4) << 1) | ((q & 8) >> 1);
    return ((size_t)t * (in / 16) + ks) * W3_BLOCK + (size_t)(32 * (pos >> 3) + n) * 8 + (pos & 7);
}

// ---- packed weights --------------------------------------------------------
// A "dense" layer (Conv1d k=1 [+BN] [+ReLU]) is stored as
//   W  : OUT*IN floats in MFMA fragment order:
//        Wpk[((jt*(IN/8) + g)*64 + lane)*4 + e] = W[jt*32 + (lane&31)][(lane>>5)*(IN/2) + 4g + e]
//   bias[OUT], alpha[OUT], beta[OUT]   (alpha=1, beta=0 when no BN)
// A dense layer in the packed blob: W as W_PLANES fp16 planes (hi, mid[, lo] of
// W * 2^s, s chosen per layer so max|W| 2^s <= 2^14) in MFMA-fragment blocks
// (w3_index) occupying W_PLANES/2*out*in floats at w (at least out*in) -- or, for
// PDSC_PRECISION_F32, W itself fp32 [out][in] in the first out*in of them --
// then bias, alpha, beta [out] and scale = {2^-s, 2^s}.
struct DenseOff {
    size_t w, bias, alpha, beta, scale;
};

struct LayerOff {
    DenseOff pcn, fc0, fc3, fc6, q, k, v;
};

struct PackLayout {
    int L, in_dim;
    size_t sigma, sigma_d;    // header scalars
    size_t l0_w, l0_b;        // layer0 plain [CH][in_dim], bias[CH]
    size_t cls0, cls2;        // DenseOff base of the two classifier dense layers
    DenseOff c0, c2;
    size_t c4_w, c4_b;        // plain [CLS], [1]
    size_t total;
    LayerOff layer[64];
};

inline DenseOff dense_at(size_t &o, int in, int out) {
    DenseOff d;
    d.w = o;
    o += (size_t)out * in * (W_PLANES > 2 ? W_PLANES : 2) / 2;
    d.bias = o;
    o += out;
    d.alpha = o;
    o += out;
    d.beta = o;
    o += out;
    o = (o + 3) & ~size_t(3);
    d.scale = o;
    o += 4;
    return d;
}

inline PackLayout make_layout(int L, int in_dim) {
    PackLayout p{};
    p.L = L;
    p.in_dim = in_dim;
    size_t o = 0;
    p.sigma = 0;
    p.sigma_d = 1;
    o = 16;
    p.l0_w = o;
    o += (size_t)CH * in_dim;
    p.l0_b = o;
    o += CH;
    o = (o + 3) & ~size_t(3);
    for (int l = 0; l < L; ++l) {
        LayerOff &lo = p.layer[l];
        lo.pcn = dense_at(o, CH, CH);
        lo.fc0 = dense_at(o, CH, CH2);
        lo.fc3 = dense_at(o, CH2, CH2);
        lo.fc6 = dense_at(o, CH2, CH);
        lo.q = dense_at(o, CH, CH);
        lo.k = dense_at(o, CH, CH);
        lo.v = dense_at(o, CH, CH);
    }
    p.c0 = dense_at(o, CH, CLS);
    p.c2 = dense_at(o, CLS, CLS);
    p.c4_w = o;
    o += CLS;
    p.c4_b = o;
    o += 4;
    p.total = o;
    return p;
}

// ---- ragged batches (pdsc_forward_testing_ragged) ----------------------------
// Every pair's buffers keep the batch stride N (the largest pair); pair b uses
// its first nv[b] rows and has sv[b] = int(nv[b] * ratio) seeds (S = the
// largest).  nv == sv == nullptr: a uniform batch (every pair N rows, S seeds).
extern thread_local int g_diag_qkv_delay;  // api.hip: pdsc_diag_qkv_delay (tests only)
struct Ragged {
    const int *nv = nullptr, *sv = nullptr;
    // the attention's pair order (longest pairs first, dealt over the XCDs), or null
    const int *po = nullptr;
    // every count equals the padded N (host-known): the attention takes the
    // uniform batch's form (stream-K on the w64 plan), so such a call is bitwise
    // the uniform entry's (same key partition, same fp32 combine order)
    bool eq = false;
    PDSC_DEV int n(int b, int N) const { return nv ? nv[b] : N; }
    PDSC_DEV int s(int b, int S) const { return sv ? sv[b] : S; }
};
constexpr int RAGGED_CHUNK = 512;  // counts per setup launch (kernel-argument array)
// counts (HOST, already validated) -> nv [B], sv [B] on the device, through
// kernel arguments (no host-to-device copy of pageable memory on the stream)
hipError_t launch_ragged_setup(const int32_t *counts_host, int B, double ratio, int *nv, int *sv, hipStream_t s);
// counts (HOST) -> po [B]: attention workgroup slot -> pair, so the workgroups
// of the largest pairs start first (each XCD's slots in decreasing pair size,
// pairs dealt to the XCD with the least N^2 so far): list scheduling of
// workgroups of unequal length, longest first
hipError_t launch_ragged_order(const int32_t *counts_host, int B, int *po, hipStream_t s);

// ---- launchers --------------------------------------------------------------
hipError_t launch_compat(const float *src, const float *tgt, int B, int N, const float *sigma_d,
                         float *M, hipStream_t s, Ragged rg = {});
// Mp: [B][mpack_floats(N)]
hipError_t launch_compat_packed(const float *src, const float *tgt, int B, int N, const float *sigma_d,
                                float *Mp, hipStream_t s, Ragged rg = {});

hipError_t launch_pack_dense(const float *w, const float *b, const float *bn_w, const float *bn_b,
                             const float *bn_rm, const float *bn_rv, int in, int out, bool f32, float *dst_w,
                             float *dst_b, float *dst_a, float *dst_beta, float *dst_scale, hipStream_t s);
hipError_t launch_copy(const float *src, float *dst, int n, hipStream_t s);

// Attention partials for one layer: opart [B][nsplit][Npad x CH], ml [B][nsplit][Npad][2];
// opart rows [Npad][CH] for f32, the fragment-block tiling of attention_h3.hpp
// (h3_opart_off) for H3.
// the split path's attention as attention_w64 (64-query waves) for this shape?
bool attention_w64(int B, int N, bool f32);
int attention_nsplit(int B, int N, bool f32, bool w64 = false);
// M's layouts: dense [B][N][N], symmetric-packed (mpack_*)
enum MLayout { M_DENSE = 0, M_PACKED = 1 };
// q, k, v: the fp16 hi/lo split layouts of attention_h3.hpp (4 B per element),
// or fp32 [B][Npad][CH] rows when f32 (exact-fp32 MFMA, attention.hpp).
// M: dense [B][N][N] or symmetric-packed [B][mpack_floats(N)] (H3), per m_layout.
// vexp: [B][Npad/32] V-tile exponents of the H3 layout (attention_h3.hpp); unused for f32.
// w64: attention_w64 (H3 and packed M only, nsplit from attention_nsplit(.., w64 = true)).
hipError_t launch_attention(const void *q, const void *k, const void *v, const float *vexp, const float *M,
                            int m_layout, bool w64, bool f32, int B, int N, int Npad, int nsplit, float *opart,
                            float *ml, hipStream_t s, Ragged rg = {}, int layer = 0);
// attention_l fused with pw_mid_l (encoder.hip: attn_pw2_kernel) for this shape?
bool attention_fused(int B, int N, bool f32);
// attention of layer `layer` on (q, k, v, vexp_in) + the pointwise chain to the
// layer-(layer+1) (qo, ko, vo, vexp_out), H3 layouts; feat updated in place.
hipError_t launch_attn_pw2(const float *packed, const PackLayout &lay, int layer, const void *q, const void *k,
                           const void *v, const float *vexp_in, const float *M, bool m_packed, int B, int N, int Npad,
                           float *feat, void *qo, void *ko, void *vo, float *vexp_out, hipStream_t s, Ragged rg = {});
// attention of the last layer on (q, k, v, vexp_in) + its fc_message, residual,
// F.normalize and classifier (encoder.hip: attn_pw2_last_kernel); outputs as launch_pw_last.
hipError_t launch_attn_pw2_last(const float *packed, const PackLayout &lay, const void *q, const void *k,
                                const void *v, const float *vexp_in, const float *M, bool m_packed, int B, int N,
                                int Npad, const float *feat, float *feat_out, float *normed, _Float16 *normed_s,
                                float *conf, hipStream_t s, Ragged rg = {});
// fp32 rows [B][N][CH] -> [B][Npad][CH], padding rows zero.
hipError_t launch_pad_rows(const float *x, int B, int N, int Npad, float *y, hipStream_t s);
// fp32 q, k, v [B][ld][CH] -> split layouts (rows N..Npad-1 zero).
hipError_t launch_split_qkv(const float *q, const float *k, const float *v, int B, int N, int ld, int Npad,
                            _Float16 *qs, _Float16 *ks, _Float16 *vs, float *vexp, hipStream_t s);
// Combine partials -> msg [B][Npad][CH] (used by the standalone attention API).
hipError_t launch_attn_combine(const float *opart, const float *ml, bool f32, int B, int N, int Npad,
                               int nsplit, float *msg, hipStream_t s);

// Pointwise chains (one workgroup per PT points); q, k, v in launch_attention's layouts.
// fused: the batch runs the fused plan (attention_fused), whatever B this call covers.
hipError_t launch_pw_first(const float *packed, const PackLayout &lay, const float *corr_pos, bool f32, int B,
                           int N, int Npad, float *feat, void *q, void *k, void *v, float *vexp, hipStream_t s,
                           Ragged rg = {}, bool fused = false);
// H3 split partials (nsplit) -> one combined split (opart1 [B][Npad][CH] in the
// h3 tiling, ml1 = (0, 1)) that pw_mid / pw_last read with nsplit = 1 (small
// batches: combine16's per-thread load chain is the pointwise launch's latency).
hipError_t launch_combine_rows(const float *opart, const float *ml, int B, int Npad, int nsplit, float *opart1,
                               float *ml1, hipStream_t s);
// feat_in: the layer's rows (the residual); feat: where the new PointCN rows
// go -- a different buffer (the Q / K / V workgroups of one point tile read
// feat_in while one of them writes feat)
hipError_t launch_pw_mid(const float *packed, const PackLayout &lay, int layer, bool f32, const float *opart,
                         const float *ml, int nsplit, int B, int N, int Npad, const float *feat_in, float *feat,
                         void *q, void *k, void *v, float *vexp, hipStream_t s);
hipError_t launch_pw_last(const float *packed, const PackLayout &lay, bool f32, const float *opart,
                          const float *ml, int nsplit, int B, int N, int Npad, const float *feat,
                          float *feat_out, float *normed, _Float16 *normed_s, float *conf, hipStream_t s);

hipError_t launch_local_max(const float *src, const float *conf, int B, int N, float radius,
                            float *lm, hipStream_t s, Ragged rg = {});
// scratch: B S N words the ranking may use (the forward's kdist), or null
hipError_t launch_seed_rank(const float *conf, const float *lm, int B, int N, int S, int *seeds,
                            hipStream_t s, Ragged rg = {}, uint32_t *scratch = nullptr);

// ns: normed as [B][N][2][128] fp16 hi/lo (qk_pos order, attention_h3.hpp)
hipError_t launch_knn_dist(const _Float16 *ns, const int *seeds, int B, int N, int S, float *dist,
                           hipStream_t s, Ragged rg = {});
hipError_t launch_split_rows(const float *x, size_t rows, _Float16 *out, hipStream_t s);
// PDSC_PRECISION_F32 seed-row distances from the fp32 normed rows [B][N][128]
hipError_t launch_knn_dist_f32(const float *normed, const int *seeds, int B, int N, int S, float *dist,
                               hipStream_t s, Ragged rg = {});
hipError_t launch_knn_select(const float *dist, int B, int N, int S, int k, int *knn, hipStream_t s,
                             Ragged rg = {});
// feats: the split normed copy [B][N][2][128] fp16 (as launch_knn_dist reads it),
// or the fp32 normed rows [B][N][128] when f32
hipError_t launch_nsm_seed(const void *feats, bool f32, const float *src, const float *tgt, const int *knn, int B,
                           int N, int S, int k, int T, const float *sigma, const float *sigma_d, float *hist,
                           unsigned *seed_flags, hipStream_t s, Ragged rg = {});
hipError_t launch_nsm_finish(const float *hist, const unsigned *seed_flags, int B, int S, int k, int T, bool batch_global,
                             float *weights, int *iters_used, hipStream_t s, Ragged rg = {});
// sums: scratch [B][S][15]
// hist != NULL (the testing forward): the NSM weights are finished inside the
// first launch (nsm_finish's arithmetic, per-pair allclose over hist /
// seed_flags) and written to wout; `weights` is then not read.
hipError_t launch_hypotheses(const float *src, const float *tgt, const int *knn, const float *weights,
                             int B, int N, int S, int k, float tau, float *seed_trans, int *counts,
                             float *sums, hipStream_t s, Ragged rg = {}, const float *hist = nullptr,
                             const unsigned *seed_flags = nullptr, int T = 0, float *wout = nullptr);
// conf / range (both may be null): the forward's fp16 range guard -- a pair
// whose logits conf[b, :n] hold a non-finite value gets range[b] = 1 (else 0),
// final_trans all NaN and labels 0; post_refine leaves such a pair alone.
hipError_t launch_select_best(const float *src, const float *tgt, const float *seed_trans,
                              const int *counts, int B, int N, int S, float tau, float *fitness,
                              int *best, float *trans, float *labels, hipStream_t s, Ragged rg = {},
                              const float *conf = nullptr, int *range = nullptr);
hipError_t launch_post_refine(float *trans, const float *src, const float *tgt, int B, int N, float thr,
                              hipStream_t s, Ragged rg = {}, const int *range = nullptr);
// launch_select_best (fitness and best not written) + launch_post_refine in one launch
hipError_t launch_best_refine(const float *src, const float *tgt, const float *seed_trans, const int *counts, int B,
                              int N, int S, float tau, float thr, float *trans, float *labels, hipStream_t s,
                              Ragged rg = {}, const float *conf = nullptr, int *range = nullptr);
hipError_t launch_rigid(const float *A, const float *Bp, const float *w, int nb, int n, float *trans,
                        hipStream_t s);

// training-mode forward pieces (training.hip)
// feats: the split normed copy [B][N][2][128] fp16 (H3) or normed [B][N][128] (f32)
hipError_t launch_feat_sim(const void *feats, bool f32, int B, int N, const float *sigma, float *M, hipStream_t s);
size_t sm_loss_partial_doubles(int B, int N);
hipError_t launch_sm_loss(const float *M, const float *labels, int B, int N, int balanced, double *part, float *loss,
                          hipStream_t s);

// descriptor stage (descriptors.hip)
struct CloudStats {
    float mn[3], mx[3];
    double centroid[3];
};
struct GridView {  // points sorted by cell key and the occupied cells
    unsigned long long *skey, *ukey;
    int *sidx, *ustart, *ucount, *nruns;
};
struct GridBufs {
    CloudStats *st;
    GridView view;
    int *err;  // [0] extent / cell >= 2^21, [1] a kNN candidate set over capacity
};
size_t grid_workspace_bytes(int n);
hipError_t build_grid(const float *pts, int n, double cell, double half, void *ws, GridBufs &G, hipStream_t s);
hipError_t launch_radius_knn(const float *pts, int n, const GridBufs &G, double radius, int K, int *nbr, double *d2,
                             int *cnt, hipStream_t s);
hipError_t launch_normals(const float *pts, int n, const int *nbr, const int *cnt, int K, const GridBufs &G,
                          int orient, const float *viewpoint, float *nrm, hipStream_t s);
hipError_t launch_voxel_reduce(const float *pts, const float *nrm, int n, const GridBufs &G, float *opts, float *onrm,
                               int *count, hipStream_t s);
hipError_t launch_fpfh(const float *pts, const float *nrm, int n, const int *nbr, const int *cnt, const double *d2,
                       int K, double *spfh, double *out, float *outn, hipStream_t s);
int ply_read_xyz(const char *path, float *xyz, int64_t capacity, int64_t *n_out, std::string &err);

// correspondence construction (corr.hip)
#define HIP_RET(expr)                         \
    do {                                      \
        hipError_t e_ = (expr);               \
        if (e_ != hipSuccess) return e_;      \
    } while (0)
// spectral-matching baseline (sm.hip)
hipError_t launch_sm(const float *corr, const float *src, const float *tgt, int N, float sig2, int S, int iters,
                     float *M, float *v, float *y, float *w, float *labels, float *trans, hipStream_t s);
hipError_t launch_sm_matvec(const float *M, const float *v, int N, float *y, hipStream_t s);
hipError_t launch_nn_argmin(const float *A, const float *B, int Na, int Nb, int D, unsigned long long *rowkey,
                            unsigned long long *colkey, hipStream_t s);
hipError_t launch_corr_build(const unsigned long long *rowkey, const unsigned long long *colkey,
                             const float *src_xyz, const float *tgt_xyz, int Na, int mutual, const double *gt,
                             double thr, int *corr, int *count, float *corr_pos, float *src_out, float *tgt_out,
                             float *labels, hipStream_t s);

}  // namespace pdsc
