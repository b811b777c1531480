/*
 * pdsc.h -- C ABI of libpdsc.so, the MI355X (gfx950) hot path of PointDSC.
 *
 * Drop-in boundary for the reference's testing-mode forward
 * (models/PointDSC.py:128-197 of AmnonDrory/PointDSC) and the functions it
 * calls.  Each entry point names the reference code it replaces.
 *
 * Conventions
 *   - Every pointer argument is a DEVICE pointer (hipMalloc / torch CUDA
 *     tensor storage) unless documented otherwise; all tensors are dense,
 *     row-major, fp32 unless stated; index tensors are int32.
 *   - B = number of independent scan pairs processed by one call (the
 *     reference's public forward is bs == 1; B > 1 is the batched API);
 *     N = correspondences per pair (same N for every pair of a call).
 *   - Calls are asynchronous on `stream` (a hipStream_t; NULL = legacy default
 *     stream), never allocate, never synchronise, and never free caller
 *     memory: scratch comes from a caller-allocated workspace whose size the
 *     matching *_workspace_bytes() query returns.  The compute functions keep
 *     no state between calls and may run concurrently on different streams;
 *     the two measurement hooks (pdsc_attention_timing, pdsc_forward_timing)
 *     are per-thread settings read by the calls of the thread that set them.
 *   - Return value: PDSC_OK or an error code; no exception crosses the ABI.
 *     pdsc_last_error() returns a thread-local message for the last failure.
 */
#ifndef PDSC_H_
#define PDSC_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef void *pdsc_stream_t; /* hipStream_t */

enum pdsc_status {
    PDSC_OK = 0,
    PDSC_ERR_ARG = 1,         /* bad shape / null pointer / unsupported hyper-parameter */
    PDSC_ERR_HIP = 2,         /* a HIP runtime call failed (launch error) */
    PDSC_ERR_UNSUPPORTED = 3, /* valid for the reference, not implemented here */
    PDSC_ERR_RANGE = 4,       /* pdsc_range_status: a pair left the fp16 range (below) */
};

/* Arithmetic of the fp32 contractions (the reference computes them in fp32).
 *   PDSC_PRECISION_H3  (default) each fp32 operand is an exact pair hi + lo of
 *                      fp16 values and each product is hi.hi + hi.lo + lo.hi on
 *                      the fp16 matrix cores with fp32 accumulation (22-bit
 *                      operands; 5.3x the fp32 MFMA rate).
 *   PDSC_PRECISION_F32 exact fp32 MFMA (v_mfma_f32_32x32x2_f32) for the 1x1
 *                      convolutions, the attention, the seed kNN and the NSM
 *                      Gram, and libm expf in the softmax: the reference's
 *                      arithmetic, used to bound the H3 mode's error.
 * Everything else (M, NMS, power iteration, Kabsch, verification) is the
 * same code in both modes.                                                   */
enum pdsc_precision {
    PDSC_PRECISION_H3 = 0,
    PDSC_PRECISION_F32 = 1,
};

/* fp16 range guard (PDSC_PRECISION_H3).  The 3xfp16 split is exact only for
 * |x| < 65520: a larger (or non-finite) activation entering a contraction --
 * features, Q / K / V, hidden layers; the encoder's are O(10) for the trained
 * networks -- becomes hi = inf, lo = -inf, and the contraction's output NaN.
 * The encoder's ReLUs propagate NaN (as torch.relu does), so such a pair ends
 * with a non-finite logit; the testing and training forwards then (on the
 * device, asynchronously) mark it in the workspace, set its final_trans to NaN
 * and its final_labels to 0, and skip its post-refinement: never a silent
 * finite result.  After the stream has run the forward, pdsc_range_status
 * reports the marks: PDSC_ERR_RANGE when any pair is marked (flags [B], HOST
 * int32, may be NULL: 1 for a marked pair), else PDSC_OK.  It synchronises
 * `stream` and must be given the forward's workspace and B.  Rerun the marked
 * pairs with PDSC_PRECISION_F32 (pointdsc_amd.PointDSC does that itself).  In
 * PDSC_PRECISION_F32 a mark means a non-finite logit (non-finite inputs), as
 * the reference's fp32 would produce.  pdsc_encoder_f32 has no workspace
 * marks: its conf output carries the NaN.                                    */
int32_t pdsc_range_status(const void *forward_workspace, int32_t B, int32_t *flags, pdsc_stream_t stream);

/* The same answer without the per-pair flags and without a copy: enqueues on
 * `stream` a one-wavefront kernel that writes whether any of the B pairs is
 * marked into a word of coherent page-locked host memory (one per host thread,
 * allocated on first use), and spins on that word until the kernel has run --
 * i.e. until everything enqueued on `stream` before it has completed -- then
 * returns PDSC_OK or PDSC_ERR_RANGE.  After 20 ms of spinning it blocks in
 * hipStreamSynchronize instead (a long queue; a faulted stream is reported as
 * PDSC_ERR_HIP).  The bs = 1 drop-in path (pointdsc_amd.PointDSC.forward) uses
 * it: the reference's forward returns with no host synchronisation at all
 * (models/PointDSC.py:128-197); this one waits only for the guard's answer. */
int32_t pdsc_range_poll(const void *forward_workspace, int32_t B, pdsc_stream_t stream);

/* Hyper-parameters of PointDSC.__init__ (models/PointDSC.py:81-100). */
typedef struct pdsc_config {
    int32_t in_dim;           /* 6 (1 .. 128; the reference's 6, 9, 12, 70) */
    int32_t num_layers;       /* 12 in both release configs */
    int32_t num_channels;     /* 128 (the only width the HIP kernels implement) */
    int32_t num_iterations;   /* power-iteration cap, 10 */
    int32_t k;                /* NSM neighbourhood, 40 (clipped to N-1 per call, :250) */
    double ratio;             /* seed ratio, 0.1: S = int(N * ratio) as Python computes it (:174) */
    float inlier_threshold;   /* tau of :328/:335 */
    float nms_radius;         /* R of :174 */
    float refine_threshold;   /* :415-418: 0.10 if inlier_threshold == 0.10 else 1.2 */
    int32_t precision;        /* enum pdsc_precision; the packed weights must be packed with the same value */
} pdsc_config;

const char *pdsc_version(void);
const char *pdsc_last_error(void);

/* ---------------------------------------------------------------- weights --
 * Packs the reference's parameters (device pointers, in the order of
 * pdsc_param_names()) into the kernels' layout: Conv1d(k=1) weights as fp16
 * hi/lo planes scaled by a per-layer power of two (PDSC_PRECISION_H3) or plain
 * fp32 [out][in] (PDSC_PRECISION_F32); eval BatchNorm turned into the per-channel
 * (alpha, beta) torch-CPU uses (alpha = w / sqrt(var + 1e-5), beta = b - mean*alpha);
 * sigma and sigma_spat copied into the blob header (read on device, no host sync).
 * Replaces: nothing in the reference (it reads nn.Module parameters directly).
 */
int32_t pdsc_param_count(const pdsc_config *cfg);
const char *pdsc_param_name(const pdsc_config *cfg, int32_t i); /* state_dict key */
size_t pdsc_packed_weights_floats(const pdsc_config *cfg);
int32_t pdsc_pack_weights(const pdsc_config *cfg, const float *const *params_host_array,
                          float *packed, pdsc_stream_t stream);

/* ---------------------------------------------------------- a1 compat ------
 * M[b,i,j] = max(0, 1 - (|s_i-s_j| - |t_i-t_j|)^2 / sigma_d^2), bit-exact with
 * torch-CPU fp32.  Replaces models/PointDSC.py:150-153.  sigma_d is read on
 * device from `sigma_d_dev` (the checkpoint's sigma_spat, :98).
 * src,tgt [B,N,3]; M [B,N,N].                                              */
int32_t pdsc_compat_f32(const float *src, const float *tgt, int32_t B, int32_t N,
                        const float *sigma_d_dev, float *M, pdsc_stream_t stream);
/* The forward's form of the same M: the upper triangle of 32 x 32 tiles, each
 * a contiguous row-major 4 KiB block, tile (ti, tj), ti <= tj, at block index
 * ti*nt - ti*(ti-1)/2 + (tj - ti), nt = ceil(N/32); M[i][j] for i > j is
 * element (j%32, i%32) of tile (j/32, i/32); entries past N are 0.
 * Mp: B * pdsc_compat_packed_floats(N) floats.                              */
size_t pdsc_compat_packed_floats(int32_t N);
int32_t pdsc_compat_packed_f32(const float *src, const float *tgt, int32_t B, int32_t N,
                               const float *sigma_d_dev, float *Mp, pdsc_stream_t stream);

/* -------------------------------------------------- a2-a4 encoder ----------
 * SCNonlocal encoder + F.normalize + classification MLP.
 * Replaces models/PointDSC.py:155-156 and :171 (NonLocalNet.forward :65-77,
 * NonLocalBlock.forward :27-45).  corr_pos [B,N,in_dim]; M [B,N,N] (must be
 * symmetric -- the spatial compatibility is; the attention kernel reads it
 * column-wise).  Outputs: feat [B,N,C] (corr_features), normed [B,N,C],
 * conf [B,N] (the classifier logits).                                        */
size_t pdsc_encoder_workspace_bytes(const pdsc_config *cfg, int32_t B, int32_t N);
int32_t pdsc_encoder_f32(const pdsc_config *cfg, const float *packed, const float *corr_pos,
                         const float *M, int32_t B, int32_t N, float *feat, float *normed,
                         float *conf, void *workspace, size_t workspace_bytes,
                         pdsc_stream_t stream);

/* The attention core of one NonLocalBlock (models/PointDSC.py:36-42) alone:
 * msg[b,i,:] = sum_j softmax_j(M_ij * q_i.k_j / sqrt(C)) v_j, heads = 1.
 * q,k,v [B,N,C]; msg [B,N,C].  C must be 128.  precision: enum pdsc_precision. */
size_t pdsc_attention_workspace_bytes(int32_t B, int32_t N, int32_t C, int32_t precision);
int32_t pdsc_attention_f32(const float *q, const float *k, const float *v, const float *M,
                           int32_t B, int32_t N, int32_t C, int32_t precision, float *msg, void *workspace,
                           size_t workspace_bytes, pdsc_stream_t stream);

/* The TESTING / TRAINING FORWARD's attention geometry for (B, N): padded rows
 * per pair and the number of key splits (partials opart [B,nsplit,Npad,C],
 * ml [B,nsplit,Npad,2] in the forward workspace).  Both this query and
 * pdsc_encoder_plan describe pdsc_forward_testing(_ragged/_debug) and
 * pdsc_forward_training only: the standalone pdsc_encoder_f32 and
 * pdsc_attention_f32 take a dense M and always run the h3 split-K plan
 * (plan 0 or 1, never 2), whose split count may differ from the one
 * reported here for shapes where the forward picks plan 2.                  */
int32_t pdsc_attention_layout(int32_t B, int32_t N, int32_t precision, int32_t *Npad, int32_t *nsplit);

/* The encoder's launch plan for (B, N, precision) (no reference counterpart):
 * *fused = 1 when every layer but the last runs its attention and the
 * following pointwise chain (fc_message, residual, PointCN, Q/K/V) as ONE
 * launch -- these are then the launches pdsc_attention_timing times -- 0
 * when attention and chain are separate launches, and 2 when they are separate
 * and the attention is the 64-query-wave kernel (one 4-wave workgroup per CU,
 * attention_w64.hpp; the forward's M symmetric-packed as for plans 0/1).    */
int32_t pdsc_encoder_plan(int32_t B, int32_t N, int32_t precision, int32_t *fused);

/* Measurement hook (bench.py): while capacity > 0, every attention launch the
 * encoder issues from the calling thread records start_events[i] / stop_events[i]
 * (hipEvent_t) around itself on its stream, i = (*count)++ while < capacity.
 * Pass capacity 0 to disable.  The caller owns the events and the counter.   */
int32_t pdsc_attention_timing(void *const *start_events, void *const *stop_events, int32_t capacity,
                              int32_t *count);
/* Measurement hook (no reference counterpart): every pdsc_forward_testing
 * call from the calling thread records PDSC_FORWARD_STAGES + 1 events on its
 * stream -- events[c + 0] before a1, then one after each stage in the order
 * a1 compat, a2-a4 encoder, a5 seeds, a6 seed kNN, a7-a8 NSM, a9-a10
 * hypotheses+verification, a11 post-refinement -- with c = *count, then
 * *count += 8, while *count + 8 <= capacity.  Capacity 0 disables.           */
#define PDSC_FORWARD_STAGES 7
int32_t pdsc_forward_timing(void *const *events, int32_t capacity, int32_t *count);
/* Test hook (no reference counterpart): the small-batch pw_mid's K / V
 * workgroups of the Q / K / V split sleep `loops` x 127 x 64 cycles before
 * their first load (0: off, the default).  A per-thread setting like the
 * timing hooks; tests/test_gpu_parity.py uses it to pin that the split's
 * readers of the residual rows cannot see the Q workgroup's new rows.       */
int32_t pdsc_diag_qkv_delay(int32_t loops);

/* ------------------------------------------------------- a5 seeds ----------
 * pick_seeds: radius NMS on the confidences then the top-S of
 * conf * is_local_max in descending order (ties: ascending index).
 * Replaces models/PointDSC.py:199-217.  src [B,N,3]; conf [B,N];
 * seeds [B,S] int32; is_local_max [B,N] (0/1 fp32; required, it hosts the
 * flags between the two launches).                                          */
int32_t pdsc_pick_seeds(const float *src, const float *conf, int32_t B, int32_t N, float radius,
                        int32_t S, int32_t *seeds, float *is_local_max, pdsc_stream_t stream);

/* ------------------------------------------------------- a6 seed kNN -------
 * For each seed row: the k nearest correspondences in feature space,
 * d_j = 2 - 2 f_s.f_j, topk(k+1, smallest)[1:] -- the FIRST of the k+1
 * (ascending distance, ascending index) is dropped positionally.
 * Replaces models/common.py:48-69 + models/PointDSC.py:250-252 (only the
 * S seed rows are computed).  normed [B,N,C]; seeds [B,S]; knn [B,S,k];
 * 1 <= k <= 63, k + 1 <= N.  precision: enum pdsc_precision (distances).
 * The workspace holds the [B,S,N] distance rows.                            */
size_t pdsc_seed_knn_workspace_bytes(int32_t B, int32_t N, int32_t S);
int32_t pdsc_seed_knn(const float *normed, const int32_t *seeds, int32_t B, int32_t N, int32_t C,
                      int32_t S, int32_t k, int32_t precision, int32_t *knn, void *workspace,
                      size_t workspace_bytes, pdsc_stream_t stream);

/* ------------------------------------------------ a7-a8 NSM weights --------
 * Local k x k feature x spatial consistency (diag 0), power iteration with
 * the batch-global allclose early exit (rtol 1e-5, atol 1e-8, evaluated over
 * all B*S seeds of the call, as torch.allclose does over the bs*S batch of one
 * cal_leading_eigenvector call), then w = v / (sum v + 1e-6); iters_used[b] is
 * the same for every b.  Replaces models/PointDSC.py:257-282, :338-358.
 * (pdsc_forward_testing exits per pair -- each pair is its own bs = 1 forward;
 * pdsc_forward_training over the whole batch -- one reference forward.)
 * sigma_dev / sigma_d_dev: device scalars (learned sigma, sigma_spat).
 * weights [B,S,k]; iters_used [B] int32 (may be NULL); 1 <= k <= min(63, N-1).
 * precision: enum pdsc_precision (the feature Gram).  The workspace holds the
 * fp16 hi/lo split of normed the H3 Gram MFMAs read.                         */
size_t pdsc_nsm_workspace_bytes(int32_t B, int32_t N, int32_t S, int32_t k, int32_t num_iterations);
int32_t pdsc_nsm_weights(const float *normed, const float *src, const float *tgt,
                         const int32_t *knn, int32_t B, int32_t N, int32_t C, int32_t S, int32_t k,
                         int32_t num_iterations, int32_t precision, const float *sigma_dev,
                         const float *sigma_d_dev, float *weights, int32_t *iters_used, void *workspace,
                         size_t workspace_bytes, pdsc_stream_t stream);

/* ------------------------------------------------------- a9 Kabsch ---------
 * rigid_transform_3d: weighted centroids, H = Am^T diag(w) Bm, R from the SVD
 * of H (3x3, fp64 Jacobi on device) with the det(V U^T) reflection fix,
 * t = c_B - R c_A, packed as 4x4.  Replaces models/common.py:7-45 (whose SVD
 * runs on the host CPU).  A,Bp [nb,n,3]; w [nb,n] (NULL = ones); trans [nb,4,4]. */
int32_t pdsc_rigid_transform_3d(const float *A, const float *Bp, const float *w, int32_t nb,
                                int32_t n, float *trans, pdsc_stream_t stream);

/* --------------------------------------------- a10 verification ------------
 * Seed hypotheses: Kabsch on each seed's kNN set with `weights`, fitness =
 * mean(|R_s src + t_s - tgt| < tau), best = first argmax, final_labels from
 * the best hypothesis.  Replaces models/PointDSC.py:287-335.
 * seed_trans [B,S,4,4] and fitness [B,S] are required (they host the per-seed
 * scratch); best [B] int32 (may be NULL); trans [B,4,4]; labels [B,N].      */
size_t pdsc_seed_hypotheses_workspace_bytes(int32_t B, int32_t S);
int32_t pdsc_seed_hypotheses(const float *src, const float *tgt, const int32_t *knn,
                             const float *weights, int32_t B, int32_t N, int32_t S, int32_t k,
                             float tau, float *seed_trans, float *fitness, int32_t *best,
                             float *trans, float *labels, void *workspace, size_t workspace_bytes,
                             pdsc_stream_t stream);

/* ------------------------------------------------ a11 post-refinement ------
 * <= 20 IRLS re-fits on the inliers of |R src + t - tgt| < thr with weights
 * 1/(1 + (L2/thr)^2), stopping when the inlier count repeats.  Device-side
 * loop, one workgroup per pair.  Replaces models/PointDSC.py:403-438.
 * trans [B,4,4] in/out.                                                      */
int32_t pdsc_post_refine(float *trans, const float *src, const float *tgt, int32_t B, int32_t N,
                         float thr, pdsc_stream_t stream);

/* ------------------------------------- f3 spectral-matching baseline -----
 * SM of baseline_scripts/baseline_3DMatch.py:19-53 for one pair: dense
 * M_ij = max(0, 4.5 - (|c_j - c_i|_xyz - |c_j - c_i|_xyz')^2 / 2 / sigma^2),
 * sigma = inlier_threshold / 3, diag 0, over corr_pos [N,6]; num_iterations
 * power iterates v <- Mv / (|Mv| + 1e-6) from v = 1; labels [N] = the
 * int(N * top_ratio) largest entries of v (ties to the lower index); trans
 * [4,4] = rigid_transform_3d(src, tgt, v * labels).  leading_eig [N] may be
 * NULL.  Workspace: the dense M (4 N^2 B) + 3 vectors.                      */
size_t pdsc_spectral_matching_workspace_bytes(int32_t N);
int32_t pdsc_spectral_matching(const float *corr_pos, const float *src, const float *tgt, int32_t N,
                               double inlier_threshold, double top_ratio, int32_t num_iterations, float *trans,
                               float *labels, float *leading_eig, void *workspace, size_t workspace_bytes,
                               pdsc_stream_t stream);
/* One M v product of the SM power iteration (the HBM-bound kernel, exposed for
 * measurement): y [N] = M [N,N] v [N].                                       */
int32_t pdsc_sm_matvec(const float *M, const float *v, int32_t N, float *y, pdsc_stream_t stream);

/* ------------------------------ f3 training-mode forward and loss ---------
 * PointDSC.forward(data) WITHOUT the 'testing' key (models/PointDSC.py:158-163,
 * 176, 182, 189-191) for B pairs (the training batch; forward only -- no
 * gradients): M = clamp(1 - (1 - F^ F^T) / sigma^2, 0, 1) with a zero diagonal
 * into M_out [B,N,N] (may be NULL), seeds = the int(N * ratio) largest logits
 * (argsort, no NMS; ties by ascending index), seed hypotheses and verification
 * as in testing, no post-refinement.  Outputs final_trans [B,4,4] and
 * confidence [B,N] (the logits the reference returns as 'final_labels');
 * seeds_out [B,int(N*ratio)] (may be NULL) receives the seed indices.       */
size_t pdsc_forward_training_workspace_bytes(const pdsc_config *cfg, int32_t B, int32_t N);
int32_t pdsc_forward_training(const pdsc_config *cfg, const float *packed, const float *corr_pos,
                              const float *src, const float *tgt, int32_t B, int32_t N, float *final_trans,
                              float *confidence, float *M_out, int32_t *seeds_out, void *workspace,
                              size_t workspace_bytes, pdsc_stream_t stream);
/* SpectralMatchingLoss (libs/loss.py:115-139) of M [B,N,N] against gt_labels
 * [B,N] (0/1): balanced != 0 -> mean over pairs of 0.5 sum gt (M-1)^2 /
 * (relu(sum gt - 1) + 1) + 0.5 sum (1-gt) M^2 / (relu(sum (1-gt) - 1) + 1), else
 * mean((M - gt)^2); gt_ij = (l_i + l_j == 2), gt_ii = 0.  Sums in fp64;
 * loss: one device float.                                                   */
size_t pdsc_spectral_matching_loss_workspace_bytes(int32_t B, int32_t N);
int32_t pdsc_spectral_matching_loss(const float *M, const float *gt_labels, int32_t B, int32_t N, int32_t balanced,
                                    float *loss, void *workspace, size_t workspace_bytes, pdsc_stream_t stream);

/* ---------------------------------- f1 correspondence construction --------
 * Mutual nearest neighbours in descriptor space and the network inputs built
 * from them: replaces datasets/ThreeDMatch.py:277-308 (3DMatch / 3DLoMatch
 * test sets), datasets/KITTI.py:85-99 and demo_registration.py:101-108.
 *   distance = sqrt(2 - 2 src_desc tgt_desc^T + 1e-6) in fp32, never stored;
 *   nn_src[i] = argmin_j, nn_tgt[j] = argmin_i (first index on ties, like
 *   numpy.argmin).  src_desc [Ns,D], tgt_desc [Nt,D], 1 <= D <= 64.
 * Workspace: 8 (Ns + Nt) bytes (64-bit key/index words).                    */
size_t pdsc_mutual_nn_workspace_bytes(int32_t Ns, int32_t Nt);
int32_t pdsc_mutual_nn(const float *src_desc, const float *tgt_desc, int32_t Ns, int32_t Nt, int32_t D,
                       int32_t *nn_src, int32_t *nn_tgt, void *workspace, size_t workspace_bytes,
                       pdsc_stream_t stream);
/* The correspondence set (mutual != 0: i with nn_tgt[nn_src[i]] == i, in
 * ascending i; else every i) and the forward's inputs: corr [Ns,2] int32
 * (first *count rows valid), src_keypts / tgt_keypts [Ns,3], corr_pos [Ns,6]
 * = [src, tgt] - their mean (numpy's sequential fp32 column mean), and, when
 * gt_trans (a device double[16], row-major 4x4) is non-NULL, labels [Ns] =
 * |R src + t - tgt| < inlier_threshold in fp64.  count: a device int32.     */
int32_t pdsc_build_correspondences(const float *src_desc, const float *tgt_desc, const float *src_xyz,
                                   const float *tgt_xyz, int32_t Ns, int32_t Nt, int32_t D, int32_t mutual,
                                   const double *gt_trans, double inlier_threshold, int32_t *corr,
                                   int32_t *count, float *corr_pos, float *src_keypts, float *tgt_keypts,
                                   float *labels, void *workspace, size_t workspace_bytes, pdsc_stream_t stream);

/* ------------------------------------------- f4 descriptor stage ----------
 * The open3d calls of demo_registration.py:37-44 / misc/cal_fpfh.py:7-36 on the
 * GPU (open3d's published algorithms restated; parity with open3d itself is
 * unpinned).  Points are fp32 [n,3] device arrays; 1 <= n <= 2^31-1.  These
 * entry points synchronise `stream` before returning (they report grid-range
 * and capacity errors found on the device).
 *
 * pdsc_ply_read_xyz (HOST memory, o3d.io.read_point_cloud): the vertex x, y, z
 * of a binary_little_endian or ascii PLY.  xyz == NULL: only *n_points.     */
int32_t pdsc_ply_read_xyz(const char *path, float *xyz, int64_t capacity, int64_t *n_points);
/* KDTreeSearchParamHybrid(radius, max_nn) for every point of the cloud: nbr
 * [n,max_nn] (ascending (d^2, index), the point itself first, -1 padded),
 * dist2 [n,max_nn] fp64 (may be NULL), count [n].  1 <= max_nn <= 128.      */
size_t pdsc_radius_knn_workspace_bytes(int32_t n);
int32_t pdsc_radius_knn(const float *pts, int32_t n, float radius, int32_t max_nn, int32_t *nbr, double *dist2,
                        int32_t *count, void *workspace, size_t workspace_bytes, pdsc_stream_t stream);
/* EstimateNormals(KDTreeSearchParamHybrid(radius, max_nn)) (utils/pointcloud.py:
 * 20-21) as open3d 0.9.0 (environment.yml:76) computes it with its default
 * fast_normal_computation: the fp64 cumulant covariance of the neighbourhood,
 * FastEigen3x3's smallest-eigenvalue eigenvector (A - l0 I)(A - l1 I) e0,
 * normalised -- so its sign gives n_x >= 0 --, (0,0,1) when that vector is 0
 * or under 3 neighbours.  orient (enum pdsc_normal_orientation):
 *   PDSC_NORMALS_OPEN3D    that sign, as open3d leaves it on a cloud without
 *                          normals (the demo's case; viewpoint unused, may be NULL)
 *   PDSC_NORMALS_VIEWPOINT flipped towards viewpoint (device float[3])
 *   PDSC_NORMALS_CENTROID  flipped towards the cloud's centroid (makes FPFH
 *                          invariant to rigid motions; not open3d's result)   */
enum pdsc_normal_orientation {
    PDSC_NORMALS_OPEN3D = 0,
    PDSC_NORMALS_VIEWPOINT = 1,
    PDSC_NORMALS_CENTROID = 2,
};
size_t pdsc_estimate_normals_workspace_bytes(int32_t n, int32_t max_nn);
int32_t pdsc_estimate_normals(const float *pts, int32_t n, float radius, int32_t max_nn, int32_t orient,
                              const float *viewpoint, float *normals, void *workspace, size_t workspace_bytes,
                              pdsc_stream_t stream);
/* VoxelDownSample(voxel_size): per-voxel means; normals summed and normalised
 * (open3d's AccumulatedPoint::GetAverageNormal: a zero sum stays 0);
 * normals / out_normals may be NULL; voxels in ascending key order; out_pts
 * [n,3] capacity; *out_count (device int32) = voxels.                        */
size_t pdsc_voxel_down_sample_workspace_bytes(int32_t n);
int32_t pdsc_voxel_down_sample(const float *pts, const float *normals, int32_t n, float voxel_size, float *out_pts,
                               float *out_normals, int32_t *out_count, void *workspace, size_t workspace_bytes,
                               pdsc_stream_t stream);
/* compute_fpfh_feature(KDTreeSearchParamHybrid(radius, max_nn)): fpfh [n,33]
 * fp64 (open3d's feature.data.T); fpfh_normalized [n,33] fp32 = f / (||f|| +
 * 1e-6) (demo_registration.py:42, may be NULL).  normals must be unit.      */
size_t pdsc_compute_fpfh_workspace_bytes(int32_t n, int32_t max_nn);
int32_t pdsc_compute_fpfh(const float *pts, const float *normals, int32_t n, float radius, int32_t max_nn,
                          double *fpfh, float *fpfh_normalized, void *workspace, size_t workspace_bytes,
                          pdsc_stream_t stream);

/* ----------------------------------------------- full testing forward ------
 * PointDSC.forward(data) with 'testing' in data (models/PointDSC.py:128-197)
 * for B independent pairs: compat -> encoder -> classifier -> seeds -> kNN ->
 * NSM -> hypotheses -> post-refinement.  corr_pos [B,N,in_dim];
 * src,tgt [B,N,3]; final_trans [B,4,4]; final_labels [B,N].
 * Optional debug outputs (NULL to skip): conf [B,N], seeds [B,S].           */
size_t pdsc_forward_workspace_bytes(const pdsc_config *cfg, int32_t B, int32_t N);
int32_t pdsc_forward_testing(const pdsc_config *cfg, const float *packed, const float *corr_pos,
                             const float *src, const float *tgt, int32_t B, int32_t N,
                             float *final_trans, float *final_labels, float *conf_out,
                             int32_t *seeds_out, void *workspace, size_t workspace_bytes,
                             pdsc_stream_t stream);
/* The same forward with the intermediates of every stage (no reference
 * counterpart: the parity tests pin each stage on the forward's own values).
 * Any member may be NULL.  k = min(cfg->k, N - 1), S = int(N * ratio).       */
typedef struct pdsc_forward_debug {
    float *conf;             /* [B,N] classifier logits (:171) */
    int32_t *seeds;          /* [B,S] (:174) */
    int32_t *knn;            /* [B,S,k] seed neighbourhoods (:250-252) */
    float *weights;          /* [B,S,k] NSM weights (:280-282) */
    float *trans_pre_refine; /* [B,4,4] the best hypothesis (:182) */
} pdsc_forward_debug;
int32_t pdsc_forward_testing_debug(const pdsc_config *cfg, const float *packed, const float *corr_pos,
                                   const float *src, const float *tgt, int32_t B, int32_t N,
                                   float *final_trans, float *final_labels, const pdsc_forward_debug *debug,
                                   void *workspace, size_t workspace_bytes, pdsc_stream_t stream);

/* ---------------------------------------------- ragged testing forward -----
 * B pairs of DIFFERENT sizes in one call: the evaluation loop's pairs
 * (datasets/ThreeDMatch.py:268-290 keeps every keypoint, so N varies per pair;
 * evaluation/test_3DMatch.py:33-53 runs them one by one at bs = 1).  Each pair
 * b occupies the first counts[b] rows of N-row buffers (corr_pos [B,N,in_dim],
 * src/tgt [B,N,3]; rows past counts[b] are ignored), and the result equals B
 * separate bs = 1 forwards: final_trans [B,4,4]; final_labels [B,N] with rows
 * past counts[b] set to 0.  counts: HOST int32 [B] (passed to the device as
 * kernel arguments, no copy on the stream), each with min(cfg->k, count - 1)
 * = min(cfg->k, N - 1) (every pair keeps the batch's k) and int(count *
 * ratio) >= 1.  debug: as pdsc_forward_testing_debug (may be NULL), with the
 * batch's strides S = int(N * ratio) and k; conf rows past counts[b], and seeds,
 * knn and weights entries past a pair's own seeds, are unspecified.
 * From 32 pairs on the fused encoder plan the encoder runs as two half batches,
 * one on `stream` and one on a per-device side stream the library owns, forked
 * from and joined back into `stream` by events (still asynchronous; the same
 * results as one stream; environment PDSC_ENC_HALVES=0 keeps one stream).
 * Workspace: pdsc_forward_workspace_bytes(cfg, B, N).                        */
int32_t pdsc_forward_testing_ragged(const pdsc_config *cfg, const float *packed, const float *corr_pos,
                                    const float *src, const float *tgt, int32_t B, int32_t N,
                                    const int32_t *counts, float *final_trans, float *final_labels,
                                    const pdsc_forward_debug *debug, void *workspace, size_t workspace_bytes,
                                    pdsc_stream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* PDSC_H_ */
