// encoder.hip -- a2-a4: SCNonlocal encoder, F.normalize and the classifier.
//
// Replaces models/PointDSC.py:9-77 (NonLocalBlock / NonLocalNet), :155-156 and
// :171.  Layout in HBM (per pair b, N padded to Npad = round_up(N,128) rows):
//   feat, Q, K, V : [B][Npad][128] fp32, point-major (row = correspondence)
//   M             : [B][N][N] fp32 (a1 output; symmetric)
//   opart, ml     : [B][nsplit][Npad][128], [B][nsplit][Npad][2] attention partials
//
// Kernels per forward: pw_first (layer0 + PointCN_0 + QKV_0), then per layer
// attention_l (+ pw_mid_l = combine + fc_message_l + residual + PointCN_{l+1}
// + QKV_{l+1}), and pw_last (combine + fc_message + residual + normalize +
// classifier).  All products run on v_mfma_f32_32x32x2_f32 (exact fp32 fma
// chains; gfx950 has no reduced-precision fp32 MFMA), so the encoder is bound
// by the 157 TFLOP/s fp32 matrix roofline: 4 N^2 C flop per layer of attention.
//
// Attention (flash-style, never materialising the N x N logits):
//   one workgroup = 4 waves x 32 queries; K/V tiles of 32 keys double-buffered
//   in LDS; S^T = K Q^T so the accumulator's column index is the query and it
//   feeds P.V as the A operand with no transpose; logits = M_ij * s_ij / sqrt(C)
//   where M is read column-wise (M symmetric => coalesced 128-B rows);
//   incompatible pairs keep logit 0 (not -inf) exactly as :41; online softmax
//   with a running max; split-K over keys when B*N is too small to fill 256 CUs.
#include "attention.hpp"

namespace pdsc {

// ============================================================ weight packing
__global__ void pack_dense_kernel(const float *__restrict__ w, const float *__restrict__ b,
                                  const float *__restrict__ bn_w, const float *__restrict__ bn_b,
                                  const float *__restrict__ bn_rm, const float *__restrict__ bn_rv,
                                  int in, int out, float *__restrict__ dw, float *__restrict__ db,
                                  float *__restrict__ da, float *__restrict__ dbeta) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    const int total = in * out;
    if (i < total) {
        const int e = i & 3, lane = (i >> 2) & 63, rest = i >> 8;  // rest = jt*(in/8) + g
        const int g = rest % (in / 8), jt = rest / (in / 8);
        const int row = jt * 32 + (lane & 31), col = (lane >> 5) * (in / 2) + 4 * g + e;
        dw[i] = w[row * in + col];
    }
    if (i < out) {
        db[i] = b[i];
        if (bn_w) {
            // torch-CPU eval BatchNorm: invstd = 1/sqrt(var+eps); alpha = invstd*w; beta = b - mean*alpha
            const float invstd = 1.0f / sqrtf(bn_rv[i] + 1e-5f);
            const float alpha = invstd * bn_w[i];
            da[i] = alpha;
            dbeta[i] = bn_b[i] - bn_rm[i] * alpha;
        } else {
            da[i] = 1.0f;
            dbeta[i] = 0.0f;
        }
    }
}

__global__ void copy_kernel(const float *__restrict__ s, float *__restrict__ d, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) d[i] = s[i];
}

hipError_t launch_pack_dense(const float *w, const float *b, const float *bn_w, const float *bn_b,
                             const float *bn_rm, const float *bn_rv, int in, int out, float *dst_w,
                             float *dst_b, float *dst_a, float *dst_beta, hipStream_t s) {
    const int n = in * out;
    hipLaunchKernelGGL(pack_dense_kernel, dim3((n + 255) / 256), dim3(256), 0, s, w, b, bn_w, bn_b,
                       bn_rm, bn_rv, in, out, dst_w, dst_b, dst_a, dst_beta);
    return hipGetLastError();
}

hipError_t launch_copy(const float *src, float *dst, int n, hipStream_t s) {
    hipLaunchKernelGGL(copy_kernel, dim3((n + 255) / 256), dim3(256), 0, s, src, dst, n);
    return hipGetLastError();
}

// ================================================================= attention
// Production variant of attention.hpp: 4 waves x 32 queries per workgroup,
// 32-key LDS stages, v_exp_f32 on log2e-prescaled logits, XCD-aware block map
// (A/B-timed against the other variants with tools/attn_bench.hip).
constexpr int ATT_NW = 4, ATT_KTS = 32;

static AttnGrid prod_grid(int B, int N) { return attention_grid<ATT_NW, ATT_KTS>(B, N, 1024); }

int attention_nsplit(int B, int N) { return prod_grid(B, N).nsplit; }

hipError_t launch_attention(const float *q, const float *k, const float *v, const float *M, int B,
                            int N, int Npad, int nsplit, float *opart, float *ml, hipStream_t s) {
    const AttnGrid g = prod_grid(B, N);
    if (g.Npad != Npad || g.nsplit != nsplit) return hipErrorInvalidValue;
    const size_t lds = attention_lds_bytes<ATT_NW, ATT_KTS>();
    auto kern = attention_kernel_t<ATT_NW, ATT_KTS, true, true>;
    hipLaunchKernelGGL(kern, dim3(g.B * g.nqb * g.nsplit), dim3(ATT_NW * 64), lds, s, q, k, v, M, g,
                       opart, ml);
    return hipGetLastError();
}

// Combine the split partials of one row segment: msg = sum_s O_s e^{m_s-m*} / sum_s l_s e^{m_s-m*}.
PDSC_DEV void combine16(const float *__restrict__ opart, const float *__restrict__ ml, int b,
                        int nsplit, int Npad, int row, int d0, float out[16]) {
    float mstar = -INFINITY;
    for (int s = 0; s < nsplit; ++s) mstar = fmaxf(mstar, ml[((size_t)(b * nsplit + s) * Npad + row) * 2]);
    float L = 0.0f;
    f32x4 acc[4] = {};
    for (int s = 0; s < nsplit; ++s) {
        const size_t base = (size_t)(b * nsplit + s) * Npad + row;
        const float w = expf(ml[base * 2] - mstar);
        L += w * ml[base * 2 + 1];
        const f32x4 *src = reinterpret_cast<const f32x4 *>(opart + base * CH + d0);
#pragma unroll
        for (int i = 0; i < 4; ++i) acc[i] += w * src[i];
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int e = 0; e < 4; ++e) out[4 * i + e] = acc[i][e] / L;
}

__global__ __launch_bounds__(256) void attn_combine_kernel(const float *__restrict__ opart,
                                                           const float *__restrict__ ml, int N,
                                                           int Npad, int nsplit,
                                                           float *__restrict__ msg) {
    const int b = blockIdx.y;
    const int row = blockIdx.x * 32 + (threadIdx.x >> 3), d0 = (threadIdx.x & 7) * 16;
    if (row >= N) return;
    float out[16];
    combine16(opart, ml, b, nsplit, Npad, row, d0, out);
    f32x4 *dst = reinterpret_cast<f32x4 *>(msg + ((size_t)b * N + row) * CH + d0);
#pragma unroll
    for (int i = 0; i < 4; ++i) dst[i] = f32x4{out[4 * i], out[4 * i + 1], out[4 * i + 2], out[4 * i + 3]};
}

hipError_t launch_attn_combine(const float *opart, const float *ml, int B, int N, int Npad,
                               int nsplit, float *msg, hipStream_t s) {
    hipLaunchKernelGGL(attn_combine_kernel, dim3((N + 31) / 32, B), dim3(256), 0, s, opart, ml, N,
                       Npad, nsplit, msg);
    return hipGetLastError();
}

// ============================================================ pointwise chain
// Dense layer on a PT=32-point tile held in LDS: Y = epi(X W^T + b).  Waves take
// 32-column output tiles round-robin.  A operand = X rows (lane -> point),
// B operand = packed W (one 1-KiB coalesced load per 4 MFMAs).
enum Epi { EPI_BIAS = 0, EPI_RELU = 1, EPI_BN_RELU = 2, EPI_RESID = 3 };

template <int IN, int OUT, int EPI>
PDSC_DEV void dense32(const float *X, int xstr, const float *__restrict__ pk, const DenseOff &off,
                      float *Y, int ystr, const float *__restrict__ resid, int wave, int lane) {
    const int h = lane >> 5, l32 = lane & 31;
    for (int jt = wave; jt < OUT / 32; jt += 4) {
        f32x16 acc = zero16();
        const float *xp = X + l32 * xstr + h * (IN / 2);
        const f32x4 *wp = reinterpret_cast<const f32x4 *>(pk + off.w) + (size_t)jt * (IN / 8) * 64 + lane;
#pragma unroll 4
        for (int g = 0; g < IN / 8; ++g) {
            const f32x4 xa = *reinterpret_cast<const f32x4 *>(xp + 4 * g);
            const f32x4 wb = wp[g * 64];
            acc = mfma32(xa[0], wb[0], acc);
            acc = mfma32(xa[1], wb[1], acc);
            acc = mfma32(xa[2], wb[2], acc);
            acc = mfma32(xa[3], wb[3], acc);
        }
        const int j = jt * 32 + l32;
        const float bias = pk[off.bias + j];
        const float al = pk[off.alpha + j], be = pk[off.beta + j];
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int row = acc_row(r, h);
            float y = acc[r] + bias;
            if (EPI == EPI_BN_RELU) y = fmaxf(y * al + be, 0.0f);
            if (EPI == EPI_RELU) y = fmaxf(y, 0.0f);
            if (EPI == EPI_RESID) y = resid[row * CH + j] + y;  // res = feat + message (:44)
            Y[row * ystr + j] = y;
        }
    }
}

// Copy a [32][CH] LDS tile (stride xstr) to global rows [p0, p0+32) of dst (row stride CH).
PDSC_DEV void store_tile32(const float *X, int xstr, float *__restrict__ dst, int p0, int nrows, int tid) {
    for (int e = tid; e < 32 * (CH / 4); e += 256) {
        const int p = e / (CH / 4), c4 = e % (CH / 4);
        if (p < nrows)
            *reinterpret_cast<f32x4 *>(dst + (size_t)(p0 + p) * CH + 4 * c4) =
                *reinterpret_cast<const f32x4 *>(X + p * xstr + 4 * c4);
    }
}

constexpr int S132 = CH + 4, S68 = CH2 + 4, S36 = CLS + 4;
constexpr int PW_LDS_FLOATS = 2 * PT * S132 + 2 * PT * S68 + 2 * PT * S36 + 64;

struct PwDense4 {  // PointCN + Q/K/V of one layer
    DenseOff pcn, q, k, v;
};
struct PwMsg {  // fc_message of one layer
    DenseOff fc0, fc3, fc6;
};

// PointCN_l then Q/K/V_l of the tile in Xin -> feat (global), Q, K, V (global).
PDSC_DEV void pcn_qkv(const float *Xin, float *Xout, const float *__restrict__ pk, const PwDense4 &d,
                      float *__restrict__ feat, float *__restrict__ Q, float *__restrict__ K,
                      float *__restrict__ V, int p0, int tid, int wave, int lane) {
    dense32<CH, CH, EPI_BN_RELU>(Xin, S132, pk, d.pcn, Xout, S132, nullptr, wave, lane);
    __syncthreads();
    store_tile32(Xout, S132, feat, p0, 32, tid);
    dense32<CH, CH, EPI_BIAS>(Xout, S132, pk, d.q, Q + (size_t)p0 * CH, CH, nullptr, wave, lane);
    dense32<CH, CH, EPI_BIAS>(Xout, S132, pk, d.k, K + (size_t)p0 * CH, CH, nullptr, wave, lane);
    dense32<CH, CH, EPI_BIAS>(Xout, S132, pk, d.v, V + (size_t)p0 * CH, CH, nullptr, wave, lane);
}

// layer0 (Conv1d in_dim -> 128) + PointCN_0 + QKV_0.
__global__ __launch_bounds__(256) void pw_first_kernel(const float *__restrict__ pk, size_t l0w,
                                                       size_t l0b, PwDense4 d,
                                                       const float *__restrict__ corr, int in_dim,
                                                       int N, int Npad, float *__restrict__ feat,
                                                       float *__restrict__ Q, float *__restrict__ K,
                                                       float *__restrict__ V) {
    extern __shared__ __attribute__((aligned(16))) float sm[];
    float *X0 = sm, *X1 = sm + PT * S132, *cp = sm + 2 * PT * S132;  // cp: [PT][in_dim]
    const int b = blockIdx.y, p0 = blockIdx.x * PT;
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const size_t boff = (size_t)b * Npad * CH;
    for (int e = tid; e < PT * in_dim; e += 256) {
        const int p = e / in_dim;
        cp[e] = (p0 + p < N) ? corr[((size_t)b * N + p0) * in_dim + e] : 0.0f;
    }
    __syncthreads();
    for (int e = tid; e < PT * CH; e += 256) {
        const int p = e / CH, j = e % CH;
        float s = 0.0f;
        for (int c = 0; c < in_dim; ++c) s = __builtin_fmaf(pk[l0w + j * in_dim + c], cp[p * in_dim + c], s);
        X0[p * S132 + j] = s + pk[l0b + j];
    }
    __syncthreads();
    pcn_qkv(X0, X1, pk, d, feat + boff, Q + boff, K + boff, V + boff, p0, tid, wave, lane);
}

// combine partials (rows p0..p0+31) into X (stride S132)
PDSC_DEV void combine_tile(const float *__restrict__ opart, const float *__restrict__ ml, int b,
                           int nsplit, int Npad, int p0, float *X, int tid) {
    const int p = tid >> 3, d0 = (tid & 7) * 16;
    float out[16];
    combine16(opart, ml, b, nsplit, Npad, p0 + p, d0, out);
#pragma unroll
    for (int i = 0; i < 4; ++i)
        *reinterpret_cast<f32x4 *>(X + p * S132 + d0 + 4 * i) =
            f32x4{out[4 * i], out[4 * i + 1], out[4 * i + 2], out[4 * i + 3]};
}

// message MLP + residual: X (msg) -> R (= feat + fc_message(msg)), scratch H1/H2.
PDSC_DEV void message_resid(const float *X, float *H1, float *H2, float *R, const float *__restrict__ pk,
                            const PwMsg &m, const float *__restrict__ feat_rows, int wave, int lane) {
    dense32<CH, CH2, EPI_BN_RELU>(X, S132, pk, m.fc0, H1, S68, nullptr, wave, lane);
    __syncthreads();
    dense32<CH2, CH2, EPI_BN_RELU>(H1, S68, pk, m.fc3, H2, S68, nullptr, wave, lane);
    __syncthreads();
    dense32<CH2, CH, EPI_RESID>(H2, S68, pk, m.fc6, R, S132, feat_rows, wave, lane);
    __syncthreads();
}

__global__ __launch_bounds__(256) void pw_mid_kernel(const float *__restrict__ pk, PwMsg m, PwDense4 d,
                                                     const float *__restrict__ opart,
                                                     const float *__restrict__ ml, int nsplit, int N,
                                                     int Npad, float *__restrict__ feat,
                                                     float *__restrict__ Q, float *__restrict__ K,
                                                     float *__restrict__ V) {
    extern __shared__ __attribute__((aligned(16))) float sm[];
    float *XA = sm, *XB = sm + PT * S132, *H1 = sm + 2 * PT * S132, *H2 = H1 + PT * S68;
    const int b = blockIdx.y, p0 = blockIdx.x * PT;
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const size_t boff = (size_t)b * Npad * CH;
    combine_tile(opart, ml, b, nsplit, Npad, p0, XA, tid);
    __syncthreads();
    message_resid(XA, H1, H2, XB, pk, m, feat + boff + (size_t)p0 * CH, wave, lane);
    pcn_qkv(XB, XA, pk, d, feat + boff, Q + boff, K + boff, V + boff, p0, tid, wave, lane);
}

__global__ __launch_bounds__(256) void pw_last_kernel(
    const float *__restrict__ pk, PwMsg m, DenseOff c0, DenseOff c2, size_t c4w, size_t c4b,
    const float *__restrict__ opart, const float *__restrict__ ml, int nsplit, int N, int Npad,
    const float *__restrict__ feat, float *__restrict__ feat_out, float *__restrict__ normed,
    float *__restrict__ conf) {
    extern __shared__ __attribute__((aligned(16))) float sm[];
    float *XA = sm, *XB = sm + PT * S132, *H1 = sm + 2 * PT * S132, *H2 = H1 + PT * S68;
    float *C1 = H2 + PT * S68, *C2 = C1 + PT * S36;
    const int b = blockIdx.y, p0 = blockIdx.x * PT;
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const size_t boff = (size_t)b * Npad * CH;
    const int nrows = min(PT, N - p0);
    combine_tile(opart, ml, b, nsplit, Npad, p0, XA, tid);
    __syncthreads();
    message_resid(XA, H1, H2, XB, pk, m, feat + boff + (size_t)p0 * CH, wave, lane);
    // XB = corr_features rows
    if (feat_out) store_tile32(XB, S132, feat_out + (size_t)b * N * CH, p0, nrows, tid);
    {   // F.normalize(p=2, dim=-1, eps=1e-12) (:156); 8 lanes per point
        const int p = tid >> 3, d0 = (tid & 7) * 16;
        float ss = 0.0f;
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const float x = XB[p * S132 + d0 + i];
            ss = __builtin_fmaf(x, x, ss);
        }
        ss += __shfl_xor(ss, 1);
        ss += __shfl_xor(ss, 2);
        ss += __shfl_xor(ss, 4);
        const float den = fmaxf(sqrtf(ss), 1e-12f);
        if (p < nrows) {
            float *dst = normed + ((size_t)b * N + p0 + p) * CH + d0;
#pragma unroll
            for (int i = 0; i < 4; ++i)
                *reinterpret_cast<f32x4 *>(dst + 4 * i) =
                    f32x4{XB[p * S132 + d0 + 4 * i] / den, XB[p * S132 + d0 + 4 * i + 1] / den,
                          XB[p * S132 + d0 + 4 * i + 2] / den, XB[p * S132 + d0 + 4 * i + 3] / den};
        }
    }
    // classification MLP 128 -> 32 -> 32 -> 1 on the unnormalised features (:171)
    dense32<CH, CLS, EPI_RELU>(XB, S132, pk, c0, C1, S36, nullptr, wave, lane);
    __syncthreads();
    dense32<CLS, CLS, EPI_RELU>(C1, S36, pk, c2, C2, S36, nullptr, wave, lane);
    __syncthreads();
    if (tid < nrows) {
        float s = 0.0f;
        for (int c = 0; c < CLS; ++c) s = __builtin_fmaf(pk[c4w + c], C2[tid * S36 + c], s);
        conf[(size_t)b * N + p0 + tid] = s + pk[c4b];
    }
}

static PwDense4 dense4(const LayerOff &l) { return PwDense4{l.pcn, l.q, l.k, l.v}; }
static PwMsg msg3(const LayerOff &l) { return PwMsg{l.fc0, l.fc3, l.fc6}; }

hipError_t launch_pw_first(const float *packed, const PackLayout &lay, const float *corr_pos, int B,
                           int N, int Npad, float *feat, float *q, float *k, float *v, hipStream_t s) {
    const size_t lds = (size_t)(2 * PT * S132 + PT * lay.in_dim) * sizeof(float);
    hipLaunchKernelGGL(pw_first_kernel, dim3(Npad / PT, B), dim3(256), lds, s, packed, lay.l0_w,
                       lay.l0_b, dense4(lay.layer[0]), corr_pos, lay.in_dim, N, Npad, feat, q, k, v);
    return hipGetLastError();
}

hipError_t launch_pw_mid(const float *packed, const PackLayout &lay, int layer, const float *opart,
                         const float *ml, int nsplit, int B, int N, int Npad, float *feat, float *q,
                         float *k, float *v, hipStream_t s) {
    const size_t lds = (size_t)(2 * PT * S132 + 2 * PT * S68) * sizeof(float);
    hipLaunchKernelGGL(pw_mid_kernel, dim3(Npad / PT, B), dim3(256), lds, s, packed,
                       msg3(lay.layer[layer]), dense4(lay.layer[layer + 1]), opart, ml, nsplit, N,
                       Npad, feat, q, k, v);
    return hipGetLastError();
}

hipError_t launch_pw_last(const float *packed, const PackLayout &lay, const float *opart,
                          const float *ml, int nsplit, int B, int N, int Npad, const float *feat,
                          float *feat_out, float *normed, float *conf, hipStream_t s) {
    const size_t lds = (size_t)(2 * PT * S132 + 2 * PT * S68 + 2 * PT * S36) * sizeof(float);
    hipLaunchKernelGGL(pw_last_kernel, dim3((N + PT - 1) / PT, B), dim3(256), lds, s, packed,
                       msg3(lay.layer[lay.L - 1]), lay.c0, lay.c2, lay.c4_w, lay.c4_b, opart, ml,
                       nsplit, N, Npad, feat, feat_out, normed, conf);
    return hipGetLastError();
}

}  // namespace pdsc
