// encoder.hip -- a2-a4: SCNonlocal encoder, F.normalize and the classifier.
//
// Replaces models/PointDSC.py:9-77 (NonLocalBlock / NonLocalNet), :155-156 and
// :171.  Layout in HBM (per pair b, N padded to Npad = round_up(N,128) rows):
//   feat          : [B][Npad][128] fp32, point-major (row = correspondence)
//   Qs, Ks, Vs    : the fp16 hi/lo split layouts of attention_h3.hpp (4 B/element)
//   M             : [B][N][N] fp32 (a1 output; symmetric)
//   opart, ml     : [B][nsplit][Npad][128], [B][nsplit][Npad][2] attention partials
//
// Kernels per forward: pw_first (layer0 + PointCN_0 + QKV_0), then per layer
// attention_l (+ pw_mid_l = combine + fc_message_l + residual + PointCN_{l+1}
// + QKV_{l+1}), and pw_last (combine + fc_message + residual + normalize +
// classifier).  The pointwise products run on v_mfma_f32_32x32x16_f16 with the
// 3-product split of attention_h3.hpp (activations split as read from LDS,
// weights pre-split and power-of-two scaled at pack time); their Q/K/V
// epilogues write the fp16 hi/lo splits that the attention consumes.
//
// Attention (attention_h3.hpp; flash-style, never materialising the N x N
// logits): 3 fp16 MFMAs per fp32 product (hi.hi + hi.lo + lo.hi, 22-bit
// operands, fp32 accumulation) -- fp32-equivalent results at 16/3 x the fp32
// matrix rate; logits = M_ij * s_ij / sqrt(C) with M read column-wise (M
// symmetric => coalesced 128-B rows); incompatible pairs keep logit 0 (not
// -inf) exactly as :41; online softmax with a lazily re-based running max;
// split-K over keys when B*N is too small to fill 256 CUs.
#include <cstdlib>

#include "attention.hpp"
#include "attention_h3.hpp"
#include "attention_w64.hpp"

namespace pdsc {

// ============================================================ weight packing
// Per-layer power-of-two scale: max|W| 2^s <= 2^14 keeps hi and (for all but
// the weights 2^-17 below the layer's largest) lo in fp16's normal range.
__global__ __launch_bounds__(256) void wscale_kernel(const float *__restrict__ w, int n, int f32,
                                                     float *__restrict__ sc) {
    __shared__ float part[4];
    if (f32) {  // exact-fp32 weights are stored unscaled
        if (threadIdx.x == 0) sc[0] = sc[1] = 1.0f;
        return;
    }
    float m = 0.0f;
    for (int i = threadIdx.x; i < n; i += 256) m = fmaxf(m, fabsf(w[i]));
    m = wave_max(m);
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) {
        m = fmaxf(fmaxf(part[0], part[1]), fmaxf(part[2], part[3]));
        int ex = 0;
        if (m > 0.0f && m < INFINITY) frexpf(m, &ex);  // m < 2^ex
        const int sh = max(-100, min(100, 14 - ex));
        sc[0] = ldexpf(1.0f, -sh);
        sc[1] = ldexpf(1.0f, sh);
    }
}

// W [out][in] (torch Conv1d weight) -> W_PLANES fp16 planes hi, mid (, lo) of
// W * 2^s ~= hi + mid (22 significant bits; with lo: 33, every fp32 weight
// exactly) in MFMA-fragment blocks (w3_index, pdsc_internal.hpp): block (t, ks)
// = outputs 32t..32t+31 x the 16 inputs of k-step ks, planes of 1 KiB
// each, lane (h, n)'s 16 B = positions 8h .. 8h+7 of output 32t + n in qk_pos
// order (bits 2 and 3 of the input index swapped: inputs {4h..4h+3,
// 8+4h..8+4h+3} of the k-step, exactly the channels a transposed product's
// accumulator half h holds).  Blocks are stored t-major, so any run of
// consecutive blocks is one contiguous copy (f32: W itself, fp32 [out][in]).
// BN folded as torch-CPU eval folds it.
__global__ void pack_dense_kernel(const float *__restrict__ w, const float *__restrict__ b,
                                  const float *__restrict__ bn_w, const float *__restrict__ bn_b,
                                  const float *__restrict__ bn_rm, const float *__restrict__ bn_rv,
                                  int in, int out, int f32, float *__restrict__ dw, float *__restrict__ db,
                                  float *__restrict__ da, float *__restrict__ dbeta,
                                  const float *__restrict__ sc) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    const int total = in * out;
    if (i < total && f32) {
        dw[i] = w[i];
    } else if (i < total) {
        _Float16 *wd = reinterpret_cast<_Float16 *>(dw);
        const int o = i / in, c = i % in;
        float x = w[i] * sc[1];  // exact (power of two)
        asm("" : "+v"(x));       // one hi for both uses (see split_h)
        const _Float16 hi = (_Float16)x;
        const float r1 = x - (float)hi;  // exact
        const _Float16 mid = (_Float16)r1;
        const size_t d = w3_index(o, c, in);
        wd[d] = hi;
        wd[d + 512] = mid;
        if (W_PLANES == 3) wd[d + 1024] = (_Float16)(r1 - (float)mid);
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
                             const float *bn_rm, const float *bn_rv, int in, int out, bool f32, float *dst_w,
                             float *dst_b, float *dst_a, float *dst_beta, float *dst_scale, hipStream_t s) {
    const int n = in * out;
    hipLaunchKernelGGL(wscale_kernel, dim3(1), dim3(256), 0, s, w, n, (int)f32, dst_scale);
    hipLaunchKernelGGL(pack_dense_kernel, dim3((n + 255) / 256), dim3(256), 0, s, w, b, bn_w, bn_b,
                       bn_rm, bn_rv, in, out, (int)f32, dst_w, dst_b, dst_a, dst_beta, dst_scale);
    return hipGetLastError();
}

hipError_t launch_copy(const float *src, float *dst, int n, hipStream_t s) {
    hipLaunchKernelGGL(copy_kernel, dim3((n + 255) / 256), dim3(256), 0, s, src, dst, n);
    return hipGetLastError();
}

// ================================================================= attention
// Production instantiation of attention_h3.hpp: 4 waves x 32 queries per
// workgroup, XCD-aware block map.  (tools/attn_bench.hip A/B-times it against
// the exact-fp32-MFMA kernel of attention.hpp.)
constexpr int ATT_NW = 4;

// Resident workgroups per round of the split-K decomposition (2 per CU on 256
// CUs; attention_split_count).  A/B knob, measurement only: PDSC_ATT_TARGET
// overrides it for the whole process.  (The exact-fp32 attention keeps its
// round-2 rule: splits = ceil(target / blocks).)
static int att_target() {
    static const int t = [] {
        const char *e = getenv("PDSC_ATT_TARGET");
        const int v = e ? atoi(e) : 0;
        return v > 0 ? v : 512;
    }();
    return t;
}
// Waves (x 32 queries) per workgroup of the h3 split-K attention: 4, except 2
// for batches of at most 16 blocks of 128 queries (single pairs up to N = 2048),
// whose launch is latency-bound: twice the query blocks, each workgroup's K/V
// stream shared by 2 waves.  Measured (ms per forward, two A/B rounds on one
// box, profiles/r06_ab_att_nw.log): 1 x 1000 0.4235 -> 0.417, 1 x 2000 0.531 ->
// 0.504, 1 x 5000 (not covered) equal; 1 wave 0.4185 / 0.515.  A/B knob
// PDSC_ATT_NW=1|2|4 (measurement only) sets the small-batch count.
static bool att_tiny(int B, int N);
static int att_nw(int B, int N) {
    static const int v = [] {
        const char *e = getenv("PDSC_ATT_NW");
        const int w = e ? atoi(e) : 2;
        return (w == 1 || w == 2) ? w : ATT_NW;
    }();
    if (att_tiny(B, N)) return 1;
    return (long)B * ((N + QB - 1) / QB) <= 16 ? v : ATT_NW;
}
// The smallest batches (at most 16 query blocks of 128 and splits of <= 24 key
// tiles: a single pair to N = 1536, two to 1024, four to 512): 32-query workgroups whose key splits fill ONE round of
// att_tiny_slots() (128) workgroups (a 1000-key pair: 32 blocks x 4 splits of 8
// tiles, run by attention_h3_ws_kernel's 4 waves) instead of 16 blocks x 16
// splits of 2 -- a quarter of the split partials, so pw_mid combines them
// itself (use_precombine: fewer than 16 splits) and the combine_rows launch goes.
// A/B knob PDSC_ATT_TINY=0 (measurement only).
static int att_tiny_slots();
static bool att_tiny(int B, int N) {
    static const int lim = [] {  // PDSC_ATT_TINY=0: off; =n: up to n blocks of 128 queries (measurement only)
        const char *e = getenv("PDSC_ATT_TINY");
        return e ? atoi(e) : 16;
    }();
    if ((long)B * ((N + QB - 1) / QB) > lim) return false;
    // splits of at most 24 key tiles (6 per wave of the wave-split kernel): ms per
    // forward, 8 -> 16-block limit (profiles/r06_ab_tiny16.log): 2 x 1000 0.431 ->
    // 0.382, 4 x 500 0.374 -> 0.324, 1 x 1500 (24 tiles) 0.456 -> 0.439, but 1 x 2000
    // (32 tiles) 0.489 -> 0.504, which keeps the two-wave split plan
    return attention_h3_grid<1>(B, N, std::min(att_target(), att_tiny_slots())).sps <= 24;
}
// The tiny plan's waves per workgroup splitting each key split's tiles
// (attention_h3_ws_kernel): 4 (default), 2, or 1 = the one-wave kernel.
// A/B knob PDSC_ATT_WS (measurement only).
static int att_ws() {
    static const int v = [] {
        const char *e = getenv("PDSC_ATT_WS");
        const int w = e ? atoi(e) : 4;
        return (w == 1 || w == 2) ? w : 4;
    }();
    return v;
}
// The tiny plan's slot target (one round of this many workgroups): 128 (ms per
// forward, wave-split kernel, profiles/r06_ab_tiny_slots.log: 1 x 1000 0.374 at
// 256 slots -> 0.366 at 128 (4 splits of 8 tiles, 2 per wave; half the partials
// again) -> 0.385 at 96, 0.415 at 64; 2 x 500 0.342 -> 0.316; 1 x 700 0.362 ->
// 0.345).  A/B knob PDSC_ATT_TINY_SLOTS (measurement only).
static int att_tiny_slots() {
    static const int v = [] {
        const char *e = getenv("PDSC_ATT_TINY_SLOTS");
        const int x = e ? atoi(e) : 0;
        return x > 0 ? x : 128;
    }();
    return v;
}
static AttnGridH3 prod_grid(int B, int N) {
    if (att_tiny(B, N)) return attention_h3_grid<1>(B, N, std::min(att_target(), att_tiny_slots()));
    switch (att_nw(B, N)) {
    case 1: return attention_h3_grid<1>(B, N, att_target());
    case 2: return attention_h3_grid<2>(B, N, att_target());
    default: return attention_h3_grid<ATT_NW>(B, N, att_target());
    }
}

// The attention's workgroup order, reversed on alternate layers (fused and
// split-K launches; the stream-K form excepted): a launch
// starts on the pairs whose M (and featL) the previous one read last, while
// they may still sit in the Infinity Cache.  A/B knob PDSC_ZIGZAG=0 (measurement
// only).
static int zigzag_rev(int layer) {
    static const int mode = [] {
        const char *e = getenv("PDSC_ZIGZAG");
        return e ? atoi(e) : 1;
    }();
    return mode == 0 ? 0 : mode == 2 ? !(layer & 1) : (layer & 1);
}

// PDSC_PRECISION_F32: attention.hpp's exact-fp32 MFMA kernel, 32-key stages, libm expf
constexpr int ATT_F32_KTS = 32;
static AttnGrid f32_grid(int B, int N) { return attention_grid<ATT_NW, ATT_F32_KTS>(B, N, att_target()); }

// The 64-query-wave attention (attention_w64.hpp, one 4-wave workgroup per CU,
// symmetric-packed M) for the split path: from 128 blocks of 256 queries
// (8 x 5000: 160 blocks, 3 key splits).  Knob PDSC_W64: 0 never, 1 wherever the
// split path runs (measurement only).
static AttnGridH3 w64_grid(int B, int N) { return attention_w64_grid(B, N, att_target() / 2); }
bool attention_w64(int B, int N, bool f32) {
    static const int mode = [] {
        const char *e = getenv("PDSC_W64");
        return e ? atoi(e) : 2;
    }();
    if (f32 || mode == 0) return false;
    return mode == 1 || (long)B * ((N + W64_QPB - 1) / W64_QPB) >= 128;
}

// Stream-K workgroups for a uniform batch on the w64 path (attention_w64_sk_kernel,
// one per CU), or 0 for the split grid: when one round of nwg workgroups of
// ceil(T / nwg) tiles (+ ~2 tiles for a workgroup's second segment) beats the
// split grid's rounds of sps tiles.  Knob PDSC_W64_SK=0: never (measurement only).
static int w64_sk_wgs(int B, int N) {
    static const int mode = [] {
        const char *e = getenv("PDSC_W64_SK");
        return e ? atoi(e) : 1;
    }();
    if (!mode) return 0;
    const int nwg = att_target() / 2;
    const AttnGridH3 g = w64_grid(B, N);
    const int nst = (N + H3_TILE - 1) / H3_TILE;
    const long T = (long)B * g.nqb * nst, rounds = ((long)B * g.nqb * g.nsplit + nwg - 1) / nwg;
    return T >= 4L * nwg && (T + nwg - 1) / nwg + 2 < rounds * g.sps ? nwg : 0;
}
// the w64 plan's partial slots: the split grid's, or the stream-K segments' if more
static int w64_nsplit(int B, int N) {
    const AttnGridH3 g = w64_grid(B, N);
    const int nwg = w64_sk_wgs(B, N);
    return nwg ? std::max(g.nsplit, w64_sk_nsplit(B, g.nqb, (N + H3_TILE - 1) / H3_TILE, nwg)) : g.nsplit;
}

int attention_nsplit(int B, int N, bool f32, bool w64) {
    return f32 ? f32_grid(B, N).nsplit : (w64 ? w64_nsplit(B, N) : prod_grid(B, N).nsplit);
}

template <int NW>
static hipError_t launch_attention_h3(const _Float16 *qs, const _Float16 *ks, const _Float16 *vs, const float *vexp,
                                      const float *M, bool m_packed, const AttnGridH3 &g, float *opart, float *ml,
                                      hipStream_t s) {
    const dim3 grid(g.B * g.nqb * g.nsplit), block(NW * 64);
    const size_t lds = attention_h3_lds_bytes<NW>();
    if (g.sps >= 3) {  // long splits: the early-issue loop (attention_h3_core's EARLY)
        if (m_packed)
            hipLaunchKernelGGL((attention_h3_kernel<NW, true, true, true>), grid, block, lds, s, qs, ks, vs, vexp, M, g,
                               opart, ml);
        else
            hipLaunchKernelGGL((attention_h3_kernel<NW, true, false, true>), grid, block, lds, s, qs, ks, vs, vexp, M, g,
                               opart, ml);
    } else if (m_packed)
        hipLaunchKernelGGL((attention_h3_kernel<NW, true, true>), grid, block, lds, s, qs, ks, vs, vexp, M, g, opart, ml);
    else
        hipLaunchKernelGGL((attention_h3_kernel<NW, true, false>), grid, block, lds, s, qs, ks, vs, vexp, M, g, opart, ml);
    return hipGetLastError();
}

hipError_t launch_attention(const void *q, const void *k, const void *v, const float *vexp, const float *M,
                            int m_layout, bool w64, bool f32, int B, int N, int Npad, int nsplit, float *opart,
                            float *ml, hipStream_t s, Ragged rg, int layer) {
    const bool m_packed = m_layout == M_PACKED;
    if (w64) {  // attention_w64 (H3 layouts, symmetric-packed M)
        if (f32 || !m_packed) return hipErrorInvalidValue;
        AttnGridH3 g = w64_grid(B, N);
        if (g.Npad != Npad || nsplit != w64_nsplit(B, N)) return hipErrorInvalidValue;
        g.nsplit = nsplit;  // slots past the split grid's own: empty splits (st0 >= st1)
        const int nwg = rg.nv && !rg.eq ? 0 : w64_sk_wgs(B, N);
        if (nwg) {
            hipLaunchKernelGGL((attention_w64_sk_kernel<true>), dim3(nwg), dim3(W64_NW * 64), W64_LDS, s,
                               static_cast<const _Float16 *>(q), static_cast<const _Float16 *>(k),
                               static_cast<const _Float16 *>(v), vexp, M, g, nwg, opart, ml);
            return hipGetLastError();
        }
        g.nv = rg.nv;
        g.po = rg.po;
        g.rev = rg.po ? 0 : zigzag_rev(layer);
        hipLaunchKernelGGL((attention_w64_kernel<true>), dim3(g.B * g.nqb * g.nsplit), dim3(W64_NW * 64), W64_LDS, s,
                           static_cast<const _Float16 *>(q), static_cast<const _Float16 *>(k),
                           static_cast<const _Float16 *>(v), vexp, M, g, opart, ml);
        return hipGetLastError();
    }
    if (f32) {  // fp32 [B][Npad][CH] rows, dense M
        AttnGrid g = f32_grid(B, N);
        g.nv = rg.nv;
        if (m_packed || g.Npad != Npad || g.nsplit != nsplit) return hipErrorInvalidValue;
        const size_t lds = attention_lds_bytes<ATT_NW, ATT_F32_KTS>();
        hipLaunchKernelGGL((attention_kernel_t<ATT_NW, ATT_F32_KTS, false, true>), dim3(g.B * g.nqb * g.nsplit),
                           dim3(ATT_NW * 64), lds, s,
                           static_cast<const float *>(q), static_cast<const float *>(k),
                           static_cast<const float *>(v), M, g, opart, ml);
        return hipGetLastError();
    }
    const _Float16 *qs = static_cast<const _Float16 *>(q), *ks = static_cast<const _Float16 *>(k),
                   *vs = static_cast<const _Float16 *>(v);
    AttnGridH3 g = prod_grid(B, N);
    g.nv = rg.nv;
    g.po = rg.po;
    g.rev = rg.po ? 0 : zigzag_rev(layer);
    if (g.Npad != Npad || g.nsplit != nsplit) return hipErrorInvalidValue;
    const int nw = att_nw(B, N);
    // the tiny plan's tiles spread over the workgroup's waves where each split has
    // at least 4 tiles (measured, ms per forward, 1 -> 4 waves: 1 x 1000 (4 tiles per
    // split) 0.393 -> 0.377; 1 x 700 (2 tiles) 0.366 -> 0.371, 2 x 500 0.347 -> 0.351,
    // so shorter splits keep the one-wave kernel; profiles/r06_ab_att_ws.log)
    if (att_tiny(B, N) && att_ws() > 1 && g.sps >= 4) {
        const dim3 grid(g.B * g.nqb * g.nsplit);
        if (att_ws() == 2) {
            if (m_packed)
                hipLaunchKernelGGL((attention_h3_ws_kernel<2, true>), grid, dim3(128), attention_h3_ws_lds_bytes<2>(), s,
                                   qs, ks, vs, vexp, M, g, opart, ml);
            else
                hipLaunchKernelGGL((attention_h3_ws_kernel<2, false>), grid, dim3(128), attention_h3_ws_lds_bytes<2>(),
                                   s, qs, ks, vs, vexp, M, g, opart, ml);
        } else {
            if (m_packed)
                hipLaunchKernelGGL((attention_h3_ws_kernel<4, true>), grid, dim3(256), attention_h3_ws_lds_bytes<4>(), s,
                                   qs, ks, vs, vexp, M, g, opart, ml);
            else
                hipLaunchKernelGGL((attention_h3_ws_kernel<4, false>), grid, dim3(256), attention_h3_ws_lds_bytes<4>(),
                                   s, qs, ks, vs, vexp, M, g, opart, ml);
        }
        return hipGetLastError();
    }
    if (nw == 1) return launch_attention_h3<1>(qs, ks, vs, vexp, M, m_packed, g, opart, ml, s);
    if (nw == 2) return launch_attention_h3<2>(qs, ks, vs, vexp, M, m_packed, g, opart, ml, s);
    return launch_attention_h3<ATT_NW>(qs, ks, vs, vexp, M, m_packed, g, opart, ml, s);
}

// fp32 rows [B][N][CH] -> [B][Npad][CH] with zero padding rows (the f32 attention's input)
__global__ void pad_rows_kernel(const float *__restrict__ x, int B, int N, int Npad, float *__restrict__ y) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (size_t)B * Npad * CH) return;
    const int c = (int)(i % CH), row = (int)((i / CH) % Npad), b = (int)(i / CH / Npad);
    y[i] = row < N ? x[((size_t)b * N + row) * CH + c] : 0.0f;
}

hipError_t launch_pad_rows(const float *x, int B, int N, int Npad, float *y, hipStream_t s) {
    const size_t n = (size_t)B * Npad * CH;
    hipLaunchKernelGGL(pad_rows_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, x, B, N, Npad, y);
    return hipGetLastError();
}

hipError_t launch_split_qkv(const float *q, const float *k, const float *v, int B, int N, int ld, int Npad,
                            _Float16 *qs, _Float16 *ks, _Float16 *vs, float *vexp, hipStream_t s) {
    const size_t n = (size_t)B * Npad * CH;
    hipLaunchKernelGGL(vexp_kernel, dim3(Npad / H3_TILE, B), dim3(256), 0, s, v, N, ld, Npad, vexp);
    hipLaunchKernelGGL(split_qkv_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, q, k, v, vexp, B, N, ld,
                       Npad, qs, ks, vs);
    return hipGetLastError();
}

// Combine the split partials of one row segment: msg = sum_s O_s e^{m_s-m*} / sum_s l_s e^{m_s-m*}.
// Channels d0 .. d0+15 (d0 % 16 == 0) as 4 runs of 4: opart rows [Npad][CH]
// (F32 attention) or the fragment-block tiling (H3, attention_h3.hpp: run a
// of the 16 sits in block 2 (d0/16) + (a >> 1), lane half a & 1).
// Loads are issued in batches (8 maxima, then 4 splits' m, l and 16 channels)
// before any is used: one L2 round trip per batch instead of one per split
// (the split loop's loads otherwise wait for each other: 10.6 of a single
// N = 1000 pair's 25 us pw_mid launch went to the 16-split combine).  Same
// arithmetic, same order as the one-load-per-split loop.
#ifndef PDSC_C16_ONE
#define PDSC_C16_ONE 8  // A/B build knob (-DPDSC_C16_ONE=0: the chunked loads only)
#endif
constexpr int C16_ONE = PDSC_C16_ONE;  // combine16: up to this many splits in one batch of loads (r06)
template <bool F32>
PDSC_DEV void combine16(const float *__restrict__ opart, const float *__restrict__ ml, int b,
                        int nsplit, int Npad, int row, int d0, float out[16]) {
    const float *mlb = ml + ((size_t)b * nsplit * Npad + row) * 2;  // split s: mlb[s * Npad * 2 + {0, 1}]
    if (nsplit <= C16_ONE) {
        // every split's m, l and 16 channels in ONE batch of loads (one round
        // trip to the partials the attention launch just left in other XCDs'
        // caches, instead of three), the maximum from the loaded m's: the same
        // operations in the same order as the chunked loop below
        f32x2 mlv[C16_ONE > 0 ? C16_ONE : 1];
        f32x4 ov[C16_ONE > 0 ? C16_ONE : 1][4];
#pragma unroll
        for (int j = 0; j < C16_ONE; ++j) {
            if (j < nsplit) {
                const size_t base = (size_t)(b * nsplit + j) * Npad + row;
                mlv[j] = *reinterpret_cast<const f32x2 *>(ml + base * 2);
                const float *ob = opart + (base - row) * CH;
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const size_t o = F32 ? (size_t)row * CH + d0 + 4 * i : h3_opart_off(row, d0 + 4 * i);
                    ov[j][i] = *reinterpret_cast<const f32x4 *>(ob + o);
                }
            }
        }
        float mstar = -INFINITY;
#pragma unroll
        for (int j = 0; j < C16_ONE; ++j)
            if (j < nsplit) mstar = fmaxf(mstar, mlv[j][0]);
        float L = 0.0f;
        f32x4 acc[4] = {};
#pragma unroll
        for (int j = 0; j < C16_ONE; ++j) {
            if (j < nsplit) {
                const float w = expf(mlv[j][0] - mstar);
                L += w * mlv[j][1];
#pragma unroll
                for (int i = 0; i < 4; ++i) acc[i] += w * ov[j][i];
            }
        }
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int e = 0; e < 4; ++e) out[4 * i + e] = acc[i][e] / L;
        return;
    }
    float mstar = -INFINITY;
    for (int s0 = 0; s0 < nsplit; s0 += 8) {
        float mv[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) mv[j] = s0 + j < nsplit ? mlb[(size_t)(s0 + j) * Npad * 2] : -INFINITY;
#pragma unroll
        for (int j = 0; j < 8; ++j) mstar = fmaxf(mstar, mv[j]);
    }
    float L = 0.0f;
    f32x4 acc[4] = {};
    constexpr int SB = 4;
    for (int s0 = 0; s0 < nsplit; s0 += SB) {
        f32x2 mlv[SB];
        f32x4 ov[SB][4];
#pragma unroll
        for (int j = 0; j < SB; ++j) {
            if (s0 + j < nsplit) {
                const size_t base = (size_t)(b * nsplit + s0 + j) * Npad + row;
                mlv[j] = *reinterpret_cast<const f32x2 *>(ml + base * 2);
                const float *ob = opart + (base - row) * CH;
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const size_t o = F32 ? (size_t)row * CH + d0 + 4 * i : h3_opart_off(row, d0 + 4 * i);
                    ov[j][i] = *reinterpret_cast<const f32x4 *>(ob + o);
                }
            }
        }
#pragma unroll
        for (int j = 0; j < SB; ++j) {
            if (s0 + j < nsplit) {
                const float w = expf(mlv[j][0] - mstar);
                L += w * mlv[j][1];
#pragma unroll
                for (int i = 0; i < 4; ++i) acc[i] += w * ov[j][i];
            }
        }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int e = 0; e < 4; ++e) out[4 * i + e] = acc[i][e] / L;
}

template <bool F32>
__global__ __launch_bounds__(256) void attn_combine_kernel(const float *__restrict__ opart,
                                                           const float *__restrict__ ml, int N,
                                                           int Npad, int nsplit,
                                                           float *__restrict__ msg) {
    const int b = blockIdx.y;
    const int row = blockIdx.x * 32 + (threadIdx.x >> 3), d0 = (threadIdx.x & 7) * 16;
    if (row >= N) return;
    float out[16];
    combine16<F32>(opart, ml, b, nsplit, Npad, row, d0, out);
    f32x4 *dst = reinterpret_cast<f32x4 *>(msg + ((size_t)b * N + row) * CH + d0);
#pragma unroll
    for (int i = 0; i < 4; ++i) dst[i] = f32x4{out[4 * i], out[4 * i + 1], out[4 * i + 2], out[4 * i + 3]};
}

hipError_t launch_attn_combine(const float *opart, const float *ml, bool f32, int B, int N, int Npad,
                               int nsplit, float *msg, hipStream_t s) {
    if (f32)
        hipLaunchKernelGGL(attn_combine_kernel<true>, dim3((N + 31) / 32, B), dim3(256), 0, s, opart, ml, N, Npad,
                           nsplit, msg);
    else
        hipLaunchKernelGGL(attn_combine_kernel<false>, dim3((N + 31) / 32, B), dim3(256), 0, s, opart, ml, N, Npad,
                           nsplit, msg);
    return hipGetLastError();
}

// Small batches (many key splits): the split partials combined ahead of the
// pointwise kernel by 32 threads per row (4 channels each), every split's
// loads of a 16-split chunk issued together -- one L2 round trip per chunk
// where combine16 (8 threads per row, 16 channels) needs six for 16 splits --
// and written back as ONE split (m = 0, l = 1) that the pointwise kernel's
// combine16 reads unchanged (w = e^0 = 1, L = 1 l = 1, acc = 1 O, O / 1).  The
// same operations in the same order per channel as combine16: bit-identical.
constexpr int CMB_SB = 16;
__global__ __launch_bounds__(256) void combine_rows_kernel(const float *__restrict__ opart,
                                                           const float *__restrict__ ml, int nsplit, int Npad,
                                                           float *__restrict__ opart1, float *__restrict__ ml1) {
    const int b = blockIdx.y, row = blockIdx.x * 8 + (threadIdx.x >> 5), d0 = 4 * (threadIdx.x & 31);
    if (row >= Npad) return;
    const float *mlb = ml + ((size_t)b * nsplit * Npad + row) * 2;  // split s: mlb[s * Npad * 2 + {0, 1}]
    const size_t oo = h3_opart_off(row, d0);
    float mstar = -INFINITY;
    if (nsplit > CMB_SB) {  // the maxima first when they do not fit one chunk
        for (int s0 = 0; s0 < nsplit; s0 += CMB_SB) {
            float mv[CMB_SB];
#pragma unroll
            for (int j = 0; j < CMB_SB; ++j) mv[j] = s0 + j < nsplit ? mlb[(size_t)(s0 + j) * Npad * 2] : -INFINITY;
#pragma unroll
            for (int j = 0; j < CMB_SB; ++j) mstar = fmaxf(mstar, mv[j]);
        }
    }
    float L = 0.0f;
    f32x4 acc = {};
    for (int s0 = 0; s0 < nsplit; s0 += CMB_SB) {
        f32x2 mlv[CMB_SB];
        f32x4 ov[CMB_SB];
#pragma unroll
        for (int j = 0; j < CMB_SB; ++j) {
            if (s0 + j < nsplit) {
                const size_t base = (size_t)(b * nsplit + s0 + j) * Npad;
                mlv[j] = *reinterpret_cast<const f32x2 *>(ml + (base + row) * 2);
                ov[j] = *reinterpret_cast<const f32x4 *>(opart + base * CH + oo);
            }
        }
        if (nsplit <= CMB_SB) {
#pragma unroll
            for (int j = 0; j < CMB_SB; ++j)
                if (j < nsplit) mstar = fmaxf(mstar, mlv[j][0]);
        }
#pragma unroll
        for (int j = 0; j < CMB_SB; ++j) {
            if (s0 + j < nsplit) {
                const float w = expf(mlv[j][0] - mstar);
                L += w * mlv[j][1];
                acc += w * ov[j];
            }
        }
    }
    const size_t base1 = (size_t)b * Npad;
    *reinterpret_cast<f32x4 *>(opart1 + base1 * CH + oo) = f32x4{acc[0] / L, acc[1] / L, acc[2] / L, acc[3] / L};
    if (d0 == 0) *reinterpret_cast<f32x2 *>(ml1 + (base1 + row) * 2) = f32x2{0.0f, 1.0f};
}

hipError_t launch_combine_rows(const float *opart, const float *ml, int B, int Npad, int nsplit, float *opart1,
                               float *ml1, hipStream_t s) {
    hipLaunchKernelGGL(combine_rows_kernel, dim3((Npad + 7) / 8, B), dim3(256), 0, s, opart, ml, nsplit, Npad, opart1,
                       ml1);
    return hipGetLastError();
}

// ============================================================ pointwise chain
// A workgroup (4 waves) owns PT = 64 points (two 32-row MFMA tiles) held in LDS
// and runs the whole per-point chain between two attention launches.
// Dense layer Y = epi(X W^T + b): A operand = X rows (lane -> point), B operand
// = packed W (one coalesced 1-KiB load per 4 MFMAs).  Wide layers (>= 128
// outputs): each wave owns column tiles and computes BOTH row tiles, so every
// weight fragment feeds two MFMAs; narrow layers (32/64 outputs): one
// (row tile, column tile) per wave so all four waves stay busy.
enum Epi { EPI_BIAS = 0, EPI_RELU = 1, EPI_BN_RELU = 2, EPI_RESID = 3, EPI_RESID_R = 4 };

// ReLU that keeps NaN (torch.relu(nan) = nan; fmaxf(nan, 0) = 0).  The fp16
// range guard relies on it: a 3xfp16 operand beyond fp16's range (hi = inf,
// lo = -inf) makes its contraction NaN, and this carries the NaN on to the
// logits, where select_best_kernel flags the pair (pdsc.h, PDSC_ERR_RANGE)
// instead of a ReLU silently zeroing it.  Same value as fmaxf(x, 0) for every
// non-NaN x (-0 -> +0).  IEEE 754-2019 maximum: one v_maximum3_f32 on gfx950.
PDSC_DEV float relu_nan(float x) { return __builtin_elementwise_maximum(x, 0.0f); }

constexpr int S132 = CH + 4, S68 = CH2 + 4, S36 = CLS + 4;
constexpr int IN_MAX = 16;     // layer0 input width held in registers (pw_first)
constexpr int IN_LIMIT = 128;  // layer0 input width supported (datasets/ThreeDMatch.py:311-315: 70)

// The wave's weight panel for output tile ct.  H3: per 16-input k-step, the hi
// and lo fragments (lane (h, n): inputs 16 ks + 8h .. +7 of output 32 ct + n).
// F32: per 8-input chunk j, lane (h, n) holds inputs 8j + 4h .. +3 of output
// 32 ct + n -- the exact-fp32 MFMA's k-step 4j + e uses input 8j + 4h + e (the
// activations are read with the same map, so the products pair up).
template <int IN, bool F32> struct WPanel;
template <int IN> struct WPanel<IN, false> {
    f16x8 h[IN / 16], m[IN / 16], l[W_PLANES == 3 ? IN / 16 : 1];  // (l: the 3-plane build only)
};
template <int IN> struct WPanel<IN, true> {
    f32x4 w[IN / 8];
};

template <int IN, int OUT, bool F32>
PDSC_DEV void load_wpanel(const float *__restrict__ pk, const DenseOff &off, int ct, int lane, WPanel<IN, F32> &p) {
    if constexpr (F32) {
        const float *W = pk + off.w;
        const size_t rowo = (size_t)(ct * 32 + (lane & 31)) * IN + 4 * (lane >> 5);
#pragma unroll
        for (int j = 0; j < IN / 8; ++j) p.w[j] = *reinterpret_cast<const f32x4 *>(W + rowo + 8 * j);
    } else {
        const _Float16 *W = reinterpret_cast<const _Float16 *>(pk + off.w) + (size_t)ct * (IN / 16) * W3_BLOCK + 8 * lane;
#pragma unroll
        for (int ks = 0; ks < IN / 16; ++ks) {
            p.h[ks] = *reinterpret_cast<const f16x8 *>(W + ks * W3_BLOCK);
            p.m[ks] = *reinterpret_cast<const f16x8 *>(W + ks * W3_BLOCK + 512);
            if constexpr (W_PLANES == 3) p.l[ks] = *reinterpret_cast<const f16x8 *>(W + ks * W3_BLOCK + 1024);
        }
    }
}

// The 8 fp32 activations at positions 8h .. 8h+7 of the k-step starting at x
// (qk_pos order: channels 4h..4h+3 and 8+4h..8+4h+3; LDS, 16-B aligned) ->
// hi / lo fp16 fragments.
PDSC_DEV void split8(const float *x, int h, f16x8 &hi, f16x8 &lo) {
    const f32x4 a = *reinterpret_cast<const f32x4 *>(x + 4 * h), b = *reinterpret_cast<const f32x4 *>(x + 8 + 4 * h);
    const float v[8] = {a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
    split8x(v, hi, lo);
}

// One 32-output tile of Y = epi(X W^T + b) for NRT row tiles.  H3: the fp16
// matrix cores with the 3-product split (attention_h3.hpp), activations split
// as they are read from LDS, weights pre-split and pre-scaled by 2^s (the
// accumulator is scaled back by the exact 2^-s before the bias).  F32: exact
// fp32 MFMA 32x32x2 on the fp32 activations and weights.
template <int IN, int OUT, int EPI, int NRT, bool F32>
PDSC_DEV void dense_tile_w(const float *X, int xstr, const WPanel<IN, F32> &wp, const float *__restrict__ pk,
                           const DenseOff &off, int rt0, int ct, float *Y, int ystr, const float *__restrict__ resid,
                           int lane, const float *rres = nullptr) {
    const int h = lane >> 5, l32 = lane & 31;
    f32x16 acc[NRT];
#pragma unroll
    for (int i = 0; i < NRT; ++i) acc[i] = zero16();
    if constexpr (F32) {
        const float *xp = X + (rt0 * 32 + l32) * xstr + 4 * h;
#pragma unroll
        for (int j = 0; j < IN / 8; ++j) {
#pragma unroll
            for (int i = 0; i < NRT; ++i) {
                const f32x4 xv = *reinterpret_cast<const f32x4 *>(xp + i * 32 * xstr + 8 * j);
#pragma unroll
                for (int e = 0; e < 4; ++e) acc[i] = mfma32(xv[e], wp.w[j][e], acc[i]);
            }
        }
    } else {
        const float *xp = X + (rt0 * 32 + l32) * xstr;
#pragma unroll
        for (int ks = 0; ks < IN / 16; ++ks) {
#pragma unroll
            for (int i = 0; i < NRT; ++i) {
                f16x8 xh, xl;
                split8(xp + i * 32 * xstr + 16 * ks, h, xh, xl);
                acc[i] = mfma_xw3(xh, xl, wp.h[ks], wp.m[ks], wp.l[W_PLANES == 3 ? ks : 0], acc[i]);
            }
        }
    }
    const int j = ct * 32 + l32;
    const float inv = pk[off.scale];
    const float bias = pk[off.bias + j];
    const float al = pk[off.alpha + j], be = pk[off.beta + j];
#pragma unroll
    for (int i = 0; i < NRT; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int row = (rt0 + i) * 32 + acc_row(r, h);
            float y = acc[i][r] * inv + bias;
            if (EPI == EPI_BN_RELU) y = relu_nan(y * al + be);  // eval BN as torch folds it, ReLU
            if (EPI == EPI_RELU) y = relu_nan(y);
            if (EPI == EPI_RESID) y = resid[row * CH + j] + y;      // res = feat + message (:44)
            if (EPI == EPI_RESID_R) y = rres[16 * i + r] + y;       // the same, rows loaded ahead (NRT = 1)
            Y[row * ystr + j] = y;
        }
}

template <int IN, int OUT, int EPI, int NRT, bool F32>
PDSC_DEV void dense_tile(const float *X, int xstr, const float *__restrict__ pk, const DenseOff &off,
                         int rt0, int ct, float *Y, int ystr, const float *__restrict__ resid, int lane) {
    WPanel<IN, F32> wp;  // the wave's whole weight panel, issued up front
    load_wpanel<IN, OUT, F32>(pk, off, ct, lane, wp);
    // keep the scheduler from sinking the loads next to their uses (each would
    // then expose a full L2 round trip per k-step); waits stay counted
    asm volatile("" ::: "memory");
    dense_tile_w<IN, OUT, EPI, NRT, F32>(X, xstr, wp, pk, off, rt0, ct, Y, ystr, resid, lane);
}

// Q/K/V projections (Conv1d 128 -> 128 + bias, :36-38) of the PT-point tile,
// written as fp16 hi/lo splits in the attention_h3 layouts.  Wave `ct` owns
// output channels ct*32..+31 of both 32-point row tiles.
//   SPLIT_Q, SPLIT_K: transposed product (accumulator rows = channels, lane =
//     point), so registers 8s..8s+7 are 8 consecutive qk_pos positions: one
//     16-B store of hi and one of lo per (row tile, s); K chunks swizzled.
//   SPLIT_V: lane = channel, registers 8s..8s+7 = 8 consecutive v_keypos
//     positions of the point tile: 16-B stores into the tile's V planes.
enum SplitMode { SPLIT_Q = 0, SPLIT_K = 1, SPLIT_V = 2 };

// The PT x 128 activation tile split once into hi / lo fp16 in LDS (row r:
// 16 hi chunks of 16 B then 16 lo chunks, chunk c stored at c ^ (r & 15) so a
// fragment read -- 32 rows, one chunk each -- is conflict-free).  Shared by the
// Q, K and V products instead of re-splitting per wave and per product.
constexpr int XS_ROWB = 2 * CH * 2;  // bytes per split row
template <int PTT, int NT = 256>
PDSC_DEV void split_tile(const float *X, int xstr, char *Xs, int tid) {
    constexpr int TPR = NT / PTT, CPT = 16 / TPR;  // threads per row, chunks per thread
    const int r = tid / TPR;
#pragma unroll
    for (int q = 0; q < CPT; ++q) {
        const int c = (tid % TPR) * CPT + q;  // chunk c = positions 8c .. 8c+7 (qk_pos order)
        f16x8 hi, lo;
        split8(X + r * xstr + 16 * (c >> 1), c & 1, hi, lo);
        const int o = r * XS_ROWB + 16 * (c ^ (r & 15));
        *reinterpret_cast<f16x8 *>(Xs + o) = hi;
        *reinterpret_cast<f16x8 *>(Xs + o + CH * 2) = lo;
    }
}

// SPLIT_V also sets the tile exponents vexp[p0/32 + i] (attention_h3.hpp) from
// the max |v| over the 4 waves' channel tiles, exchanged through `red` (LDS,
// 4 * NRT floats no other wave reads at this point; one barrier).
// active = false (8-wave workgroups, SPLIT_V): the wave only joins the barrier.
template <int MODE, int NRT>
PDSC_DEV void dense_split(const char *Xs, const WPanel<CH, false> &wp, const float *__restrict__ pk,
                          const DenseOff &off, int ct, _Float16 *__restrict__ dst, int p0, int lane,
                          float *red = nullptr, float *__restrict__ vexp = nullptr, bool active = true) {
    const int h = lane >> 5, l32 = lane & 31;
    f32x16 acc[NRT];
#pragma unroll
    for (int i = 0; i < NRT; ++i) acc[i] = zero16();
    if (active)
#pragma unroll
    for (int ks = 0; ks < CH / 16; ++ks) {
#pragma unroll
        for (int i = 0; i < NRT; ++i) {
            const int r = 32 * i + l32;
            const char *xr = Xs + r * XS_ROWB + 16 * ((2 * ks + h) ^ (r & 15));
            const f16x8 xh = *reinterpret_cast<const f16x8 *>(xr);
            const f16x8 xl = *reinterpret_cast<const f16x8 *>(xr + CH * 2);
            acc[i] = MODE == SPLIT_V ? mfma_xw3(xh, xl, wp.h[ks], wp.m[ks], wp.l[W_PLANES == 3 ? ks : 0], acc[i])
                                     : mfma_w3x(wp.h[ks], wp.m[ks], wp.l[W_PLANES == 3 ? ks : 0], xh, xl, acc[i]);
        }
    }
    const float inv = pk[off.scale];
    if constexpr (MODE == SPLIT_V) {
        const int c = ct * 32 + l32;
        const float bias = pk[off.bias + c];
        int ev[NRT];
        if (active)
#pragma unroll
        for (int i = 0; i < NRT; ++i) {
            float m = 0.0f;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                acc[i][r] = acc[i][r] * inv + bias;
                m = fmaxf(m, fabsf(acc[i][r]));
            }
            m = wave_max(m);
            if (lane == 0) red[4 * i + ct] = m;
        }
        __syncthreads();
        if (!active) return;
#pragma unroll
        for (int i = 0; i < NRT; ++i) {
            ev[i] = h3_vexp(fmaxf(fmaxf(red[4 * i], red[4 * i + 1]), fmaxf(red[4 * i + 2], red[4 * i + 3])));
            if (ct == 0 && lane == 0) vexp[(p0 >> 5) + i] = (float)ev[i];
        }
#pragma unroll
        for (int i = 0; i < NRT; ++i) {
            _Float16 *tile = dst + (size_t)((p0 >> 5) + i) * H3_TILE_H;
#pragma unroll
            for (int s = 0; s < 2; ++s) {
                f16x8 hi, lo;
#pragma unroll
                for (int e = 0; e < 8; ++e) {
                    _Float16 a, b;
                    split_h(ldexpf(acc[i][8 * s + e], ev[i]), a, b);
                    hi[e] = a;
                    lo[e] = b;
                }
                *reinterpret_cast<f16x8 *>(tile + h3_frag(2 * ct + s, 0, lane)) = hi;
                *reinterpret_cast<f16x8 *>(tile + h3_frag(2 * ct + s, 1, lane)) = lo;
            }
        }
    } else {
        float bias[16];
#pragma unroll
        for (int r = 0; r < 16; ++r) bias[r] = pk[off.bias + ct * 32 + acc_row(r, h)];
#pragma unroll
        for (int i = 0; i < NRT; ++i) {
            _Float16 *tile = dst + (size_t)((p0 >> 5) + i) * H3_TILE_H;
#pragma unroll
            for (int s = 0; s < 2; ++s) {
                f16x8 hi, lo;
#pragma unroll
                for (int e = 0; e < 8; ++e) {
                    _Float16 a, b;
                    const float y = acc[i][8 * s + e] * inv + bias[8 * s + e];
                    split_h(MODE == SPLIT_Q && ATT_QFMA ? y * H3_QSCALE : y, a, b);
                    hi[e] = a;
                    lo[e] = b;
                }
                *reinterpret_cast<f16x8 *>(tile + h3_frag(2 * ct + s, 0, lane)) = hi;
                *reinterpret_cast<f16x8 *>(tile + h3_frag(2 * ct + s, 1, lane)) = lo;
            }
        }
    }
}

// Y = epi(X W^T + b) over a PTT-point tile (PTT/32 row tiles) by 4 waves.
template <int IN, int OUT, int EPI, int PTT, bool F32, int NWV = 4>
PDSC_DEV void dense64(const float *X, int xstr, const float *__restrict__ pk, const DenseOff &off, float *Y,
                      int ystr, const float *__restrict__ resid, int wave, int lane) {
    constexpr int NCT = OUT / 32, NRT = PTT / 32;
    static_assert(NWV == 4 || NRT == 1, "8-wave workgroups take 32-point tiles");
    if constexpr (NCT >= 4) {
        for (int ct = wave; ct < NCT; ct += NWV)
            dense_tile<IN, OUT, EPI, NRT, F32>(X, xstr, pk, off, 0, ct, Y, ystr, resid, lane);
    } else if constexpr (NRT == 2) {
        const int rt = wave & 1, ct = wave >> 1;
        if (ct < NCT) dense_tile<IN, OUT, EPI, 1, F32>(X, xstr, pk, off, rt, ct, Y, ystr, resid, lane);
    } else {
        if (wave < NCT) dense_tile<IN, OUT, EPI, 1, F32>(X, xstr, pk, off, 0, wave, Y, ystr, resid, lane);
    }
}

// Copy a [PT][CH] LDS tile (stride xstr) to global rows [p0, p0 + nrows) (row stride CH).
template <int PTT, int NT = 256>
PDSC_DEV void store_rows(const float *X, int xstr, float *__restrict__ dst, int p0, int nrows, int tid) {
    for (int e = tid; e < PTT * (CH / 4); e += NT) {
        const int p = e / (CH / 4), c4 = e % (CH / 4);
        if (p < nrows)
            *reinterpret_cast<f32x4 *>(dst + (size_t)(p0 + p) * CH + 4 * c4) =
                *reinterpret_cast<const f32x4 *>(X + p * xstr + 4 * c4);
    }
}

struct PwDense4 {  // PointCN + Q/K/V of one layer
    DenseOff pcn, q, k, v;
};
struct PwMsg {  // fc_message of one layer
    DenseOff fc0, fc3, fc6;
};

// LDS: A, B = [PT][S132] (67,584 B -> 2 workgroups per CU).  The fc_message
// hidden tile C [PT][S68] and pw_first's corr_pos tile live in B, which is free
// until the residual add writes it.
template <int PTT> constexpr size_t pw_lds() { return (size_t)(2 * PTT * S132) * sizeof(float); }

// PointCN_l (Xin -> Xout) then Q/K/V_l (Xout -> the attention's input layouts);
// Xout rows -> feat.  Q, K, V point at the pair's buffers: the fp16 hi/lo split
// layouts (H3) or fp32 [Npad][CH] rows (F32, same bytes).
// only = 0 / 1 / 2 (H3): this workgroup writes Q / K / V alone (feat only with
// Q), as pcn_qkv8's `only` (pw_first_kernel's z dimension).
template <int PTT, bool F32>
PDSC_DEV void pcn_qkv(const float *Xin, float *Xout, const float *__restrict__ pk, const PwDense4 &d,
                      float *__restrict__ feat, _Float16 *__restrict__ Q, _Float16 *__restrict__ K,
                      _Float16 *__restrict__ V, float *__restrict__ vexp, int p0, int tid, int wave, int lane,
                      int only = -1) {
    // four 128 -> 128 products with the same wave -> output-tile map (ct = wave):
    // each one's weight panel is fetched while the previous one computes
    WPanel<CH, F32> pa, pb;
    if constexpr (!F32) {
        if (only >= 0) {  // workgroup-uniform
            load_wpanel<CH, CH, F32>(pk, d.pcn, wave, lane, pa);
            load_wpanel<CH, CH, F32>(pk, only == 0 ? d.q : (only == 1 ? d.k : d.v), wave, lane, pb);
            asm volatile("" ::: "memory");
            dense_tile_w<CH, CH, EPI_BN_RELU, PTT / 32, F32>(Xin, S132, pa, pk, d.pcn, 0, wave, Xout, S132, nullptr,
                                                             lane);
            __syncthreads();  // Xout complete; Xin is dead (it now holds the split copy of Xout)
            char *Xs = reinterpret_cast<char *>(const_cast<float *>(Xin));
            split_tile<PTT>(Xout, S132, Xs, tid);
            if (only == 0) store_rows<PTT>(Xout, S132, feat, p0, PTT, tid);
            __syncthreads();
            if (only == 0)
                dense_split<SPLIT_Q, PTT / 32>(Xs, pb, pk, d.q, wave, Q, p0, lane);
            else if (only == 1)
                dense_split<SPLIT_K, PTT / 32>(Xs, pb, pk, d.k, wave, K, p0, lane);
            else
                dense_split<SPLIT_V, PTT / 32>(Xs, pb, pk, d.v, wave, V, p0, lane, Xout, vexp);  // Xout is dead
            return;
        }
    }
    load_wpanel<CH, CH, F32>(pk, d.pcn, wave, lane, pa);
    load_wpanel<CH, CH, F32>(pk, d.q, wave, lane, pb);
    asm volatile("" ::: "memory");
    dense_tile_w<CH, CH, EPI_BN_RELU, PTT / 32, F32>(Xin, S132, pa, pk, d.pcn, 0, wave, Xout, S132, nullptr, lane);
    __syncthreads();  // Xout complete; Xin is dead (H3: it now holds the split copy of Xout)
    CH_STAMP(155);
    if constexpr (F32) {
        float *Qf = reinterpret_cast<float *>(Q) + (size_t)p0 * CH, *Kf = reinterpret_cast<float *>(K) + (size_t)p0 * CH,
              *Vf = reinterpret_cast<float *>(V) + (size_t)p0 * CH;
        load_wpanel<CH, CH, F32>(pk, d.k, wave, lane, pa);
        asm volatile("" ::: "memory");
        store_rows<PTT>(Xout, S132, feat, p0, PTT, tid);
        dense_tile_w<CH, CH, EPI_BIAS, PTT / 32, F32>(Xout, S132, pb, pk, d.q, 0, wave, Qf, CH, nullptr, lane);
        load_wpanel<CH, CH, F32>(pk, d.v, wave, lane, pb);
        asm volatile("" ::: "memory");
        dense_tile_w<CH, CH, EPI_BIAS, PTT / 32, F32>(Xout, S132, pa, pk, d.k, 0, wave, Kf, CH, nullptr, lane);
        dense_tile_w<CH, CH, EPI_BIAS, PTT / 32, F32>(Xout, S132, pb, pk, d.v, 0, wave, Vf, CH, nullptr, lane);
    } else {
        char *Xs = reinterpret_cast<char *>(const_cast<float *>(Xin));
        split_tile<PTT>(Xout, S132, Xs, tid);
        load_wpanel<CH, CH, F32>(pk, d.k, wave, lane, pa);
        asm volatile("" ::: "memory");
        store_rows<PTT>(Xout, S132, feat, p0, PTT, tid);
        __syncthreads();
        CH_STAMP(156);
        dense_split<SPLIT_Q, PTT / 32>(Xs, pb, pk, d.q, wave, Q, p0, lane);
        load_wpanel<CH, CH, F32>(pk, d.v, wave, lane, pb);
        asm volatile("" ::: "memory");
        CH_STAMP(157);
        dense_split<SPLIT_K, PTT / 32>(Xs, pa, pk, d.k, wave, K, p0, lane);
        CH_STAMP(158);
        dense_split<SPLIT_V, PTT / 32>(Xs, pb, pk, d.v, wave, V, p0, lane, Xout, vexp);  // Xout is dead
        CH_STAMP(159);
    }
}

// pcn_qkv for 8-wave workgroups (H3, 32-point tiles; small batches): PointCN on
// waves 0-3, then Q (waves 0-3) and K (waves 4-7) at once, then V (waves 0-3).
// Every output tile is the same dense_tile_w / dense_split code as the 4-wave
// form, so the same bits.  only = 0 / 1 / 2: this workgroup writes Q / K / V
// alone (and feat only for Q): three workgroups per point tile share the
// projections (pw_mid_kernel's z dimension), each streaming 4 of the chain's
// 7 weight panels instead of all 7 -- the single pair's chain is bound by
// each CU streaming its panels.
template <int PTT>
PDSC_DEV void pcn_qkv8(const float *Xin, float *Xout, const float *__restrict__ pk, const PwDense4 &d,
                       float *__restrict__ feat, _Float16 *__restrict__ Q, _Float16 *__restrict__ K,
                       _Float16 *__restrict__ V, float *__restrict__ vexp, int p0, int tid, int wave, int lane,
                       int only = -1) {
    static_assert(PTT == 32, "8-wave chain: 32-point tiles");
    const int w4 = wave & 3;
    const bool lo = wave < 4;
    WPanel<CH, false> pa, pb;
    if (only >= 0) {  // workgroup-uniform
        if (lo) {
            load_wpanel<CH, CH, false>(pk, d.pcn, w4, lane, pa);
            load_wpanel<CH, CH, false>(pk, only == 0 ? d.q : (only == 1 ? d.k : d.v), w4, lane, pb);
        }
        asm volatile("" ::: "memory");
        if (lo) dense_tile_w<CH, CH, EPI_BN_RELU, 1, false>(Xin, S132, pa, pk, d.pcn, 0, w4, Xout, S132, nullptr, lane);
        __syncthreads();  // Xout complete; Xin is dead (it now holds the split copy of Xout)
        CH_STAMP(155);
        char *Xs = reinterpret_cast<char *>(const_cast<float *>(Xin));
        split_tile<PTT, 512>(Xout, S132, Xs, tid);
        if (only == 0) store_rows<PTT, 512>(Xout, S132, feat, p0, PTT, tid);
        __syncthreads();
        CH_STAMP(156);
        CH_STAMP(157);
        CH_STAMP(158);
        if (only == 0) {
            if (lo) dense_split<SPLIT_Q, 1>(Xs, pb, pk, d.q, w4, Q, p0, lane);
        } else if (only == 1) {
            if (lo) dense_split<SPLIT_K, 1>(Xs, pb, pk, d.k, w4, K, p0, lane);
        } else {
            dense_split<SPLIT_V, 1>(Xs, pb, pk, d.v, w4, V, p0, lane, Xout, vexp, lo);  // Xout is dead
        }
        CH_STAMP(159);
        return;
    }
    if (lo) {
        load_wpanel<CH, CH, false>(pk, d.pcn, w4, lane, pa);
        load_wpanel<CH, CH, false>(pk, d.q, w4, lane, pb);
    } else {
        load_wpanel<CH, CH, false>(pk, d.k, w4, lane, pb);
    }
    asm volatile("" ::: "memory");
    if (lo) dense_tile_w<CH, CH, EPI_BN_RELU, 1, false>(Xin, S132, pa, pk, d.pcn, 0, w4, Xout, S132, nullptr, lane);
    __syncthreads();  // Xout complete; Xin is dead (it now holds the split copy of Xout)
    CH_STAMP(155);
    char *Xs = reinterpret_cast<char *>(const_cast<float *>(Xin));
    split_tile<PTT, 512>(Xout, S132, Xs, tid);
    if (lo) load_wpanel<CH, CH, false>(pk, d.v, w4, lane, pa);
    asm volatile("" ::: "memory");
    store_rows<PTT, 512>(Xout, S132, feat, p0, PTT, tid);
    __syncthreads();
    CH_STAMP(156);
    CH_STAMP(157);  // (Q and K run at once: the "k" phase of tools/pw_stamps.py)
    if (lo)
        dense_split<SPLIT_Q, 1>(Xs, pb, pk, d.q, w4, Q, p0, lane);
    else
        dense_split<SPLIT_K, 1>(Xs, pb, pk, d.k, w4, K, p0, lane);
    CH_STAMP(158);
    dense_split<SPLIT_V, 1>(Xs, pa, pk, d.v, w4, V, p0, lane, Xout, vexp, lo);  // Xout is dead
    CH_STAMP(159);
}

// layer0 (Conv1d in_dim -> 128, :54, :73) + PointCN_0 + QKV_0.
template <int PTT, bool F32>
__global__ __launch_bounds__(256, 2) void pw_first_kernel(const float *__restrict__ pk, size_t l0w,
                                                       size_t l0b, PwDense4 d,
                                                       const float *__restrict__ corr, int in_dim,
                                                       int N, int Npad, float *__restrict__ feat,
                                                       _Float16 *__restrict__ Q, _Float16 *__restrict__ K,
                                                       _Float16 *__restrict__ V, float *__restrict__ vexp,
                                                       const int *__restrict__ nv) {
    extern __shared__ __attribute__((aligned(16))) float sm[];
    float *XA = sm, *XB = sm + PTT * S132, *cp = XB;  // cp: [PTT][in_dim], consumed before XB is written
    const int b = blockIdx.y, p0 = blockIdx.x * PTT;
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const size_t boff = (size_t)b * Npad * CH;
    const int n = nv ? nv[b] : N;  // this pair's rows (ragged batches); N: the row stride
    for (int e = tid; e < PTT * in_dim; e += 256) {
        const int p = e / in_dim;
        cp[e] = (p0 + p < n) ? corr[((size_t)b * N + p0) * in_dim + e] : 0.0f;
    }
    // thread -> output channel j (both halves of the block cover rows of opposite parity)
    const int j = tid & (CH - 1), p_off = tid >> 7;
    const float bj = pk[l0b + j];
    if (in_dim <= IN_MAX) {  // the weights in registers
        float w[IN_MAX];
#pragma unroll
        for (int c = 0; c < IN_MAX; ++c) w[c] = (c < in_dim) ? pk[l0w + j * in_dim + c] : 0.0f;
        __syncthreads();
        for (int p = p_off; p < PTT; p += 2) {
            float s = 0.0f;
#pragma unroll
            for (int c = 0; c < IN_MAX; ++c)
                if (c < in_dim) s = __builtin_fmaf(w[c], cp[p * in_dim + c], s);
            XA[p * S132 + j] = s + bj;
        }
    } else {  // wide inputs (in_dim <= IN_LIMIT): the same ascending fma chain, weights from L1
        __syncthreads();
        const float *wj = pk + l0w + (size_t)j * in_dim;
        for (int p = p_off; p < PTT; p += 2) {
            float s = 0.0f;
            for (int c = 0; c < in_dim; ++c) s = __builtin_fmaf(wj[c], cp[p * in_dim + c], s);
            XA[p * S132 + j] = s + bj;
        }
    }
    __syncthreads();
    pcn_qkv<PTT, F32>(XA, XB, pk, d, feat + boff, Q + 2 * boff, K + 2 * boff, V + 2 * boff,
                      vexp + (size_t)b * (Npad / 32), p0, tid, wave, lane, gridDim.z == 3 ? (int)blockIdx.z : -1);
}

// Combine the split partials of rows p0..p0+63 into X (stride S132); 4 threads per row.
template <int PTT, bool F32>
PDSC_DEV void combine_tile(const float *__restrict__ opart, const float *__restrict__ ml, int b,
                           int nsplit, int Npad, int p0, float *X, int tid) {
    constexpr int TPR = 256 / PTT, NH = 8 / TPR;  // threads per row, 16-channel pieces per thread
    const int p = tid / TPR;
#pragma unroll
    for (int half = 0; half < NH; ++half) {
        const int d0 = (tid % TPR) * (16 * NH) + half * 16;
        float out[16];
        combine16<F32>(opart, ml, b, nsplit, Npad, p0 + p, d0, out);
#pragma unroll
        for (int i = 0; i < 4; ++i)
            *reinterpret_cast<f32x4 *>(X + p * S132 + d0 + 4 * i) =
                f32x4{out[4 * i], out[4 * i + 1], out[4 * i + 2], out[4 * i + 3]};
    }
}

// fc_message + residual (:43-44): X = msg (A) -> C -> A (stride S68) -> R (B);
// C may alias R: it is dead once fc3 has read it (barrier before fc6).
template <int PTT, bool F32, int NWV = 4>
PDSC_DEV void message_resid(float *A, float *C, float *R, const float *__restrict__ pk, const PwMsg &m,
                            const float *__restrict__ feat_rows, int wave, int lane) {
    dense64<CH, CH2, EPI_BN_RELU, PTT, F32, NWV>(A, S132, pk, m.fc0, C, S68, nullptr, wave, lane);
    __syncthreads();
    CH_STAMP(152);
    dense64<CH2, CH2, EPI_BN_RELU, PTT, F32, NWV>(C, S68, pk, m.fc3, A, S68, nullptr, wave, lane);
    __syncthreads();
    CH_STAMP(153);
    dense64<CH2, CH, EPI_RESID, PTT, F32, NWV>(A, S68, pk, m.fc6, R, S132, feat_rows, wave, lane);
    __syncthreads();
    CH_STAMP(154);
}

// pw_mid's chain for the 8-wave workgroups of a Q / K / V split (three
// workgroups per 32-point tile, `only` = blockIdx.z), each wave's weight panel
// loaded a phase ahead of its layer instead of at its start (the single pair's
// chain is a sequence of L2 round trips: every layer of the message chain paid
// one before its MFMAs).  Roles: fc0 on waves 4-5 and fc3 on waves 6-7 (panels
// loaded before the combine), fc6 on waves 0-3 (panel and residual rows loaded
// before the combine), PointCN on waves 4-7 (panel loaded once fc0 / fc3 are
// done, during fc6), the projection on waves 0-3 (panel loaded after fc6,
// during PointCN).  Every output tile is the same dense_tile_w / dense_split
// arithmetic as message_resid + pcn_qkv8: the same bits.
PDSC_DEV void mid_split8(float *XA, float *XB, const float *__restrict__ pk, const PwMsg &m, const PwDense4 &d,
                         const float *__restrict__ opart, const float *__restrict__ ml, int b, int nsplit, int Npad,
                         int p0, const float *__restrict__ feat_rows, float *__restrict__ feat,
                         _Float16 *__restrict__ Q, _Float16 *__restrict__ K, _Float16 *__restrict__ V,
                         float *__restrict__ vexp, int only, int tid, int wave, int lane) {
    constexpr int PTT = 32;
    float *XC = XB;
    const int w4 = wave & 3, h = lane >> 5, l32 = lane & 31;
    WPanel<CH, false> pa;   // fc0 (waves 4-5), then PointCN (waves 4-7) / the projection (waves 0-3)
    WPanel<CH2, false> pb;  // fc3 (waves 6-7) / fc6 (waves 0-3)
    float res[16];          // fc6's residual rows (waves 0-3)
    if (wave >= 6)
        load_wpanel<CH2, CH2, false>(pk, m.fc3, wave - 6, lane, pb);
    else if (wave >= 4)
        load_wpanel<CH, CH2, false>(pk, m.fc0, wave - 4, lane, pa);
    asm volatile("" ::: "memory");
    if (tid < 256) {
        combine_tile<PTT, false>(opart, ml, b, nsplit, Npad, p0, XA, tid);
        // (after the combine: its loads and these do not share the register file)
        load_wpanel<CH2, CH, false>(pk, m.fc6, wave, lane, pb);
#pragma unroll
        for (int r = 0; r < 16; ++r) res[r] = feat_rows[acc_row(r, h) * CH + wave * 32 + l32];
    }
    asm volatile("" ::: "memory");
    __syncthreads();
    CH_STAMP(151);
    if (wave == 4 || wave == 5)  // fc0: XA -> XC
        dense_tile_w<CH, CH2, EPI_BN_RELU, 1, false>(XA, S132, pa, pk, m.fc0, 0, wave - 4, XC, S68, nullptr, lane);
    __syncthreads();
    CH_STAMP(152);
    if (wave >= 4) load_wpanel<CH, CH, false>(pk, d.pcn, w4, lane, pa);  // (waves 4-5 are done with fc0's)
    asm volatile("" ::: "memory");
    if (wave >= 6)  // fc3: XC -> XA
        dense_tile_w<CH2, CH2, EPI_BN_RELU, 1, false>(XC, S68, pb, pk, m.fc3, 0, wave - 6, XA, S68, nullptr, lane);
    __syncthreads();
    CH_STAMP(153);
    if (wave < 4)  // fc6 + residual: XA -> XB
        dense_tile_w<CH2, CH, EPI_RESID_R, 1, false>(XA, S68, pb, pk, m.fc6, 0, wave, XB, S132, nullptr, lane, res);
    __syncthreads();
    CH_STAMP(154);
    if (wave < 4) load_wpanel<CH, CH, false>(pk, only == 0 ? d.q : (only == 1 ? d.k : d.v), wave, lane, pa);
    asm volatile("" ::: "memory");
    if (wave >= 4)  // PointCN: XB -> XA
        dense_tile_w<CH, CH, EPI_BN_RELU, 1, false>(XB, S132, pa, pk, d.pcn, 0, w4, XA, S132, nullptr, lane);
    __syncthreads();  // XA complete; XB is dead (it now holds the split copy of XA)
    CH_STAMP(155);
    char *Xs = reinterpret_cast<char *>(XB);
    split_tile<PTT, 512>(XA, S132, Xs, tid);
    if (only == 0) store_rows<PTT, 512>(XA, S132, feat, p0, PTT, tid);
    __syncthreads();
    CH_STAMP(156);
    CH_STAMP(157);
    CH_STAMP(158);
    if (only == 0) {
        if (wave < 4) dense_split<SPLIT_Q, 1>(Xs, pa, pk, d.q, wave, Q, p0, lane);
    } else if (only == 1) {
        if (wave < 4) dense_split<SPLIT_K, 1>(Xs, pa, pk, d.k, wave, K, p0, lane);
    } else {
        dense_split<SPLIT_V, 1>(Xs, pa, pk, d.v, w4, V, p0, lane, XA, vexp, wave < 4);  // XA is dead
    }
    CH_STAMP(159);
}

// A/B knob (measurement only): PDSC_PW_PREFETCH=0 runs the Q / K / V split
// chain without the panel prefetch (message_resid + pcn_qkv8).
static bool pw_prefetch_on() {
    static const bool off = [] {
        const char *e = getenv("PDSC_PW_PREFETCH");
        return e && e[0] == '0';
    }();
    return !off;
}

template <int PTT, bool F32, int NWV = 4>
__global__ __launch_bounds__(NWV * 64, NWV == 4 ? 2 : 1) void pw_mid_kernel(const float *__restrict__ pk, PwMsg m, PwDense4 d,
                                                     const float *__restrict__ opart,
                                                     const float *__restrict__ ml, int nsplit, int N,
                                                     int Npad, const float *__restrict__ feat_in,
                                                     float *__restrict__ feat,
                                                     _Float16 *__restrict__ Q, _Float16 *__restrict__ K,
                                                     _Float16 *__restrict__ V, float *__restrict__ vexp,
                                                     int diag_delay, int prefetch) {
    // feat_in != feat: with gridDim.z == 3 the three workgroups of a point tile
    // read feat_in's rows as fc6's residual while the z = 0 one writes feat
    extern __shared__ __attribute__((aligned(16))) float sm[];
    float *XA = sm, *XB = sm + PTT * S132, *XC = XB;
    const int b = blockIdx.y, p0 = blockIdx.x * PTT;
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    // diagnostic (PDSC_DIAG_QKV_DELAY, tests only): the K / V workgroups start
    // late, after the Q one has stored its PointCN rows
    if (diag_delay > 0 && blockIdx.z != 0)
        for (int i = 0; i < diag_delay; ++i) __builtin_amdgcn_s_sleep(127);
    const size_t boff = (size_t)b * Npad * CH;
#ifdef ATT_STAMPS
    unsigned long long *stp = att_stamp_ptr(wave);
    ATT_RSTAMP(stp, 186);
    ATT_STAMP(stp, 150);
#endif
    if constexpr (NWV == 8 && PTT == 32 && !F32) {
        if (prefetch && gridDim.z == 3) {  // workgroup-uniform
            mid_split8(XA, XB, pk, m, d, opart, ml, b, nsplit, Npad, p0, feat_in + boff + (size_t)p0 * CH, feat + boff,
                       Q + 2 * boff, K + 2 * boff, V + 2 * boff, vexp + (size_t)b * (Npad / 32), (int)blockIdx.z, tid,
                       wave, lane);
            ATT_RSTAMP(stp, 187);
            return;
        }
    }
    if (tid < 256) combine_tile<PTT, F32>(opart, ml, b, nsplit, Npad, p0, XA, tid);
    __syncthreads();
    ATT_STAMP(stp, 151);
    message_resid<PTT, F32, NWV>(XA, XC, XB, pk, m, feat_in + boff + (size_t)p0 * CH, wave, lane);
    if constexpr (NWV == 8)
        pcn_qkv8<PTT>(XB, XA, pk, d, feat + boff, Q + 2 * boff, K + 2 * boff, V + 2 * boff,
                      vexp + (size_t)b * (Npad / 32), p0, tid, wave, lane, gridDim.z == 3 ? (int)blockIdx.z : -1);
    else
        pcn_qkv<PTT, F32>(XB, XA, pk, d, feat + boff, Q + 2 * boff, K + 2 * boff, V + 2 * boff,
                          vexp + (size_t)b * (Npad / 32), p0, tid, wave, lane);
    ATT_RSTAMP(stp, 187);
}

template <int PTT, bool F32>
__global__ __launch_bounds__(256, 2) void pw_last_kernel(
    const float *__restrict__ pk, PwMsg m, DenseOff c0, DenseOff c2, size_t c4w, size_t c4b,
    const float *__restrict__ opart, const float *__restrict__ ml, int nsplit, int N, int Npad,
    const float *__restrict__ feat, float *__restrict__ feat_out, float *__restrict__ normed,
    _Float16 *__restrict__ normed_s, float *__restrict__ conf) {
    extern __shared__ __attribute__((aligned(16))) float sm[];
    float *XA = sm, *XB = sm + PTT * S132, *XC = XB;
    float *C1 = XA, *C2 = XA + PTT * S36;  // classifier hidden layers reuse A
    const int b = blockIdx.y, p0 = blockIdx.x * PTT;
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const size_t boff = (size_t)b * Npad * CH;
    const int nrows = min(PTT, N - p0);
    combine_tile<PTT, F32>(opart, ml, b, nsplit, Npad, p0, XA, tid);
    __syncthreads();
    message_resid<PTT, F32>(XA, XC, XB, pk, m, feat + boff + (size_t)p0 * CH, wave, lane);
    // XB = corr_features rows
    if (feat_out) store_rows<PTT>(XB, S132, feat_out + (size_t)b * N * CH, p0, nrows, tid);
    {   // F.normalize(p=2, dim=-1, eps=1e-12) (:156); LPP lanes per point
        constexpr int LPP = 256 / PTT, CPL = CH / LPP;  // lanes per point, channels per lane
        const int p = tid / LPP, d0 = (tid % LPP) * CPL;
        float ss = 0.0f;
#pragma unroll
        for (int i = 0; i < CPL; ++i) {
            const float x = XB[p * S132 + d0 + i];
            ss = __builtin_fmaf(x, x, ss);
        }
#pragma unroll
        for (int o = 1; o < LPP; o <<= 1) ss += __shfl_xor(ss, o);
        const float den = fmaxf(sqrtf(ss), 1e-12f);
        if (p < nrows) {
            float *dst = normed + ((size_t)b * N + p0 + p) * CH + d0;
#pragma unroll
            for (int i = 0; i < CPL / 4; ++i)
                *reinterpret_cast<f32x4 *>(dst + 4 * i) =
                    f32x4{XB[p * S132 + d0 + 4 * i] / den, XB[p * S132 + d0 + 4 * i + 1] / den,
                          XB[p * S132 + d0 + 4 * i + 2] / den, XB[p * S132 + d0 + 4 * i + 3] / den};
            if (!F32 && normed_s) {  // the fp16 hi/lo split copy (qk_pos order) the H3 seed kNN consumes
                _Float16 *ds = normed_s + ((size_t)b * N + p0 + p) * 2 * CH;
#pragma unroll
                for (int q = 0; q < CPL / 8; ++q) {
                    f16x8 hi, lo;
#pragma unroll
                    for (int e = 0; e < 8; ++e) {
                        _Float16 a, c;
                        split_h(XB[p * S132 + qk_pos(d0 + 8 * q + e)] / den, a, c);
                        hi[e] = a;
                        lo[e] = c;
                    }
                    *reinterpret_cast<f16x8 *>(ds + d0 + 8 * q) = hi;
                    *reinterpret_cast<f16x8 *>(ds + CH + d0 + 8 * q) = lo;
                }
            }
        }
    }
    // classification MLP 128 -> 32 -> 32 -> 1 on the unnormalised features (:171)
    dense64<CH, CLS, EPI_RELU, PTT, F32>(XB, S132, pk, c0, C1, S36, nullptr, wave, lane);
    __syncthreads();
    dense64<CLS, CLS, EPI_RELU, PTT, F32>(C1, S36, pk, c2, C2, S36, nullptr, wave, lane);
    __syncthreads();
    if (tid < nrows) {
        float s = 0.0f;
        for (int c = 0; c < CLS; ++c) s = __builtin_fmaf(pk[c4w + c], C2[tid * S36 + c], s);
        conf[(size_t)b * N + p0 + tid] = s + pk[c4b];
    }
}

// ============================================== pw2: register-chained pointwise chain
// The large-launch form of pw_first / pw_mid / pw_last (H3 precision).  A
// workgroup is PW2_W waves; wave w owns the 32 consecutive points p0 + 32 w ..
// +31 (lane l32 <-> point: one MFMA tile) and carries their whole per-point
// chain in registers.  Dense layers run transposed, Y^T = W X^T (A = weights,
// B = activations): accumulator register r of lane (h, l32) of output tile t is
// channel 32 t + acc_row(r, h) of point l32, and registers 8u .. 8u+7 of tile t
// are exactly the fragment of k-step 2t + u that the next layer's B operand
// takes (inputs in qk_pos order -- the packed weights' order), so layers chain
// with no data movement between lanes.  V runs untransposed (A = activations,
// B = weights) to come out in the attention's V-tile layout.
//
// Weights: the kernel's layers are cut into chunks of <= PW2_CB weight blocks
// (w3_index: one block = 32 outputs x 16 inputs x W_PLANES planes of 1 KiB,
// contiguous per chunk), listed in consumption order by the host (W2Sched).
// Chunks are copied into a 2-slot LDS ring by LDS-DMA and shared by the
// workgroup's waves: right after the barrier that retires chunk c, chunk c + 2
// is queued into the slot c just freed -- before any epilogue work -- so the
// barrier at the end of chunk c + 1 waits only for that DMA (vmcnt counts the
// epilogue's later stores out), and no store is ever waited for.  Per-channel
// epilogue coefficients (bias, BN alpha / beta) sit in LDS for the launch.
// Two workgroups per CU (~55 KiB of LDS and <= 256 VGPRs each) overlap one's
// HBM phases and epilogues with the other's MFMAs.
#ifndef PW2_WAVES
#define PW2_WAVES 4
#endif
// The fused kernels' attention with attention_h3_core's early-issue loop
// (measured, one box: 128 x 1000 forward 3.802 vs 3.831 ms over three A/B
// pairs, attn_pw2 290.3 vs 291.7 us; ragged 4.51 vs 4.58 ms).  A/B build
// -DPW2_EARLY=0: the plain loop.
#ifndef PW2_EARLY
#define PW2_EARLY 1
#endif
constexpr int PW2_W = PW2_WAVES;                      // waves per workgroup (32 points each)
constexpr int PW2_OCC = PW2_W >= 8 ? 1 : 2;           // workgroups per CU (<= 256 VGPRs: 2 waves per SIMD)
// 16 two-plane blocks = 32 KiB chunks (r04, A/B: -0.7 % per step at 128 x 1000
// against 8, equal at 8 x 5000 and one pair): half the chunk barriers per chain
#ifndef PW2_CHUNK_BLOCKS
#define PW2_CHUNK_BLOCKS 16
#endif
constexpr int PW2_CB = PW2_CHUNK_BLOCKS;              // blocks per chunk (W_PLANES KiB each)
constexpr int PW2_BLKB = W_PLANES * 1024;             // bytes per block (W_PLANES planes)
constexpr int PW2_SLOT = PW2_CB * PW2_BLKB;
constexpr int PW2_PTS = PW2_W * 32;
constexpr int PW2_COEF = 1536;                        // floats of epilogue coefficients in LDS
constexpr int PW2_NSLOT = 2;                          // weight-ring slots
constexpr size_t PW2_LDS = PW2_NSLOT * PW2_SLOT + PW2_COEF * sizeof(float);
constexpr int W2_MAXCH = 24;

struct W2Sched {                 // chunk c: np[c] pieces of 1 KiB starting at pk-halfs off[c]
    uint32_t off[W2_MAXCH];
    int32_t np[W2_MAXCH];
    int32_t n;
};

// output tiles per chunk of an IN -> OUT layer
constexpr int w2_nt(int in, int out) {
    return PW2_CB / (in / 16) < 1 ? 1 : (PW2_CB / (in / 16) < out / 32 ? PW2_CB / (in / 16) : out / 32);
}

// Host: append a layer's chunks to the schedule (same cut as w2_layer).
static void w2_sched_add(W2Sched &S, const DenseOff &o, int in, int out) {
    const int nks = in / 16, nt = w2_nt(in, out);
    for (int c = 0; c < out / 32 / nt; ++c) {
        S.off[S.n] = (uint32_t)(2 * o.w + (size_t)c * nt * nks * W3_BLOCK);
        S.np[S.n] = W_PLANES * nt * nks;
        ++S.n;
    }
}

// LDS-DMA of chunk c into `slot` (nothing past the schedule): piece i = 1 KiB =
// one wave instruction, lane-linear on both sides.
PDSC_DEV void w2_stage(const float *pk, const W2Sched &S, int c, char *slot, int wave, int lane) {
    if (c >= S.n) return;
#if ATT_BUFDMA
    // the piece's offset in the SGPR operand: no per-piece address VALU
    const __amdgpu_buffer_rsrc_t r = h3_rsrc(pk, 0xFFFFFFFFu);
    for (int i = wave; i < S.np[c]; i += PW2_W)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void *)(slot + 1024 * i), 16,
                                                 16 * lane, (int)(2 * S.off[c]) + 1024 * i, 0, 0);
#else
    const _Float16 *src = reinterpret_cast<const _Float16 *>(pk) + S.off[c] + 8 * lane;
    for (int i = wave; i < S.np[c]; i += PW2_W)
        __builtin_amdgcn_global_load_lds(src + 512 * i, slot + 1024 * i, 16, 0, 0);
#endif
}

struct W2Pipe {
    char *base;
    int c;  // chunk being multiplied
    PDSC_DEV char *slot(int k) const { return base + (k % PW2_NSLOT) * PW2_SLOT; }
};

// End of a chunk: this wave's DMA of the next chunk has landed (all but its
// NST youngest vector-memory ops -- the stores issued after that DMA -- are
// done) and its LDS reads have returned, then the barrier.
template <int NST>
PDSC_DEV void w2_sync(bool active) {
    if (NST > 0 && active)
        asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" ::"n"(NST) : "memory");
    else
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

PDSC_DEV void w2_frag(const char *bp, f16x8 (&w)[3]) {
    w[0] = *reinterpret_cast<const f16x8 *>(bp);
    w[1] = *reinterpret_cast<const f16x8 *>(bp + 1024);
    if constexpr (W_PLANES == 3) w[2] = *reinterpret_cast<const f16x8 *>(bp + 2048);
}

// acc[t0 + t] += W_t X over the chunk's NT tiles x NKS k-steps (TRANS: A = W,
// B = X).  The fragments of block j + 2 are read while block j's MFMAs run (a
// ring of three register sets with compile-time indices); sched_barrier(0)
// pins that order (left alone, the scheduler sinks every read next to its
// MFMA and exposes the LDS latency each time).
template <int NKS, int NT, bool TRANS, int NACC>
PDSC_DEV void w2_mma(const char *slot, const f16x8 *xh, const f16x8 *xl, f32x16 (&acc)[NACC], int t0, int lane) {
    constexpr int NB = NT * NKS;
    const char *bp = slot + 16 * lane;
    f16x8 w[3][3];
    w2_frag(bp, w[0]);
    if (NB > 1) w2_frag(bp + PW2_BLKB, w[1]);
#pragma unroll
    for (int j = 0; j < NB; ++j) {
        if (j + 2 < NB) w2_frag(bp + (j + 2) * PW2_BLKB, w[(j + 2) % 3]);
        const int t = j / NKS, ks = j % NKS;
        const f16x8(&f)[3] = w[j % 3];
        const f32x16 c = ks == 0 ? zero16() : acc[t0 + t];  // k-step 0 starts from the inline-constant 0
        acc[t0 + t] = TRANS ? mfma_w3x(f[0], f[1], f[2], xh[ks], xl[ks], c) : mfma_xw3(xh[ks], xl[ks], f[0], f[1], f[2], c);
        __builtin_amdgcn_sched_barrier(0);
    }
}

// One dense layer IN -> OUT.  Per chunk: multiply, sync (NST: the stores the
// caller issued since the previous barrier), queue chunk + 2 into the slot just
// retired.
template <int IN, int OUT, bool TRANS, int NST = 0>
PDSC_DEV void w2_layer(W2Pipe &P, const float *pk, const W2Sched &S, const f16x8 *xh, const f16x8 *xl,
                       f32x16 (&acc)[OUT / 32], bool active, int wave, int lane) {
    constexpr int NKS = IN / 16, NT = w2_nt(IN, OUT), NCH = OUT / 32 / NT;
    static_assert(NCH * NT == OUT / 32, "chunk tiling");
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
        CH_STAMP(192 + 3 * min(P.c, 20));  // (diagnostic build: chunk P.c's MFMAs, its sync, tools/att_stamps.py)
        if (active) w2_mma<NKS, NT, TRANS>(P.slot(P.c), xh, xl, acc, c * NT, lane);
        CH_STAMP(193 + 3 * min(P.c, 20));
        if (c == 0)
            w2_sync<NST>(active);
        else
            w2_sync<0>(active);
        CH_STAMP(194 + 3 * min(P.c, 20));
        w2_stage(pk, S, P.c + PW2_NSLOT, P.slot(P.c), wave, lane);
        asm volatile("" ::: "memory");
        ++P.c;
    }
}

// The epilogue coefficients (bias, alpha, beta: 3 * out contiguous floats from
// DenseOff::bias) of one layer into LDS at `dst`.
PDSC_DEV void w2_coef(float *dst, const float *__restrict__ pk, const DenseOff &o, int out, int tid) {
    for (int i = tid; i < 3 * out; i += PW2_W * 64) dst[i] = pk[o.bias + i];
}

// fp32 -> fp16 hi / lo of 8 values
PDSC_DEV void split8v(const float (&v)[8], f16x8 &hi, f16x8 &lo) { split8x(v, hi, lo); }

// Channel of register 8u + e of output tile t for lane half h (transposed layout).
PDSC_DEV int w2_chan(int t, int u, int e, int h) { return 32 * t + 16 * u + 8 * (e >> 2) + 4 * h + (e & 3); }

// Epilogue of a transposed layer: y = epi(acc 2^-s + b) (EPI_BIAS / RELU /
// BN_RELU, as dense_tile_w; EPI_RESID adds resid[t][r]) back into acc, and
// (SPLIT) the hi / lo split of every k-step fragment into xh / xl.  cf = the
// layer's LDS coefficients (bias[out], alpha[out], beta[out]).  SPLIT is a
// compile-time flag: a run-time null test of xh would keep the caller's arrays
// out of registers.
template <int OUT, int EPI, bool SPLIT = true>
PDSC_DEV void w2_epilogue(f32x16 (&acc)[OUT / 32], float inv, const float *cf, const f32x16 *resid, f16x8 *xh,
                          f16x8 *xl, int lane) {
    const int h = lane >> 5;
#pragma unroll
    for (int t = 0; t < OUT / 32; ++t)
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const int c0 = 32 * t + 16 * u + 4 * h;
            const f32x4 b0 = *reinterpret_cast<const f32x4 *>(cf + c0), b1 = *reinterpret_cast<const f32x4 *>(cf + c0 + 8);
            f32x4 a0, a1, e0, e1;
            if (EPI == EPI_BN_RELU) {
                a0 = *reinterpret_cast<const f32x4 *>(cf + OUT + c0);
                a1 = *reinterpret_cast<const f32x4 *>(cf + OUT + c0 + 8);
                e0 = *reinterpret_cast<const f32x4 *>(cf + 2 * OUT + c0);
                e1 = *reinterpret_cast<const f32x4 *>(cf + 2 * OUT + c0 + 8);
            }
            float v[8];
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                const int r = 8 * u + e;
                float y = __builtin_fmaf(acc[t][r], inv, e < 4 ? b0[e] : b1[e - 4]);  // exact acc 2^-s, one rounding
                if (EPI == EPI_BN_RELU) y = relu_nan(y * (e < 4 ? a0[e] : a1[e - 4]) + (e < 4 ? e0[e] : e1[e - 4]));
                if (EPI == EPI_RELU) y = relu_nan(y);
                if (EPI == EPI_RESID) y = resid[t][r] + y;  // res = feat + message (:44)
                acc[t][r] = y;
                v[e] = y;
            }
            if constexpr (SPLIT) split8v(v, xh[2 * t + u], xl[2 * t + u]);
        }
}

// Combine the split partials of this lane's point into the k-step fragments of
// the 128 message channels (as combine16: sum_s w_s O_s / sum_s w_s l_s).  The
// partials are in the fragment-block tiling (attention_h3.hpp): k-step ks is
// blocks 2 ks and 2 ks + 1 at this lane, 16 coalesced 1-KiB loads per split.
PDSC_DEV void w2_combine(const float *__restrict__ opart, const float *__restrict__ ml, int b, int nsplit, int Npad,
                         int row, f16x8 *xh, f16x8 *xl, int lane) {
    float mstar = -INFINITY;
    for (int s = 0; s < nsplit; ++s) mstar = fmaxf(mstar, ml[((size_t)(b * nsplit + s) * Npad + row) * 2]);
    float L = 0.0f;
    f32x4 acc[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[i] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
    // (r06: both splits of a pair issued before either is used measured no
    // faster at 8 x 5000, 4.34 vs 4.33 ms per forward: not kept)
    for (int s = 0; s < nsplit; ++s) {
        const size_t base = (size_t)(b * nsplit + s) * Npad + row;
        const float ms = ml[base * 2];
        // an empty split (m = -inf: past a ragged pair's keys, or a stream-K slot past
        // the block's segments, attention_w64.hpp) has w = 0: its O is not read
        // (uniform over the wave's 32 rows, which share one query block)
        if (ms == -INFINITY) continue;
        const float w = expf(ms - mstar);
        L += w * ml[base * 2 + 1];
        const float *src = opart + (base - (row & 31)) * CH + 4 * lane;  // the tile's first block
#pragma unroll
        for (int i = 0; i < 16; ++i) acc[i] += w * *reinterpret_cast<const f32x4 *>(src + 256 * i);
    }
    const float rl = 1.0f / L;  // the softmax denominator once (the reference divides e by its sum first)
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) {
        float v[8];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            v[e] = acc[2 * ks][e] * rl;
            v[4 + e] = acc[2 * ks + 1][e] * rl;
        }
        split8v(v, xh[ks], xl[ks]);
    }
}

// The O^T accumulators of the attention core -> the message's k-step fragments
// (msg = O / l; registers 8u .. 8u+7 of tile t = k-step 2t + u).
PDSC_DEV void w2_msg_frags(const f32x16 (&O)[4], float l_run, f16x8 *xh, f16x8 *xl) {
    const float rl = 1.0f / l_run;
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) {
        float v[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = O[ks >> 1][8 * (ks & 1) + e] * rl;
        split8v(v, xh[ks], xl[ks]);
    }
}

// This lane's 64 fp32 values of a 128-channel row.  featL keeps the lane-register
// order of a transposed 128-output layer in the fragment-block tiling of the
// attention partials (per 32-row tile, block 4t + q = registers 4q .. 4q+3 of
// tile t for the 64 lanes): 16 coalesced 1-KiB accesses each way.
PDSC_DEV void w2_load_row(const float *__restrict__ featL, int row, int lane, f32x16 (&y)[4]) {
    const f32x4 *src = reinterpret_cast<const f32x4 *>(featL + (size_t)(row >> 5) * (32 * CH)) + lane;
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const f32x4 v = src[64 * (4 * t + q)];
#pragma unroll
            for (int e = 0; e < 4; ++e) y[t][4 * q + e] = v[e];
        }
}
PDSC_DEV void w2_store_row(float *__restrict__ featL, int row, int lane, const f32x16 (&y)[4]) {
    f32x4 *dst = reinterpret_cast<f32x4 *>(featL + (size_t)(row >> 5) * (32 * CH)) + lane;
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int q = 0; q < 4; ++q) dst[64 * (4 * t + q)] = f32x4{y[t][4 * q], y[t][4 * q + 1], y[t][4 * q + 2], y[t][4 * q + 3]};
}

// Q / K outputs (transposed, bias only) in the attention_h3 fragment-block
// tiling: registers 8u .. 8u+7 of tile t = fragment 2t + u of this lane (qk_pos
// positions 32t + 16u + 8h .. +7 of its point): 16 coalesced 1-KiB stores.
template <bool QSCALE>  // Q: times log2(e)/sqrt(C) (ATT_QFMA: the attention's softmax scale)
PDSC_DEV void w2_store_qk(const f32x16 (&acc)[4], float inv, const float *bias, _Float16 *__restrict__ dst, int row,
                          int lane) {
    const int h = lane >> 5;
    _Float16 *dtile = dst + (size_t)(row >> 5) * H3_TILE_H;
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const int c0 = 32 * t + 16 * u + 4 * h;
            const f32x4 b0 = *reinterpret_cast<const f32x4 *>(bias + c0), b1 = *reinterpret_cast<const f32x4 *>(bias + c0 + 8);
            float v[8];
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                v[e] = __builtin_fmaf(acc[t][8 * u + e], inv, e < 4 ? b0[e] : b1[e - 4]);
                if (QSCALE && ATT_QFMA) v[e] *= H3_QSCALE;
            }
            f16x8 hi, lo;
            split8v(v, hi, lo);
            *reinterpret_cast<f16x8 *>(dtile + h3_frag(2 * t + u, 0, lane)) = hi;
            *reinterpret_cast<f16x8 *>(dtile + h3_frag(2 * t + u, 1, lane)) = lo;
        }
}

// V output (untransposed: lane l32 <-> channel 32t + l32, registers 8s .. 8s+7
// <-> the key tile's v_keypos positions 16s + 8h .. +7) = fragment 2t + s of
// this lane in the V tiling, scaled by the tile's 2^vexp (the tile's max |v| is
// wave-local here): 16 coalesced 1-KiB stores.
PDSC_DEV void w2_store_v(f32x16 (&acc)[4], float inv, const float *bias, _Float16 *__restrict__ Vt,
                         float *__restrict__ vexp_t, int lane) {
    const int h = lane >> 5, l32 = lane & 31;
    float m = 0.0f;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
        const float bs = bias[32 * t + l32];
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            acc[t][r] = __builtin_fmaf(acc[t][r], inv, bs);
            m = fmaxf(m, fabsf(acc[t][r]));
        }
    }
    const int ev = h3_vexp(wave_max(m));
    if (lane == 0) *vexp_t = (float)ev;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
#pragma unroll
        for (int s = 0; s < 2; ++s) {
            float v[8];
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] = ldexpf(acc[t][8 * s + e], ev);
            f16x8 hi, lo;
            split8v(v, hi, lo);
            *reinterpret_cast<f16x8 *>(Vt + h3_frag(2 * t + s, 0, lane)) = hi;
            *reinterpret_cast<f16x8 *>(Vt + h3_frag(2 * t + s, 1, lane)) = lo;
        }
    }
}

// LDS coefficient table of a PointCN + QKV stage (PW2_COEF floats available).
struct W2CoefQKV {
    static constexpr int pcn = 0, q = 3 * CH, k = 4 * CH, v = 5 * CH, end = 6 * CH;
};
PDSC_DEV void w2_coef_qkv(float *cf, const float *pk, const PwDense4 &d, int tid) {
    w2_coef(cf + W2CoefQKV::pcn, pk, d.pcn, CH, tid);
    for (int i = tid; i < CH; i += PW2_W * 64) {  // Q / K / V: bias only
        cf[W2CoefQKV::q + i] = pk[d.q.bias + i];
        cf[W2CoefQKV::k + i] = pk[d.k.bias + i];
        cf[W2CoefQKV::v + i] = pk[d.v.bias + i];
    }
}

// PointCN (BN, ReLU) of the fragments x, then the Q/K/V projections; the
// PointCN rows go to featL.  The pipeline is at the PointCN layer's first chunk.
PDSC_DEV void w2_pcn_qkv(W2Pipe &P, const float *__restrict__ pk, const W2Sched &S, const float *cf, const PwDense4 &d,
                         const f16x8 *xh, const f16x8 *xl, float *__restrict__ featL, _Float16 *__restrict__ Q,
                         _Float16 *__restrict__ K, _Float16 *__restrict__ V, float *__restrict__ vexp, int row,
                         bool active, int wave, int lane) {
    const int h = lane >> 5;
    f32x16 acc[4];
    f16x8 yh[8], yl[8];
    const float sp = pk[d.pcn.scale], sq = pk[d.q.scale], sk = pk[d.k.scale], sv = pk[d.v.scale];
    w2_layer<CH, CH, true>(P, pk, S, xh, xl, acc, active, wave, lane);
    if (active) {
        w2_epilogue<CH, EPI_BN_RELU>(acc, sp, cf + W2CoefQKV::pcn, nullptr, yh, yl, lane);
        w2_store_row(featL, row, lane, acc);
    }
    CH_STAMP(175);
    w2_layer<CH, CH, true, 16>(P, pk, S, yh, yl, acc, active, wave, lane);
    if (active) w2_store_qk<true>(acc, sq, cf + W2CoefQKV::q, Q, row, lane);
    CH_STAMP(176);
    w2_layer<CH, CH, true, 16>(P, pk, S, yh, yl, acc, active, wave, lane);
    if (active) w2_store_qk<false>(acc, sk, cf + W2CoefQKV::k, K, row, lane);
    CH_STAMP(177);
    w2_layer<CH, CH, false, 16>(P, pk, S, yh, yl, acc, active, wave, lane);
    if (active) w2_store_v(acc, sv, cf + W2CoefQKV::v, V + (size_t)(row >> 5) * H3_TILE_H, vexp + (row >> 5), lane);
    CH_STAMP(178);
}

// Coefficients of combine + fc_message + PointCN + QKV (pw2_mid / attn_pw2).
struct W2CoefMid {
    static constexpr int f0 = W2CoefQKV::end, f3 = f0 + 3 * CH2, f6 = f3 + 3 * CH2, end = f6 + 3 * CH;
};
static_assert(W2CoefMid::end <= PW2_COEF, "coefficient table");
PDSC_DEV void w2_coef_mid(float *cf, const float *__restrict__ pk, const PwMsg &m, const PwDense4 &d, int tid) {
    w2_coef_qkv(cf, pk, d, tid);
    w2_coef(cf + W2CoefMid::f0, pk, m.fc0, CH2, tid);
    w2_coef(cf + W2CoefMid::f3, pk, m.fc3, CH2, tid);
    w2_coef(cf + W2CoefMid::f6, pk, m.fc6, CH, tid);
}

// fc_message + residual + PointCN + QKV from the message fragments x (after the
// combine); the pipeline is at fc0's first chunk.  featL, Q, K, V, vexp: the pair's.
PDSC_DEV void w2_mid_chain(W2Pipe &P, const float *__restrict__ pk, const W2Sched &S, const float *cf, const PwMsg &m,
                           const PwDense4 &d, f16x8 *xh, f16x8 *xl, const float *featL_in, float *featL,
                           _Float16 *__restrict__ Q, _Float16 *__restrict__ K, _Float16 *__restrict__ V,
                           float *__restrict__ vexp, int row, bool active, int wave, int lane) {
    // featL_in: the residual rows; featL: where the PointCN rows go (each lane
    // reads and writes only its own row, so the two may be one buffer)
    f32x16 a2[2], a4[4], res[4];
    f16x8 yh[8], yl[8];
    w2_layer<CH, CH2, true>(P, pk, S, xh, xl, a2, active, wave, lane);
    if (active) w2_epilogue<CH2, EPI_BN_RELU>(a2, pk[m.fc0.scale], cf + W2CoefMid::f0, nullptr, yh, yl, lane);
    CH_STAMP(172);
    w2_layer<CH2, CH2, true>(P, pk, S, yh, yl, a2, active, wave, lane);
    if (active) {
        w2_epilogue<CH2, EPI_BN_RELU>(a2, pk[m.fc3.scale], cf + W2CoefMid::f3, nullptr, xh, xl, lane);
        w2_load_row(featL_in, row, lane, res);  // the residual: lands during fc6's MFMAs
    }
    CH_STAMP(173);
    w2_layer<CH2, CH, true, 16>(P, pk, S, xh, xl, a4, active, wave, lane);
    if (active) w2_epilogue<CH, EPI_RESID>(a4, pk[m.fc6.scale], cf + W2CoefMid::f6, res, yh, yl, lane);
    CH_STAMP(174);
    w2_pcn_qkv(P, pk, S, cf, d, yh, yl, featL, Q, K, V, vexp, row, active, wave, lane);
}

#define PW2_PROLOGUE                                                                              \
    extern __shared__ __attribute__((aligned(16))) char w2smem[];                                 \
    const int b = blockIdx.y, tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, h = lane >> 5; \
    const int row = blockIdx.x * PW2_PTS + wave * 32 + (lane & 31);                               \
    const bool active = blockIdx.x * PW2_PTS + wave * 32 < Npad; /* wave-uniform */               \
    const size_t boff = (size_t)b * Npad * CH;                                                    \
    W2Pipe P{w2smem, 0};                                                                          \
    float *cf = reinterpret_cast<float *>(w2smem + PW2_NSLOT * PW2_SLOT);                         \
    for (int c_ = 0; c_ < PW2_NSLOT; ++c_) w2_stage(pk, S, c_, P.slot(c_), wave, lane);

// layer0 (Conv1d in_dim -> 128 on exact fp32 MFMA 32x32x2, k-step j: inputs 2j + h)
// + PointCN_0 + QKV_0.
__global__ __launch_bounds__(PW2_W * 64, PW2_OCC) void pw2_first_kernel(const float *__restrict__ pk, W2Sched S, size_t l0w,
                                                                 size_t l0b, PwDense4 d, const float *__restrict__ corr,
                                                                 int in_dim, int N, int Npad, float *__restrict__ featL,
                                                                 _Float16 *__restrict__ Q, _Float16 *__restrict__ K,
                                                                 _Float16 *__restrict__ V, float *__restrict__ vexp,
                                                                 const int *__restrict__ nv) {
    // ragged batches: a workgroup wholly past its pair's rows has nothing any later
    // kernel reads (the attention's key tiles end at round_up(n, 32) <= its first
    // row; its query blocks past n exit) -- leave before staging any weights
    if (nv && (int)blockIdx.x * PW2_PTS >= nv[blockIdx.y]) return;  // workgroup-uniform
    PW2_PROLOGUE
    const int l32 = lane & 31;
    const int n = nv ? nv[b] : N;  // this pair's rows (ragged batches); N: the row stride
    w2_coef_qkv(cf, pk, d, tid);
    f16x8 xh[8], xl[8];
    if (active) {
        const float *cp = corr + ((size_t)b * N + min(row, n - 1)) * in_dim;
        const bool in = row < n;
        f32x16 acc[4] = {zero16(), zero16(), zero16(), zero16()};
        for (int j = 0; j < (in_dim + 1) / 2; ++j) {
            const int i = 2 * j + h;
            const float x = (in && i < in_dim) ? cp[i] : 0.0f;
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                const float w = i < in_dim ? pk[l0w + (32 * t + l32) * in_dim + i] : 0.0f;
                acc[t] = mfma32(w, x, acc[t]);
            }
        }
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                float v[8];
#pragma unroll
                for (int e = 0; e < 8; ++e) v[e] = acc[t][8 * u + e] + pk[l0b + w2_chan(t, u, e, h)];
                split8v(v, xh[2 * t + u], xl[2 * t + u]);
            }
    }
    __syncthreads();
    w2_pcn_qkv(P, pk, S, cf, d, xh, xl, featL + boff, Q + 2 * boff, K + 2 * boff, V + 2 * boff,
               vexp + (size_t)b * (Npad / 32), row, active, wave, lane);
}

// combine_l + fc_message_l + residual + PointCN_{l+1} + QKV_{l+1}.
__global__ __launch_bounds__(PW2_W * 64, PW2_OCC) void pw2_mid_kernel(const float *__restrict__ pk, W2Sched S, PwMsg m,
                                                               PwDense4 d, const float *__restrict__ opart,
                                                               const float *__restrict__ ml, int nsplit, int N,
                                                               int Npad, const float *__restrict__ featL_in,
                                                               float *__restrict__ featL,
                                                               _Float16 *__restrict__ Q, _Float16 *__restrict__ K,
                                                               _Float16 *__restrict__ V, float *__restrict__ vexp) {
    PW2_PROLOGUE
    w2_coef_mid(cf, pk, m, d, tid);
    f16x8 xh[8], xl[8];
    if (active) w2_combine(opart, ml, b, nsplit, Npad, row, xh, xl, lane);
    __syncthreads();
    w2_mid_chain(P, pk, S, cf, m, d, xh, xl, featL_in + boff, featL + boff, Q + 2 * boff, K + 2 * boff,
                 V + 2 * boff, vexp + (size_t)b * (Npad / 32), row, active, wave, lane);
}

// attention_l + fc_message_l + residual + PointCN_{l+1} + QKV_{l+1} in ONE
// launch (one key split: the workgroup's 128 queries are the 128 points of its
// chain): the O^T accumulators the attention core leaves in registers are the
// message's k-step fragments, so the partials never touch HBM, and workgroups
// in their attention phase overlap others' store-heavy chain phase.  Reads the
// layer-l Q/K/V (Qs, Ks, Vs, vexp_in) and writes the layer-(l+1) ones to other
// buffers (Q, K, V, vexp): other workgroups of the pair still read layer l.
// Bit-identical to attention_h3_kernel + pw2_mid_kernel (a one-split combine
// is O * (1 / l) exactly).  LDS: the K/V ring, then the weight ring.
template <bool PACKED>
__global__ __launch_bounds__(PW2_W * 64, PW2_OCC) void attn_pw2_kernel(
    const _Float16 *__restrict__ Qs, const _Float16 *__restrict__ Ks, const _Float16 *__restrict__ Vs,
    const float *__restrict__ vexp_in, const float *__restrict__ M, AttnGridH3 g, const float *__restrict__ pk,
    W2Sched S, PwMsg m, PwDense4 d, float *__restrict__ featL, _Float16 *__restrict__ Q, _Float16 *__restrict__ K,
    _Float16 *__restrict__ V, float *__restrict__ vexp) {
    extern __shared__ __attribute__((aligned(16))) char w2smem[];
    const AttnBlock blk = attention_h3_block(g, true);
    if (blk.qb * PW2_PTS >= g.n(blk.b)) return;  // past a ragged pair's end (workgroup-uniform)
    const int b = blk.b, Npad = g.Npad, tid = threadIdx.x, wave = __builtin_amdgcn_readfirstlane(tid >> 6),
              lane = tid & 63;
    const int row = blk.qb * PW2_PTS + wave * 32 + (lane & 31);
    const bool active = blk.qb * PW2_PTS + wave * 32 < Npad;  // wave-uniform
    const size_t boff = (size_t)b * Npad * CH;
#ifdef ATT_STAMPS
    unsigned long long *stp = att_stamp_ptr(wave);
    ATT_RSTAMP(stp, 188);
    ATT_STAMP(stp, 0);
#endif
    f32x16 O[4];
    float m_run, l_run;
    attention_h3_core<PW2_W, PACKED, PW2_EARLY>(Qs, Ks, Vs, vexp_in, M, g, blk, w2smem, wave, lane, O, m_run, l_run);
    ATT_STAMP(stp, 170);
    // the K/V ring is free (the core ends on a barrier): weight chunks 0, 1 and the coefficients
    W2Pipe P{w2smem, 0};
    float *cf = reinterpret_cast<float *>(w2smem + PW2_NSLOT * PW2_SLOT);
    for (int c = 0; c < PW2_NSLOT; ++c) w2_stage(pk, S, c, P.slot(c), wave, lane);
    w2_coef_mid(cf, pk, m, d, tid);
    f16x8 xh[8], xl[8];
    if (active) w2_msg_frags(O, l_run, xh, xl);  // msg = O / l
    __syncthreads();
    ATT_STAMP(stp, 171);
    w2_mid_chain(P, pk, S, cf, m, d, xh, xl, featL + boff, featL + boff, Q + 2 * boff, K + 2 * boff,
                 V + 2 * boff, vexp + (size_t)b * (Npad / 32), row, active, wave, lane);
    ATT_STAMP(stp, 180);
    ATT_RSTAMP(stp, 189);
}

#ifdef ATT_STAMPS
extern "C" int pdsc_diag_att_stamps(void *host, size_t bytes) {
    const size_t n = std::min(bytes, sizeof(g_att_stamps));
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_att_stamps), n, 0, hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}
extern "C" int pdsc_diag_att_stamps_clear() {
    static unsigned long long zero[ST_WGS * 4 * ST_PER_WAVE];
    return hipMemcpyToSymbol(HIP_SYMBOL(g_att_stamps), zero, sizeof(zero), 0, hipMemcpyHostToDevice) == hipSuccess ? 0
                                                                                                             : -1;
}
#endif

// Coefficients of the last layer's fc_message + classifier (pw2_last / attn_pw2_last).
struct W2CoefLast {
    static constexpr int f0 = 0, f3 = f0 + 3 * CH2, f6 = f3 + 3 * CH2, c0 = f6 + 3 * CH, c2 = c0 + 3 * CLS,
                         c4 = c2 + 3 * CLS, end = c4 + CLS;
};
static_assert(W2CoefLast::end <= PW2_COEF, "coefficient table");
PDSC_DEV void w2_coef_last(float *cf, const float *__restrict__ pk, const PwMsg &m, const DenseOff &c0,
                           const DenseOff &c2, size_t c4w, int tid) {
    w2_coef(cf + W2CoefLast::f0, pk, m.fc0, CH2, tid);
    w2_coef(cf + W2CoefLast::f3, pk, m.fc3, CH2, tid);
    w2_coef(cf + W2CoefLast::f6, pk, m.fc6, CH, tid);
    w2_coef(cf + W2CoefLast::c0, pk, c0, CLS, tid);
    w2_coef(cf + W2CoefLast::c2, pk, c2, CLS, tid);
    for (int i = tid; i < CLS; i += PW2_W * 64) cf[W2CoefLast::c4 + i] = pk[c4w + i];
}

// fc_message + residual from the message fragments x, then F.normalize (:156)
// and the classifier (:171); the pipeline is at fc0's first chunk.  featL: the pair's.
PDSC_DEV void w2_last_chain(W2Pipe &P, const float *__restrict__ pk, const W2Sched &S, const float *cf, const PwMsg &m,
                            const DenseOff &c0, const DenseOff &c2, size_t c4b, f16x8 *xh, f16x8 *xl,
                            const float *__restrict__ featL, float *__restrict__ feat_out, float *__restrict__ normed,
                            _Float16 *__restrict__ normed_s, float *__restrict__ conf, int b, int N, int row,
                            bool active, int wave, int lane) {
    constexpr int CF0 = W2CoefLast::f0, CF3 = W2CoefLast::f3, CF6 = W2CoefLast::f6, CC0 = W2CoefLast::c0,
                  CC2 = W2CoefLast::c2, CC4 = W2CoefLast::c4;
    const int h = lane >> 5;
    f32x16 a1[1], a2[2], a4[4], res[4];
    f16x8 yh[8], yl[8];
    w2_layer<CH, CH2, true>(P, pk, S, xh, xl, a2, active, wave, lane);
    if (active) w2_epilogue<CH2, EPI_BN_RELU>(a2, pk[m.fc0.scale], cf + CF0, nullptr, yh, yl, lane);
    w2_layer<CH2, CH2, true>(P, pk, S, yh, yl, a2, active, wave, lane);
    if (active) {
        w2_epilogue<CH2, EPI_BN_RELU>(a2, pk[m.fc3.scale], cf + CF3, nullptr, xh, xl, lane);
        w2_load_row(featL, row, lane, res);
    }
    w2_layer<CH2, CH, true, 16>(P, pk, S, xh, xl, a4, active, wave, lane);
    const bool in = row < N;
    if (active) {
        w2_epilogue<CH, EPI_RESID>(a4, pk[m.fc6.scale], cf + CF6, res, yh, yl, lane);  // a4 = corr_features (:155)
        float ss = 0.0f;  // F.normalize(p=2, dim=-1, eps=1e-12) (:156)
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
            for (int r = 0; r < 16; ++r) ss = __builtin_fmaf(a4[t][r], a4[t][r], ss);
        ss = halves_sum(ss);
        const float den = fmaxf(sqrtf(ss), 1e-12f);
        if (in) {
            float *dst = normed + ((size_t)b * N + row) * CH;
            _Float16 *ds = normed_s ? normed_s + ((size_t)b * N + row) * 2 * CH : nullptr;
#pragma unroll
            for (int t = 0; t < 4; ++t)
#pragma unroll
                for (int u = 0; u < 2; ++u) {
                    float v[8];
#pragma unroll
                    for (int e = 0; e < 8; ++e) v[e] = a4[t][8 * u + e] / den;
                    *reinterpret_cast<f32x4 *>(dst + 32 * t + 16 * u + 4 * h) = f32x4{v[0], v[1], v[2], v[3]};
                    *reinterpret_cast<f32x4 *>(dst + 32 * t + 16 * u + 8 + 4 * h) = f32x4{v[4], v[5], v[6], v[7]};
                    if (ds) {  // the fp16 hi/lo split copy (qk_pos order) the seed kNN consumes
                        f16x8 hi, lo;
                        split8v(v, hi, lo);
                        const int chk = 4 * t + 2 * u + h;
                        *reinterpret_cast<f16x8 *>(ds + 8 * chk) = hi;
                        *reinterpret_cast<f16x8 *>(ds + CH + 8 * chk) = lo;
                    }
                }
            if (feat_out) {  // natural channel order (the standalone encoder API only)
                float *fo = feat_out + ((size_t)b * N + row) * CH;
#pragma unroll
                for (int t = 0; t < 4; ++t)
#pragma unroll
                    for (int g = 0; g < 4; ++g)
                        *reinterpret_cast<f32x4 *>(fo + 32 * t + 8 * g + 4 * h) =
                            f32x4{a4[t][4 * g], a4[t][4 * g + 1], a4[t][4 * g + 2], a4[t][4 * g + 3]};
            }
        }
    }
    // classification MLP 128 -> 32 -> 32 -> 1 on the unnormalised features (:171)
    w2_layer<CH, CLS, true>(P, pk, S, yh, yl, a1, active, wave, lane);
    if (active) w2_epilogue<CLS, EPI_RELU>(a1, pk[c0.scale], cf + CC0, nullptr, xh, xl, lane);
    w2_layer<CLS, CLS, true>(P, pk, S, xh, xl, a1, active, wave, lane);
    if (active) {
        w2_epilogue<CLS, EPI_RELU, false>(a1, pk[c2.scale], cf + CC2, nullptr, nullptr, nullptr, lane);
        float s = 0.0f;  // this half's 16 channels, then the other half's
#pragma unroll
        for (int u = 0; u < 2; ++u)
#pragma unroll
            for (int e = 0; e < 8; ++e) s = __builtin_fmaf(cf[CC4 + w2_chan(0, u, e, h)], a1[0][8 * u + e], s);
        s = halves_sum(s);
        if (in && h == 0) conf[(size_t)b * N + row] = s + pk[c4b];
    }
}

// combine + fc_message + residual, then F.normalize (:156) and the classifier (:171).
__global__ __launch_bounds__(PW2_W * 64, PW2_OCC) void pw2_last_kernel(
    const float *__restrict__ pk, W2Sched S, PwMsg m, DenseOff c0, DenseOff c2, size_t c4w, size_t c4b,
    const float *__restrict__ opart, const float *__restrict__ ml, int nsplit, int N, int Npad,
    const float *__restrict__ featL, float *__restrict__ feat_out, float *__restrict__ normed,
    _Float16 *__restrict__ normed_s, float *__restrict__ conf) {
    PW2_PROLOGUE
    w2_coef_last(cf, pk, m, c0, c2, c4w, tid);
    f16x8 xh[8], xl[8];
    if (active) w2_combine(opart, ml, b, nsplit, Npad, row, xh, xl, lane);
    __syncthreads();
    w2_last_chain(P, pk, S, cf, m, c0, c2, c4b, xh, xl, featL + boff, feat_out, normed, normed_s, conf, b, N, row,
                  active, wave, lane);
}

// attention_{L-1} + fc_message_{L-1} + residual + normalize + classifier in ONE
// launch (as attn_pw2_kernel for the last layer): bit-identical to
// attention_h3_kernel + pw2_last_kernel with one key split.
template <bool PACKED>
__global__ __launch_bounds__(PW2_W * 64, PW2_OCC) void attn_pw2_last_kernel(
    const _Float16 *__restrict__ Qs, const _Float16 *__restrict__ Ks, const _Float16 *__restrict__ Vs,
    const float *__restrict__ vexp_in, const float *__restrict__ M, AttnGridH3 g, const float *__restrict__ pk,
    W2Sched S, PwMsg m, DenseOff c0, DenseOff c2, size_t c4w, size_t c4b, const float *__restrict__ featL,
    float *__restrict__ feat_out, float *__restrict__ normed, _Float16 *__restrict__ normed_s,
    float *__restrict__ conf) {
    extern __shared__ __attribute__((aligned(16))) char w2smem[];
    const AttnBlock blk = attention_h3_block(g, true);
    if (blk.qb * PW2_PTS >= g.n(blk.b)) return;  // past a ragged pair's end (workgroup-uniform)
    const int b = blk.b, N = g.N, Npad = g.Npad, tid = threadIdx.x, wave = __builtin_amdgcn_readfirstlane(tid >> 6),
              lane = tid & 63;
    const int row = blk.qb * PW2_PTS + wave * 32 + (lane & 31);
    const bool active = blk.qb * PW2_PTS + wave * 32 < Npad;  // wave-uniform
    f32x16 O[4];
    float m_run, l_run;
    attention_h3_core<PW2_W, PACKED, PW2_EARLY>(Qs, Ks, Vs, vexp_in, M, g, blk, w2smem, wave, lane, O, m_run, l_run);
    W2Pipe P{w2smem, 0};
    float *cf = reinterpret_cast<float *>(w2smem + PW2_NSLOT * PW2_SLOT);
    for (int c = 0; c < PW2_NSLOT; ++c) w2_stage(pk, S, c, P.slot(c), wave, lane);
    w2_coef_last(cf, pk, m, c0, c2, c4w, tid);
    f16x8 xh[8], xl[8];
    if (active) w2_msg_frags(O, l_run, xh, xl);
    __syncthreads();
    w2_last_chain(P, pk, S, cf, m, c0, c2, c4b, xh, xl, featL + (size_t)b * Npad * CH, feat_out, normed, normed_s,
                  conf, b, N, row, active, wave, lane);
}
#undef PW2_PROLOGUE

// pw2 for launches of at least 320 128-point workgroups, 1.25 per CU (knob
// PDSC_PW2: 0 never, 2 always, else this rule; measurement only).  Measured
// encoder ms, pw2 vs pw_mid chains: 8 x N=5000 (320 WGs; 3 key splits) 4.48
// vs 4.61; 40 x 1000 (320, fused) 1.47 vs 1.78; 56 x 1000 (448, fused) 1.68 vs
// 2.12; 32 x 1000 (256) 1.26 vs 1.22 and 1.24 fused; 16 x 1000 (128) 0.95 vs 0.80.
static bool use_pw2(int B, int Npad, bool f32) {
    static const int mode = [] {
        const char *e = getenv("PDSC_PW2");
        return e ? atoi(e) : 1;
    }();
    if (f32 || mode == 0) return false;
    return mode == 2 || (long)B * ((Npad + PW2_PTS - 1) / PW2_PTS) >= 320;
}

static W2Sched sched_qkv(W2Sched S, const PwDense4 &d) {
    w2_sched_add(S, d.pcn, CH, CH);
    w2_sched_add(S, d.q, CH, CH);
    w2_sched_add(S, d.k, CH, CH);
    w2_sched_add(S, d.v, CH, CH);
    return S;
}
static W2Sched sched_msg(const PwMsg &m) {
    W2Sched S{};
    w2_sched_add(S, m.fc0, CH, CH2);
    w2_sched_add(S, m.fc3, CH2, CH2);
    w2_sched_add(S, m.fc6, CH2, CH);
    return S;
}

static PwDense4 dense4(const LayerOff &l) { return PwDense4{l.pcn, l.q, l.k, l.v}; }
static PwMsg msg3(const LayerOff &l) { return PwMsg{l.fc0, l.fc3, l.fc6}; }

// attn_pw2 wherever pw2 runs and the attention has one key split (knob
// PDSC_FUSE=0 keeps the two launches; measurement only).
static AttnGridH3 fused_grid(int B, int N) { return attention_h3_grid<PW2_W>(B, N, att_target() * 4 / PW2_W); }
// the fused launches' grid: one key split always (attention_fused chose the plan
// on the whole batch; a part of it -- run_encoder_part's halves -- keeps it)
static AttnGridH3 fused_launch_grid(int B, int N) {
    AttnGridH3 g = fused_grid(B, N);
    const int nst = (N + H3_TILE - 1) / H3_TILE;
    g.sps = nst;
    g.nsplit = 1;
    return g;
}
bool attention_fused(int B, int N, bool f32) {
    static const bool off = [] {
        const char *e = getenv("PDSC_FUSE");
        return e && e[0] == '0';
    }();
    const int Npad = round_up(N, QB);
    const AttnGridH3 g = fused_grid(B, N);
    return !off && use_pw2(B, Npad, f32) && g.nsplit == 1 && g.nqb * PW2_PTS == Npad;
}

hipError_t launch_attn_pw2(const float *packed, const PackLayout &lay, int layer, const void *q, const void *k,
                           const void *v, const float *vexp_in, const float *M, bool m_packed, int B, int N, int Npad,
                           float *feat, void *qo, void *ko, void *vo, float *vexp_out, hipStream_t s, Ragged rg) {
    AttnGridH3 g = fused_launch_grid(B, N);
    g.nv = rg.nv;
    g.po = rg.po;
    g.rev = rg.po ? 0 : zigzag_rev(layer);  // (ragged batches keep their longest-first order)
    if (g.nsplit != 1 || g.Npad != Npad || g.nqb * PW2_PTS != Npad || layer + 1 >= lay.L) return hipErrorInvalidValue;
    const W2Sched S = sched_qkv(sched_msg(msg3(lay.layer[layer])), dense4(lay.layer[layer + 1]));
    const size_t lds = std::max(attention_h3_lds_bytes<PW2_W>(), PW2_LDS);
    const _Float16 *qs = static_cast<const _Float16 *>(q), *ks = static_cast<const _Float16 *>(k),
                   *vs = static_cast<const _Float16 *>(v);
    _Float16 *Q = static_cast<_Float16 *>(qo), *K = static_cast<_Float16 *>(ko), *V = static_cast<_Float16 *>(vo);
    if (m_packed)
        hipLaunchKernelGGL(attn_pw2_kernel<true>, dim3(g.B * g.nqb), dim3(PW2_W * 64), lds, s, qs, ks, vs, vexp_in, M,
                           g, packed, S, msg3(lay.layer[layer]), dense4(lay.layer[layer + 1]), feat, Q, K, V, vexp_out);
    else
        hipLaunchKernelGGL(attn_pw2_kernel<false>, dim3(g.B * g.nqb), dim3(PW2_W * 64), lds, s, qs, ks, vs, vexp_in, M,
                           g, packed, S, msg3(lay.layer[layer]), dense4(lay.layer[layer + 1]), feat, Q, K, V, vexp_out);
    return hipGetLastError();
}

hipError_t launch_attn_pw2_last(const float *packed, const PackLayout &lay, const void *q, const void *k,
                                const void *v, const float *vexp_in, const float *M, bool m_packed, int B, int N,
                                int Npad, const float *feat, float *feat_out, float *normed, _Float16 *normed_s,
                                float *conf, hipStream_t s, Ragged rg) {
    AttnGridH3 g = fused_launch_grid(B, N);
    g.nv = rg.nv;
    g.po = rg.po;
    g.rev = rg.po ? 0 : zigzag_rev(lay.L - 1);
    if (g.nsplit != 1 || g.Npad != Npad || g.nqb * PW2_PTS != Npad) return hipErrorInvalidValue;
    W2Sched S = sched_msg(msg3(lay.layer[lay.L - 1]));
    w2_sched_add(S, lay.c0, CH, CLS);
    w2_sched_add(S, lay.c2, CLS, CLS);
    const size_t lds = std::max(attention_h3_lds_bytes<PW2_W>(), PW2_LDS);
    const _Float16 *qs = static_cast<const _Float16 *>(q), *ks = static_cast<const _Float16 *>(k),
                   *vs = static_cast<const _Float16 *>(v);
    const PwMsg m = msg3(lay.layer[lay.L - 1]);
    if (m_packed)
        hipLaunchKernelGGL(attn_pw2_last_kernel<true>, dim3(g.B * g.nqb), dim3(PW2_W * 64), lds, s, qs, ks, vs, vexp_in,
                           M, g, packed, S, m, lay.c0, lay.c2, lay.c4_w, lay.c4_b, feat, feat_out, normed, normed_s,
                           conf);
    else
        hipLaunchKernelGGL(attn_pw2_last_kernel<false>, dim3(g.B * g.nqb), dim3(PW2_W * 64), lds, s, qs, ks, vs,
                           vexp_in, M, g, packed, S, m, lay.c0, lay.c2, lay.c4_w, lay.c4_b, feat, feat_out, normed,
                           normed_s, conf);
    return hipGetLastError();
}

// Point-tile size: 64 points (two 32-row MFMA tiles per wave, 2 workgroups per
// CU) once the launch has >= 2 workgroups per CU, else 32 (twice the
// workgroups for single pairs and small batches).
static bool small_tiles(int B, int Npad) {
    static const long lim = [] {  // A/B knob (measurement only): PDSC_PW_SMALL_LIMIT
        const char *e = getenv("PDSC_PW_SMALL_LIMIT");
        return e ? atol(e) : 512L;
    }();
    return (long)B * (Npad / 64) < lim;
}

// 8-wave pw_mid workgroups (32 points each) when the launch has at most one
// workgroup per CU (a single N = 1000 pair: 32): the chain's output tiles
// spread over twice the waves (A/B knob PDSC_PW_WAVES=4: never).
static bool pw_waves8(int B, int Npad) {
    static const bool off = [] {
        const char *e = getenv("PDSC_PW_WAVES");
        return e && atoi(e) == 4;
    }();
    return !off && (long)B * (Npad / 32) <= 256;
}

// 8-wave pw_mid with Q, K and V in three workgroups per point tile (pcn_qkv8's
// `only`) while that stays within one workgroup per CU.  A/B knob
// PDSC_PW_QKV_SPLIT=0 (measurement only; the same bits either way).
static bool pw_qkv_split(int B, int Npad) {
    static const bool off = [] {
        const char *e = getenv("PDSC_PW_QKV_SPLIT");
        return e && e[0] == '0';
    }();
    return !off && 3L * B * (Npad / 32) <= 256;
}

// One launch of pointwise kernel K<PTT, F32> with PTT and F32 picked at run time.
#define PW_LAUNCH(K, rows, ...)                                                                         \
    do {                                                                                                \
        const bool st_ = small_tiles(B, Npad);                                                          \
        const int pt_ = st_ ? 32 : 64;                                                                  \
        const dim3 g_(((rows) + pt_ - 1) / pt_, B);                                                     \
        if (st_ && f32)                                                                                 \
            hipLaunchKernelGGL((K<32, true>), g_, dim3(256), pw_lds<32>(), s, __VA_ARGS__);             \
        else if (st_)                                                                                   \
            hipLaunchKernelGGL((K<32, false>), g_, dim3(256), pw_lds<32>(), s, __VA_ARGS__);            \
        else if (f32)                                                                                   \
            hipLaunchKernelGGL((K<64, true>), g_, dim3(256), pw_lds<64>(), s, __VA_ARGS__);             \
        else                                                                                            \
            hipLaunchKernelGGL((K<64, false>), g_, dim3(256), pw_lds<64>(), s, __VA_ARGS__);            \
    } while (0)

hipError_t launch_pw_first(const float *packed, const PackLayout &lay, const float *corr_pos, bool f32, int B,
                           int N, int Npad, float *feat, void *q, void *k, void *v, float *vexp, hipStream_t s,
                           Ragged rg, bool fused) {
    if (lay.in_dim > IN_LIMIT) return hipErrorInvalidValue;
    _Float16 *Q = static_cast<_Float16 *>(q), *K = static_cast<_Float16 *>(k), *V = static_cast<_Float16 *>(v);
    if (fused || use_pw2(B, Npad, f32)) {  // the fused plan's layouts (a part of a batch: the batch's plan)
        const W2Sched S = sched_qkv(W2Sched{}, dense4(lay.layer[0]));
        hipLaunchKernelGGL(pw2_first_kernel, dim3((Npad + PW2_PTS - 1) / PW2_PTS, B), dim3(PW2_W * 64), PW2_LDS, s,
                           packed, S, lay.l0_w, lay.l0_b, dense4(lay.layer[0]), corr_pos, lay.in_dim, N, Npad, feat, Q, K,
                           V, vexp, rg.nv);
        return hipGetLastError();
    }
    if (!f32 && small_tiles(B, Npad) && pw_qkv_split(B, Npad)) {  // Q / K / V in three workgroups per tile
        hipLaunchKernelGGL((pw_first_kernel<32, false>), dim3(Npad / 32, B, 3), dim3(256), pw_lds<32>(), s, packed,
                           lay.l0_w, lay.l0_b, dense4(lay.layer[0]), corr_pos, lay.in_dim, N, Npad, feat, Q, K, V, vexp,
                           rg.nv);
        return hipGetLastError();
    }
    PW_LAUNCH(pw_first_kernel, Npad, packed, lay.l0_w, lay.l0_b, dense4(lay.layer[0]), corr_pos, lay.in_dim, N, Npad,
              feat, Q, K, V, vexp, rg.nv);
    return hipGetLastError();
}

hipError_t launch_pw_mid(const float *packed, const PackLayout &lay, int layer, bool f32, const float *opart,
                         const float *ml, int nsplit, int B, int N, int Npad, const float *feat_in, float *feat,
                         void *q, void *k, void *v, float *vexp, hipStream_t s) {
    const int delay = g_diag_qkv_delay;  // tests only (pdsc_diag_qkv_delay): delay the split's K / V workgroups
    _Float16 *Q = static_cast<_Float16 *>(q), *K = static_cast<_Float16 *>(k), *V = static_cast<_Float16 *>(v);
    if (use_pw2(B, Npad, f32)) {
        const W2Sched S = sched_qkv(sched_msg(msg3(lay.layer[layer])), dense4(lay.layer[layer + 1]));
        hipLaunchKernelGGL(pw2_mid_kernel, dim3((Npad + PW2_PTS - 1) / PW2_PTS, B), dim3(PW2_W * 64), PW2_LDS, s,
                           packed, S, msg3(lay.layer[layer]), dense4(lay.layer[layer + 1]), opart, ml, nsplit, N, Npad,
                           feat_in, feat, Q, K, V, vexp);
        return hipGetLastError();
    }
    if (!f32 && pw_waves8(B, Npad)) {
        hipLaunchKernelGGL((pw_mid_kernel<32, false, 8>), dim3(Npad / 32, B, pw_qkv_split(B, Npad) ? 3 : 1), dim3(512),
                           pw_lds<32>(), s, packed,
                           msg3(lay.layer[layer]), dense4(lay.layer[layer + 1]), opart, ml, nsplit, N, Npad, feat_in,
                           feat, Q, K, V, vexp, delay, (int)pw_prefetch_on());
        return hipGetLastError();
    }
    PW_LAUNCH(pw_mid_kernel, Npad, packed, msg3(lay.layer[layer]), dense4(lay.layer[layer + 1]), opart, ml, nsplit,
              N, Npad, feat_in, feat, Q, K, V, vexp, 0, 0);
    return hipGetLastError();
}

hipError_t launch_pw_last(const float *packed, const PackLayout &lay, bool f32, const float *opart,
                          const float *ml, int nsplit, int B, int N, int Npad, const float *feat,
                          float *feat_out, float *normed, _Float16 *normed_s, float *conf, hipStream_t s) {
    if (use_pw2(B, Npad, f32)) {
        W2Sched S = sched_msg(msg3(lay.layer[lay.L - 1]));
        w2_sched_add(S, lay.c0, CH, CLS);
        w2_sched_add(S, lay.c2, CLS, CLS);
        hipLaunchKernelGGL(pw2_last_kernel, dim3((Npad + PW2_PTS - 1) / PW2_PTS, B), dim3(PW2_W * 64), PW2_LDS, s,
                           packed, S, msg3(lay.layer[lay.L - 1]), lay.c0, lay.c2, lay.c4_w, lay.c4_b, opart, ml, nsplit, N,
                           Npad, feat, feat_out, normed, normed_s, conf);
        return hipGetLastError();
    }
    PW_LAUNCH(pw_last_kernel, N, packed, msg3(lay.layer[lay.L - 1]), lay.c0, lay.c2, lay.c4_w, lay.c4_b, opart, ml,
              nsplit, N, Npad, feat, feat_out, normed, normed_s, conf);
    return hipGetLastError();
}
#undef PW_LAUNCH
}  // namespace pdsc
