// api.hip -- the C ABI of libpdsc.so (declared in include/pdsc.h).
//
// Host-side orchestration only: argument checks, workspace carving and kernel
// launches on the caller's stream.  No allocation, no synchronisation.
#include <algorithm>
#include <chrono>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <mutex>
#include <string>
#include <vector>

#include "pdsc_internal.hpp"

using namespace pdsc;

namespace pdsc {
thread_local int g_diag_qkv_delay = 0;  // pdsc_diag_qkv_delay (tests only)
}

namespace {

thread_local std::string g_err;
thread_local std::string g_name;

// measurement hook (pdsc_attention_timing): events recorded around attention launches
thread_local hipEvent_t *g_tstart = nullptr, *g_tstop = nullptr;
thread_local int g_tcap = 0;
thread_local int32_t *g_tcount = nullptr;
// pdsc_forward_timing: PDSC_FORWARD_STAGES + 1 events per forward call
thread_local hipEvent_t *g_fev = nullptr;
thread_local int g_fcap = 0;
thread_local int32_t *g_fcount = nullptr;

int fail(int code, const char *fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}

#define HIPCHK(expr)                                                                          \
    do {                                                                                      \
        hipError_t e_ = (expr);                                                               \
        if (e_ != hipSuccess) return fail(PDSC_ERR_HIP, "%s: %s", #expr, hipGetErrorString(e_)); \
    } while (0)

hipStream_t S_(pdsc_stream_t s) { return reinterpret_cast<hipStream_t>(s); }

// Bump allocator over a caller workspace (256-B aligned slices).
struct Carve {
    char *base;
    size_t off = 0;
    explicit Carve(void *p) : base(static_cast<char *>(p)) {}
    template <typename T> T *take(size_t n) {
        T *p = base ? reinterpret_cast<T *>(base + off) : nullptr;
        off += align_bytes(n * sizeof(T));
        return p;
    }
};

// A/B knob (measurement only): PDSC_DENSE_M=1 makes the forward write and read M dense.
bool dense_m_requested() {
    static const bool v = [] {
        const char *e = getenv("PDSC_DENSE_M");
        return e && e[0] == '1';
    }();
    return v;
}

// The forward's M layout: symmetric-packed for the H3 plans, dense for exact fp32
// (and PDSC_DENSE_M=1 on the h3 plans other than attention_w64's, measurement only).
struct Dims;
int forward_m_layout(const Dims &d);

int check_cfg(const pdsc_config *cfg) {
    if (!cfg) return fail(PDSC_ERR_ARG, "cfg is NULL");
    if (cfg->num_channels != CH)
        return fail(PDSC_ERR_UNSUPPORTED, "num_channels=%d: only %d is implemented", cfg->num_channels, CH);
    if (cfg->num_layers < 1 || cfg->num_layers > 64)
        return fail(PDSC_ERR_UNSUPPORTED, "num_layers=%d not in [1, 64]", cfg->num_layers);
    if (cfg->in_dim < 1 || cfg->in_dim > 128) return fail(PDSC_ERR_UNSUPPORTED, "in_dim=%d not in [1, 128]", cfg->in_dim);
    if (cfg->num_iterations < 0 || cfg->num_iterations > 31)
        return fail(PDSC_ERR_UNSUPPORTED, "num_iterations=%d not in [0, 31]", cfg->num_iterations);
    if (cfg->k < 1) return fail(PDSC_ERR_ARG, "k=%d", cfg->k);
    if (cfg->precision != PDSC_PRECISION_H3 && cfg->precision != PDSC_PRECISION_F32)
        return fail(PDSC_ERR_ARG, "precision=%d (PDSC_PRECISION_H3 or PDSC_PRECISION_F32)", cfg->precision);
    return PDSC_OK;
}

// The tiniest batches (<= 16 query blocks of 128, >= 16 key splits: a single
// N = 1000 pair) combine the attention partials in their own launch
// (combine_rows) rather than in the pointwise kernel's prologue: measured
// 0.511 -> 0.482 ms per single-pair forward, but slower from 4 pairs of
// N = 1000 on (an extra launch per layer).  A/B knob PDSC_PRECOMBINE=0 (never).
static bool use_precombine(int B, int Npad, int nsplit, bool f32, bool fuse) {
    static const bool off = [] {
        const char *e = getenv("PDSC_PRECOMBINE");
        return e && e[0] == '0';
    }();
    return !off && !f32 && !fuse && nsplit >= 16 && (long)B * (Npad / QB) <= 16;
}

struct Dims {
    int B, N, Npad, S, k, T, nsplit;
    bool f32;   // PDSC_PRECISION_F32
    bool fuse;  // attention + pointwise chain in one launch per layer (attention_fused)
    bool w64;   // split path with attention_w64 (64-query waves)
    bool precombine;  // split partials combined by combine_rows ahead of the pointwise kernels
};

int make_dims(const pdsc_config *cfg, int B, int N, Dims &d) {
    if (B < 1 || N < 2) return fail(PDSC_ERR_ARG, "B=%d N=%d (need B >= 1, N >= 2)", B, N);
    if (N > 32767) return fail(PDSC_ERR_UNSUPPORTED, "N=%d > 32767 (32-bit buffer descriptors over M)", N);
    d.B = B;
    d.N = N;
    d.Npad = round_up(N, QB);
    d.S = (int)((double)N * cfg->ratio);  // int(num_corr * self.ratio) (:174)
    d.k = std::min(cfg->k, N - 1);        // (:250)
    d.T = cfg->num_iterations;
    d.f32 = cfg->precision == PDSC_PRECISION_F32;
    d.fuse = attention_fused(B, N, d.f32);
    d.w64 = !d.fuse && attention_w64(B, N, d.f32);
    d.nsplit = attention_nsplit(B, N, d.f32, d.w64);
    d.precombine = use_precombine(B, d.Npad, d.nsplit, d.f32, d.fuse);
    if (d.S < 1) return fail(PDSC_ERR_ARG, "int(N*ratio) = 0 seeds for N=%d", N);
    if (d.k > 63) return fail(PDSC_ERR_UNSUPPORTED, "k=%d > 63", d.k);
    return PDSC_OK;
}

int forward_m_layout(const Dims &d) {
    if (d.w64) return M_PACKED;
    return (!dense_m_requested() && !d.f32) ? M_PACKED : M_DENSE;
}

struct EncBufs {
    float *feat, *opart, *ml, *vexp, *vexp2;
    float *feat2;            // the split path's second feat buffer (pw_mid reads one, writes the other), else null
    _Float16 *q, *k, *v;     // attention_h3 split layouts (hi + lo per element), or fp32 rows (F32)
    _Float16 *q2, *k2, *v2;  // the other Q/K/V set of the fused path (layers alternate), else null
    float *opart1, *ml1;     // the combined split (Dims::precombine), else null
};

EncBufs carve_encoder(Carve &c, const Dims &d) {
    EncBufs e;
    const size_t rows = (size_t)d.B * d.Npad * CH;
    e.feat = c.take<float>(rows);
    e.q = c.take<_Float16>(2 * rows);
    e.k = c.take<_Float16>(2 * rows);
    e.v = c.take<_Float16>(2 * rows);
    e.opart = c.take<float>(rows * d.nsplit);
    e.ml = c.take<float>((size_t)d.B * d.Npad * d.nsplit * 2);
    e.vexp = c.take<float>((size_t)d.B * (d.Npad / 32));
    e.opart1 = d.precombine ? c.take<float>(rows) : nullptr;
    e.ml1 = d.precombine ? c.take<float>((size_t)d.B * d.Npad * 2) : nullptr;
    e.q2 = e.k2 = e.v2 = nullptr;
    e.vexp2 = nullptr;
    // pw_mid's three Q / K / V workgroups per point tile all read the layer's
    // residual rows while one of them writes the new PointCN rows: the rows
    // ping-pong between feat and feat2 so no workgroup overwrites what another
    // still reads
    e.feat2 = d.fuse ? nullptr : c.take<float>(rows);
    if (d.fuse) {
        e.q2 = c.take<_Float16>(2 * rows);
        e.k2 = c.take<_Float16>(2 * rows);
        e.v2 = c.take<_Float16>(2 * rows);
        e.vexp2 = c.take<float>((size_t)d.B * (d.Npad / 32));
    }
    return e;
}

int run_encoder(const PackLayout &lay, const float *packed, const float *corr_pos, const float *M,
                int m_layout, const Dims &d, const EncBufs &e, float *feat_out, float *normed,
                _Float16 *normed_s, float *conf, hipStream_t s, Ragged rg = {}) {
    const bool m_packed = m_layout == M_PACKED;
    const bool w64 = d.w64 && !d.fuse;
    if (w64 && m_layout != M_PACKED) return fail(PDSC_ERR_ARG, "M layout %d for this plan", m_layout);
    HIPCHK(launch_pw_first(packed, lay, corr_pos, d.f32, d.B, d.N, d.Npad, e.feat, e.q, e.k, e.v, e.vexp, s, rg,
                           d.fuse));
    if (d.fuse) {  // every layer fused (0 .. L-2 with the next layer's PointCN/QKV, Q/K/V alternating between the two sets)
        _Float16 *q = e.q, *k = e.k, *v = e.v, *q2 = e.q2, *k2 = e.k2, *v2 = e.v2;
        float *vx = e.vexp, *vx2 = e.vexp2;
        for (int l = 0; l + 1 < lay.L; ++l) {
            const bool timed = g_tcap > 0 && g_tcount && *g_tcount < g_tcap;
            if (timed) HIPCHK(hipEventRecord(g_tstart[*g_tcount], s));
            HIPCHK(launch_attn_pw2(packed, lay, l, q, k, v, vx, M, m_packed, d.B, d.N, d.Npad, e.feat, q2, k2, v2, vx2,
                                   s, rg));
            if (timed) HIPCHK(hipEventRecord(g_tstop[(*g_tcount)++], s));
            std::swap(q, q2);
            std::swap(k, k2);
            std::swap(v, v2);
            std::swap(vx, vx2);
        }
        HIPCHK(launch_attn_pw2_last(packed, lay, q, k, v, vx, M, m_packed, d.B, d.N, d.Npad, e.feat, feat_out, normed,
                                    normed_s, conf, s, rg));
        return PDSC_OK;
    }
    float *feat = e.feat, *feat_alt = e.feat2;
    for (int l = 0; l < lay.L; ++l) {
        const bool timed = g_tcap > 0 && g_tcount && *g_tcount < g_tcap;
        if (timed) HIPCHK(hipEventRecord(g_tstart[*g_tcount], s));
        HIPCHK(launch_attention(e.q, e.k, e.v, e.vexp, M, m_layout, w64, d.f32, d.B, d.N, d.Npad, d.nsplit, e.opart,
                                e.ml, s, rg, l));
        if (timed) HIPCHK(hipEventRecord(g_tstop[(*g_tcount)++], s));
        const float *op = e.opart, *mlp = e.ml;
        int ns = d.nsplit;
        if (d.precombine) {
            HIPCHK(launch_combine_rows(e.opart, e.ml, d.B, d.Npad, d.nsplit, e.opart1, e.ml1, s));
            op = e.opart1;
            mlp = e.ml1;
            ns = 1;
        }
        if (l + 1 < lay.L) {
            HIPCHK(launch_pw_mid(packed, lay, l, d.f32, op, mlp, ns, d.B, d.N, d.Npad, feat, feat_alt, e.q, e.k, e.v,
                                 e.vexp, s));
            std::swap(feat, feat_alt);
        } else {
            HIPCHK(launch_pw_last(packed, lay, d.f32, op, mlp, ns, d.B, d.N, d.Npad, feat, feat_out, normed,
                                  d.f32 ? nullptr : normed_s, conf, s));
        }
    }
    return PDSC_OK;
}

// Ragged batches run the fused encoder as P parts of the batch (contiguous pair
// ranges of equal pair counts), each on its own
// stream -- the caller's and P - 1 per-device side streams, forked and joined
// by events -- so one part's launches fill the others' dispatch tails: a ragged
// batch's attention launches end in a tail of a few long workgroups per XCD
// (DESIGN.md §7).  Pairs are independent through the encoder, so each part is
// the same arithmetic on its own pointer range (bitwise equal results).
// 128 pairs, N in [700, 1300], two halves: 4.54 -> 4.12 ms per forward (three
// parts 4.23, four 4.32 vs two 4.19 on another box); uniform batches (two full
// rounds of workgroups, no tail to fill) measured 3.77 -> 3.83 ms, so they stay
// on one stream.  Knobs: PDSC_ENC_HALVES 0 never, 1 uniform batches too;
// PDSC_ENC_PARTS P in [2, 4] (default 2).  Every part keeps the whole batch's
// plan (the fused launches' one key split, pw2_first's layouts).
static int enc_halves_mode() {
    static const int v = [] {
        const char *e = getenv("PDSC_ENC_HALVES");
        return e && e[0] == '0' ? 0 : (e && e[0] == '1' ? 2 : 1);
    }();
    return v;
}
constexpr int ENC_MAX_PARTS = 4;
static int enc_parts() {
    static const int v = [] {
        const char *e = getenv("PDSC_ENC_PARTS");
        const int p = e ? atoi(e) : 2;
        return std::min(std::max(p, 2), ENC_MAX_PARTS);
    }();
    return v;
}
// Parts of equal pair counts; A/B knob PDSC_ENC_BAL=1: parts of equal work
// sum(n^2) instead (measured slower: 128 pairs, N in [700, 1300], 4.150 / 4.159
// vs 4.021 / 4.056 ms per forward, one stream 4.423 / 4.437).
static bool enc_work_balanced() {
    static const bool on = [] {
        const char *e = getenv("PDSC_ENC_BAL");
        return e && e[0] == '1';
    }();
    return on;
}
static bool enc_halves(const Dims &d, bool ragged) {
    const int mode = enc_halves_mode();
    return d.fuse && d.B >= 16 * enc_parts() && (mode == 2 || (mode == 1 && ragged));
}
// Part boundaries bounds[0 .. P]: bounds[i] = the first pair whose work prefix
// reaches i/P of the total (counts: HOST sizes, or NULL for a uniform batch).
static void enc_bounds(const int32_t *counts, int B, int P, int *bounds) {
    std::vector<double> pre(B + 1, 0.0);
    for (int b = 0; b < B; ++b) pre[b + 1] = pre[b] + (counts ? (double)counts[b] * counts[b] : 1.0);
    bounds[0] = 0;
    bounds[P] = B;
    for (int i = 1; i < P; ++i) {
        const double goal = pre[B] * i / P;
        int h = bounds[i - 1] + 1;
        while (h < B - (P - i) && std::abs(pre[h + 1] - goal) < std::abs(pre[h] - goal)) ++h;
        bounds[i] = h;
    }
}

struct SideStream {
    std::mutex mu;  // one fork / join enqueued at a time per device
    hipStream_t s2[ENC_MAX_PARTS - 1] = {};
    hipEvent_t fork = nullptr, join[ENC_MAX_PARTS - 1] = {};
    bool ok = false;
};
// The side streams of the device that stream s runs on (the current device for
// the legacy default stream), created there on first use.
static SideStream *side_stream(hipStream_t s) {
    static SideStream ss[64];
    hipDevice_t dev = 0;
    if (!s || hipStreamGetDevice(s, &dev) != hipSuccess)
        if (hipGetDevice(&dev) != hipSuccess) return nullptr;
    if (dev < 0 || dev >= 64) return nullptr;
    SideStream &x = ss[dev];
    static std::mutex create_mu;
    std::lock_guard<std::mutex> lock(create_mu);
    if (!x.ok) {  // all or none (a failure leaves the forward on one stream)
        int cur = dev;
        if (hipGetDevice(&cur) != hipSuccess || (cur != dev && hipSetDevice(dev) != hipSuccess)) return nullptr;
        bool ok = x.fork || hipEventCreateWithFlags(&x.fork, hipEventDisableTiming) == hipSuccess;
        for (int i = 0; ok && i < ENC_MAX_PARTS - 1; ++i) {
            if (!x.s2[i]) ok = hipStreamCreateWithFlags(&x.s2[i], hipStreamNonBlocking) == hipSuccess;
            if (ok && !x.join[i]) ok = hipEventCreateWithFlags(&x.join[i], hipEventDisableTiming) == hipSuccess;
        }
        if (cur != dev) (void)hipSetDevice(cur);
        x.ok = ok;
    }
    return x.ok ? &x : nullptr;
}

// The fused plan's encoder over pairs [b0, b0 + nb): every per-pair pointer
// moved to pair b0 (the pair-major layouts of carve_encoder / carve_forward).
static int run_encoder_part(const PackLayout &lay, const float *packed, const float *corr_pos, const float *M,
                            int m_layout, const Dims &d, const EncBufs &e, float *normed, _Float16 *normed_s,
                            float *conf, hipStream_t s, Ragged rg, int b0, int nb) {
    Dims dh = d;
    dh.B = nb;
    const size_t rows = (size_t)b0 * d.Npad * CH;
    EncBufs eh = e;
    eh.feat = e.feat + rows;
    eh.q = e.q + 2 * rows;
    eh.k = e.k + 2 * rows;
    eh.v = e.v + 2 * rows;
    eh.q2 = e.q2 + 2 * rows;
    eh.k2 = e.k2 + 2 * rows;
    eh.v2 = e.v2 + 2 * rows;
    eh.vexp = e.vexp + (size_t)b0 * (d.Npad / 32);
    eh.vexp2 = e.vexp2 + (size_t)b0 * (d.Npad / 32);
    const size_t mstr = m_layout == M_PACKED ? mpack_floats(d.N) : (size_t)d.N * d.N;
    Ragged rh = rg;
    if (rg.nv) rh.nv = rg.nv + b0;
    if (rg.sv) rh.sv = rg.sv + b0;
    if (rg.po) rh.po = rg.po + b0;
    return run_encoder(lay, packed, corr_pos + (size_t)b0 * d.N * lay.in_dim, M + (size_t)b0 * mstr, m_layout, dh,
                       eh, nullptr, normed + (size_t)b0 * d.N * CH, normed_s + (size_t)b0 * d.N * 2 * CH,
                       conf + (size_t)b0 * d.N, s, rh);
}

// run_encoder for the forward: the fused plan as P concurrent parts given side
// streams ss and the part boundaries (enc_halves / enc_bounds; rg.po, when set,
// must then order each part's pairs on its own: launch_ragged_order per part),
// else run_encoder itself.
static int run_encoder_fwd(const PackLayout &lay, const float *packed, const float *corr_pos, const float *M,
                           int m_layout, const Dims &d, const EncBufs &e, float *normed, _Float16 *normed_s,
                           float *conf, hipStream_t s, Ragged rg, SideStream *ss, const int *bounds, int P) {
    if (!ss) return run_encoder(lay, packed, corr_pos, M, m_layout, d, e, nullptr, normed, normed_s, conf, s, rg);
    std::lock_guard<std::mutex> lock(ss->mu);
    // The side streams are shared by every caller stream of the device.  A side
    // stream forked into another thread's graph capture stays in that capture
    // until it ends: enqueueing there from a stream outside that capture would
    // record into (or invalidate) the other graph, so such a call runs on one
    // stream (bitwise the same results).
    {
        hipStreamCaptureStatus cs = hipStreamCaptureStatusNone, c2 = hipStreamCaptureStatusNone;
        unsigned long long id = 0, id2 = 0;
        HIPCHK(hipStreamGetCaptureInfo(s, &cs, &id));
        for (int i = 1; i < P; ++i) {
            HIPCHK(hipStreamGetCaptureInfo(ss->s2[i - 1], &c2, &id2));
            if (c2 != hipStreamCaptureStatusNone && (cs != hipStreamCaptureStatusActive || id2 != id))
                return run_encoder(lay, packed, corr_pos, M, m_layout, d, e, nullptr, normed, normed_s, conf, s, rg);
        }
    }
    HIPCHK(hipEventRecord(ss->fork, s));
    int forked = 1, r = PDSC_OK;
    for (; forked < P; ++forked)
        if (hipStreamWaitEvent(ss->s2[forked - 1], ss->fork, 0) != hipSuccess) {
            r = fail(PDSC_ERR_HIP, "hipStreamWaitEvent (fork)");
            break;
        }
    for (int i = 0; r == PDSC_OK && i < P; ++i)
        r = run_encoder_part(lay, packed, corr_pos, M, m_layout, d, e, normed, normed_s, conf,
                             i ? ss->s2[i - 1] : s, rg, bounds[i], bounds[i + 1] - bounds[i]);
    // join every side stream that was forked, on success AND on error: the
    // caller's stream must not run ahead of work a side stream may still do in
    // the workspace, and a capture must not end with an unjoined fork
    for (int i = 1; i < forked; ++i) {
        const hipError_t a = hipEventRecord(ss->join[i - 1], ss->s2[i - 1]);
        const hipError_t b = a == hipSuccess ? hipStreamWaitEvent(s, ss->join[i - 1], 0) : a;
        if (b != hipSuccess && r == PDSC_OK) r = fail(PDSC_ERR_HIP, "join: %s", hipGetErrorString(b));
    }
    return r;
}

struct NsmBufs {
    float *hist, *weights;
    _Float16 *ns;  // split normed copy (standalone API only; the forward passes pw_last's)
    unsigned *mask;
};

NsmBufs carve_nsm(Carve &c, int B, int N, int S, int k, int T, bool own_split) {
    NsmBufs n;
    n.ns = own_split ? c.take<_Float16>((size_t)B * N * 2 * CH) : nullptr;
    n.hist = c.take<float>((size_t)B * S * std::max(T, 1) * k);
    n.mask = c.take<unsigned>((size_t)B * S);  // per-seed allclose bits
    n.weights = c.take<float>((size_t)B * S * k);
    return n;
}

// normed_s: the split normed copy, or NULL to build it here from normed (H3);
// f32: the Gram reads normed itself
int run_nsm(const float *normed, const _Float16 *normed_s, bool f32, const float *src, const float *tgt,
            const int *knn, int B, int N, int S, int k, int T, const float *sigma, const float *sigma_d,
            const NsmBufs &nb, float *weights, int *iters, bool batch_global, hipStream_t s, Ragged rg = {}) {
    if (!f32 && !normed_s) {
        HIPCHK(launch_split_rows(normed, (size_t)B * N, nb.ns, s));
        normed_s = nb.ns;
    }
    const void *feats = f32 ? static_cast<const void *>(normed) : static_cast<const void *>(normed_s);
    if (T > 0)
        HIPCHK(launch_nsm_seed(feats, f32, src, tgt, knn, B, N, S, k, T, sigma, sigma_d, nb.hist, nb.mask, s, rg));
    HIPCHK(launch_nsm_finish(nb.hist, nb.mask, B, S, k, T, batch_global, weights, iters, s, rg));
    return PDSC_OK;
}

// The testing forward's fused tail launches (nsm_finish inside the hypotheses'
// first launch, select_best + post_refine in one): the same bits, two launches
// fewer per forward.  A/B knob PDSC_TAIL_FUSED=0 (measurement only).
static bool tail_fused() {
    static const bool off = [] {
        const char *e = getenv("PDSC_TAIL_FUSED");
        return e && e[0] == '0';
    }();
    return !off;
}

// A/B knob (measurement only): PDSC_RAGGED_ORDER=0 keeps the ragged attention
// workgroups in pair order.
static bool ragged_order_on() {
    static const bool off = [] {
        const char *e = getenv("PDSC_RAGGED_ORDER");
        return e && e[0] == '0';
    }();
    return !off;
}

struct FwdBufs {
    int *range;  // [B] the fp16 range guard's per-pair flags: the workspace's first bytes (pdsc_range_status)
    float *M, *normed, *conf, *lm, *kdist, *seed_trans, *weights, *hsums;
    _Float16 *normed_s;
    int *seeds, *knn, *counts;
    int *nv, *sv, *po;  // ragged batches: per-pair correspondences and seeds, attention pair order
    EncBufs enc;
    NsmBufs nsm;
};

FwdBufs carve_forward(Carve &c, const Dims &d) {
    FwdBufs f;
    f.range = c.take<int>((size_t)d.B);  // first: at the workspace's base
    // symmetric-packed tiles (PDSC_DENSE_M=1: the dense [N][N] form, for A/B measurement)
    f.M = c.take<float>((size_t)d.B * std::max(mpack_floats(d.N), (size_t)d.N * d.N));  // packed or dense
    f.enc = carve_encoder(c, d);
    f.normed = c.take<float>((size_t)d.B * d.N * CH);
    f.normed_s = c.take<_Float16>((size_t)d.B * d.N * 2 * CH);
    f.conf = c.take<float>((size_t)d.B * d.N);
    f.lm = c.take<float>((size_t)d.B * d.N);
    f.seeds = c.take<int>((size_t)d.B * d.S);
    f.kdist = c.take<float>((size_t)d.B * d.S * d.N);
    f.knn = c.take<int>((size_t)d.B * d.S * d.k);
    f.nsm = carve_nsm(c, d.B, d.N, d.S, d.k, d.T, false);
    f.weights = f.nsm.weights;
    f.seed_trans = c.take<float>((size_t)d.B * d.S * 16);
    f.counts = c.take<int>((size_t)d.B * d.S);
    f.hsums = c.take<float>((size_t)d.B * d.S * 15);
    f.nv = c.take<int>((size_t)d.B);
    f.sv = c.take<int>((size_t)d.B);
    f.po = c.take<int>((size_t)d.B);
    return f;
}

int need_ws(size_t have, size_t need) {
    if (have < need) return fail(PDSC_ERR_ARG, "workspace too small: %zu < %zu bytes", have, need);
    return PDSC_OK;
}

}  // namespace

#define RET_IF(x)                  \
    do {                           \
        int r_ = (x);              \
        if (r_ != PDSC_OK) return r_; \
    } while (0)

namespace {
int32_t check_nn_args(const float *a, const float *b, int32_t Ns, int32_t Nt, int32_t D, void *ws, size_t ws_bytes) {
    if (!a || !b || !ws) return fail(PDSC_ERR_ARG, "null pointer");
    if (Ns < 1 || Nt < 1 || D < 1 || D > 64) return fail(PDSC_ERR_ARG, "Ns=%d Nt=%d D=%d (1 <= D <= 64)", Ns, Nt, D);
    return need_ws(ws_bytes, pdsc_mutual_nn_workspace_bytes(Ns, Nt));
}

__global__ void unpack_nn_kernel(const unsigned long long *key, int n, int32_t *out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = (int32_t)(uint32_t)key[i];
}
}  // namespace

extern "C" {

const char *pdsc_version(void) { return "pdsc 0.1.0 gfx950"; }
const char *pdsc_last_error(void) { return g_err.c_str(); }

// ------------------------------------------------------------------ weights
int32_t pdsc_param_count(const pdsc_config *cfg) { return cfg ? 10 + 26 * cfg->num_layers : -1; }

const char *pdsc_param_name(const pdsc_config *cfg, int32_t i) {
    if (!cfg || i < 0 || i >= pdsc_param_count(cfg)) return nullptr;
    static const char *bn[] = {"weight", "bias", "running_mean", "running_var"};
    static const char *per[] = {"fc_message.0.weight", "fc_message.0.bias", "fc_message.1.weight",
                                "fc_message.1.bias", "fc_message.1.running_mean", "fc_message.1.running_var",
                                "fc_message.3.weight", "fc_message.3.bias", "fc_message.4.weight",
                                "fc_message.4.bias", "fc_message.4.running_mean", "fc_message.4.running_var",
                                "fc_message.6.weight", "fc_message.6.bias", "projection_q.weight",
                                "projection_q.bias", "projection_k.weight", "projection_k.bias",
                                "projection_v.weight", "projection_v.bias"};
    static const char *tail[] = {"encoder.layer0.weight", "encoder.layer0.bias", "classification.0.weight",
                                 "classification.0.bias", "classification.2.weight", "classification.2.bias",
                                 "classification.4.weight", "classification.4.bias"};
    const int L = cfg->num_layers;
    if (i == 0) return "sigma";
    if (i == 1) return "sigma_spat";
    i -= 2;
    if (i < 26 * L) {
        const int l = i / 26, o = i % 26;
        char buf[128];
        if (o < 2)
            snprintf(buf, sizeof(buf), "encoder.blocks.PointCN_layer_%d.0.%s", l, o == 0 ? "weight" : "bias");
        else if (o < 6)
            snprintf(buf, sizeof(buf), "encoder.blocks.PointCN_layer_%d.1.%s", l, bn[o - 2]);
        else
            snprintf(buf, sizeof(buf), "encoder.blocks.NonLocal_layer_%d.%s", l, per[o - 6]);
        g_name = buf;
        return g_name.c_str();
    }
    return tail[i - 26 * L];
}

size_t pdsc_packed_weights_floats(const pdsc_config *cfg) {
    if (check_cfg(cfg) != PDSC_OK) return 0;
    return make_layout(cfg->num_layers, cfg->in_dim).total;
}

int32_t pdsc_pack_weights(const pdsc_config *cfg, const float *const *P, float *packed,
                          pdsc_stream_t stream) {
    RET_IF(check_cfg(cfg));
    if (!P || !packed) return fail(PDSC_ERR_ARG, "null params/packed");
    const int n = pdsc_param_count(cfg);
    for (int i = 0; i < n; ++i)
        if (!P[i]) return fail(PDSC_ERR_ARG, "param %d (%s) is NULL", i, pdsc_param_name(cfg, i));
    hipStream_t s = S_(stream);
    const PackLayout lay = make_layout(cfg->num_layers, cfg->in_dim);
    HIPCHK(hipMemsetAsync(packed, 0, lay.total * sizeof(float), s));
    HIPCHK(launch_copy(P[0], packed + lay.sigma, 1, s));
    HIPCHK(launch_copy(P[1], packed + lay.sigma_d, 1, s));
    const bool f32 = cfg->precision == PDSC_PRECISION_F32;
    auto dense = [&](const DenseOff &o, int wi, int in, int out, bool has_bn) -> hipError_t {
        return launch_pack_dense(P[wi], P[wi + 1], has_bn ? P[wi + 2] : nullptr,
                                 has_bn ? P[wi + 3] : nullptr, has_bn ? P[wi + 4] : nullptr,
                                 has_bn ? P[wi + 5] : nullptr, in, out, f32, packed + o.w, packed + o.bias,
                                 packed + o.alpha, packed + o.beta, packed + o.scale, s);
    };
    for (int l = 0; l < cfg->num_layers; ++l) {
        const int b = 2 + 26 * l;
        const LayerOff &lo = lay.layer[l];
        HIPCHK(dense(lo.pcn, b + 0, CH, CH, true));
        HIPCHK(dense(lo.fc0, b + 6, CH, CH2, true));
        HIPCHK(dense(lo.fc3, b + 12, CH2, CH2, true));
        HIPCHK(dense(lo.fc6, b + 18, CH2, CH, false));
        HIPCHK(dense(lo.q, b + 20, CH, CH, false));
        HIPCHK(dense(lo.k, b + 22, CH, CH, false));
        HIPCHK(dense(lo.v, b + 24, CH, CH, false));
    }
    const int t = 2 + 26 * cfg->num_layers;
    HIPCHK(launch_copy(P[t], packed + lay.l0_w, CH * cfg->in_dim, s));
    HIPCHK(launch_copy(P[t + 1], packed + lay.l0_b, CH, s));
    HIPCHK(dense(lay.c0, t + 2, CH, CLS, false));
    HIPCHK(dense(lay.c2, t + 4, CLS, CLS, false));
    HIPCHK(launch_copy(P[t + 6], packed + lay.c4_w, CLS, s));
    HIPCHK(launch_copy(P[t + 7], packed + lay.c4_b, 1, s));
    return PDSC_OK;
}

// ------------------------------------------------------------------- a1
int32_t pdsc_compat_f32(const float *src, const float *tgt, int32_t B, int32_t N,
                        const float *sigma_d_dev, float *M, pdsc_stream_t stream) {
    if (!src || !tgt || !sigma_d_dev || !M) return fail(PDSC_ERR_ARG, "null pointer");
    if (B < 1 || N < 1) return fail(PDSC_ERR_ARG, "B=%d N=%d", B, N);
    HIPCHK(launch_compat(src, tgt, B, N, sigma_d_dev, M, S_(stream)));
    return PDSC_OK;
}

size_t pdsc_compat_packed_floats(int32_t N) { return N < 1 ? 0 : mpack_floats(N); }

int32_t pdsc_compat_packed_f32(const float *src, const float *tgt, int32_t B, int32_t N,
                               const float *sigma_d_dev, float *Mp, pdsc_stream_t stream) {
    if (!src || !tgt || !sigma_d_dev || !Mp) return fail(PDSC_ERR_ARG, "null pointer");
    if (B < 1 || N < 1) return fail(PDSC_ERR_ARG, "B=%d N=%d", B, N);
    HIPCHK(launch_compat_packed(src, tgt, B, N, sigma_d_dev, Mp, S_(stream)));
    return PDSC_OK;
}

// ---------------------------------------------------------------- a2-a4
// the standalone encoder takes the caller's dense M: its plan never runs attention_w64
static void dims_dense_m(Dims &d) {
    d.w64 = false;
    d.nsplit = attention_nsplit(d.B, d.N, d.f32, false);
    d.precombine = use_precombine(d.B, d.Npad, d.nsplit, d.f32, d.fuse);
}

size_t pdsc_encoder_workspace_bytes(const pdsc_config *cfg, int32_t B, int32_t N) {
    Dims d;
    if (check_cfg(cfg) != PDSC_OK || make_dims(cfg, B, N, d) != PDSC_OK) return 0;
    dims_dense_m(d);
    Carve c(nullptr);
    carve_encoder(c, d);
    return c.off;
}

int32_t pdsc_encoder_f32(const pdsc_config *cfg, const float *packed, const float *corr_pos,
                         const float *M, int32_t B, int32_t N, float *feat, float *normed, float *conf,
                         void *ws, size_t ws_bytes, pdsc_stream_t stream) {
    RET_IF(check_cfg(cfg));
    Dims d;
    RET_IF(make_dims(cfg, B, N, d));
    dims_dense_m(d);
    if (!packed || !corr_pos || !M || !normed || !conf || !ws) return fail(PDSC_ERR_ARG, "null pointer");
    RET_IF(need_ws(ws_bytes, pdsc_encoder_workspace_bytes(cfg, B, N)));
    Carve c(ws);
    const EncBufs e = carve_encoder(c, d);
    const PackLayout lay = make_layout(cfg->num_layers, cfg->in_dim);
    return run_encoder(lay, packed, corr_pos, M, M_DENSE, d, e, feat, normed, nullptr, conf, S_(stream));
}

size_t pdsc_attention_workspace_bytes(int32_t B, int32_t N, int32_t C, int32_t precision) {
    if (C != CH || B < 1 || N < 1 || (precision != PDSC_PRECISION_H3 && precision != PDSC_PRECISION_F32)) return 0;
    const int Npad = round_up(N, QB), ns = attention_nsplit(B, N, precision == PDSC_PRECISION_F32);
    Carve c(nullptr);
    for (int i = 0; i < 3; ++i) c.take<_Float16>((size_t)2 * B * Npad * CH);
    c.take<float>((size_t)B * Npad * CH * ns);
    c.take<float>((size_t)B * Npad * ns * 2);
    c.take<float>((size_t)B * (Npad / 32));
    return c.off;
}

int32_t pdsc_attention_f32(const float *q, const float *k, const float *v, const float *M, int32_t B,
                           int32_t N, int32_t C, int32_t precision, float *msg, void *ws, size_t ws_bytes,
                           pdsc_stream_t stream) {
    if (C != CH) return fail(PDSC_ERR_UNSUPPORTED, "C=%d (only %d)", C, CH);
    if (!q || !k || !v || !M || !msg || !ws) return fail(PDSC_ERR_ARG, "null pointer");
    if (B < 1 || N < 1 || N > 32767) return fail(PDSC_ERR_ARG, "B=%d N=%d", B, N);
    if (precision != PDSC_PRECISION_H3 && precision != PDSC_PRECISION_F32)
        return fail(PDSC_ERR_ARG, "precision=%d", precision);
    RET_IF(need_ws(ws_bytes, pdsc_attention_workspace_bytes(B, N, C, precision)));
    hipStream_t s = S_(stream);
    const bool f32 = precision == PDSC_PRECISION_F32;
    const int Npad = round_up(N, QB), ns = attention_nsplit(B, N, f32);
    Carve c(ws);
    _Float16 *qs = c.take<_Float16>((size_t)2 * B * Npad * CH);
    _Float16 *ks = c.take<_Float16>((size_t)2 * B * Npad * CH);
    _Float16 *vs = c.take<_Float16>((size_t)2 * B * Npad * CH);
    float *op = c.take<float>((size_t)B * Npad * CH * ns);
    float *ml = c.take<float>((size_t)B * Npad * ns * 2);
    float *vexp = c.take<float>((size_t)B * (Npad / 32));
    if (f32) {  // the caller's rows, zero-padded to Npad rows (the same bytes as the split layouts)
        HIPCHK(launch_pad_rows(q, B, N, Npad, reinterpret_cast<float *>(qs), s));
        HIPCHK(launch_pad_rows(k, B, N, Npad, reinterpret_cast<float *>(ks), s));
        HIPCHK(launch_pad_rows(v, B, N, Npad, reinterpret_cast<float *>(vs), s));
    } else {  // the caller's fp32 [B][N][C] rows -> the kernel's padded fp16 hi/lo layouts
        HIPCHK(launch_split_qkv(q, k, v, B, N, N, Npad, qs, ks, vs, vexp, s));
    }
    HIPCHK(launch_attention(qs, ks, vs, vexp, M, M_DENSE, false, f32, B, N, Npad, ns, op, ml, s));
    HIPCHK(launch_attn_combine(op, ml, f32, B, N, Npad, ns, msg, s));
    return PDSC_OK;
}

int32_t pdsc_attention_timing(void *const *start_events, void *const *stop_events, int32_t capacity,
                              int32_t *count) {
    if (capacity > 0 && (!start_events || !stop_events || !count))
        return fail(PDSC_ERR_ARG, "null events/count with capacity %d", capacity);
    g_tstart = reinterpret_cast<hipEvent_t *>(const_cast<void **>(start_events));
    g_tstop = reinterpret_cast<hipEvent_t *>(const_cast<void **>(stop_events));
    g_tcap = capacity;
    g_tcount = count;
    return PDSC_OK;
}

int32_t pdsc_diag_qkv_delay(int32_t loops) {
    if (loops < 0) return fail(PDSC_ERR_ARG, "loops=%d", loops);
    g_diag_qkv_delay = loops;
    return PDSC_OK;
}

int32_t pdsc_forward_timing(void *const *events, int32_t capacity, int32_t *count) {
    if (capacity > 0 && (!events || !count)) return fail(PDSC_ERR_ARG, "null events/count with capacity %d", capacity);
    g_fev = reinterpret_cast<hipEvent_t *>(const_cast<void **>(events));
    g_fcap = capacity;
    g_fcount = count;
    return PDSC_OK;
}

int32_t pdsc_attention_layout(int32_t B, int32_t N, int32_t precision, int32_t *Npad, int32_t *nsplit) {
    if (precision != PDSC_PRECISION_H3 && precision != PDSC_PRECISION_F32)
        return fail(PDSC_ERR_ARG, "precision %d (enum pdsc_precision)", precision);
    if (B < 1 || N < 1 || !Npad || !nsplit) return fail(PDSC_ERR_ARG, "B=%d N=%d", B, N);
    *Npad = round_up(N, QB);
    const bool f32 = precision == PDSC_PRECISION_F32;
    *nsplit = attention_nsplit(B, N, f32, !attention_fused(B, N, f32) && attention_w64(B, N, f32));
    return PDSC_OK;
}

int32_t pdsc_encoder_plan(int32_t B, int32_t N, int32_t precision, int32_t *fused) {
    if (precision != PDSC_PRECISION_H3 && precision != PDSC_PRECISION_F32)
        return fail(PDSC_ERR_ARG, "precision %d (enum pdsc_precision)", precision);
    if (B < 1 || N < 1 || !fused) return fail(PDSC_ERR_ARG, "B=%d N=%d", B, N);
    const bool f32 = precision == PDSC_PRECISION_F32, fu = attention_fused(B, N, f32);
    *fused = fu ? 1 : (attention_w64(B, N, f32) ? 2 : 0);
    return PDSC_OK;
}

// -------------------------------------------------------------------- a5
int32_t pdsc_pick_seeds(const float *src, const float *conf, int32_t B, int32_t N, float radius,
                        int32_t S, int32_t *seeds, float *is_local_max, pdsc_stream_t stream) {
    if (!src || !conf || !seeds || !is_local_max) return fail(PDSC_ERR_ARG, "null pointer (is_local_max is used as scratch)");
    if (B < 1 || N < 1 || S < 1 || S > N) return fail(PDSC_ERR_ARG, "B=%d N=%d S=%d", B, N, S);
    hipStream_t s = S_(stream);
    HIPCHK(launch_local_max(src, conf, B, N, radius, is_local_max, s));
    HIPCHK(launch_seed_rank(conf, is_local_max, B, N, S, seeds, s));
    return PDSC_OK;
}

// -------------------------------------------------------------------- a6
// a6 (:250-252) for the forwards: knn [B][S][k]; dist [B][S][N] scratch
int run_seed_knn(const float *normed, const _Float16 *normed_s, bool f32, const int *seeds, int B, int N, int S,
                 int k, float *dist, int *knn, hipStream_t s, Ragged rg = {}) {
    // (no zero fill of knn: knn_select writes all k entries of every seed row it
    // owns -- ranks 1 .. k of k + 1 distinct (key, index) candidates -- and the
    // rows past a ragged pair's own seeds are never read; readers clamp indices)
    if (f32) {
        HIPCHK(launch_knn_dist_f32(normed, seeds, B, N, S, dist, s, rg));
    } else {
        HIPCHK(launch_knn_dist(normed_s, seeds, B, N, S, dist, s, rg));
    }
    HIPCHK(launch_knn_select(dist, B, N, S, k, knn, s, rg));
    return PDSC_OK;
}

size_t pdsc_seed_knn_workspace_bytes(int32_t B, int32_t N, int32_t S) {
    return align_bytes((size_t)B * S * N * sizeof(float)) + align_bytes((size_t)B * N * 2 * CH * sizeof(_Float16));
}

int32_t pdsc_seed_knn(const float *normed, const int32_t *seeds, int32_t B, int32_t N, int32_t C,
                      int32_t S, int32_t k, int32_t precision, int32_t *knn, void *ws, size_t ws_bytes,
                      pdsc_stream_t stream) {
    if (precision != PDSC_PRECISION_H3 && precision != PDSC_PRECISION_F32)
        return fail(PDSC_ERR_ARG, "precision=%d", precision);
    if (C != CH) return fail(PDSC_ERR_UNSUPPORTED, "C=%d (only %d)", C, CH);
    if (!normed || !seeds || !knn || !ws) return fail(PDSC_ERR_ARG, "null pointer");
    if (B < 1 || S < 1 || k < 1 || k + 1 > N || k > 63) return fail(PDSC_ERR_ARG, "B=%d N=%d S=%d k=%d", B, N, S, k);
    RET_IF(need_ws(ws_bytes, pdsc_seed_knn_workspace_bytes(B, N, S)));
    hipStream_t s = S_(stream);
    Carve c(ws);
    float *dist = c.take<float>((size_t)B * S * N);
    _Float16 *ns = c.take<_Float16>((size_t)B * N * 2 * CH);
    const bool f32 = precision == PDSC_PRECISION_F32;
    if (!f32) HIPCHK(launch_split_rows(normed, (size_t)B * N, ns, s));
    return run_seed_knn(normed, ns, f32, seeds, B, N, S, k, dist, knn, s);
}

// ----------------------------------------------------------------- a7-a8
size_t pdsc_nsm_workspace_bytes(int32_t B, int32_t N, int32_t S, int32_t k, int32_t T) {
    Carve c(nullptr);
    carve_nsm(c, B, N, S, k, T, true);
    return c.off;
}

int32_t pdsc_nsm_weights(const float *normed, const float *src, const float *tgt, const int32_t *knn,
                         int32_t B, int32_t N, int32_t C, int32_t S, int32_t k, int32_t T, int32_t precision,
                         const float *sigma, const float *sigma_d, float *weights, int32_t *iters,
                         void *ws, size_t ws_bytes, pdsc_stream_t stream) {
    if (C != CH) return fail(PDSC_ERR_UNSUPPORTED, "C=%d (only %d)", C, CH);
    if (!normed || !src || !tgt || !knn || !sigma || !sigma_d || !weights || !ws)
        return fail(PDSC_ERR_ARG, "null pointer");
    if (B < 1 || S < 1 || k < 1 || k > 63 || N < k + 1 || T < 0 || T > 31)
        return fail(PDSC_ERR_ARG, "B=%d N=%d S=%d k=%d T=%d (1 <= k <= min(63, N-1), 0 <= T <= 31)", B, N, S, k, T);
    if (precision != PDSC_PRECISION_H3 && precision != PDSC_PRECISION_F32)
        return fail(PDSC_ERR_ARG, "precision=%d", precision);
    RET_IF(need_ws(ws_bytes, pdsc_nsm_workspace_bytes(B, N, S, k, T)));
    Carve c(ws);
    NsmBufs nb = carve_nsm(c, B, N, S, k, T, true);
    return run_nsm(normed, nullptr, precision == PDSC_PRECISION_F32, src, tgt, knn, B, N, S, k, T, sigma, sigma_d,
                   nb, weights, iters, true, S_(stream));
}

// -------------------------------------------------------------------- a9
int32_t pdsc_rigid_transform_3d(const float *A, const float *Bp, const float *w, int32_t nb, int32_t n,
                                float *trans, pdsc_stream_t stream) {
    if (!A || !Bp || !trans) return fail(PDSC_ERR_ARG, "null pointer");
    if (nb < 1 || n < 0) return fail(PDSC_ERR_ARG, "nb=%d n=%d", nb, n);
    HIPCHK(launch_rigid(A, Bp, w, nb, n, trans, S_(stream)));
    return PDSC_OK;
}

// ------------------------------------------------------------------- a10
size_t pdsc_seed_hypotheses_workspace_bytes(int32_t B, int32_t S) {
    return align_bytes((size_t)B * S * 15 * sizeof(float));
}

int32_t pdsc_seed_hypotheses(const float *src, const float *tgt, const int32_t *knn, const float *weights,
                             int32_t B, int32_t N, int32_t S, int32_t k, float tau, float *seed_trans,
                             float *fitness, int32_t *best, float *trans, float *labels, void *ws,
                             size_t ws_bytes, pdsc_stream_t stream) {
    if (!src || !tgt || !knn || !weights || !trans || !labels || !seed_trans)
        return fail(PDSC_ERR_ARG, "null pointer (seed_trans is required as scratch)");
    if (B < 1 || S < 1 || k < 1 || k > 63 || N < k + 1)
        return fail(PDSC_ERR_ARG, "B=%d N=%d S=%d k=%d (1 <= k <= min(63, N-1))", B, N, S, k);
    hipStream_t s = S_(stream);
    // the integer inlier counts live in the caller's fitness buffer until select_best turns
    // each into count / N (same thread, same element)
    if (!fitness) return fail(PDSC_ERR_ARG, "fitness [B,S] buffer is required (hosts the inlier counts)");
    int *counts = reinterpret_cast<int *>(fitness);
    if (!ws || ws_bytes < pdsc_seed_hypotheses_workspace_bytes(B, S))
        return fail(PDSC_ERR_ARG, "workspace too small");
    HIPCHK(launch_hypotheses(src, tgt, knn, weights, B, N, S, k, tau, seed_trans, counts,
                             static_cast<float *>(ws), s));
    HIPCHK(launch_select_best(src, tgt, seed_trans, counts, B, N, S, tau, fitness, best, trans, labels, s));
    return PDSC_OK;
}

// ------------------------------------------------------------------- a11
int32_t pdsc_post_refine(float *trans, const float *src, const float *tgt, int32_t B, int32_t N, float thr,
                         pdsc_stream_t stream) {
    if (!trans || !src || !tgt) return fail(PDSC_ERR_ARG, "null pointer");
    if (B < 1 || N < 1) return fail(PDSC_ERR_ARG, "B=%d N=%d", B, N);
    HIPCHK(launch_post_refine(trans, src, tgt, B, N, thr, S_(stream)));
    return PDSC_OK;
}

// --------------------------------------------------------------- forward
size_t pdsc_forward_workspace_bytes(const pdsc_config *cfg, int32_t B, int32_t N) {
    Dims d;
    if (check_cfg(cfg) != PDSC_OK || make_dims(cfg, B, N, d) != PDSC_OK) return 0;
    Carve c(nullptr);
    carve_forward(c, d);
    return c.off;
}

int32_t pdsc_forward_testing(const pdsc_config *cfg, const float *packed, const float *corr_pos,
                             const float *src, const float *tgt, int32_t B, int32_t N, float *final_trans,
                             float *final_labels, float *conf_out, int32_t *seeds_out, void *ws,
                             size_t ws_bytes, pdsc_stream_t stream) {
    pdsc_forward_debug dbg{};
    dbg.conf = conf_out;
    dbg.seeds = seeds_out;
    return pdsc_forward_testing_debug(cfg, packed, corr_pos, src, tgt, B, N, final_trans, final_labels, &dbg, ws,
                                      ws_bytes, stream);
}

// The testing forward of B pairs; counts (HOST, may be NULL) makes it ragged:
// pair b uses the first counts[b] rows of its N-row buffers.
static int32_t forward_testing_impl(const pdsc_config *cfg, const float *packed, const float *corr_pos,
                                    const float *src, const float *tgt, int32_t B, int32_t N, const int32_t *counts,
                                    float *final_trans, float *final_labels, const pdsc_forward_debug *dbg, void *ws,
                                    size_t ws_bytes, pdsc_stream_t stream) {
    const pdsc_forward_debug no{};
    if (!dbg) dbg = &no;
    RET_IF(check_cfg(cfg));
    Dims d;
    RET_IF(make_dims(cfg, B, N, d));
    if (!packed || !corr_pos || !src || !tgt || !final_trans || !final_labels || !ws)
        return fail(PDSC_ERR_ARG, "null pointer");
    if (counts)
        for (int b = 0; b < B; ++b) {
            // every pair must keep the batch's k = min(cfg k, N - 1) and have >= 1 seed
            const int n = counts[b];
            if (n < 2 || n > N || std::min(cfg->k, n - 1) != d.k || (int)((double)n * cfg->ratio) < 1)
                return fail(PDSC_ERR_ARG, "counts[%d] = %d: need k + 1 = %d <= count <= N = %d and int(count * ratio) >= 1",
                            b, n, d.k + 1, N);
        }
    RET_IF(need_ws(ws_bytes, pdsc_forward_workspace_bytes(cfg, B, N)));
    hipStream_t s = S_(stream);
    Carve c(ws);
    const FwdBufs f = carve_forward(c, d);
    Ragged rg;
    SideStream *halves = enc_halves(d, counts != nullptr) ? side_stream(s) : nullptr;
    const int parts = halves ? enc_parts() : 1;
    int bounds[ENC_MAX_PARTS + 1] = {0, B};
    if (halves) enc_bounds(enc_work_balanced() ? counts : nullptr, B, parts, bounds);
    if (counts) {
        HIPCHK(launch_ragged_setup(counts, B, cfg->ratio, f.nv, f.sv, s));
        rg.nv = f.nv;
        rg.sv = f.sv;
        rg.eq = std::all_of(counts, counts + B, [N](int32_t n) { return n == N; });
        if (ragged_order_on()) {  // each part's attention launches order that part's pairs
            for (int i = 0; i < parts; ++i)
                HIPCHK(launch_ragged_order(counts + bounds[i], bounds[i + 1] - bounds[i], f.po + bounds[i], s));
            rg.po = f.po;
        }
    }
    const PackLayout lay = make_layout(cfg->num_layers, cfg->in_dim);
    const float *sigma = packed + lay.sigma, *sigma_d = packed + lay.sigma_d;
    const bool timed = g_fcap > 0 && g_fcount && *g_fcount + PDSC_FORWARD_STAGES + 1 <= g_fcap;
    hipEvent_t *ev = timed ? g_fev + *g_fcount : nullptr;
    if (timed) *g_fcount += PDSC_FORWARD_STAGES + 1;
#define STAGE(i) \
    if (ev) HIPCHK(hipEventRecord(ev[i], s))
    STAGE(0);
    // a1 (:150-153).  (r04: a1 on a second stream beside the encoder's first
    // launch measured no gain at 128 x 1000 / 8 x 5000 and +44 us per single
    // pair -- the cross-stream event pair -- so the forward stays on one stream.)
    const int mlay = forward_m_layout(d);
    if (mlay == M_PACKED)
        HIPCHK(launch_compat_packed(src, tgt, d.B, d.N, sigma_d, f.M, s, rg));
    else
        HIPCHK(launch_compat(src, tgt, d.B, d.N, sigma_d, f.M, s, rg));
    STAGE(1);
    // a2-a4 (:155-156, :171)
    RET_IF(run_encoder_fwd(lay, packed, corr_pos, f.M, mlay, d, f.enc, f.normed, f.normed_s, f.conf, s, rg, halves,
                           bounds, parts));
    STAGE(2);
    // a5 (:174)
    HIPCHK(launch_local_max(src, f.conf, d.B, d.N, cfg->nms_radius, f.lm, s, rg));
    // (kdist, written by the seed kNN next, is the ranking's scratch)
    HIPCHK(launch_seed_rank(f.conf, f.lm, d.B, d.N, d.S, f.seeds, s, rg, reinterpret_cast<uint32_t *>(f.kdist)));
    STAGE(3);
    // a6 (:250-252)
    RET_IF(run_seed_knn(f.normed, f.normed_s, d.f32, f.seeds, d.B, d.N, d.S, d.k, f.kdist, f.knn, s, rg));
    STAGE(4);
    // a7-a8 (:257-282)
    // per pair: each pair is its own bs = 1 forward, whose allclose spans its S seeds.
    // The power iterates here; nsm_finish's step (t*, the normalised weights) runs
    // inside the hypotheses' first launch below (the same bits, one launch fewer).
    const bool tail = tail_fused();
    if (!tail) {
        RET_IF(run_nsm(f.normed, f.normed_s, d.f32, src, tgt, f.knn, d.B, d.N, d.S, d.k, d.T, sigma, sigma_d, f.nsm,
                       f.weights, nullptr, false, s, rg));
    } else if (d.T > 0)
        HIPCHK(launch_nsm_seed(d.f32 ? static_cast<const void *>(f.normed) : static_cast<const void *>(f.normed_s),
                               d.f32, src, tgt, f.knn, d.B, d.N, d.S, d.k, d.T, sigma, sigma_d, f.nsm.hist, f.nsm.mask,
                               s, rg));
    STAGE(5);
    // a9-a10 (:280-282, :287-335)
    HIPCHK(launch_hypotheses(src, tgt, f.knn, f.weights, d.B, d.N, d.S, d.k, cfg->inlier_threshold,
                             f.seed_trans, f.counts, f.hsums, s, rg, tail ? f.nsm.hist : nullptr, f.nsm.mask, d.T,
                             f.weights));
    if (dbg->trans_pre_refine || !tail) {  // the pose before refinement: the two launches
        HIPCHK(launch_select_best(src, tgt, f.seed_trans, f.counts, d.B, d.N, d.S, cfg->inlier_threshold,
                                  nullptr, nullptr, final_trans, final_labels, s, rg, f.conf, f.range));
        if (dbg->trans_pre_refine)
            HIPCHK(hipMemcpyAsync(dbg->trans_pre_refine, final_trans, sizeof(float) * 16 * d.B, hipMemcpyDeviceToDevice,
                                  s));
        STAGE(6);
        // a11 (:186, :403-438)
        HIPCHK(launch_post_refine(final_trans, src, tgt, d.B, d.N, cfg->refine_threshold, s, rg, f.range));
    } else {
        // a10 best + a11 in one launch (select_best's and post_refine's workgroup
        // bodies back to back; the stage split of the two is then not measured)
        STAGE(6);
        HIPCHK(launch_best_refine(src, tgt, f.seed_trans, f.counts, d.B, d.N, d.S, cfg->inlier_threshold,
                                  cfg->refine_threshold, final_trans, final_labels, s, rg, f.conf, f.range));
    }
    STAGE(7);
#undef STAGE
    if (dbg->conf) HIPCHK(hipMemcpyAsync(dbg->conf, f.conf, sizeof(float) * d.B * d.N, hipMemcpyDeviceToDevice, s));
    if (dbg->seeds) HIPCHK(hipMemcpyAsync(dbg->seeds, f.seeds, sizeof(int) * d.B * d.S, hipMemcpyDeviceToDevice, s));
    if (dbg->knn) HIPCHK(hipMemcpyAsync(dbg->knn, f.knn, sizeof(int) * d.B * d.S * d.k, hipMemcpyDeviceToDevice, s));
    if (dbg->weights)
        HIPCHK(hipMemcpyAsync(dbg->weights, f.weights, sizeof(float) * d.B * d.S * d.k, hipMemcpyDeviceToDevice, s));
    return PDSC_OK;
}

int32_t pdsc_forward_testing_debug(const pdsc_config *cfg, const float *packed, const float *corr_pos,
                                   const float *src, const float *tgt, int32_t B, int32_t N, float *final_trans,
                                   float *final_labels, const pdsc_forward_debug *dbg, void *ws, size_t ws_bytes,
                                   pdsc_stream_t stream) {
    return forward_testing_impl(cfg, packed, corr_pos, src, tgt, B, N, nullptr, final_trans, final_labels, dbg, ws,
                                ws_bytes, stream);
}

int32_t pdsc_forward_testing_ragged(const pdsc_config *cfg, const float *packed, const float *corr_pos,
                                    const float *src, const float *tgt, int32_t B, int32_t N, const int32_t *counts,
                                    float *final_trans, float *final_labels, const pdsc_forward_debug *dbg, void *ws,
                                    size_t ws_bytes, pdsc_stream_t stream) {
    if (!counts) return fail(PDSC_ERR_ARG, "counts is NULL");
    return forward_testing_impl(cfg, packed, corr_pos, src, tgt, B, N, counts, final_trans, final_labels, dbg, ws,
                                ws_bytes, stream);
}


// ------------------------------------------- f3 training-mode forward and loss
size_t pdsc_forward_training_workspace_bytes(const pdsc_config *cfg, int32_t B, int32_t N) {
    return pdsc_forward_workspace_bytes(cfg, B, N);
}

int32_t pdsc_forward_training(const pdsc_config *cfg, const float *packed, const float *corr_pos, const float *src,
                              const float *tgt, int32_t B, int32_t N, float *final_trans, float *confidence,
                              float *M_out, int32_t *seeds_out, void *ws, size_t ws_bytes, pdsc_stream_t stream) {
    RET_IF(check_cfg(cfg));
    Dims d;
    RET_IF(make_dims(cfg, B, N, d));
    if (!packed || !corr_pos || !src || !tgt || !final_trans || !confidence || !ws)
        return fail(PDSC_ERR_ARG, "null pointer");
    RET_IF(need_ws(ws_bytes, pdsc_forward_training_workspace_bytes(cfg, B, N)));
    hipStream_t s = S_(stream);
    Carve c(ws);
    const FwdBufs f = carve_forward(c, d);
    const PackLayout lay = make_layout(cfg->num_layers, cfg->in_dim);
    const float *sigma = packed + lay.sigma, *sigma_d = packed + lay.sigma_d;
    // a1-a4 as in testing (:150-156, :171)
    const int mlay = forward_m_layout(d);
    if (mlay == M_PACKED)
        HIPCHK(launch_compat_packed(src, tgt, d.B, d.N, sigma_d, f.M, s));
    else
        HIPCHK(launch_compat(src, tgt, d.B, d.N, sigma_d, f.M, s));
    RET_IF(run_encoder(lay, packed, corr_pos, f.M, mlay, d, f.enc, nullptr, f.normed, f.normed_s, f.conf, s));
    // the loss's feature-similarity M (:158-163)
    if (M_out)
        HIPCHK(launch_feat_sim(d.f32 ? static_cast<const void *>(f.normed) : static_cast<const void *>(f.normed_s),
                               d.f32, d.B, d.N, sigma, M_out, s));
    // seeds = argsort(confidence, descending)[:, :S] (:176): the ranking with every flag 1
    HIPCHK(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(f.lm), 0x3f800000u, (size_t)d.B * d.N, s));
    HIPCHK(launch_seed_rank(f.conf, f.lm, d.B, d.N, d.S, f.seeds, s));
    // a6-a10 as in testing (:182 -> cal_seed_trans), no post-refinement (:185-186)
    // (f.counts: the hypotheses' inlier counts later, the overflow flags here)
    RET_IF(run_seed_knn(f.normed, f.normed_s, d.f32, f.seeds, d.B, d.N, d.S, d.k, f.kdist, f.knn, s));
    // the training batch is ONE reference forward: torch.allclose over all B * S seeds (:354)
    RET_IF(run_nsm(f.normed, f.normed_s, d.f32, src, tgt, f.knn, d.B, d.N, d.S, d.k, d.T, sigma, sigma_d, f.nsm,
                   f.weights, nullptr, true, s));
    HIPCHK(launch_hypotheses(src, tgt, f.knn, f.weights, d.B, d.N, d.S, d.k, cfg->inlier_threshold, f.seed_trans,
                             f.counts, f.hsums, s));
    // the labels of the best hypothesis are not returned in training mode (:189-191): f.lm is scratch
    HIPCHK(launch_select_best(src, tgt, f.seed_trans, f.counts, d.B, d.N, d.S, cfg->inlier_threshold, nullptr,
                              nullptr, final_trans, f.lm, s, {}, f.conf, f.range));
    HIPCHK(hipMemcpyAsync(confidence, f.conf, sizeof(float) * d.B * d.N, hipMemcpyDeviceToDevice, s));
    if (seeds_out) HIPCHK(hipMemcpyAsync(seeds_out, f.seeds, sizeof(int) * d.B * d.S, hipMemcpyDeviceToDevice, s));
    return PDSC_OK;
}

int32_t pdsc_range_status(const void *ws, int32_t B, int32_t *flags, pdsc_stream_t stream) {
    if (!ws || B < 1) return fail(PDSC_ERR_ARG, "ws=%p B=%d", ws, B);
    std::vector<int32_t> h((size_t)B);
    hipStream_t s = S_(stream);
    HIPCHK(hipMemcpyAsync(h.data(), ws, sizeof(int32_t) * B, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    int bad = 0;
    for (int b = 0; b < B; ++b) {
        if (flags) flags[b] = h[b];
        bad += h[b] != 0;
    }
    if (bad) return fail(PDSC_ERR_RANGE, "%d of %d pairs left the fp16 range (rerun them with PDSC_PRECISION_F32)", bad, B);
    return PDSC_OK;
}

// pdsc_range_poll: one wavefront ORs the B marks and stores (seq << 1) | any into
// a word of coherent page-locked host memory (a system-scope release store);
// the host spins on the word instead of a D2H copy + stream synchronisation
// (the copy alone: 12.6 us on an idle MI355X stream, tools/dropin_breakdown.py).
__global__ __launch_bounds__(64) void range_publish_kernel(const int32_t *__restrict__ range, int B,
                                                           uint32_t *word, uint32_t seq) {
    bool any = false;
    for (int b = threadIdx.x; b < B; b += 64) any |= range[b] != 0;
    const bool m = __ballot(any) != 0;
    if (threadIdx.x == 0) __hip_atomic_store(word, (seq << 1) | (m ? 1u : 0u), __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

namespace {
struct PollWord {
    uint32_t *host = nullptr, *dev = nullptr;
    uint32_t seq = 0;
    ~PollWord() {
        if (host) (void)hipHostFree(host);
    }
};
thread_local PollWord g_poll;  // one word per host thread: its calls wait one at a time
}  // namespace

int32_t pdsc_range_poll(const void *ws, int32_t B, pdsc_stream_t stream) {
    if (!ws || B < 1) return fail(PDSC_ERR_ARG, "ws=%p B=%d", ws, B);
    hipStream_t s = S_(stream);
    PollWord &w = g_poll;
    if (!w.host) {
        void *h = nullptr, *dp = nullptr;
        HIPCHK(hipHostMalloc(&h, 64, hipHostMallocPortable | hipHostMallocMapped | hipHostMallocCoherent));
        if (hipHostGetDevicePointer(&dp, h, 0) != hipSuccess) {
            (void)hipHostFree(h);
            return fail(PDSC_ERR_HIP, "hipHostGetDevicePointer");
        }
        w.host = static_cast<uint32_t *>(h);
        w.dev = static_cast<uint32_t *>(dp);
        __atomic_store_n(w.host, 0u, __ATOMIC_RELEASE);
    }
    w.seq = (w.seq + 1) & 0x7fffffffu;
    if (w.seq == 0) w.seq = 1;  // 0 is the word's initial value
    const uint32_t seq = w.seq;
    hipLaunchKernelGGL(range_publish_kernel, dim3(1), dim3(64), 0, s, static_cast<const int32_t *>(ws), (int)B, w.dev,
                       seq);
    HIPCHK(hipGetLastError());
    // spin ~20 ms at most (the forward's own device time is well below), then
    // block in hipStreamSynchronize: it also reports a faulted stream
    uint32_t v = 0;
    bool seen = false;
    const auto t0 = std::chrono::steady_clock::now();
    for (unsigned it = 1;; ++it) {
        v = __atomic_load_n(w.host, __ATOMIC_ACQUIRE);
        if ((v >> 1) == seq) {
            seen = true;
            break;
        }
        __builtin_ia32_pause();
        if ((it & 1023u) == 0 && std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(20)) break;
    }
    if (!seen) {
        HIPCHK(hipStreamSynchronize(s));
        v = __atomic_load_n(w.host, __ATOMIC_ACQUIRE);
        if ((v >> 1) != seq) return fail(PDSC_ERR_HIP, "range word %u after the stream drained (expected %u)", v >> 1, seq);
    }
    if (v & 1u) return fail(PDSC_ERR_RANGE, "a pair of %d left the fp16 range (rerun it with PDSC_PRECISION_F32)", B);
    return PDSC_OK;
}

size_t pdsc_spectral_matching_loss_workspace_bytes(int32_t B, int32_t N) {
    return (B < 1 || N < 1) ? 0 : align_bytes(sm_loss_partial_doubles(B, N) * sizeof(double));
}

int32_t pdsc_spectral_matching_loss(const float *M, const float *gt_labels, int32_t B, int32_t N, int32_t balanced,
                                    float *loss, void *ws, size_t ws_bytes, pdsc_stream_t stream) {
    if (!M || !gt_labels || !loss || !ws) return fail(PDSC_ERR_ARG, "null pointer");
    if (B < 1 || N < 1) return fail(PDSC_ERR_ARG, "B=%d N=%d", B, N);
    RET_IF(need_ws(ws_bytes, pdsc_spectral_matching_loss_workspace_bytes(B, N)));
    HIPCHK(launch_sm_loss(M, gt_labels, B, N, balanced, static_cast<double *>(ws), loss, S_(stream)));
    return PDSC_OK;
}

// ------------------------------------------------------ f4 descriptor stage
int32_t pdsc_ply_read_xyz(const char *path, float *xyz, int64_t capacity, int64_t *n_points) {
    if (!path || !n_points) return fail(PDSC_ERR_ARG, "null pointer");
    std::string err;
    if (ply_read_xyz(path, xyz, capacity, n_points, err) != 0) return fail(PDSC_ERR_ARG, "PLY: %s", err.c_str());
    return PDSC_OK;
}

static int check_cloud(const float *pts, int32_t n, float r, int32_t max_nn) {
    if (!pts) return fail(PDSC_ERR_ARG, "null points");
    if (n < 1) return fail(PDSC_ERR_ARG, "n=%d", n);
    if (!(r > 0.0f) || !std::isfinite(r)) return fail(PDSC_ERR_ARG, "radius / voxel size %g must be > 0", (double)r);
    if (max_nn < 1 || max_nn > 128) return fail(PDSC_ERR_UNSUPPORTED, "max_nn=%d not in [1, 128]", max_nn);
    return PDSC_OK;
}

// the device error flags of a grid pass, after the stream drained
static int grid_status(const GridBufs &G, hipStream_t s) {
    int e[2] = {0, 0};
    HIPCHK(hipMemcpyAsync(e, G.err, sizeof e, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    if (e[0]) return fail(PDSC_ERR_ARG, "cloud extent / cell size >= 2^21 cells per axis");
    if (e[1]) return fail(PDSC_ERR_UNSUPPORTED, "a radius neighbourhood holds > 1024 points within one d^2 bin");
    return PDSC_OK;
}

size_t pdsc_radius_knn_workspace_bytes(int32_t n) { return n < 1 ? 0 : grid_workspace_bytes(n); }

int32_t pdsc_radius_knn(const float *pts, int32_t n, float radius, int32_t max_nn, int32_t *nbr, double *dist2,
                        int32_t *count, void *ws, size_t ws_bytes, pdsc_stream_t stream) {
    RET_IF(check_cloud(pts, n, radius, max_nn));
    if (!nbr || !count || !ws) return fail(PDSC_ERR_ARG, "null pointer");
    RET_IF(need_ws(ws_bytes, pdsc_radius_knn_workspace_bytes(n)));
    hipStream_t s = S_(stream);
    GridBufs G;
    HIPCHK(build_grid(pts, n, radius, 0.0, ws, G, s));
    HIPCHK(launch_radius_knn(pts, n, G, radius, max_nn, nbr, dist2, count, s));
    return grid_status(G, s);
}

size_t pdsc_estimate_normals_workspace_bytes(int32_t n, int32_t max_nn) {
    if (n < 1 || max_nn < 1) return 0;
    return grid_workspace_bytes(n) + align_bytes((size_t)n * max_nn * sizeof(int)) + align_bytes((size_t)n * sizeof(int));
}

int32_t pdsc_estimate_normals(const float *pts, int32_t n, float radius, int32_t max_nn, int32_t orient,
                              const float *viewpoint, float *normals, void *ws, size_t ws_bytes, pdsc_stream_t stream) {
    RET_IF(check_cloud(pts, n, radius, max_nn));
    if (!normals || !ws) return fail(PDSC_ERR_ARG, "null pointer");
    if (orient != PDSC_NORMALS_OPEN3D && orient != PDSC_NORMALS_VIEWPOINT && orient != PDSC_NORMALS_CENTROID)
        return fail(PDSC_ERR_ARG, "orient=%d (enum pdsc_normal_orientation)", orient);
    if (orient == PDSC_NORMALS_VIEWPOINT && !viewpoint) return fail(PDSC_ERR_ARG, "PDSC_NORMALS_VIEWPOINT needs a viewpoint");
    RET_IF(need_ws(ws_bytes, pdsc_estimate_normals_workspace_bytes(n, max_nn)));
    hipStream_t s = S_(stream);
    char *w = static_cast<char *>(ws);
    int *nbr = reinterpret_cast<int *>(w + grid_workspace_bytes(n));
    int *cnt = reinterpret_cast<int *>(reinterpret_cast<char *>(nbr) + align_bytes((size_t)n * max_nn * sizeof(int)));
    GridBufs G;
    HIPCHK(build_grid(pts, n, radius, 0.0, ws, G, s));
    HIPCHK(launch_radius_knn(pts, n, G, radius, max_nn, nbr, nullptr, cnt, s));
    HIPCHK(launch_normals(pts, n, nbr, cnt, max_nn, G, orient, viewpoint, normals, s));
    return grid_status(G, s);
}

size_t pdsc_voxel_down_sample_workspace_bytes(int32_t n) { return n < 1 ? 0 : grid_workspace_bytes(n); }

int32_t pdsc_voxel_down_sample(const float *pts, const float *normals, int32_t n, float voxel_size, float *out_pts,
                               float *out_normals, int32_t *out_count, void *ws, size_t ws_bytes,
                               pdsc_stream_t stream) {
    RET_IF(check_cloud(pts, n, voxel_size, 1));
    if (!out_pts || !out_count || !ws) return fail(PDSC_ERR_ARG, "null pointer");
    RET_IF(need_ws(ws_bytes, pdsc_voxel_down_sample_workspace_bytes(n)));
    hipStream_t s = S_(stream);
    GridBufs G;
    HIPCHK(build_grid(pts, n, voxel_size, 0.5 * (double)voxel_size, ws, G, s));
    HIPCHK(launch_voxel_reduce(pts, normals, n, G, out_pts, out_normals, out_count, s));
    return grid_status(G, s);
}

size_t pdsc_compute_fpfh_workspace_bytes(int32_t n, int32_t max_nn) {
    if (n < 1 || max_nn < 1) return 0;
    return grid_workspace_bytes(n) + align_bytes((size_t)n * max_nn * sizeof(int)) +
           align_bytes((size_t)n * max_nn * sizeof(double)) + align_bytes((size_t)n * sizeof(int)) +
           align_bytes((size_t)n * 33 * sizeof(double));
}

int32_t pdsc_compute_fpfh(const float *pts, const float *normals, int32_t n, float radius, int32_t max_nn,
                          double *fpfh, float *fpfh_normalized, void *ws, size_t ws_bytes, pdsc_stream_t stream) {
    RET_IF(check_cloud(pts, n, radius, max_nn));
    if (!normals || !fpfh || !ws) return fail(PDSC_ERR_ARG, "null pointer");
    RET_IF(need_ws(ws_bytes, pdsc_compute_fpfh_workspace_bytes(n, max_nn)));
    hipStream_t s = S_(stream);
    char *w = static_cast<char *>(ws) + grid_workspace_bytes(n);
    int *nbr = reinterpret_cast<int *>(w);
    w += align_bytes((size_t)n * max_nn * sizeof(int));
    double *d2 = reinterpret_cast<double *>(w);
    w += align_bytes((size_t)n * max_nn * sizeof(double));
    int *cnt = reinterpret_cast<int *>(w);
    w += align_bytes((size_t)n * sizeof(int));
    double *spfh = reinterpret_cast<double *>(w);
    GridBufs G;
    HIPCHK(build_grid(pts, n, radius, 0.0, ws, G, s));
    HIPCHK(launch_radius_knn(pts, n, G, radius, max_nn, nbr, d2, cnt, s));
    HIPCHK(launch_fpfh(pts, normals, n, nbr, cnt, d2, max_nn, spfh, fpfh, fpfh_normalized, s));
    return grid_status(G, s);
}

// ------------------------------------------------- f1 correspondence construction
size_t pdsc_mutual_nn_workspace_bytes(int32_t Ns, int32_t Nt) {
    return align_bytes((size_t)Ns * 8) + align_bytes((size_t)Nt * 8);
}


int32_t pdsc_mutual_nn(const float *src_desc, const float *tgt_desc, int32_t Ns, int32_t Nt, int32_t D,
                       int32_t *nn_src, int32_t *nn_tgt, void *ws, size_t ws_bytes, pdsc_stream_t stream) {
    RET_IF(check_nn_args(src_desc, tgt_desc, Ns, Nt, D, ws, ws_bytes));
    if (!nn_src || !nn_tgt) return fail(PDSC_ERR_ARG, "null pointer");
    hipStream_t s = S_(stream);
    Carve c(ws);
    unsigned long long *rk = c.take<unsigned long long>(Ns), *ck = c.take<unsigned long long>(Nt);
    HIPCHK(launch_nn_argmin(src_desc, tgt_desc, Ns, Nt, D, rk, ck, s));
    hipLaunchKernelGGL(unpack_nn_kernel, dim3((Ns + 255) / 256), dim3(256), 0, s, rk, Ns, nn_src);
    hipLaunchKernelGGL(unpack_nn_kernel, dim3((Nt + 255) / 256), dim3(256), 0, s, ck, Nt, nn_tgt);
    HIPCHK(hipGetLastError());
    return PDSC_OK;
}

int32_t pdsc_build_correspondences(const float *src_desc, const float *tgt_desc, const float *src_xyz,
                                   const float *tgt_xyz, int32_t Ns, int32_t Nt, int32_t D, int32_t mutual,
                                   const double *gt_trans, double inlier_threshold, int32_t *corr,
                                   int32_t *count, float *corr_pos, float *src_keypts, float *tgt_keypts,
                                   float *labels, void *ws, size_t ws_bytes, pdsc_stream_t stream) {
    RET_IF(check_nn_args(src_desc, tgt_desc, Ns, Nt, D, ws, ws_bytes));
    if (!src_xyz || !tgt_xyz || !corr || !count || !corr_pos || !src_keypts || !tgt_keypts)
        return fail(PDSC_ERR_ARG, "null pointer");
    if (gt_trans && !labels) return fail(PDSC_ERR_ARG, "gt_trans given without labels");
    hipStream_t s = S_(stream);
    Carve c(ws);
    unsigned long long *rk = c.take<unsigned long long>(Ns), *ck = c.take<unsigned long long>(Nt);
    HIPCHK(launch_nn_argmin(src_desc, tgt_desc, Ns, Nt, D, rk, ck, s));
    HIPCHK(launch_corr_build(rk, ck, src_xyz, tgt_xyz, Ns, mutual ? 1 : 0, gt_trans, inlier_threshold, corr, count,
                             corr_pos, src_keypts, tgt_keypts, gt_trans ? labels : nullptr, s));
    return PDSC_OK;
}

// ------------------------------------------------ f3 spectral-matching baseline
size_t pdsc_spectral_matching_workspace_bytes(int32_t N) {
    return align_bytes((size_t)N * N * sizeof(float)) + 3 * align_bytes((size_t)N * sizeof(float));
}

int32_t pdsc_spectral_matching(const float *corr_pos, const float *src, const float *tgt, int32_t N,
                               double inlier_threshold, double top_ratio, int32_t iters, float *trans,
                               float *labels, float *leading_eig, void *ws, size_t ws_bytes, pdsc_stream_t stream) {
    if (!corr_pos || !src || !tgt || !trans || !labels || !ws) return fail(PDSC_ERR_ARG, "null pointer");
    if (N < 1 || N > 46340 || iters < 0 || !(top_ratio >= 0.0 && top_ratio <= 1.0) || !(inlier_threshold > 0.0))
        return fail(PDSC_ERR_ARG, "N=%d iters=%d top_ratio=%g inlier_threshold=%g", N, iters, top_ratio,
                    inlier_threshold);
    RET_IF(need_ws(ws_bytes, pdsc_spectral_matching_workspace_bytes(N)));
    Carve c(ws);
    float *M = c.take<float>((size_t)N * N), *v = c.take<float>(N), *y = c.take<float>(N), *w = c.take<float>(N);
    if (leading_eig) v = leading_eig;
    const double sigma = inlier_threshold / 3.0;  // :34 (python float)
    const float sig2 = (float)(sigma * sigma);    // tensor / python scalar -> fp32 divisor
    const int S = (int)(N * top_ratio);           // int(leading_eig.shape[1] * top_ratio) (:46)
    HIPCHK(launch_sm(corr_pos, src, tgt, N, sig2, S, iters, M, v, y, w, labels, trans, S_(stream)));
    return PDSC_OK;
}

int32_t pdsc_sm_matvec(const float *M, const float *v, int32_t N, float *y, pdsc_stream_t stream) {
    if (!M || !v || !y) return fail(PDSC_ERR_ARG, "null pointer");
    if (N < 1) return fail(PDSC_ERR_ARG, "N=%d", N);
    HIPCHK(launch_sm_matvec(M, v, N, y, S_(stream)));
    return PDSC_OK;
}

}  // extern "C"
