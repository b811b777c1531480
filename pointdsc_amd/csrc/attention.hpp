// attention.hpp -- the SCNonlocal attention core (models/PointDSC.py:36-42),
// flash-style on fp32 MFMA, as a template so variants can be A/B-timed in one
// process (tools/attn_bench.hip).  The production instantiation is chosen in
// encoder.hip.
//
//   msg_i = sum_j softmax_j( M_ij * (q_i . k_j) / sqrt(C) ) v_j,   C = 128, heads = 1
//
// Work decomposition: a workgroup = NW waves x 32 queries of one pair and a
// contiguous range ("split") of key stages; a stage = KTS keys staged in LDS
// (double-buffered, register-staged); each stage is consumed as KTS/32
// sub-tiles of 32 keys.  Per wave and sub-tile: S^T = K Q^T (64 MFMA
// 32x32x2 f32, lane <-> query), logits scaled by M (read column-wise: M is
// symmetric, so M[q][key] = M[key][q] and one 128-B row segment per key),
// online softmax with a lazily re-based running max, O += P V (64 MFMA, P in
// the S^T accumulator layout is already the A operand).
//
// Numerics: fp32 throughout; exp via v_exp_f32 on log2e-prescaled logits
// (FASTEXP) or libm expf; the max is re-based only when it grows by more than
// DEFER (log2 units) -- exact in real arithmetic, bounded growth 2^DEFER.
#pragma once
#include "pdsc_internal.hpp"

namespace pdsc {

constexpr int A_KSTR = CH + 4;  // K row stride in LDS: conflict-free ds_read_b128 columns
constexpr int A_VSTR = CH;

template <int NW, int KTS, bool GLDS = false>
constexpr size_t attention_lds_bytes() {
    return GLDS ? (size_t)2 * KTS * (2 * CH) * sizeof(float) : (size_t)2 * KTS * (A_KSTR + A_VSTR) * sizeof(float);
}

PDSC_DEV __amdgpu_buffer_rsrc_t make_rsrc(const void *base, uint32_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(base), 0, (int)bytes, 0x00020000);
}
PDSC_DEV float buf_ld(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff) {
    return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, voff, soff, 0));
}
PDSC_DEV f32x4 buf_ld4(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff) {
    return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, voff, soff, 0));
}

struct AttnGrid {
    int B, N, Npad, nqb, nsplit, sps;  // sps = stages per split
    const int *nv;  // ragged batches: pair b's correspondences (N, Npad: the strides), or null
    PDSC_DEV int n(int b) const { return nv ? nv[b] : N; }
};

// Host: split-K factor so that the grid fills the chip (~`target` workgroups).
template <int NW, int KTS>
inline AttnGrid attention_grid(int B, int N, int target) {
    AttnGrid g;
    g.nv = nullptr;
    g.B = B;
    g.N = N;
    g.Npad = round_up(N, QB);
    g.nqb = (N + NW * 32 - 1) / (NW * 32);
    const int nst = (N + KTS - 1) / KTS;
    int ns = (target + B * g.nqb - 1) / (B * g.nqb);
    ns = std::max(1, std::min(ns, std::max(1, nst / 2)));
    g.sps = (nst + ns - 1) / ns;
    g.nsplit = (nst + g.sps - 1) / g.sps;
    return g;
}

// blockIdx.x -> logical (pair, query block, split), keeping a pair's blocks on
// one XCD (blocks b and b+8 share an XCD under round-robin dispatch; speed only).
PDSC_DEV void attention_block_coords(const AttnGrid &g, bool xcd, int &b, int &qb, int &split) {
    const int G = g.B * g.nqb * g.nsplit;
    int lid = blockIdx.x;
    if (xcd) {
        const int full = G & ~7;
        if (lid < full) lid = (lid & 7) * (full >> 3) + (lid >> 3);
    }
    split = lid % g.nsplit;
    const int r = lid / g.nsplit;
    qb = r % g.nqb;
    b = r / g.nqb;
}

// GLDS: stage K/V with LDS-DMA (global_load_lds_dwordx4, one 1-KiB piece = two
// 512-B rows per wave-instruction, no staging registers).  K rows are stored
// unpadded with their 16-B chunks XOR-swizzled by (row & 15) -- the swizzle is
// applied to the SOURCE address (the DMA writes LDS lane-linearly) and undone on
// the ds_read_b128 side, keeping the column reads conflict-free.
template <int NW, int KTS, bool FASTEXP, bool XCD, int BUF = 3, bool GLDS = false>
__global__ __launch_bounds__(NW * 64, (NW == 4 ? 2 : 1)) void attention_kernel_t(
    const float *__restrict__ q, const float *__restrict__ k, const float *__restrict__ v,
    const float *__restrict__ M, AttnGrid g, float *__restrict__ opart, float *__restrict__ ml) {
    constexpr int NT = NW * 64;                       // threads
    constexpr int LD4 = KTS * CH / 4 / NT;           // float4 per thread per stage, per K and per V
    static_assert(LD4 * NT * 4 == KTS * CH, "stage must split evenly");
    constexpr float DEFER = FASTEXP ? 8.0f : 5.5f;    // log2 / ln units
    extern __shared__ __attribute__((aligned(16))) float smem[];
    constexpr int KSTR_ = GLDS ? CH : A_KSTR;
    float *Kl0 = smem, *Kl1 = smem + KTS * KSTR_;
    float *Vl0 = smem + 2 * KTS * KSTR_, *Vl1 = Vl0 + KTS * A_VSTR;

    int b, qb, split;
    attention_block_coords(g, XCD, b, qb, split);
    // N: this pair's keys (a ragged batch's pairs differ); Ns, Npad: the batch's strides
    const int N = g.n(b), Ns = g.N, Npad = g.Npad;
    if (qb * (NW * 32) >= N) return;  // past a ragged pair's end (workgroup-uniform)
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, h = lane >> 5, l32 = lane & 31;
    const int q0 = qb * (NW * 32) + wave * 32;
    const int nst = (N + KTS - 1) / KTS;
    const int st0 = split * g.sps, st1 = min(nst, st0 + g.sps);
    const size_t pbase = (size_t)b * Npad * CH;
    const __amdgpu_buffer_rsrc_t rK = make_rsrc(k + pbase, (uint32_t)Npad * CH * 4);
    const __amdgpu_buffer_rsrc_t rV = make_rsrc(v + pbase, (uint32_t)Npad * CH * 4);
    // M of this pair (N <= 32767 so the byte range fits the 32-bit descriptor);
    // rows >= N read 0 through the range check (and are masked to -inf below)
    const __amdgpu_buffer_rsrc_t rM = make_rsrc(M + (size_t)b * Ns * Ns, (uint32_t)Ns * (uint32_t)Ns * 4u);
    const size_t obase = (size_t)(b * g.nsplit + split) * Npad;
    const int qq = q0 + l32;
    const bool active = q0 < Npad;  // waves past the padded end (NW*32 > 128 granularity)

    float qf[64];
    if (active) {
        const f32x4 *src4 = reinterpret_cast<const f32x4 *>(q + pbase + (size_t)qq * CH + h * 64);
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const f32x4 t = src4[i];
            qf[4 * i] = t[0];
            qf[4 * i + 1] = t[1];
            qf[4 * i + 2] = t[2];
            qf[4 * i + 3] = t[3];
        }
    } else {
#pragma unroll
        for (int i = 0; i < 64; ++i) qf[i] = 0.0f;
    }

    f32x4 sk[GLDS ? 1 : LD4], sv[GLDS ? 1 : LD4];
    // LDS-DMA staging: the stage is KTS*CH*4*2 bytes = 2*KTS/2 pieces of 1 KiB
    constexpr int PIECES = KTS;  // KTS/2 K pieces + KTS/2 V pieces
    auto glds_stage = [&](int st, float *Kl, float *Vl) {
#pragma unroll
        for (int i = 0; i < PIECES / NW; ++i) {
            const int piece = wave * (PIECES / NW) + i;
            const bool isV = piece >= PIECES / 2;
            const int pp = isV ? piece - PIECES / 2 : piece;
            const int row = 2 * pp + (lane >> 5), cpos = lane & 31;
            const int csrc = isV ? cpos : (cpos ^ (row & 15));
            const float *g = (isV ? v : k) + pbase + (size_t)(st * KTS + row) * CH + 4 * csrc;
            float *l = (isV ? Vl : Kl) + pp * 256;
            __builtin_amdgcn_global_load_lds(g, l, 16, 0, 0);
        }
    };
    auto load_stage = [&](int st) {
#pragma unroll
        for (int i = 0; i < LD4; ++i) {
            const int idx = tid + NT * i, row = idx >> 5, c4 = idx & 31;
            const uint32_t off = ((uint32_t)(st * KTS + row) * CH + 4 * c4) * 4;
            if (BUF & 1) {
                sk[i] = buf_ld4(rK, off, 0);
                sv[i] = buf_ld4(rV, off, 0);
            } else {
                sk[i] = *reinterpret_cast<const f32x4 *>(reinterpret_cast<const char *>(k + pbase) + off);
                sv[i] = *reinterpret_cast<const f32x4 *>(reinterpret_cast<const char *>(v + pbase) + off);
            }
        }
    };
    auto store_stage = [&](float *Kl, float *Vl) {
#pragma unroll
        for (int i = 0; i < LD4; ++i) {
            const int idx = tid + NT * i, row = idx >> 5, c4 = idx & 31;
            *reinterpret_cast<f32x4 *>(Kl + row * A_KSTR + 4 * c4) = sk[i];
            *reinterpret_cast<f32x4 *>(Vl + row * A_VSTR + 4 * c4) = sv[i];
        }
    };

    f32x16 O0 = zero16(), O1 = zero16(), O2 = zero16(), O3 = zero16();
    float m_run = -INFINITY, l_run = 0.0f;
    // FASTEXP: logits in log2 units (log2(e)/sqrt(128)); else natural units (1/sqrt(128))
    const float scale = FASTEXP ? 0.12751743082459868f : 0.08838834764831845f;
    const uint32_t Nb = (uint32_t)Ns * 4;

    auto subtile = [&](const float *Kl, const float *Vl, int key0) {
        // M[key][q] for this lane's 16 keys (rows acc_row(r, h)) -- issued before the MFMAs
        float mv[16];
        const uint32_t vo = ((uint32_t)(key0 + 4 * h) * (uint32_t)Ns + (uint32_t)qq) * 4;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const uint32_t o = vo + (uint32_t)((r & 3) + 8 * (r >> 2)) * Nb;
            if (BUF & 2) {
                mv[r] = buf_ld(rM, o, 0);
            } else {
                const int key = key0 + acc_row(r, h);
                mv[r] = key < N ? *reinterpret_cast<const float *>(reinterpret_cast<const char *>(M + (size_t)b * Ns * Ns) + o) : 0.0f;
            }
        }
        f32x16 S = zero16();
        const float *Kp = Kl + l32 * KSTR_ + h * 64;
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const f32x4 kv = *reinterpret_cast<const f32x4 *>(Kp + 4 * (GLDS ? (i ^ (l32 & 15)) : i));
            S = mfma32(kv[0], qf[4 * i], S);
            S = mfma32(kv[1], qf[4 * i + 1], S);
            S = mfma32(kv[2], qf[4 * i + 2], S);
            S = mfma32(kv[3], qf[4 * i + 3], S);
        }
        float p[16];
        float mx = -INFINITY;
        const bool tail = key0 + 32 > N;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            float x = mv[r] * (S[r] * scale);  // (:39) then * M (:41); 0, not -inf, off-support
            if (tail && key0 + acc_row(r, h) >= N) x = -INFINITY;
            p[r] = x;
            mx = fmaxf(mx, x);
        }
        mx = fmaxf(mx, __shfl_xor(mx, 32));
        if (__any(mx > m_run + DEFER)) {  // re-base the running max (wave-uniform branch)
            const float m_new = fmaxf(m_run, mx);
            const float alpha = FASTEXP ? __builtin_amdgcn_exp2f(m_run - m_new) : expf(m_run - m_new);
            m_run = m_new;
            l_run *= alpha;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const float a = __shfl(alpha, acc_row(r, h));
                O0[r] *= a;
                O1[r] *= a;
                O2[r] *= a;
                O3[r] *= a;
            }
        }
        float psum = 0.0f;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            p[r] = FASTEXP ? __builtin_amdgcn_exp2f(p[r] - m_run) : expf(p[r] - m_run);
            psum += p[r];
        }
        l_run += psum;
        const float *Vp = Vl + 4 * l32 + 4 * h * A_VSTR;
#pragma unroll
        for (int s = 0; s < 16; ++s) {
            const f32x4 vv = *reinterpret_cast<const f32x4 *>(Vp + ((s & 3) + 8 * (s >> 2)) * A_VSTR);
            O0 = mfma32(p[s], vv[0], O0);
            O1 = mfma32(p[s], vv[1], O1);
            O2 = mfma32(p[s], vv[2], O2);
            O3 = mfma32(p[s], vv[3], O3);
        }
    };

    if (st0 < st1) {
        if (GLDS) {
            glds_stage(st0, Kl0, Vl0);
        } else {
            load_stage(st0);
            store_stage(Kl0, Vl0);
        }
    }
    __syncthreads();
    for (int st = st0; st < st1; ++st) {
        const int buf = (st - st0) & 1;
        const float *Kl = buf ? Kl1 : Kl0;
        const float *Vl = buf ? Vl1 : Vl0;
        if (st + 1 < st1) {
            if (GLDS)
                glds_stage(st + 1, buf ? Kl0 : Kl1, buf ? Vl0 : Vl1);
            else
                load_stage(st + 1);
        }
        if (active) {
#pragma unroll
            for (int sub = 0; sub < KTS / 32; ++sub) {
                const int key0 = st * KTS + sub * 32;
                if (key0 < N) subtile(Kl + sub * 32 * KSTR_, Vl + sub * 32 * A_VSTR, key0);
            }
        }
        if (!GLDS && st + 1 < st1) store_stage(buf ? Kl0 : Kl1, buf ? Vl0 : Vl1);
        __syncthreads();
    }
    if (!active) return;

    l_run += __shfl_xor(l_run, 32);
    float *Ob = opart + obase * CH;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const int row = q0 + acc_row(r, h);
        *reinterpret_cast<f32x4 *>(Ob + (size_t)row * CH + 4 * l32) = f32x4{O0[r], O1[r], O2[r], O3[r]};
    }
    if (h == 0) {
        // partial max in natural-log units so the combine is variant-independent
        ml[(obase + qq) * 2] = FASTEXP ? m_run * 0.6931471805599453f : m_run;
        ml[(obase + qq) * 2 + 1] = l_run;
    }
}

}  // namespace pdsc
