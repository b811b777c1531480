// attention_h3.hpp -- the SCNonlocal attention core (models/PointDSC.py:36-42)
// on the fp16 matrix cores with fp32-equivalent accuracy ("3xf16").
//
//   msg_i = sum_j softmax_j( M_ij * (q_i . k_j) / sqrt(C) ) v_j,   C = 128, heads = 1
//
// gfx950 has no reduced-precision fp32 MFMA (v_mfma_f32_32x32x2_f32 runs at
// the fp32 vector rate, 1/16 of v_mfma_f32_32x32x16_f16).  Every fp32 operand
// x is stored as an exact-sum pair x = hi + lo of fp16 values (hi = fp16(x),
// lo = fp16(x - hi): 22 significant bits) and each product is formed from the
// three significant partial products
//      a.b ~= a_hi.b_hi + a_hi.b_lo + a_lo.b_hi        (the a_lo.b_lo term is 2^-22 relative)
// accumulated in fp32 by the MFMA -- 3 fp16 MFMAs instead of 16 fp32 ones.
// Validated against the reference's golden features (tools/emulate_h3.py):
// the error vs the reference is the same as a plain fp32 re-ordering.
//
// Range: |Q|, |K|, |V| < 65504 (fp16 max; the features of the BN-normalised
// encoder are O(10)); a value outside turns the result into inf/NaN (loud,
// never silently wrong).  Softmax weights are kept as p = 2^(x - m + PSHIFT)
// <= 2^(DEFER + PSHIFT) = 2^15, so they too sit in fp16's normal range.
// Small V: each 32-key tile of V is stored as V * 2^e (vexp[tile] = e in
// [0, H3_VEXP_MAX], chosen by the producer from the tile's max |v|) so its lo
// halves stay normal fp16; the tile's p are formed as 2^(x - m + PSHIFT - e)
// (one add) and its sum re-scaled by 2^e (one ldexp): sum p v is unchanged.
// The scale trades V's resolution against p's: both halves bottom out at fp16's
// 2^-24, V' relative to the tile's max 2^(e + log2 max|v|), p' relative to the
// row sum >= 2^(PSHIFT - e).  e lifts max|v'| only to [2^4, 2^5): a larger e
// (r03: max|v'| up to 2^14, e = 8 for any |v| < 64) pushed the p' of keys far
// below the row max under 2^-24 -- lost mass that grows with the key chain,
// measured 5x the fp32 envelope at one 1000-key split (tools/emulate_attn.py).
// Small Q or K only shrink the logits' absolute error, which is what the
// softmax is sensitive to.
//
// HBM layouts (written by the pointwise kernels' epilogues, encoder.hip, or
// by split_qkv_kernel for the standalone API), per pair, in 32-row tiles of
// 16 KiB made of 16 "fragment blocks" of 1 KiB: block (f, plane) holds, for
// each lane (h, n) of a wave in lane order, the 16 B (8 fp16) that lane feeds
// the MFMA as operand fragment f -- so a producer's store of one fragment and
// a consumer's load of it (or LDS-DMA + ds_read) are one contiguous 1 KiB:
//   Qs, Ks  fragment j (k-step, 0..7), lane (h, n): row n of the tile,
//           positions 16 j + 8h .. +7 of the row in qk_pos order (bits 2 and 3
//           of the channel index swapped); plane 0 = hi, 1 = lo
//   Vs      fragment i = 2t + s, lane (h, n): channel 32 t + n, the tile's
//           keys at v_keypos positions 16 s + 8h .. +7
// Each layout equals the fp32 tensor's size (4 B per element).
// The partial outputs (opart) use the same tiling for fp32: per 32-query tile
// 16 blocks (2 ks + g) of 64 lanes x 4 floats, lane (h, n) = query n,
// qk_pos positions 16 ks + 8h + 4g .. +3 (h3_opart_off) -- the k-step
// fragments of the message layer that consumes them.
//
// Work decomposition (as attention.hpp): a workgroup = NW waves x 32 queries
// of one pair and a contiguous split of 32-key tiles; K and V tiles (16 KiB
// each, contiguous in HBM) are copied into a 2-deep LDS ring by LDS-DMA.  Per
// wave and tile:
//   S^T = K Q^T      8 k-steps x 3 MFMA 32x32x16 (lane <-> query)
//   logits, online softmax with a lazily re-based max (as attention.hpp)
//   O^T += V^T P^T   the S^T accumulator registers 8s..8s+7 ARE the B operand
//                    of k-step s (key order = v_keypos), 4 channel tiles x 2 x 3
//                    MFMA; lane <-> query again, so the softmax re-scale is a
//                    per-lane multiply and O^T registers 8u..8u+7 of tile t are
//                    the consuming layer's k-step 2t + u fragment
#pragma once
#include "pdsc_internal.hpp"

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));

namespace pdsc {

constexpr int H3_ROWB = 2 * CH * 2;          // bytes per Qs/Ks row (hi + lo)
constexpr int H3_TILE = 32;                  // keys per LDS tile
constexpr int H3_KTB = H3_TILE * H3_ROWB;    // K tile bytes (16 KiB)
constexpr int H3_VTB = 2 * CH * H3_TILE * 2; // V tile bytes (16 KiB)
constexpr int H3_PSHIFT = 7;                 // p = 2^(x - m + PSHIFT)
constexpr float H3_DEFER = 8.0f;             // re-base the max when it grows by > 2^8
#ifndef ATT_SOFTMAX_PRIO
#define ATT_SOFTMAX_PRIO 1  // s_setprio of the softmax section (build knob; 0 = off)
#endif
#ifndef ATT_QFMA
#define ATT_QFMA 1  // Q pre-scaled by log2(e)/sqrt(C) at production; logits minus the running base by one fma
#endif
#ifndef ATT_BUFDMA
#define ATT_BUFDMA 1  // K/V (and pw2 weight) LDS-DMA by buffer_load ... lds (no per-piece 64-bit address VALU)
#endif
constexpr float H3_QSCALE = 0.12751743082459868f;  // log2(e) / sqrt(128): the softmax's scale, in base 2
constexpr int H3_VEXP_MAX = 8;               // V tile pre-scale 2^e, 0 <= e <= 8
constexpr int H3_VEXP_TARGET = 5;            // ... lifting the tile's max |v| below 2^5

// The V-tile exponent for a tile whose max |v| is vmax: the largest e <= 8 with
// vmax 2^e < 2^H3_VEXP_TARGET (0 for vmax >= 2^4, vmax == 0 or non-finite vmax).
PDSC_DEV int h3_vexp(float vmax) {
    if (!(vmax > 0.0f) || !(vmax < 8192.0f)) return 0;
    int ex;
    frexpf(vmax, &ex);  // vmax < 2^ex
    return max(0, min(H3_VEXP_MAX, H3_VEXP_TARGET - ex));
}

// channel -> position in a Qs/Ks row: swap bits 2 and 3
PDSC_DEV constexpr int qk_pos(int c) { return (c & ~12) | ((c & 4) << 1) | ((c & 8) >> 1); }
// key (0..31 within a tile) -> position in a Vs plane row: swap bits 2 and 3
PDSC_DEV constexpr int v_keypos(int k) { return (k & ~12) | ((k & 4) << 1) | ((k & 8) >> 1); }
// Fragment-block tiling (above): 32 rows x 128 channels x (hi, lo) per tile;
// element offset of (fragment f, plane, lane) in fp16 units within the tile.
constexpr int H3_TILE_H = 2 * CH * H3_TILE;  // fp16 per tile (8192)
PDSC_DEV constexpr int h3_frag(int f, int plane, int lane) { return ((2 * f + plane) * 64 + lane) * 8; }

// element offsets (in fp16 units) inside one pair's buffers
PDSC_DEV size_t qs_off(int row, int half, int c) {
    const int p = qk_pos(c);
    return (size_t)(row >> 5) * H3_TILE_H + h3_frag(p >> 4, half, 32 * ((p >> 3) & 1) + (row & 31)) + (p & 7);
}
PDSC_DEV size_t ks_off(int row, int half, int c) { return qs_off(row, half, c); }
PDSC_DEV size_t vs_off(int key, int half, int c) {
    const int kp = v_keypos(key & 31);
    return (size_t)(key >> 5) * H3_TILE_H + h3_frag(2 * (c >> 5) + (kp >> 4), half, 32 * ((kp >> 3) & 1) + (c & 31)) +
           (kp & 7);
}
// fp32 offset of (row, channel c) in one (pair, split)'s opart of Npad rows
PDSC_DEV size_t h3_opart_off(int row, int c) {
    const int p = qk_pos(c);
    return (size_t)(row >> 5) * (H3_TILE * CH) + ((2 * (p >> 4) + ((p >> 2) & 1)) * 64 + 32 * ((p >> 3) & 1) + (row & 31)) * 4 +
           (p & 3);
}

// x = hi + lo (fp16 pair).  The empty asm pins x as the rounded fp32 value:
// without it the compiler folds a producing multiply into the hi conversion
// (v_fma_mixlo_f16: one rounding of the exact product) while lo is formed from the
// fp32-rounded product, so where that product rounds onto an fp16 tie, hi and
// lo disagree by one fp16 ulp (measured: 1 channel in ~10^4, 1e-4 errors).
PDSC_DEV void split_h(float x, _Float16 &hi, _Float16 &lo) {
    asm("" : "+v"(x));
    hi = (_Float16)x;
    lo = (_Float16)(x - (float)hi);
}

// Two values at once: hi = {f16(x0), f16(x1)} (one v_cvt_pk_f16_f32) and lo =
// {f16(x0 - hi0), f16(x1 - hi1)} by v_fma_mixlo / v_fma_mixhi, which form the
// exact difference of the fp32 value and the fp16 hi operand and round once --
// bit-identical to split_h (x - hi is exact in fp32), 1.5 instead of ~2.5 VALU
// per value.  Inline asm: the inputs are the rounded fp32 values by
// construction, and every use sees the same hi register.  ONE asm statement:
// the closing s_nop 1 gives both hi and lo the 2 wait states a VALU write needs
// before an MFMA reads the register as A/B (hipcc pads nothing inside asm, and
// its hazard recognizer does not see asm-written VGPRs); as separate statements
// the scheduler could move the hi.hi MFMA right after the cvt.
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
PDSC_DEV void split2(float x0, float x1, uint32_t &hi, uint32_t &lo) {
    asm("v_cvt_pk_f16_f32 %0, %2, %3\n\t"
        "v_fma_mixlo_f16 %1, %2, 1.0, -%0 op_sel_hi:[0,0,1]\n\t"
        "v_fma_mixhi_f16 %1, %3, 1.0, -%0 op_sel:[0,0,1] op_sel_hi:[0,0,1]\n\t"
        "s_nop 1"
        : "=&v"(hi), "=&v"(lo)
        : "v"(x0), "v"(x1));
}
// 8 values (v[e] -> element e of the fragments)
PDSC_DEV void split8x(const float (&v)[8], f16x8 &hi, f16x8 &lo) {
    u32x4 h, l;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        uint32_t a, b;
        split2(v[2 * e], v[2 * e + 1], a, b);
        h[e] = a;
        l[e] = b;
    }
    hi = __builtin_bit_cast(f16x8, h);
    lo = __builtin_bit_cast(f16x8, l);
}

// x (op) x of the lane 32 apart, on every lane, by v_permlane32_swap (no LDS
// round trip, unlike __shfl_xor's ds_bpermute); bit-identical to the shuffle
// form since max and + commute.
PDSC_DEV float halves_max(float x) {
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
PDSC_DEV float halves_sum(float x) {
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

PDSC_DEV f32x16 mfma_h(f16x8 a, f16x8 b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
}
// a.b with a = ah + al, b = bh + bl: small terms first
PDSC_DEV f32x16 mfma_h3(f16x8 ah, f16x8 al, f16x8 bh, f16x8 bl, f32x16 c) {
    c = mfma_h(al, bh, c);
    c = mfma_h(ah, bl, c);
    return mfma_h(ah, bh, c);
}

// Products with a W_PLANES-plane weight w = wh + wm (+ wl) (encoder.hip:
// pack_dense_kernel) and a two-plane activation x = xh + xl:
// x.w ~= xh.(wh + wm (+ wl)) + xl.wh, small terms first.  The dropped xl.wm is
// 2^-22 relative, as is a 2-plane weight's representation error (r01-r03 kept
// the lo plane: every fp32 weight exactly, one more product; r04 measured the
// two forms inside the same fp32 noise, tools/emulate_conv.py).
// mfma_xw3: A = activations (rows = points), B = weights; mfma_w3x: transposed.
PDSC_DEV f32x16 mfma_xw3(f16x8 xh, f16x8 xl, f16x8 wh, f16x8 wm, f16x8 wl, f32x16 c) {
    if constexpr (W_PLANES == 3) c = mfma_h(xh, wl, c);
    c = mfma_h(xh, wm, c);
    c = mfma_h(xl, wh, c);
    return mfma_h(xh, wh, c);
}
PDSC_DEV f32x16 mfma_w3x(f16x8 wh, f16x8 wm, f16x8 wl, f16x8 xh, f16x8 xl, f32x16 c) {
    if constexpr (W_PLANES == 3) c = mfma_h(wl, xh, c);
    c = mfma_h(wm, xh, c);
    c = mfma_h(wh, xl, c);
    return mfma_h(wh, xh, c);
}

// Diagnostic build only (-DATT_STAMPS, tools/att_stamps.py): s_memtime stamps of
// the waves of every 16th workgroup (the first 64 of them) -- per key tile: top,
// S and M ready, softmax done, PV issued, barrier passed; then the chain phase.
// Stamps go to a buffer of their own that nothing in the kernel reads.
#ifdef ATT_STAMPS
constexpr int ST_PER_WAVE = 256, ST_WGS = 64;  // (192 + 3 c .. : the fused chain's chunk c, w2_layer)
static __device__ unsigned long long g_att_stamps[ST_WGS * 4 * ST_PER_WAVE];
PDSC_DEV unsigned long long *att_stamp_ptr(int wave) {
    return (blockIdx.x % 16 == 0 && blockIdx.x / 16 < ST_WGS && wave < 4 && blockIdx.z == 0)
               ? g_att_stamps + ((blockIdx.x / 16) * 4 + wave) * ST_PER_WAVE
               : nullptr;
}
#define ATT_STAMP(stp, i)                                                       \
    do {                                                                        \
        __builtin_amdgcn_sched_barrier(0);                                      \
        if (stp) {                                                              \
            const unsigned long long t_ = __builtin_amdgcn_s_memtime();         \
            if (lane == 0) stp[i] = t_;                                         \
        }                                                                       \
        __builtin_amdgcn_sched_barrier(0);                                      \
    } while (0)
#define ATT_RSTAMP(stp, i)                                                      \
    do {                                                                        \
        if (stp) {                                                              \
            const unsigned long long t_ = __builtin_amdgcn_s_memrealtime();     \
            if (lane == 0) stp[i] = t_;                                         \
        }                                                                       \
    } while (0)
#define CH_STAMP(i)                                       \
    do {                                                  \
        unsigned long long *stc_ = att_stamp_ptr(wave);   \
        ATT_STAMP(stc_, i);                               \
    } while (0)
#else
#define CH_STAMP(i) \
    do {            \
    } while (0)
#define ATT_STAMP(stp, i) \
    do {                  \
    } while (0)
#define ATT_RSTAMP(stp, i) \
    do {                   \
    } while (0)
#endif

// K/V ring: 2 slots (tile t + 1 lands while tile t is consumed)
constexpr int H3_NSLOT = 2;
template <int NW>
constexpr size_t attention_h3_lds_bytes() { return (size_t)H3_NSLOT * (H3_KTB + H3_VTB); }

PDSC_DEV __amdgpu_buffer_rsrc_t h3_rsrc(const void *base, uint32_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(base), 0, (int)bytes, 0x00020000);
}

struct AttnGridH3 {
    int B, N, Npad, nqb, nsplit, sps;  // sps = 32-key tiles per split
    // ragged batches: pair b's correspondences (N, Npad: the batch's strides), or null
    const int *nv;
    const int *po;  // ragged batches: workgroup pair slot -> pair (Ragged::po), or null
    int rev = 0;    // the workgroup order reversed (alternate layers: attn_pw2 ZIGZAG)
    PDSC_DEV int n(int b) const { return nv ? nv[b] : N; }
};

// Key splits per query block: the count that minimises the estimated launch
// time  ceil(workgroups / slots) x (key tiles per split + H3_SPLIT_C0)  --
// whole rounds of `slots` resident workgroups (2 per CU), each as long as its
// workgroups' tile loop plus a fixed per-workgroup cost (prologue, first DMA,
// partial stores, the combine's extra reads) of about H3_SPLIT_C0 tiles.
// Measured (A/B, one box): N = 5000 x 8 pairs 313 us per layer at 4 splits
// (2.5 rounds) against 350 at 2 (1.25 rounds: a quarter-full last round) and
// 324-326 at 5 / 8; 16 x 1000 best at 4 (one round).  Ties: fewer splits.
constexpr int H3_SPLIT_C0 = 15;
inline int attention_split_count(long blocks, int nst, int slots) {
    int best = 1;
    long best_cost = -1;
    for (int ns = 1; ns <= std::max(1, nst / 2); ++ns) {
        const int sps = (nst + ns - 1) / ns;
        if ((nst + sps - 1) / sps != ns) continue;  // an equivalent smaller count exists
        const long rounds = (blocks * ns + slots - 1) / slots;
        const long cost = rounds * (sps + H3_SPLIT_C0);
        if (best_cost < 0 || cost < best_cost) {
            best = ns;
            best_cost = cost;
        }
    }
    return best;
}

template <int NW>
inline AttnGridH3 attention_h3_grid(int B, int N, int slots) {
    AttnGridH3 g;
    g.nv = nullptr;
    g.po = nullptr;
    g.B = B;
    g.N = N;
    g.Npad = round_up(N, QB);
    g.nqb = (N + NW * 32 - 1) / (NW * 32);
    const int nst = (N + H3_TILE - 1) / H3_TILE;
    const int ns = attention_split_count((long)B * g.nqb, nst, slots);
    g.sps = (nst + ns - 1) / ns;
    g.nsplit = (nst + g.sps - 1) / g.sps;
    return g;
}

// Workgroup -> (pair, query block, split), a pair's blocks kept on one XCD
// (consecutive workgroup ids round-robin over the 8 XCDs).
struct AttnBlock {
    int b, qb, split;
    int st0 = 0, st1 = -1;  // key tiles [st0, st1) when st1 >= 0 (attention_w64_sk_kernel), else the split's
};
PDSC_DEV AttnBlock attention_h3_block(const AttnGridH3 &g, bool xcd) {
    const int G = g.B * g.nqb * g.nsplit;
    int lid = blockIdx.x;
    if (xcd) {
        // g.rev: each XCD walks its own logical range backwards (pairs keep their XCD)
        const int full = G & ~7;
        if (lid < full) {
            const int loc = lid >> 3;
            lid = (lid & 7) * (full >> 3) + (g.rev ? (full >> 3) - 1 - loc : loc);
        }
    } else if (g.rev) {
        lid = G - 1 - lid;
    }
    const int slot = lid / g.nsplit / g.nqb;
    return AttnBlock{g.po ? g.po[slot] : slot, (lid / g.nsplit) % g.nqb, lid % g.nsplit};
}

// The attention of one workgroup (NW waves x 32 queries of pair b, query block
// qb, key-tile split `split`): every wave runs the tile loop (the barriers)
// and, for queries < Npad, leaves this lane's un-normalised O^T (lane <-> query,
// tile t register r <-> channel 32t + acc_row(r, h)), the running max m (log2
// units, + PSHIFT) and the full row sum l (both lane halves).  smem: the K/V
// ring (attention_h3_lds_bytes), free again when this returns.
// PACKED: M in the symmetric-packed tile layout (pdsc_internal.hpp); else dense [N][N].
// vexp: [B][Npad/32] V-tile exponents (see above).
// EARLY (the split-K kernel on splits of >= 3 tiles, launch_attention): the
// first two tiles' LDS-DMA and the first tile's M issued with the Q loads, ahead
// of the one wait before the loop, and each later tile's M issued one tile
// ahead.  Measured (A/B, one box): 4 x 5000 forward 2.405 vs 2.460 ms; on the
// single pair's 2-tile splits 0.419 vs 0.417 ms, so those keep the plain loop.
// The same arithmetic on the same operands: bit-identical either way.
// WS > 0 (attention_h3_ws_kernel, the tiny plan): the workgroup's WS waves
// share ONE block of 32 queries and split the key split's tiles between them
// (wave w: the w-th of WS contiguous runs); each wave stages its own tiles into
// a single LDS slot of its own (h3smem + w (KTB + VTB)) with no workgroup
// barrier, and the caller merges the waves' (O, m, l) (NW must be 1).
template <int NW, bool PACKED, bool EARLY = false, int WS = 0>
PDSC_DEV void attention_h3_core(const _Float16 *__restrict__ Qs, const _Float16 *__restrict__ Ks,
                                const _Float16 *__restrict__ Vs, const float *__restrict__ vexp,
                                const float *__restrict__ M, const AttnGridH3 &g, const AttnBlock &blk, char *h3smem,
                                int wave, int lane, f32x16 (&O)[4], float &m_run, float &l_run) {
    static_assert(WS == 0 || (NW == 1 && !EARLY), "wave-split: one 32-query block, the plain loop");
    const int b = blk.b, qb = blk.qb, split = blk.split;
    const int N = g.n(b), Npad = g.Npad;  // this pair's keys; the batch's row stride
    const int h = lane >> 5, l32 = lane & 31;
    const int q0 = WS ? qb * 32 : qb * (NW * 32) + wave * 32;
    const int nst = (N + H3_TILE - 1) / H3_TILE;
    int st0 = split * g.sps, st1 = min(nst, st0 + g.sps);
    if constexpr (WS > 0) {  // this wave's run of the split's tiles (wave-uniform)
        const int tpw = (st1 - st0 + WS - 1) / WS, a = min(st1, st0 + wave * tpw);
        st1 = min(st1, a + tpw);
        st0 = a;
    }
    const int qq = q0 + l32;
    const bool active = q0 < Npad;

    const char *Kp = reinterpret_cast<const char *>(Ks + (size_t)b * Npad * 2 * CH);
    const char *Vp = reinterpret_cast<const char *>(Vs + (size_t)b * Npad * 2 * CH);
    const int mnt = mpack_ntile(g.N);  // M's layout is the batch stride's
    const size_t mper = PACKED ? (size_t)mnt * (mnt + 1) / 2 * MPACK_T * MPACK_T : (size_t)g.N * g.N;
    const __amdgpu_buffer_rsrc_t rM = h3_rsrc(M + (size_t)b * mper, (uint32_t)(mper * 4u));

    // this lane's query: 8 k-steps x (hi, lo) fragments (16 coalesced 1-KiB loads)
    f16x8 qh[8], ql[8];
    {
        const _Float16 *qt = Qs + (size_t)b * Npad * 2 * CH + (size_t)(min(q0, Npad - 32) >> 5) * H3_TILE_H;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            qh[j] = *reinterpret_cast<const f16x8 *>(qt + h3_frag(j, 0, lane));
            ql[j] = *reinterpret_cast<const f16x8 *>(qt + h3_frag(j, 1, lane));
        }
    }

    // LDS-DMA copy of tile st (K 16 KiB + V 16 KiB = 32 pieces of 1 KiB) into ring slot `slot`
#if ATT_BUFDMA
    const __amdgpu_buffer_rsrc_t rK = h3_rsrc(Kp, (uint32_t)Npad * H3_ROWB), rV = h3_rsrc(Vp, (uint32_t)Npad * H3_ROWB);
#endif
    auto stage = [&](int st, int slot) {
        char *dst = h3smem + (WS ? wave : slot) * (H3_KTB + H3_VTB);
        constexpr int PIECES = (H3_KTB + H3_VTB) / 1024;
#pragma unroll
        for (int i = 0; i < PIECES / NW; ++i) {
            const int piece = WS ? i : wave * (PIECES / NW) + i;  // wave-uniform (SGPR)
#if ATT_BUFDMA
            // the piece's offset in the SGPR operand: no per-piece address VALU
            if (piece < H3_KTB / 1024)
                __builtin_amdgcn_raw_ptr_buffer_load_lds(rK, (__attribute__((address_space(3))) void *)(dst + piece * 1024),
                                                         16, 16 * lane, st * H3_KTB + piece * 1024, 0, 0);
            else
                __builtin_amdgcn_raw_ptr_buffer_load_lds(rV, (__attribute__((address_space(3))) void *)(dst + piece * 1024),
                                                         16, 16 * lane, st * H3_VTB + (piece - H3_KTB / 1024) * 1024, 0, 0);
#else
            const char *src = piece < H3_KTB / 1024
                                  ? Kp + (size_t)st * H3_KTB + piece * 1024
                                  : Vp + (size_t)st * H3_VTB + (piece - H3_KTB / 1024) * 1024;
            __builtin_amdgcn_global_load_lds(src + 16 * lane, dst + piece * 1024, 16, 0, 0);
#endif
        }
    };

#pragma unroll
    for (int t = 0; t < 4; ++t) O[t] = zero16();
    m_run = -INFINITY;
    l_run = 0.0f;
    const float scale = ATT_QFMA ? 1.0f : H3_QSCALE;  // (QFMA: Q carries it)
    const uint32_t Nb = (uint32_t)g.N * 4;

#ifdef ATT_STAMPS
    unsigned long long *stp = att_stamp_ptr(wave);
#endif
    int st_si = 0;  // the current tile's first stamp index (diagnostic build)
    (void)st_si;
    const float *vexp_b = vexp + (size_t)b * (Npad / H3_TILE);
    const __amdgpu_buffer_rsrc_t rE = h3_rsrc(vexp_b, (uint32_t)(Npad / H3_TILE) * 4u);
    // M[key][q] = M[q][key] (M symmetric) for this lane's 16 keys of tile key0
    auto load_m = [&](int key0, float (&mv)[16], float &ev) {
        if constexpr (PACKED) {
            // the wave's 32 x 32 block IS one packed tile: (kt, qt) row-major when
            // kt <= qt (rows = keys: 16 loads, each 32 consecutive queries of a key
            // row), else tile (qt, kt) read transposed (rows = queries: the lane's
            // 16 keys are 4 runs of 4 in its query's row).  Scalar branch (q0 is
            // wave-uniform in an SGPR).
            static_assert(MPACK_T == 32, "one packed tile per wave step");
            const int kt = key0 / MPACK_T, qt = q0 / MPACK_T;
            const int kr = 4 * h, qr = l32;
            if (kt <= qt) {  // rows = keys
                const uint32_t vo =
                    ((uint32_t)mpack_tile(kt, qt, mnt) * (MPACK_T * MPACK_T) + (uint32_t)(kr * MPACK_T + qr)) * 4;
#pragma unroll
                for (int r = 0; r < 16; ++r)
                    mv[r] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                                          rM, vo + (uint32_t)((r & 3) + 8 * (r >> 2)) * (MPACK_T * 4), 0, 0));
            } else {  // rows = queries
                const uint32_t vo =
                    ((uint32_t)mpack_tile(qt, kt, mnt) * (MPACK_T * MPACK_T) + (uint32_t)(qr * MPACK_T + kr)) * 4;
#pragma unroll
                for (int g = 0; g < 4; ++g) {
                    const f32x4 v4 = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rM, vo + 32 * g, 0, 0));
#pragma unroll
                    for (int e = 0; e < 4; ++e) mv[4 * g + e] = v4[e];
                }
            }
        } else {
            const uint32_t vo = ((uint32_t)(key0 + 4 * h) * (uint32_t)g.N + (uint32_t)qq) * 4;
#pragma unroll
            for (int r = 0; r < 16; ++r)
                mv[r] = __builtin_bit_cast(
                    float, __builtin_amdgcn_raw_buffer_load_b32(rM, vo + (uint32_t)((r & 3) + 8 * (r >> 2)) * Nb, 0, 0));
        }
        // the tile's V exponent as a vector load with the M loads (a scalar load
        // here was waited for with lgkmcnt(0) in the middle of the softmax)
        ev = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rE, (uint32_t)(key0 / H3_TILE) * 4u, 0, 0));
    };
    // One key tile: M loads first (they land while QK^T runs), K and V fragments
    // read two blocks ahead of their MFMAs (three register sets; sched_barrier
    // keeps the compiler from sinking each read onto its MFMA).  (Prefetching M
    // a whole tile ahead, or queueing the next DMA after the softmax, measured
    // no faster: DESIGN.md §7.)
    // (the tile's V exponent is a vector load issued with the M loads: a scalar
    // load here is waited for with lgkmcnt(0) in the middle of the softmax)
    // QK^T + online softmax of one key tile -> this lane's P fragments (ph, pl)
    auto qk_softmax = [&](const char *Kl, int key0, float (&mv)[16], float ev, f16x8(&ph)[2], f16x8(&pl)[2],
                          bool first, auto after_qk) {
        // S^T[key][query] = sum_c K[key][c] Q[query][c]
        f32x16 S = zero16();
        f16x8 kf[3][2];
        auto kread = [&](int j, f16x8(&f)[2]) {
            f[0] = *reinterpret_cast<const f16x8 *>(Kl + 2 * h3_frag(j, 0, lane));
            f[1] = *reinterpret_cast<const f16x8 *>(Kl + 2 * h3_frag(j, 1, lane));
        };
        kread(0, kf[0]);
        kread(1, kf[1]);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            if (j + 2 < 8) kread(j + 2, kf[(j + 2) % 3]);
            S = mfma_h3(kf[j % 3][0], kf[j % 3][1], qh[j], ql[j], S);
            __builtin_amdgcn_sched_barrier(0);
        }
        after_qk();  // (WS: the next tile's K into the K half of the wave's slot)
        // the softmax's VALU at raised issue priority (the partner wave on this
        // SIMD is then mostly in its MFMA phase): -1.8 % per fused launch, measured
        if (ATT_SOFTMAX_PRIO > 0) __builtin_amdgcn_s_setprio(ATT_SOFTMAX_PRIO);
        float p[16];
        float mx = -INFINITY;
        // p = the exponent of this tile's softmax weights relative to the base
        // mb = m_run - PSHIFT + ev (log2 units); the running max m_run is
        // re-based (lazily) when the tile's max exceeds it by > DEFER.
        float ex[16];
        if (ATT_QFMA && !first) {  // wave-uniform (scalar): every tile but the first (m_run = -inf there)
            // logit * M - mb in one rounding (Q carries log2(e)/sqrt(C), :39 and :41)
            const float mb0 = m_run - (float)H3_PSHIFT + ev;
#pragma unroll
            for (int r = 0; r < 16; ++r) p[r] = __builtin_fmaf(mv[r], S[r], -mb0);
            ATT_STAMP(stp, st_si + 1);
            ATT_STAMP(stp, st_si + 2);
            if (key0 + 32 > N) {  // wave-uniform: only the last key tile has padding keys
#pragma unroll
                for (int r = 0; r < 16; ++r)
                    if (key0 + acc_row(r, h) >= N) p[r] = -INFINITY;
            }
#pragma unroll
            for (int r = 0; r < 16; ++r) mx = fmaxf(mx, p[r]);
            mx = halves_max(mx);
            // logit max > m_run + DEFER  <=>  mx > DEFER + PSHIFT - ev
            if (__any(mx > H3_DEFER + (float)H3_PSHIFT - ev)) {
                const float m_new = fmaxf(m_run, mx + mb0);
                const float alpha = __builtin_amdgcn_exp2f(m_run - m_new);
                const float dm = m_new - m_run;
                m_run = m_new;
                l_run *= alpha;
#pragma unroll
                for (int t = 0; t < 4; ++t)
#pragma unroll
                    for (int r = 0; r < 16; ++r) O[t][r] *= alpha;  // lane = query
#pragma unroll
                for (int r = 0; r < 16; ++r) p[r] -= dm;
            }
        } else {
#pragma unroll
            for (int r = 0; r < 16; ++r) p[r] = S[r] * scale;  // (:39)
            ATT_STAMP(stp, st_si + 1);
#pragma unroll
            for (int r = 0; r < 16; ++r) p[r] = mv[r] * p[r];  // then * M (:41); 0, not -inf, off-support
            ATT_STAMP(stp, st_si + 2);
            if (key0 + 32 > N) {  // wave-uniform: only the last key tile has padding keys
#pragma unroll
                for (int r = 0; r < 16; ++r)
                    if (key0 + acc_row(r, h) >= N) p[r] = -INFINITY;
            }
#pragma unroll
            for (int r = 0; r < 16; ++r) mx = fmaxf(mx, p[r]);
            mx = halves_max(mx);
            if (__any(mx > m_run + H3_DEFER)) {  // wave-uniform re-base of the running max
                const float m_new = fmaxf(m_run, mx);
                const float alpha = __builtin_amdgcn_exp2f(m_run - m_new);
                m_run = m_new;
                l_run *= alpha;
#pragma unroll
                for (int t = 0; t < 4; ++t)
#pragma unroll
                    for (int r = 0; r < 16; ++r) O[t][r] *= alpha;  // lane = query
            }
            const float mb = m_run - (float)H3_PSHIFT + ev;
#pragma unroll
            for (int r = 0; r < 16; ++r) p[r] -= mb;
        }
        float psum = 0.0f;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            ex[r] = __builtin_amdgcn_exp2f(p[r]);
            psum += ex[r];
        }
#pragma unroll
        for (int s = 0; s < 2; ++s) {
            float v[8];
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] = ex[8 * s + e];
            split8x(v, ph[s], pl[s]);
        }
        l_run += ldexpf(psum, (int)ev);
        if (ATT_SOFTMAX_PRIO > 0) __builtin_amdgcn_s_setprio(0);
    };
    // O^T[32 t + m][query] += sum_key V[key][32 t + m] P[query][key]
    auto pv = [&](const char *Vl, const f16x8(&ph)[2], const f16x8(&pl)[2]) {
        f16x8 vf[3][2];
        auto vread = [&](int i, f16x8(&f)[2]) {  // fragment i = (t, s) = (i / 2, i % 2)
            f[0] = *reinterpret_cast<const f16x8 *>(Vl + 2 * h3_frag(i, 0, lane));
            f[1] = *reinterpret_cast<const f16x8 *>(Vl + 2 * h3_frag(i, 1, lane));
        };
        vread(0, vf[0]);
        vread(1, vf[1]);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            if (i + 2 < 8) vread(i + 2, vf[(i + 2) % 3]);
            // the three products in the order of P V's mfma_h3 (pl.vh, ph.vl, ph.vh)
            f32x16 o = mfma_h(vf[i % 3][0], pl[i & 1], O[i >> 1]);
            o = mfma_h(vf[i % 3][1], ph[i & 1], o);
            O[i >> 1] = mfma_h(vf[i % 3][0], ph[i & 1], o);
            __builtin_amdgcn_sched_barrier(0);
        }
    };

    // End of a tile: this wave's DMA of the next tile has landed and its LDS
    // reads returned, then the workgroup barrier -- as an s_waitcnt builtin
    // (not asm, not __syncthreads) so the compiler's counter model learns that
    // the DMA is done and adds no vmcnt(0) before the next tile's LDS reads.
    // Immediate (gfx9 simm16): vmcnt[3:0] | expcnt(7) << 4 | lgkmcnt(0) << 8.
    auto sync = [&] {
        __builtin_amdgcn_s_waitcnt(0x0070);  // vmcnt(0) lgkmcnt(0)
#ifndef ATT_DIAG_NOBAR
        if constexpr (WS == 0) __builtin_amdgcn_s_barrier();  // (WS: the wave's own slot only)
#endif
    };

    // (Measured and reverted: M and the exponent loaded by inline asm with an
    // explicit vmcnt -- the compiler waits vmcnt(0), the next tile's DMA
    // included, because it does not count LDS-DMA -- issued at the tile start
    // or at the end of the previous tile: no faster, and the compiler copies
    // asm-loaded registers before the wait.  DESIGN.md section 7.)
    auto slot_base = [&](int st) {
        return h3smem + (WS ? wave : (st - st0) % H3_NSLOT) * (H3_KTB + H3_VTB);
    };
    if constexpr (WS > 0) {
        // One slot per wave, its K and V halves refilled separately: tile t+1's K
        // is staged once tile t's QK^T has read its K (hidden behind tile t's
        // softmax and P.V), its M and V once P.V has read V (behind tile t+1's
        // QK^T).  Waits: the 16 V pieces issued last may stay in flight at a
        // tile's top, the next tile's 16 K pieces before P.V.
        char *slot = h3smem + wave * (H3_KTB + H3_VTB);
        auto stage_half = [&](int st, bool v) {  // 16 pieces of 1 KiB
#pragma unroll
            for (int i = 0; i < 16; ++i) {
#if ATT_BUFDMA
                __builtin_amdgcn_raw_ptr_buffer_load_lds(v ? rV : rK,
                                                         (__attribute__((address_space(3))) void *)(slot + (v ? H3_KTB : 0) + i * 1024),
                                                         16, 16 * lane, st * (v ? H3_VTB : H3_KTB) + i * 1024, 0, 0);
#else
                const char *src = (v ? Vp + (size_t)st * H3_VTB : Kp + (size_t)st * H3_KTB) + i * 1024;
                __builtin_amdgcn_global_load_lds(src + 16 * lane, slot + (v ? H3_KTB : 0) + i * 1024, 16, 0, 0);
#endif
            }
        };
        float mvA[16], evA;
        if (st0 < st1) {
            stage_half(st0, false);
            load_m(st0 * H3_TILE, mvA, evA);
            stage_half(st0, true);
        }
        for (int st = st0; st < st1; ++st) {
            float mv[16], ev;
            f16x8 ph[2], pl[2];
            __builtin_amdgcn_s_waitcnt(0x4F70);  // vmcnt(16): K and M of this tile landed (V may not have)
#pragma unroll
            for (int r = 0; r < 16; ++r) mv[r] = mvA[r];
            ev = evA;
            const bool more = st + 1 < st1;
            qk_softmax(slot, st * H3_TILE, mv, ev, ph, pl, st == st0, [&] {
                if (more) {
                    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): this tile's K reads returned
                    stage_half(st + 1, false);
                }
            });
            if (more)
                __builtin_amdgcn_s_waitcnt(0x4F70);  // vmcnt(16): this tile's V landed (the next K may not have)
            else
                __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
            pv(slot + H3_KTB, ph, pl);
            if (more) {
                load_m((st + 1) * H3_TILE, mvA, evA);
                __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): this tile's V reads returned
                stage_half(st + 1, true);
            }
        }
        l_run = halves_sum(l_run);
        return;
    }
    float mvA[16], evA;  // EARLY: the next tile's M, loaded a tile ahead
    if (st0 < st1) {
        stage(st0, 0);
        if constexpr (EARLY) {
            load_m(st0 * H3_TILE, mvA, evA);
            if (st0 + 1 < st1) stage(st0 + 1, 1);
        }
    }
    sync();
    for (int st = st0; st < st1; ++st) {
        float mv[16], ev;
        f16x8 ph[2], pl[2];
        const int si = 1 + 6 * min(st - st0, 23);
        st_si = si;
        ATT_STAMP(stp, si);
        if constexpr (EARLY) {
#pragma unroll
            for (int r = 0; r < 16; ++r) mv[r] = mvA[r];
            ev = evA;
            if (st + 1 < st1) load_m((st + 1) * H3_TILE, mvA, evA);
            // tile st0 + 1 went out before the loop; tile st + 1's slot held tile
            // st - 1, released by the barrier that ended iteration st - 1
            if (st > st0 && st + 1 < st1) stage(st + 1, ((st + 1 - st0) % H3_NSLOT));
        } else {
            load_m(st * H3_TILE, mv, ev);  // (padding waves' reads stay inside the pair's M)
            if (st + 1 < st1) stage(st + 1, ((st + 1 - st0) % H3_NSLOT));
        }
        // padding waves (q0 >= Npad) compute on clamped operands and store nothing
        qk_softmax(slot_base(st), st * H3_TILE, mv, ev, ph, pl, st == st0, [] {});
        ATT_STAMP(stp, si + 3);
        pv(slot_base(st) + H3_KTB, ph, pl);
        ATT_STAMP(stp, si + 4);
        sync();
        ATT_STAMP(stp, si + 5);
    }
    l_run = halves_sum(l_run);
}

template <int NW, bool XCD, bool PACKED, bool EARLY = false>
__global__ __launch_bounds__(NW * 64, 2) void attention_h3_kernel(
    const _Float16 *__restrict__ Qs, const _Float16 *__restrict__ Ks, const _Float16 *__restrict__ Vs,
    const float *__restrict__ vexp, const float *__restrict__ M, AttnGridH3 g, float *__restrict__ opart,
    float *__restrict__ ml) {
    extern __shared__ __attribute__((aligned(16))) char h3smem[];
    const AttnBlock blk = attention_h3_block(g, XCD);
    if (blk.qb * (NW * 32) >= g.n(blk.b)) return;  // past a ragged pair's end (workgroup-uniform)
    const int b = blk.b, split = blk.split, Npad = g.Npad;
    // wave in an SGPR: every wave-uniform branch (M orientation, active, the
    // barrier's count) is then a scalar branch, never an exec-masked one
    const int tid = threadIdx.x, wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63, h = lane >> 5;
    const int q0 = blk.qb * (NW * 32) + wave * 32, qq = q0 + (lane & 31);
#ifdef ATT_STAMPS
    unsigned long long *stp = att_stamp_ptr(wave);
    ATT_RSTAMP(stp, 184);
    ATT_STAMP(stp, 160);
#endif
    f32x16 O[4];
    float m_run, l_run;
    attention_h3_core<NW, PACKED, EARLY>(Qs, Ks, Vs, vexp, M, g, blk, h3smem, wave, lane, O, m_run, l_run);
    ATT_STAMP(stp, 161);
    ATT_RSTAMP(stp, 185);
    if (q0 >= Npad) return;
    const size_t obase = (size_t)(b * g.nsplit + split) * Npad;
    // registers 8u + 4g .. +3 of tile t = fragment block 2 (2t + u) + g (16 coalesced 1-KiB stores)
    float *Ob = opart + obase * CH + (size_t)(q0 >> 5) * (H3_TILE * CH) + 4 * lane;
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int q = 0; q < 4; ++q)
            *reinterpret_cast<f32x4 *>(Ob + (4 * t + q) * 256) =
                f32x4{O[t][4 * q], O[t][4 * q + 1], O[t][4 * q + 2], O[t][4 * q + 3]};
    if (h == 0) {
        // partial max in natural-log units (the p's carry the 2^PSHIFT factor)
        ml[(obase + qq) * 2] = (m_run - (float)H3_PSHIFT) * 0.6931471805599453f;
        ml[(obase + qq) * 2 + 1] = l_run;
    }
}

// The tiny plan's split-K attention with the split's key tiles spread over the
// workgroup's WS waves (attention_h3_core's WS mode; one 32-query block per
// workgroup): each wave runs its run of tiles alone on its SIMD (no partner
// wave, no workgroup barrier per tile), then the waves' (O, m, l) are merged
// through LDS into the workgroup's ONE partial -- the split count and the
// partials the pointwise kernel combines stay those of the one-wave plan.
//   O = sum_w 2^(m_w - m*) O_w,  l = sum_w 2^(m_w - m*) l_w,  m = m* = max_w m_w
// (waves in ascending order; an empty run has m = -inf: weight 0).  LDS: WS
// single-tile slots of 32 KiB, each wave's slot reused for its merge record.
template <int WS>
constexpr size_t attention_h3_ws_lds_bytes() { return (size_t)WS * (H3_KTB + H3_VTB); }

template <int WS, bool PACKED>
__global__ __launch_bounds__(WS * 64) void attention_h3_ws_kernel(
    const _Float16 *__restrict__ Qs, const _Float16 *__restrict__ Ks, const _Float16 *__restrict__ Vs,
    const float *__restrict__ vexp, const float *__restrict__ M, AttnGridH3 g, float *__restrict__ opart,
    float *__restrict__ ml) {
    extern __shared__ __attribute__((aligned(16))) char h3smem[];
    const AttnBlock blk = attention_h3_block(g, true);
    if (blk.qb * 32 >= g.n(blk.b)) return;  // past a ragged pair's end (workgroup-uniform)
    const int b = blk.b, split = blk.split, Npad = g.Npad;
    const int tid = threadIdx.x, wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63, h = lane >> 5;
    const int q0 = blk.qb * 32, qq = q0 + (lane & 31);
    f32x16 O[4];
    float m_run, l_run;
    attention_h3_core<1, PACKED, false, WS>(Qs, Ks, Vs, vexp, M, g, blk, h3smem, wave, lane, O, m_run, l_run);
    // merge record in this wave's own slot: O[t][r] at ((16 t + r) * 64 + lane), then m, l
    float *rec = reinterpret_cast<float *>(h3smem + wave * (H3_KTB + H3_VTB));
    __builtin_amdgcn_s_waitcnt(0xc07f);  // this wave's last LDS reads of its slot returned
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) rec[(16 * t + r) * 64 + lane] = O[t][r];
    rec[4096 + lane] = m_run;
    rec[4096 + 64 + lane] = l_run;
    __syncthreads();
    if (q0 >= Npad) return;
    float mw[WS], ms = -INFINITY;
#pragma unroll
    for (int w = 0; w < WS; ++w) {
        mw[w] = reinterpret_cast<const float *>(h3smem + w * (H3_KTB + H3_VTB))[4096 + lane];
        ms = fmaxf(ms, mw[w]);
    }
    float a[WS];
#pragma unroll
    for (int w = 0; w < WS; ++w) a[w] = ms == -INFINITY ? 0.0f : __builtin_amdgcn_exp2f(mw[w] - ms);
    const size_t obase = (size_t)(b * g.nsplit + split) * Npad;
    float *Ob = opart + obase * CH + (size_t)(q0 >> 5) * (H3_TILE * CH) + 4 * lane;
    for (int t = wave; t < 4; t += WS) {  // this wave's output tiles (registers 4q .. 4q+3 -> block 4t + q)
        float acc[16];
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[r] = 0.0f;
#pragma unroll
        for (int w = 0; w < WS; ++w) {
            const float *rw = reinterpret_cast<const float *>(h3smem + w * (H3_KTB + H3_VTB));
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[r] = __builtin_fmaf(a[w], rw[(16 * t + r) * 64 + lane], acc[r]);
        }
#pragma unroll
        for (int q = 0; q < 4; ++q)
            *reinterpret_cast<f32x4 *>(Ob + (4 * t + q) * 256) = f32x4{acc[4 * q], acc[4 * q + 1], acc[4 * q + 2], acc[4 * q + 3]};
    }
    if (wave == 0 && h == 0) {
        float l = 0.0f;
#pragma unroll
        for (int w = 0; w < WS; ++w)
            l = __builtin_fmaf(a[w], reinterpret_cast<const float *>(h3smem + w * (H3_KTB + H3_VTB))[4096 + 64 + lane], l);
        // partial max in natural-log units (the p's carry the 2^PSHIFT factor)
        ml[(obase + qq) * 2] = (ms - (float)H3_PSHIFT) * 0.6931471805599453f;
        ml[(obase + qq) * 2 + 1] = l;
    }
}

// vexp of every 32-key tile of fp32 v [B][ld][CH] (rows >= N count as 0):
// one workgroup per (tile, pair).
static __global__ __launch_bounds__(256) void vexp_kernel(const float *__restrict__ v, int N, int ld, int Npad,
                                                         float *__restrict__ vexp) {
    __shared__ float part[4];
    const int t = blockIdx.x, b = blockIdx.y, tid = threadIdx.x;
    float m = 0.0f;
    for (int e = tid; e < H3_TILE * CH; e += 256) {
        const int row = t * H3_TILE + e / CH;
        if (row < N) m = fmaxf(m, fabsf(v[((size_t)b * ld + row) * CH + e % CH]));
    }
    m = wave_max(m);
    if ((tid & 63) == 0) part[tid >> 6] = m;
    __syncthreads();
    if (tid == 0) vexp[(size_t)b * (Npad / H3_TILE) + t] = (float)h3_vexp(fmaxf(fmaxf(part[0], part[1]), fmaxf(part[2], part[3])));
}

// fp32 q, k, v [B][ld][CH] (ld >= N rows per pair; rows >= N of the padded
// layouts become zero) -> Qs, Ks, Vs (V scaled by its tile's 2^vexp).  One
// thread per (pair, row, channel).
static __global__ void split_qkv_kernel(const float *__restrict__ q, const float *__restrict__ k,
                                 const float *__restrict__ v, const float *__restrict__ vexp, int B, int N,
                                 int ld, int Npad, _Float16 *__restrict__ Qs, _Float16 *__restrict__ Ks,
                                 _Float16 *__restrict__ Vs) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (size_t)B * Npad * CH) return;
    const int c = (int)(i % CH);
    const int row = (int)((i / CH) % Npad);
    const int b = (int)(i / CH / Npad);
    const size_t src = ((size_t)b * ld + row) * CH + c, pb = (size_t)b * Npad * 2 * CH;
    const bool in = row < N;
    _Float16 hi, lo;
    split_h(in ? (ATT_QFMA ? q[src] * H3_QSCALE : q[src]) : 0.0f, hi, lo);
    Qs[pb + qs_off(row, 0, c)] = hi;
    Qs[pb + qs_off(row, 1, c)] = lo;
    split_h(in ? k[src] : 0.0f, hi, lo);
    Ks[pb + ks_off(row, 0, c)] = hi;
    Ks[pb + ks_off(row, 1, c)] = lo;
    const float ev = vexp[(size_t)b * (Npad / H3_TILE) + row / H3_TILE];
    split_h(in ? ldexpf(v[src], (int)ev) : 0.0f, hi, lo);
    Vs[pb + vs_off(row, 0, c)] = hi;
    Vs[pb + vs_off(row, 1, c)] = lo;
}

}  // namespace pdsc
