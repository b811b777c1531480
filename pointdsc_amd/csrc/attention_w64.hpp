// attention_w64.hpp -- the SCNonlocal attention core (models/PointDSC.py:36-42)
// with 64 queries per wave and one 4-wave workgroup per CU.
//
// Same arithmetic as attention_h3_core (attention_h3.hpp: 3xf16 products,
// online softmax with the lazy re-base, V tiles pre-scaled by 2^vexp) and the
// same HBM layouts, per query bit for bit; what changes is the schedule:
//
//   * a wave owns TWO 32-query blocks (A = queries q0 .. q0+31, B = q0+32 ..
//     q0+63), so every K or V fragment read from LDS feeds both blocks' MFMAs,
//     and a workgroup of 4 waves (one per SIMD) covers 256 queries -- the same
//     256 queries per CU as two 128-query workgroups of attention_h3, with ONE
//     K/V stream per CU instead of two;
//   * the wave has the whole 512-register file (launch bound 1 wave per SIMD):
//     Q fragments and O accumulators of both blocks (256 registers) sit in the
//     accumulator file, MFMA operands in place;
//   * with no partner wave on the SIMD, the wave overlaps its own softmax with
//     its own MFMAs: per key tile  QK_A | QK_B + softmax_A | PV_A + softmax_B |
//     PV_B  (each softmax's VALU beside the other block's matrix work);
//   * the K/V ring has 3 slots and tile t + 2 is queued at the top of tile t,
//     so the one barrier per tile waits only for a DMA issued a tile earlier;
//     the next tile's M is loaded at the top of the current one (two register
//     sets), ahead of that DMA, so the softmax's M waits never include it.
#pragma once
#include "attention_h3.hpp"

namespace pdsc {

// f(integral_constant<int, i>) for i = 0 .. N-1 (compile-time indices)
template <typename F, int... I> PDSC_DEV void static_for_(F &f, std::integer_sequence<int, I...>) {
    (f(std::integral_constant<int, I>{}), ...);
}
template <int N, typename F> PDSC_DEV void static_for(F &&f) { static_for_(f, std::make_integer_sequence<int, N>{}); }

// Pin x at this point of the instruction stream: an empty volatile asm that
// "modifies" x keeps IR passes from sinking its computation past here and the
// scheduler from hoisting its consumers above (the softmax slices' placement).
template <typename T> PDSC_DEV void w64_pin(T &x) { asm volatile("" : "+v"(x)); }

constexpr int W64_NW = 4;                    // waves per workgroup (one per SIMD)
constexpr int W64_QW = 64;                   // queries per wave (two 32-query blocks)
constexpr int W64_QPB = W64_NW * W64_QW;     // queries per workgroup
constexpr int W64_NSLOT = 4;                 // K/V ring slots (V(t-1) is read in tile t)
constexpr size_t W64_RING = (size_t)W64_NSLOT * (H3_KTB + H3_VTB);  // 128 KiB
constexpr int W64_MAXT = 1024;                                       // V-tile exponents in LDS (N <= 32767)
constexpr size_t W64_LDS = W64_RING + W64_MAXT * sizeof(float);

// ---- the accumulator file, asm-owned ----------------------------------------
// The wave's Q fragments and O accumulators (256 registers) live in fixed
// AGPRs, named literally by the inline-asm MFMAs below:
//   O of block u, channel tile t:       a[64 u + 16 t .. + 15]
//   Q of block u, k-step j, plane p:    a[128 + 64 u + 8 j + 4 p .. + 3]
// hipcc allocates the VGPRs (softmax, M, K/V and P fragments, S) and must not
// use an AGPR itself: w64_claim_agprs() makes the kernel descriptor allocate all
// 256, and the kernel is audited for compiler-generated v_accvgpr_* / scratch
// ("asm-owned accumulators").  hipcc models none of these asm
// MFMAs, so each hazard is padded inside the strings: an MFMA result read by
// VALU (8-pass XDL: 12 wait states, s_nop 11); an AGPR written by
// v_accvgpr_write read by an MFMA (2: s_nop 1).  Chains D -> next C need none;
// operands from ds_read are waited for by the compiler (it sees the "v" input);
// P fragments come out of split2, which ends on its own s_nop 1.
constexpr int W64_AO = 0, W64_AQ = 128;
#define W64_AGPRS "a0","a1","a2","a3","a4","a5","a6","a7","a8","a9","a10","a11","a12","a13","a14","a15","a16","a17","a18","a19","a20","a21","a22","a23","a24","a25","a26","a27","a28","a29","a30","a31","a32","a33","a34","a35","a36","a37","a38","a39","a40","a41","a42","a43","a44","a45","a46","a47","a48","a49","a50","a51","a52","a53","a54","a55","a56","a57","a58","a59","a60","a61","a62","a63","a64","a65","a66","a67","a68","a69","a70","a71","a72","a73","a74","a75","a76","a77","a78","a79","a80","a81","a82","a83","a84","a85","a86","a87","a88","a89","a90","a91","a92","a93","a94","a95","a96","a97","a98","a99","a100","a101","a102","a103","a104","a105","a106","a107","a108","a109","a110","a111","a112","a113","a114","a115","a116","a117","a118","a119","a120","a121","a122","a123","a124","a125","a126","a127","a128","a129","a130","a131","a132","a133","a134","a135","a136","a137","a138","a139","a140","a141","a142","a143","a144","a145","a146","a147","a148","a149","a150","a151","a152","a153","a154","a155","a156","a157","a158","a159","a160","a161","a162","a163","a164","a165","a166","a167","a168","a169","a170","a171","a172","a173","a174","a175","a176","a177","a178","a179","a180","a181","a182","a183","a184","a185","a186","a187","a188","a189","a190","a191","a192","a193","a194","a195","a196","a197","a198","a199","a200","a201","a202","a203","a204","a205","a206","a207","a208","a209","a210","a211","a212","a213","a214","a215","a216","a217","a218","a219","a220","a221","a222","a223","a224","a225","a226","a227","a228","a229","a230","a231","a232","a233","a234","a235","a236","a237","a238","a239","a240","a241","a242","a243","a244","a245","a246","a247","a248","a249","a250","a251","a252","a253","a254","a255"
PDSC_DEV void w64_claim_agprs() { asm volatile("" ::: W64_AGPRS); }

// S^T (+)= K Q^T, one fp16 product: K fragment (VGPRs) x Q fragment a[QA..QA+3]
template <int QA> PDSC_DEV void w64_kq0(f32x16 &c, const f16x8 &k) {
    asm volatile("v_mfma_f32_32x32x16_f16 %0, %1, a[%c2:%c3], 0" : "=&v"(c) : "v"(k), "i"(QA), "i"(QA + 3));
}
template <int QA> PDSC_DEV void w64_kq(f32x16 &c, const f16x8 &k) {
    asm volatile("v_mfma_f32_32x32x16_f16 %0, %1, a[%c2:%c3], %0" : "+v"(c) : "v"(k), "i"(QA), "i"(QA + 3));
}
template <int QA> PDSC_DEV void w64_kq_last(f32x16 &c, const f16x8 &k) {
    asm volatile("v_mfma_f32_32x32x16_f16 %0, %1, a[%c2:%c3], %0\n\ts_nop 11" : "+v"(c) : "v"(k), "i"(QA), "i"(QA + 3));
}
// one k-step j of block u's S^T (= mfma_h3(kh, kl, qh, ql, S): kl.qh, kh.ql, kh.qh)
template <int U, int J> PDSC_DEV void w64_qk_step(f32x16 &S, const f16x8 (&kf)[2]) {
    constexpr int QH = W64_AQ + 64 * U + 8 * J, QL = QH + 4;
    if constexpr (J == 0)
        w64_kq0<QH>(S, kf[1]);
    else
        w64_kq<QH>(S, kf[1]);
    w64_kq<QL>(S, kf[0]);
    if constexpr (J == 7)
        w64_kq_last<QH>(S, kf[0]);
    else
        w64_kq<QH>(S, kf[0]);
}
// O^T tile a[OA..OA+15] += V^T P^T, one fp16 product
template <int OA> PDSC_DEV void w64_vp(const f16x8 &v, const f16x8 &p) {
    asm volatile("v_mfma_f32_32x32x16_f16 a[%c0:%c1], %2, %3, a[%c0:%c1]" ::"i"(OA), "i"(OA + 15), "v"(v), "v"(p));
}
// fragment i = (t, s) of block u's P V: pl.vh, ph.vl, ph.vh (P V's mfma_h3 order)
template <int U, int I> PDSC_DEV void w64_pv_step(const f16x8 (&vf)[2], const f16x8 (&ph)[2], const f16x8 (&pl)[2]) {
    constexpr int OA = W64_AO + 64 * U + 16 * (I >> 1);
    w64_vp<OA>(vf[0], pl[I & 1]);
    w64_vp<OA>(vf[1], ph[I & 1]);
    w64_vp<OA>(vf[0], ph[I & 1]);
}
// Q fragment (16 B per lane at p) straight into a[A..A+3]
template <int A> PDSC_DEV void w64_load_q(const void *p) {
    asm volatile("global_load_dwordx4 a[%c0:%c1], %2, off" ::"i"(A), "i"(A + 3), "v"(p) : "memory");
}
// a[A] = 0
template <int A> PDSC_DEV void w64_zero_a() { asm volatile("v_accvgpr_write_b32 a%c0, 0" ::"i"(A)); }
// a[A] *= alpha (the re-base of a running max)
template <int A> PDSC_DEV void w64_scale_a(float alpha) {
    float t;
    asm volatile("v_accvgpr_read_b32 %0, a%c1\n\tv_mul_f32 %0, %0, %2\n\tv_accvgpr_write_b32 a%c1, %0"
                 : "=&v"(t)
                 : "i"(A), "v"(alpha));
}
template <int A> PDSC_DEV float w64_read_a() {
    float x;
    asm volatile("v_accvgpr_read_b32 %0, a%c1" : "=v"(x) : "i"(A));
    return x;
}
// ---- M, asm-owned VGPRs -------------------------------------------------------
// The two M register sets (tile t's and tile t + 1's, both blocks) live in
// v[192:255]: set s, block u at v[W64_VM + 32 s + 16 u .. + 15], register r =
// this lane's M[32 kt + acc_row(r, h)][32 qt + l32].  hipcc is capped below them
// (amdgpu_num_vgpr) and never sees them: the loads, their waits and the two
// softmax instructions that read them are asm, so the register-to-load binding
// cannot be broken by a copy or a reuse while a load is in flight, and the two
// load shapes below (one of them four 4-byte ops) fill the same registers.
constexpr int W64_VM = 192;
PDSC_DEV void w64_claim_vm() {
    asm volatile("" ::: "v192","v193","v194","v195","v196","v197","v198","v199","v200","v201","v202","v203","v204","v205","v206","v207","v208","v209","v210","v211","v212","v213","v214","v215","v216","v217","v218","v219","v220","v221","v222","v223","v224","v225","v226","v227","v228","v229","v230","v231","v232","v233","v234","v235","v236","v237","v238","v239","v240","v241","v242","v243","v244","v245","v246","v247","v248","v249","v250","v251","v252","v253","v254","v255");
}
// M quad G (registers R + 4 G ..) of a lane from the symmetric-packed layout
// (row-major 32 x 32 tiles, pdsc_internal.hpp mpack_tile).  Rows = queries (tile
// (qt, kt), kt > qt): 16 B of the lane's row, one op.  Rows = keys (tile (kt,
// qt), kt <= qt): 4 words of the lane's column 128 B apart, four ops (each a
// coalesced 128-B row piece per half-wave).  hipcc does not count these loads:
// their waits are the kernel's own.
template <int R, int G> PDSC_DEV void w64_mload_row(__amdgpu_buffer_rsrc_t r, uint32_t voff) {
    asm volatile("buffer_load_dwordx4 v[%c0:%c1], %2, %3, 0 offen offset:%c4" ::"i"(R + 4 * G), "i"(R + 4 * G + 3),
                 "v"(voff), "s"(r), "i"(32 * G)
                 : "memory");
}
template <int R, int G> PDSC_DEV void w64_mload_col(__amdgpu_buffer_rsrc_t r, uint32_t voff) {
    asm volatile("buffer_load_dword v%c0, %4, %5, 0 offen offset:%c6\n\t"
                 "buffer_load_dword v%c1, %4, %5, 0 offen offset:%c7\n\t"
                 "buffer_load_dword v%c2, %4, %5, 0 offen offset:%c8\n\t"
                 "buffer_load_dword v%c3, %4, %5, 0 offen offset:%c9" ::"i"(R + 4 * G), "i"(R + 4 * G + 1),
                 "i"(R + 4 * G + 2), "i"(R + 4 * G + 3), "v"(voff), "s"(r), "i"(1024 * G), "i"(1024 * G + 128),
                 "i"(1024 * G + 256), "i"(1024 * G + 384)
                 : "memory");
}
// all but the N youngest vector-memory ops done
template <int N> PDSC_DEV void w64_vmwait() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }
// a block's M ready: 8 + (4 or 16) younger ops -- the DMA pieces around the
// other block's M, whose op count depends on its orientation (scalar branch)
PDSC_DEV void w64_mwait_after(bool other_keyrows) {
    if (other_keyrows)
        w64_vmwait<8 + 16>();
    else
        w64_vmwait<8 + 4>();
}
// p = M[r] s - mb (softmax part 1), p = M[r] p (the first tile)
template <int R> PDSC_DEV float w64_fma_m(float sv, float mb) {
    float p;
    asm volatile("v_fma_f32 %0, v%c1, %2, -%3" : "=v"(p) : "i"(R), "v"(sv), "v"(mb));
    return p;
}
template <int R> PDSC_DEV void w64_mul_m(float &p) { asm volatile("v_mul_f32 %0, v%c1, %0" : "+v"(p) : "i"(R)); }

// Diagnostic build only (-DW64_STAMPS, tools/att_w64_bench.hip): s_memtime at
// region boundaries of every tile, kept in LDS past W64_LDS (no vector-memory
// op: the kernel's vmcnt counts stay as in the product), copied out at the end
// for the first W64_ST_WGS workgroups into a buffer nothing else reads.
#ifdef W64_STAMPS
constexpr int W64_ST_PER_TILE = 6, W64_ST_TILES = 40, W64_ST_WGS = 64;
constexpr int W64_ST_PER_WAVE = W64_ST_PER_TILE * W64_ST_TILES + 8;
constexpr size_t W64_ST_LDS = (size_t)W64_NW * W64_ST_PER_WAVE * 8;
static __device__ unsigned long long g_w64_stamps[W64_ST_WGS * W64_NW * W64_ST_PER_WAVE];
#define W64_ST(i)                                                                                   \
    do {                                                                                            \
        __builtin_amdgcn_sched_barrier(0);                                                          \
        const unsigned long long t_ = __builtin_amdgcn_s_memtime();                                 \
        if (lane == 0 && (i) < W64_ST_PER_WAVE) st_lds[i] = t_;                                     \
        __builtin_amdgcn_sched_barrier(0);                                                          \
    } while (0)
#else
constexpr int W64_ST_PER_TILE = 6;
constexpr size_t W64_ST_LDS = 0;
#define W64_ST(i) \
    do {          \
    } while (0)
#endif

// split2 (attention_h3.hpp) as three single-instruction statements, so a
// softmax slice carries one of them: hi = {f16(x0), f16(x1)}, then lo's halves
// by v_fma_mixlo / v_fma_mixhi (x - hi exact, one rounding).  No s_nop: the P
// fragments are read by the MFMAs of the NEXT region, many states later.
PDSC_DEV void w64_cvt_hi(float x0, float x1, uint32_t &hi) {
    asm volatile("v_cvt_pk_f16_f32 %0, %1, %2" : "=v"(hi) : "v"(x0), "v"(x1));
}
PDSC_DEV void w64_mix_lo(float x0, uint32_t hi, uint32_t &lo) {
    asm volatile("v_fma_mixlo_f16 %0, %1, 1.0, -%2 op_sel_hi:[0,0,1]" : "=&v"(lo) : "v"(x0), "v"(hi));
}
PDSC_DEV void w64_mix_hi(float x1, uint32_t hi, uint32_t &lo) {
    asm volatile("v_fma_mixhi_f16 %0, %1, 1.0, -%2 op_sel:[0,0,1] op_sel_hi:[0,0,1]" : "+v"(lo) : "v"(x1), "v"(hi));
}

// split-K grid of 256-query blocks (slots = resident workgroups: one per CU)
inline AttnGridH3 attention_w64_grid(int B, int N, int slots) { return attention_h3_grid<W64_QPB / 32>(B, N, slots); }

// The attention of one workgroup (4 waves x 64 queries of pair blk.b, query
// block blk.qb, key-tile split blk.split).  Leaves, per block u of this wave,
// this lane's un-normalised O^T in a[64 u .. 64 u + 63] (w64_read_o; lane <->
// query, tile t register r <-> channel 32 t + acc_row(r, h), as
// attention_h3_core), the running max m (log2 units, + PSHIFT) and the full
// row sum l.  smem: W64_LDS bytes, free again when this returns.
//
// Software pipeline (block B half a tile behind block A), per key tile t:
//   R1  QK_A(t)    beside  softmax_B(t-1), part 2 (2^p, row sum, P split)
//   R2  PV_B(t-1)  beside  softmax_A(t),   part 1 (logits, max, re-base test)
//                          + the M loads of tile t+1 and the DMA of tile t+2
//       [re-base of block A, rare]
//   R3  QK_B(t)    beside  softmax_A(t),   part 2
//       [barrier: tile t+1 landed; V(t-1) retired by every wave]
//   R4  PV_A(t)    beside  softmax_B(t),   part 1
//       [re-base of block B, rare]
// Each region is 24 MFMAs; its VALU is dealt out one slice after each MFMA
// (sched_barrier-fenced: hipcc neither knows the asm MFMA's 32 cycles nor may
// it move the slices), the K / V fragments read two k-steps ahead, across
// region boundaries.  The K/V ring has 4 slots (V(t-1) is read in tile t).
PDSC_DEV void attention_w64_core(const _Float16 *__restrict__ Qs, const _Float16 *__restrict__ Ks,
                                 const _Float16 *__restrict__ Vs, const float *__restrict__ vexp,
                                 const float *__restrict__ M, const AttnGridH3 &g, const AttnBlock &blk, char *smem,
                                 int wave, int lane, float (&m_run)[2], float (&l_run)[2]) {
    const int b = blk.b, qb = blk.qb, split = blk.split;
    const int N = g.n(b), Npad = g.Npad;  // this pair's keys; the batch's row stride
    const int h = lane >> 5;
    const int q0 = qb * W64_QPB + wave * W64_QW;  // block u: queries q0 + 32 u ..
    const int nst = (N + H3_TILE - 1) / H3_TILE;
    const int st0 = blk.st1 >= 0 ? blk.st0 : split * g.sps, st1 = blk.st1 >= 0 ? blk.st1 : min(nst, st0 + g.sps);

    const char *Kp = reinterpret_cast<const char *>(Ks + (size_t)b * Npad * 2 * CH);
    const char *Vp = reinterpret_cast<const char *>(Vs + (size_t)b * Npad * 2 * CH);
    const int mnt = mpack_ntile(g.N);  // M's layout is the batch stride's
    const size_t mper = mpack_floats(g.N);
#ifdef W64_EXP_MSHARED  // diagnostic: every pair reads pair 0's M (L2 / MALL resident)
    const __amdgpu_buffer_rsrc_t rM = h3_rsrc(M, (uint32_t)(mper * 4u));
#else
    const __amdgpu_buffer_rsrc_t rM = h3_rsrc(M + (size_t)b * mper, (uint32_t)(mper * 4u));
#endif
    const float *vexp_b = vexp + (size_t)b * (Npad / H3_TILE);
    const __amdgpu_buffer_rsrc_t rK = h3_rsrc(Kp, (uint32_t)Npad * H3_ROWB), rV = h3_rsrc(Vp, (uint32_t)Npad * H3_ROWB);

#ifdef W64_STAMPS
    unsigned long long *st_lds = reinterpret_cast<unsigned long long *>(smem + W64_LDS) + wave * W64_ST_PER_WAVE;
    const unsigned long long st_c0 = __builtin_amdgcn_s_memtime(), st_r0 = __builtin_amdgcn_s_memrealtime();
#endif
    w64_claim_agprs();
    w64_claim_vm();
    static_for<128>([&](auto ic) { w64_zero_a<W64_AO + decltype(ic)::value>(); });
#pragma unroll
    for (int u = 0; u < 2; ++u) {
        m_run[u] = -INFINITY;
        l_run[u] = 0.0f;
    }
    // a split wholly past a ragged pair's key tiles (workgroup-uniform): O = 0,
    // m = -inf, l = 0, as attention_h3_core's empty tile loop leaves them
    if (st0 >= st1) return;
    // both blocks' queries (2 x 8 k-steps x (hi, lo) fragments) into the
    // accumulator file
    static_for<2>([&](auto uc) {
        constexpr int u = decltype(uc)::value;
        const _Float16 *qt =
            Qs + (size_t)b * Npad * 2 * CH + (size_t)(min(q0 + 32 * u, Npad - 32) >> 5) * H3_TILE_H;
        static_for<8>([&](auto jc) {
            constexpr int j = decltype(jc)::value;
            w64_load_q<W64_AQ + 64 * u + 8 * j>(qt + h3_frag(j, 0, lane));
            w64_load_q<W64_AQ + 64 * u + 8 * j + 4>(qt + h3_frag(j, 1, lane));
        });
    });

    auto slot_of = [&](int st) { return smem + ((st - st0) & (W64_NSLOT - 1)) * (H3_KTB + H3_VTB); };
    // LDS-DMA piece i (0 .. 7) of this wave's share of tile st.  Issued
    // unconditionally (a tile past the split's end reads past the K/V resource,
    // or a tile nobody reads: zeros or unused bytes into a free slot) -- a branch
    // here would cost hipcc its vmcnt bookkeeping of the DMA.
    constexpr int DMA_PW = (H3_KTB + H3_VTB) / 1024 / W64_NW;  // pieces per wave and tile (8)
    // waves 0, 1 copy K, waves 2, 3 copy V: one resource per wave, chosen once
    // (a per-piece branch would again cost the vmcnt bookkeeping)
    static_assert(H3_KTB == H3_VTB && W64_NW * DMA_PW == 2 * H3_KTB / 1024, "K / V split over the waves");
    const __amdgpu_buffer_rsrc_t rS = wave < W64_NW / 2 ? rK : rV;
    const int pbase = (wave * DMA_PW) % (H3_KTB / 1024);  // this wave's first piece within its K or V tile
    auto stage_piece = [&](int st, int i) {
        char *dst = slot_of(st) + (wave * DMA_PW + i) * 1024;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rS, (__attribute__((address_space(3))) void *)dst, 16, 16 * lane,
                                                 st * H3_KTB + (pbase + i) * 1024, 0, 0);
    };
    // M of tile st, block u, quad gg: this lane's 16 values M[32 st + acc_row(r, h)]
    // [32 qt + l32] from packed tile (st, qt) (rows = keys: column l32, rows 4 h +
    // 8 gg ..) or (qt, st) (rows = queries: row l32, columns 4 h + 8 gg ..).  The
    // offsets of attention_h3_core's packed loads (a block past the layout reads
    // past the resource: zeros).
    const int qt0 = q0 >> 5;  // block A's query tile (wave-uniform)
    const uint32_t vcol = (uint32_t)(4 * h * MPACK_T + (lane & 31)) * 4u;
    const uint32_t vrow = (uint32_t)((lane & 31) * MPACK_T + 4 * h) * 4u;
    auto keyrows = [&](int st, int u) { return st <= qt0 + u; };  // tile st of block u is read by columns
    // the load shape of tile st, block u under a tile step's shape SH: 1 = every
    // block by columns (st <= qt0), 2 = every block by rows (st > qt0 + 1),
    // 0 = per block at run time.  The key tiles of a query block run through
    // shape 1, one or two mixed steps, then shape 2: the kernel's tile steps
    // come in those three compiled forms, so the hot loops carry no per-load
    // branch (per-load scalar branches measured 300 vs 274 us per launch).
    auto kr = [&](auto shc, int st, int u) {
        constexpr int SH = decltype(shc)::value;
        if constexpr (SH == 1)
            return true;
        else if constexpr (SH == 2)
            return false;
        else
            return keyrows(st, u);
    };
    using SH0 = std::integral_constant<int, 0>;
    using SH1 = std::integral_constant<int, 1>;
    using SH2 = std::integral_constant<int, 2>;
    // quad gg of block u's M of tile st into register set ms
    auto load_mq = [&](auto shc, auto msc, auto uc, auto gc, int st) {
        constexpr int R = W64_VM + 32 * decltype(msc)::value + 16 * decltype(uc)::value, gg = decltype(gc)::value;
        const int qt = qt0 + decltype(uc)::value;
        if (kr(shc, st, decltype(uc)::value))
            w64_mload_col<R, gg>(rM, vcol + (uint32_t)mpack_tile(st, qt, mnt) * (MPACK_T * MPACK_T * 4u));
        else
            w64_mload_row<R, gg>(rM, vrow + (uint32_t)mpack_tile(qt, st, mnt) * (MPACK_T * MPACK_T * 4u));
    };
    const float *ev_lds = reinterpret_cast<const float *>(smem + W64_RING);
    auto load_ev = [&](int st) { return ev_lds[st]; };  // (wave-uniform address: one broadcast read)

#ifdef W64_EXP_NO_LDSREAD  // diagnostic: fragments read once, then reused (no ds_read in the loop)
    bool lds_once = true;
#endif
    auto kread = [&](const char *Kl, int j, f16x8(&f)[2]) {
#ifdef W64_EXP_NO_LDSREAD
        if (!lds_once) return;
#endif
        f[0] = *reinterpret_cast<const f16x8 *>(Kl + 2 * h3_frag(j, 0, lane));
        f[1] = *reinterpret_cast<const f16x8 *>(Kl + 2 * h3_frag(j, 1, lane));
    };
    auto vread = [&](const char *Vl, int i, f16x8(&f)[2]) {  // fragment i = (t, s) = (i / 2, i % 2)
#ifdef W64_EXP_NO_LDSREAD
        if (!lds_once) return;
#endif
        f[0] = *reinterpret_cast<const f16x8 *>(Vl + 2 * h3_frag(i, 0, lane));
        f[1] = *reinterpret_cast<const f16x8 *>(Vl + 2 * h3_frag(i, 1, lane));
    };

    // per-block softmax state between the two parts
    struct SmA {
        float p[16];  // logit exponents relative to the base (part 1 -> part 2)
        float mx, mb0;
        bool resc;
    };
    // softmax part 1, slice k (0 .. 23) of block u (tile key0, its M and ev):
    // p = M S - base (one fma), the tile's max, the re-base test (attention_h3_core
    // arithmetic, not the first tile)
    auto sm1_slice = [&](auto kc, int u, const f32x16 &S, auto mrc, float ev, int key0, SmA &a) {
        constexpr int k = decltype(kc)::value, MR = decltype(mrc)::value;  // MR: the block's M registers
#ifdef W64_EXP_NO_SM1  // diagnostic: no part-1 VALU (p = S)
        if constexpr (k >= 1 && k <= 16) a.p[k - 1] = S[k - 1];
        if constexpr (k == 22) a.resc = false;
        return;
#endif
        if constexpr (k == 0) {
            a.mb0 = m_run[u] - (float)H3_PSHIFT + ev;
            a.mx = -INFINITY;
            w64_pin(a.mb0);
        } else if constexpr (k <= 16) {
            constexpr int r = k - 1;
            a.p[r] = w64_fma_m<MR + r>(S[r], a.mb0);
            w64_pin(a.p[r]);
        } else if constexpr (k <= 20) {
            if constexpr (k == 17) {
                if (__builtin_expect(key0 + 32 > N, 0)) {  // wave-uniform: only the last key tile has padding keys
#pragma unroll
                    for (int r = 0; r < 16; ++r)
                        if (key0 + acc_row(r, h) >= N) a.p[r] = -INFINITY;
                }
            }
#pragma unroll
            for (int r = 4 * (k - 17); r < 4 * (k - 16); ++r) a.mx = fmaxf(a.mx, a.p[r]);
            w64_pin(a.mx);
        } else if constexpr (k == 21) {
            a.mx = halves_max(a.mx);
            w64_pin(a.mx);
        } else if constexpr (k == 22) {
            a.resc = __any(a.mx > H3_DEFER + (float)H3_PSHIFT - ev);  // logit max > m_run + DEFER
        }
    };
    // the re-base of block u's running max (rare; after part 1, before its P V)
    auto rebase = [&](auto uc, SmA &a) {
        constexpr int u = decltype(uc)::value;
        if (a.resc) {
            const float m_new = fmaxf(m_run[u], a.mx + a.mb0);
            const float alpha = __builtin_amdgcn_exp2f(m_run[u] - m_new);
            const float dm = m_new - m_run[u];
            m_run[u] = m_new;
            l_run[u] *= alpha;
            static_for<64>([&](auto ic) { w64_scale_a<W64_AO + 64 * u + decltype(ic)::value>(alpha); });
            asm volatile("s_nop 1");  // v_accvgpr_write -> MFMA C
#pragma unroll
            for (int r = 0; r < 16; ++r) a.p[r] -= dm;
        }
    };
    // the first tile's part 1 (m_run = -inf, O = 0: attention_h3_core's first-tile arithmetic)
    auto sm1_first = [&](int u, const f32x16 &S, auto mrc, float ev, int key0, SmA &a) {
        constexpr int MR = decltype(mrc)::value;
        const float scale = ATT_QFMA ? 1.0f : H3_QSCALE;
        float mx = -INFINITY;
#pragma unroll
        for (int r = 0; r < 16; ++r) a.p[r] = S[r] * scale;
        static_for<16>([&](auto rc) { w64_mul_m<MR + decltype(rc)::value>(a.p[decltype(rc)::value]); });
        if (key0 + 32 > N) {
#pragma unroll
            for (int r = 0; r < 16; ++r)
                if (key0 + acc_row(r, h) >= N) a.p[r] = -INFINITY;
        }
#pragma unroll
        for (int r = 0; r < 16; ++r) mx = fmaxf(mx, a.p[r]);
        mx = halves_max(mx);
        if (__any(mx > m_run[u] + H3_DEFER)) {  // (O = 0: its re-scale by alpha = 0 is a no-op)
            const float m_new = fmaxf(m_run[u], mx);
            const float alpha = __builtin_amdgcn_exp2f(m_run[u] - m_new);
            m_run[u] = m_new;
            l_run[u] *= alpha;
        }
        const float mb = m_run[u] - (float)H3_PSHIFT + ev;
#pragma unroll
        for (int r = 0; r < 16; ++r) a.p[r] -= mb;
    };
    // softmax part 2, slice k: the weights 2^p, their row sum (in key order),
    // the fp16 hi / lo P fragments, the row-sum update
    struct SmB {
        float ex[16], psum;
        uint32_t hi[8], lo[8];
    };
    auto sm2_slice = [&](auto kc, int u, const SmA &a, float ev, SmB &w, f16x8(&ph)[2], f16x8(&pl)[2]) {
        constexpr int k = decltype(kc)::value;
#ifdef W64_EXP_NO_SM2  // diagnostic: no part-2 VALU (P = the bits of p)
        if constexpr (k < 8) {
            auto hs = __builtin_bit_cast(u32x4, ph[k >> 2]);
            hs[k & 3] = __builtin_bit_cast(uint32_t, a.p[2 * k]);
            ph[k >> 2] = pl[k >> 2] = __builtin_bit_cast(f16x8, hs);
        }
        return;
#endif
        if constexpr (k == 0) w.psum = 0.0f;
        if constexpr (k < 16) {
            w.ex[k] = __builtin_amdgcn_exp2f(a.p[k]);
            w64_pin(w.ex[k]);
        }
        if constexpr (k >= 1 && k <= 16) {
            w.psum += w.ex[k - 1];
            w64_pin(w.psum);
        }
        // pair i = (ex[2i], ex[2i+1]): hi at slice 2i + 3, lo's halves at 2i + 4, 2i + 5
        if constexpr (k >= 3 && k <= 17 && (k & 1)) {
            constexpr int i = (k - 3) / 2;
            w64_cvt_hi(w.ex[2 * i], w.ex[2 * i + 1], w.hi[i]);
        }
        if constexpr (k >= 4 && k <= 18 && !(k & 1)) {
            constexpr int i = (k - 4) / 2;
            w64_mix_lo(w.ex[2 * i], w.hi[i], w.lo[i]);
        }
        if constexpr (k >= 5 && k <= 19 && (k & 1)) {
            constexpr int i = (k - 5) / 2;
            w64_mix_hi(w.ex[2 * i + 1], w.hi[i], w.lo[i]);
            // fragment s = i / 4, element pair (2 (i % 4), +1)
            auto hs = __builtin_bit_cast(u32x4, ph[i >> 2]);
            auto ls = __builtin_bit_cast(u32x4, pl[i >> 2]);
            hs[i & 3] = w.hi[i];
            ls[i & 3] = w.lo[i];
            ph[i >> 2] = __builtin_bit_cast(f16x8, hs);
            pl[i >> 2] = __builtin_bit_cast(f16x8, ls);
        }
        if constexpr (k == 20) {
            l_run[u] += ldexpf(w.psum, (int)ev);
            w64_pin(l_run[u]);
        }
    };

    // MFMA k (0 .. 23) of the QK^T of block U from K fragments kf; kread
    // ahead: the ring's k-step j + 2, or (kn) the next region's first two.
    float dummy = 0.0f;
    (void)dummy;

    struct Frag {
        f16x8 f[3][2];
    };
    Frag kf, vf;

    // The regions.  nxt(k): the fragment read issued after MFMA k (k % 3 == 2
    // reads k-step k / 3 + 3's fragment ... as below)
    auto qk_region = [&](auto uc, const char *Kl, f32x16 &S, auto nextread, auto slice) {
        constexpr int U = decltype(uc)::value;
        static_for<24>([&](auto kc) {
            constexpr int k = decltype(kc)::value, j = k / 3, m = k % 3;
            if constexpr (m == 0) {
                if constexpr (j + 2 < 8)
                    kread(Kl, j + 2, kf.f[(j + 2) % 3]);
                else
                    nextread(std::integral_constant<int, j - 6>{});  // the next region's fragment 0 / 1
            }
            constexpr int QH = W64_AQ + 64 * U + 8 * j, QL = QH + 4;
            const f16x8(&f)[2] = kf.f[j % 3];
            if constexpr (m == 0) {
                if constexpr (j == 0)
                    w64_kq0<QH>(S, f[1]);
                else
                    w64_kq<QH>(S, f[1]);
            } else if constexpr (m == 1) {
                w64_kq<QL>(S, f[0]);
            } else {
                if constexpr (j == 7)
                    w64_kq_last<QH>(S, f[0]);
                else
                    w64_kq<QH>(S, f[0]);
            }
            slice(kc);
            __builtin_amdgcn_sched_barrier(0);
        });
    };
    auto pv_region = [&](auto uc, const char *Vl, const f16x8 (&ph)[2], const f16x8 (&pl)[2], auto nextread, auto slice) {
        constexpr int U = decltype(uc)::value;
        static_for<24>([&](auto kc) {
            constexpr int k = decltype(kc)::value, i = k / 3, m = k % 3;
            if constexpr (m == 0) {
                if constexpr (i + 2 < 8)
                    vread(Vl, i + 2, vf.f[(i + 2) % 3]);
                else
                    nextread(std::integral_constant<int, i - 6>{});
            }
            constexpr int OA = W64_AO + 64 * U + 16 * (i >> 1);
            const f16x8(&f)[2] = vf.f[i % 3];
            if constexpr (m == 0)
                w64_vp<OA>(f[0], pl[i & 1]);
            else if constexpr (m == 1)
                w64_vp<OA>(f[1], ph[i & 1]);
            else
                w64_vp<OA>(f[0], ph[i & 1]);
            slice(kc);
            __builtin_amdgcn_sched_barrier(0);
        });
    };
    // next-region fragment reads: K of tile Kl into kf, V of tile Vl into vf
    auto next_k = [&](const char *Kl) { return [&, Kl](auto ic) { kread(Kl, decltype(ic)::value, kf.f[decltype(ic)::value]); }; };
    auto next_v = [&](const char *Vl) { return [&, Vl](auto ic) { vread(Vl, decltype(ic)::value, vf.f[decltype(ic)::value]); }; };
    auto none = [](auto) {};

    // end of R3: tile t + 1's DMA (issued in R2 and R4 of tile t - 1) has landed;
    // younger than it: R2(t)'s block A M ops (of tile tn) and 4 DMA pieces.
    // vmcnt(8) or vmcnt(20), no lgkm / exp wait.
    auto mid_barrier = [&](auto shc, int tn) {
        if (kr(shc, tn, 0))
            __builtin_amdgcn_s_waitcnt(0x4F74);  // vmcnt(20) = 16 + 4
        else
            __builtin_amdgcn_s_waitcnt(0x0F78);  // vmcnt(8) = 4 + 4
        __builtin_amdgcn_s_barrier();
    };

    using MSX = std::integral_constant<int, 0>;  // the M register sets
    using MSY = std::integral_constant<int, 1>;
    auto mregs = [](auto msc, auto uc) { return std::integral_constant<int, W64_VM + 32 * decltype(msc)::value + 16 * decltype(uc)::value>{}; };
    float eX, eY;
    f32x16 S[2];
    SmA sa[2];
    SmB sb;
    f16x8 ph[2][2], pl[2][2];

    // The vector-memory issue of a tile, one M quad (1 or 4 ops) or DMA piece
    // per 3 MFMAs: in R2 block A's 4 M quads of tile tn and DMA pieces 0-3 of
    // tile td, in R4 block B's quads and pieces 4-7 (slices 1, 4, 7, 10: M; 13,
    // 16, 19, 22: DMA).  A block's M wait finds 8 + (the other block's M ops)
    // younger ops (its half's 4 pieces, the other half's M and 4 pieces), the
    // barrier 4 + (R2's M ops).
    auto issue_half = [&](auto shc, auto kc, auto hc, int tn, int td, auto msn) {
        constexpr int k = decltype(kc)::value, half = decltype(hc)::value;
#ifndef W64_EXP_NO_M
        if constexpr (k % 3 == 1 && k <= 10) load_mq(shc, msn, hc, std::integral_constant<int, k / 3>{}, tn);
#endif
#ifndef W64_EXP_NO_DMA
        if constexpr (k % 3 == 1 && k >= 13) stage_piece(td, 4 * half + (k - 13) / 3);
#endif
    };
    using H0 = std::integral_constant<int, 0>;
    using H1 = std::integral_constant<int, 1>;

    // ---- prologue: tiles st0, st0 + 1 in flight, the first tile's M ----
#pragma unroll
    for (int i = 0; i < DMA_PW; ++i) stage_piece(st0, i);
#pragma unroll
    for (int i = 0; i < DMA_PW; ++i) stage_piece(st0 + 1, i);
    static_for<2>([&](auto uc) { static_for<4>([&](auto gc) { load_mq(SH0{}, MSX{}, uc, gc, st0); }); });
    {
        float *evw = reinterpret_cast<float *>(smem + W64_RING);
        for (int i = threadIdx.x; i < Npad / H3_TILE; i += W64_NW * 64) evw[i] = vexp_b[i];
    }
    w64_vmwait<0>();  // (the Q and M loads are asm: hipcc does not count them)
    __builtin_amdgcn_s_waitcnt(0x0070);               // vmcnt(0) lgkmcnt(0)
    __builtin_amdgcn_s_barrier();
    eX = load_ev(st0);

    // ---- tile st0 (the first: m_run = -inf, O = 0) ----
    {
        const int t = st0, key0 = t * H3_TILE;
        const char *L = slot_of(t);
        kread(L, 0, kf.f[0]);
        kread(L, 1, kf.f[1]);
        // R1: QK_A
        qk_region(std::integral_constant<int, 0>{}, L, S[0], none, none);
        // R2: softmax_A part 1 (first tile) + the issue of tile t + 1's M and tile t + 2's DMA
        static_for<24>([&](auto kc) { issue_half(SH0{}, kc, H0{}, min(t + 1, st1 - 1), t + 2, MSY{}); });
        eY = load_ev(min(t + 1, st1 - 1));
        kread(L, 0, kf.f[0]);  // (QK_A's last k-steps held kf[0], kf[1]: R3's first two only now)
        kread(L, 1, kf.f[1]);
        sm1_first(0, S[0], mregs(MSX{}, H0{}), eX, key0, sa[0]);
        // R3: QK_B + softmax_A part 2
        qk_region(std::integral_constant<int, 1>{}, L, S[1], next_v(L + H3_KTB),
                  [&](auto kc) { sm2_slice(kc, 0, sa[0], eX, sb, ph[0], pl[0]); });
        mid_barrier(SH0{}, min(t + 1, st1 - 1));
        // R4: PV_A + softmax_B part 1 (first tile)
        pv_region(std::integral_constant<int, 0>{}, L + H3_KTB, ph[0], pl[0], next_k(slot_of(t + 1)),
                  [&](auto kc) { issue_half(SH0{}, kc, H1{}, min(t + 1, st1 - 1), t + 2, MSY{}); });
        sm1_first(1, S[1], mregs(MSX{}, H1{}), eX, key0, sa[1]);
    }
    // ---- steady state: tile t (its M in mc, ev ec; the next tile's into mn, en) ----
    auto tile = [&](int t, auto msc, float &ec, float &ep, auto msn, float &en, auto shc) {
        const int key0 = t * H3_TILE;
        const int si = W64_ST_PER_TILE * min(t - st0, 39);
        (void)si;
        W64_ST(si);
        const char *L = slot_of(t), *Lp = slot_of(t - 1);
        // R1: QK_A(t) + softmax_B(t - 1) part 2 (ep: tile t - 1's V exponent)
        qk_region(std::integral_constant<int, 0>{}, L, S[0], next_v(Lp + H3_KTB),
                  [&](auto kc) { sm2_slice(kc, 1, sa[1], ep, sb, ph[1], pl[1]); });
        W64_ST(si + 1);
        // R2: PV_B(t - 1) + softmax_A(t) part 1 + tile t + 1's M, tile t + 2's DMA
        pv_region(std::integral_constant<int, 1>{}, Lp + H3_KTB, ph[1], pl[1], next_k(L), [&](auto kc) {
            // block A's M of tile t (issued in R2 of tile t - 1; younger: 8 + block B's)
            if constexpr (decltype(kc)::value == 0) w64_mwait_after(kr(shc, t, 1));
            if constexpr (decltype(kc)::value == 2) en = load_ev(min(t + 1, st1 - 1));
            sm1_slice(kc, 0, S[0], mregs(msc, H0{}), ec, key0, sa[0]);
            issue_half(shc, kc, H0{}, min(t + 1, st1 - 1), t + 2, msn);
        });
        rebase(std::integral_constant<int, 0>{}, sa[0]);
        W64_ST(si + 2);
        // R3: QK_B(t) + softmax_A(t) part 2
        qk_region(std::integral_constant<int, 1>{}, L, S[1], next_v(L + H3_KTB),
                  [&](auto kc) { sm2_slice(kc, 0, sa[0], ec, sb, ph[0], pl[0]); });
        W64_ST(si + 3);
        mid_barrier(shc, min(t + 1, st1 - 1));
        W64_ST(si + 4);
        // R4: PV_A(t) + softmax_B(t) part 1
        pv_region(std::integral_constant<int, 0>{}, L + H3_KTB, ph[0], pl[0], next_k(slot_of(t + 1)), [&](auto kc) {
            // block B's M of tile t (issued in R4 of tile t - 1; younger: 8 + block A's
            // of tile t + 1, issued in R2)
            if constexpr (decltype(kc)::value == 0) w64_mwait_after(kr(shc, min(t + 1, st1 - 1), 0));
            sm1_slice(kc, 1, S[1], mregs(msc, H1{}), ec, key0, sa[1]);
            issue_half(shc, kc, H1{}, min(t + 1, st1 - 1), t + 2, msn);
        });
        rebase(std::integral_constant<int, 1>{}, sa[1]);
        W64_ST(si + 5);
    };
#ifdef W64_EXP_NO_LDSREAD
    lds_once = false;
#endif
    int t = st0 + 1;
    for (; t + 1 < st1; t += 2) {
        // the step's shape (see kr): 1 if its next tile's M are by columns for
        // both blocks (then so is the current tile's block B), 2 if the current
        // tile is past both blocks' query tiles
        auto shape = [&](int tt) { return min(tt + 1, st1 - 1) <= qt0 ? 1 : (tt >= qt0 + 2 ? 2 : 0); };
        const int s0 = shape(t), s1 = shape(t + 1);
        auto two = [&](auto shc) {
            tile(t, MSY{}, eY, eX, MSX{}, eX, shc);
            tile(t + 1, MSX{}, eX, eY, MSY{}, eY, shc);
        };
        if (s0 == 1 && s1 == 1)
            two(SH1{});
        else if (s0 == 2 && s1 == 2)
            two(SH2{});
        else
            two(SH0{});
    }
    // (ep of the pair's first tile above: eX before it is overwritten in R2 --
    // part 2 of block B reads it in R1, ahead of the loads)
    if (t < st1) {
        tile(t, MSY{}, eY, eX, MSX{}, eX, SH0{});
        ++t;
    }
    // ---- epilogue: softmax_B(last) part 2, PV_B(last) ----
    // The last tile loaded a "next" M that nothing reads: landed before the
    // core returns (the registers are the next segment's).
    w64_vmwait<0>();
    {
        const float el = ((t - st0) & 1) ? eX : eY;  // the last tile's exponent
        const char *Lp = slot_of(t - 1);
        static_for<24>([&](auto kc) { sm2_slice(kc, 1, sa[1], el, sb, ph[1], pl[1]); });
        vread(Lp + H3_KTB, 0, vf.f[0]);
        vread(Lp + H3_KTB, 1, vf.f[1]);
        pv_region(std::integral_constant<int, 1>{}, Lp + H3_KTB, ph[1], pl[1], none, none);
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) l_run[u] = halves_sum(l_run[u]);
    // every wave's LDS reads and this wave's (past-the-end) DMA done before the
    // caller reuses the LDS; the last P V MFMA's result -> v_accvgpr_read (w64_read_o)
    __builtin_amdgcn_s_waitcnt(0x0070);  // vmcnt(0) lgkmcnt(0)
    __builtin_amdgcn_s_barrier();
    asm volatile("s_nop 15");
#ifdef W64_STAMPS
    {
        const unsigned long long st_c1 = __builtin_amdgcn_s_memtime(), st_r1 = __builtin_amdgcn_s_memrealtime();
        if (lane == 0) {
            st_lds[W64_ST_PER_WAVE - 4] = st_c0;
            st_lds[W64_ST_PER_WAVE - 3] = st_c1;
            st_lds[W64_ST_PER_WAVE - 2] = st_r0;
            st_lds[W64_ST_PER_WAVE - 1] = st_r1;
        }
        const int wg = blockIdx.x;
        if (wg < W64_ST_WGS)
            for (int i = lane; i < W64_ST_PER_WAVE; i += 64)
                g_w64_stamps[(wg * W64_NW + wave) * W64_ST_PER_WAVE + i] = st_lds[i];
    }
#endif
}

// block u's O^T tiles out of the accumulator file
template <int U> PDSC_DEV void w64_read_o(f32x16 (&O)[4]) {
    static_for<64>([&](auto ic) {
        constexpr int i = decltype(ic)::value;
        O[i >> 4][i & 15] = w64_read_a<W64_AO + 64 * U + i>();
    });
}

// This workgroup's partial (split blk.split of query block blk.qb): O^T rows in
// the fragment-block tiling of attention_h3_kernel, m (natural-log units) and l.
PDSC_DEV void w64_store_partial(const AttnGridH3 &g, const AttnBlock &blk, float *__restrict__ opart,
                                float *__restrict__ ml, int wave, int lane, const float (&m_run)[2],
                                const float (&l_run)[2]) {
    const int Npad = g.Npad, h = lane >> 5;
    const size_t obase = (size_t)(blk.b * g.nsplit + blk.split) * Npad;
    static_for<2>([&](auto uc) {
        constexpr int u = decltype(uc)::value;
        const int q0 = blk.qb * W64_QPB + wave * W64_QW + 32 * u, qq = q0 + (lane & 31);
        f32x16 O[4];
        w64_read_o<u>(O);
        if (q0 < Npad) {
            float *Ob = opart + obase * CH + (size_t)(q0 >> 5) * (H3_TILE * CH) + 4 * lane;
#pragma unroll
            for (int t = 0; t < 4; ++t)
#pragma unroll
                for (int q = 0; q < 4; ++q)
                    *reinterpret_cast<f32x4 *>(Ob + (4 * t + q) * 256) =
                        f32x4{O[t][4 * q], O[t][4 * q + 1], O[t][4 * q + 2], O[t][4 * q + 3]};
            if (h == 0) {
                ml[(obase + qq) * 2] = (m_run[u] - (float)H3_PSHIFT) * 0.6931471805599453f;
                ml[(obase + qq) * 2 + 1] = l_run[u];
            }
        }
    });
}

// Split-K attention with 64-query waves: partials as attention_h3_kernel.
template <bool XCD>
__global__ __launch_bounds__(W64_NW * 64, 1) __attribute__((amdgpu_num_vgpr(W64_VM))) void attention_w64_kernel(
    const _Float16 *__restrict__ Qs, const _Float16 *__restrict__ Ks, const _Float16 *__restrict__ Vs,
    const float *__restrict__ vexp, const float *__restrict__ M, AttnGridH3 g, float *__restrict__ opart,
    float *__restrict__ ml) {
    extern __shared__ __attribute__((aligned(16))) char w64smem[];
    const AttnBlock blk = attention_h3_block(g, XCD);
    if (blk.qb * W64_QPB >= g.n(blk.b)) return;  // past a ragged pair's end (workgroup-uniform)
    const int tid = threadIdx.x, wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
    float m_run[2], l_run[2];
    attention_w64_core(Qs, Ks, Vs, vexp, M, g, blk, w64smem, wave, lane, m_run, l_run);
    w64_store_partial(g, blk, opart, ml, wave, lane, m_run, l_run);
}

// ---- stream-K form (uniform batches) ------------------------------------------
// The split grid runs ceil(B nqb nsplit / slots) rounds of whole splits: 8 x 5000
// is 480 workgroups of 53 key tiles on 256 CUs, a second round 7/8 full.  Here
// one round of `nwg` workgroups (one per CU) shares the T = B nqb nst (query
// block, key tile) pairs evenly: logical workgroup w owns the block-major tiles
// [w T / nwg, (w + 1) T / nwg), XCD-major (logical ids w .. of one XCD hold
// consecutive tiles, so a pair's blocks stay in one L2).  Each maximal run of
// those tiles inside one query block is a segment, stored as split
// s = w - (owner of the block's first tile); the owner of the block's last tile
// also writes the slots past its own as an empty split leaves them (O = 0,
// m = -inf, l = 0), so the combine reads nsplit slots as before.
__host__ __device__ inline int w64_sk_owner(long x, long T, int nwg) { return (int)(((x + 1) * nwg - 1) / T); }
inline int w64_sk_nsplit(int B, int nqb, int nst, int nwg) {
    const long T = (long)B * nqb * nst;
    int ns = 1;
    for (long k = 0; k < (long)B * nqb; ++k)
        ns = std::max(ns, w64_sk_owner(k * nst + nst - 1, T, nwg) - w64_sk_owner(k * nst, T, nwg) + 1);
    return ns;
}

// split s of query block (b, qb) as an empty split leaves it
PDSC_DEV void w64_zero_partial(const AttnGridH3 &g, int b, int qb, int s, float *__restrict__ opart,
                               float *__restrict__ ml, int tid) {
    const int Npad = g.Npad;
    const size_t obase = (size_t)(b * g.nsplit + s) * Npad;
    const int r0 = qb * W64_QPB, r1 = min(Npad, r0 + W64_QPB);  // rows (multiples of 32)
    f32x4 *Ob = reinterpret_cast<f32x4 *>(opart + (obase + r0) * CH);
    for (int i = tid; i < (r1 - r0) * CH / 4; i += W64_NW * 64) Ob[i] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
    for (int r = r0 + tid; r < r1; r += W64_NW * 64) {
        ml[(obase + r) * 2] = -INFINITY;
        ml[(obase + r) * 2 + 1] = 0.0f;
    }
}

template <bool XCD>
__global__ __launch_bounds__(W64_NW * 64, 1) __attribute__((amdgpu_num_vgpr(W64_VM))) void attention_w64_sk_kernel(
    const _Float16 *__restrict__ Qs, const _Float16 *__restrict__ Ks, const _Float16 *__restrict__ Vs,
    const float *__restrict__ vexp, const float *__restrict__ M, AttnGridH3 g, int nwg, float *__restrict__ opart,
    float *__restrict__ ml) {
    extern __shared__ __attribute__((aligned(16))) char w64smem[];
    int w = blockIdx.x;
    if (XCD && (nwg & 7) == 0) w = (w & 7) * (nwg >> 3) + (w >> 3);
    const int nst = (g.N + H3_TILE - 1) / H3_TILE;
    const long T = (long)g.B * g.nqb * nst;
    const long hi = (long)(w + 1) * T / nwg;
    const int tid = threadIdx.x, wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
    for (long x = (long)w * T / nwg; x < hi;) {
        const int k = (int)(x / nst);
        const long k0 = (long)k * nst, x1 = min(hi, k0 + nst);
        AttnBlock blk{k / g.nqb, k % g.nqb, w - w64_sk_owner(k0, T, nwg)};
        blk.st0 = (int)(x - k0);
        blk.st1 = (int)(x1 - k0);
        __builtin_amdgcn_s_waitcnt(0x0070);  // the previous segment's stores: the core starts with none in flight
        float m_run[2], l_run[2];
        attention_w64_core(Qs, Ks, Vs, vexp, M, g, blk, w64smem, wave, lane, m_run, l_run);
        w64_store_partial(g, blk, opart, ml, wave, lane, m_run, l_run);
        if (x1 == k0 + nst)
            for (int s = blk.split + 1; s < g.nsplit; ++s) w64_zero_partial(g, blk.b, blk.qb, s, opart, ml, tid);
        x = x1;
    }
}

}  // namespace pdsc
