// tools/att_w64_bench.hip -- attention_w64_kernel (64-query waves, one 4-wave
// workgroup per CU) against attention_h3_kernel on the same inputs: timing and
// a bitwise comparison of the partials (diagnostics; bench.py has the numbers
// that count).
// Build: hipcc -O3 --offload-arch=gfx950 -std=c++17 -ffp-contract=off -I pointdsc_amd/csrc \
//        tools/att_w64_bench.hip -o tools/att_w64_bench
// Run:   att_w64_bench [B=128] [N=1000] [reps=20] [nsplit_w64=auto]
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <vector>

#include "attention_w64.hpp"

using namespace pdsc;

#define CK(x)                                                                \
    do {                                                                     \
        hipError_t e_ = (x);                                                 \
        if (e_ != hipSuccess) {                                              \
            printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); \
            exit(1);                                                         \
        }                                                                    \
    } while (0)

__global__ void fill_h(_Float16 *p, size_t n, unsigned seed, float scale) {
    const size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (i >= n) return;
    unsigned x = (unsigned)i * 2654435761u ^ seed;
    x ^= x >> 13;
    x *= 0x5bd1e995u;
    x ^= x >> 15;
    p[i] = (_Float16)(((x & 0xffff) / 65536.0f - 0.5f) * scale);
}
__global__ void fill_f(float *p, size_t n, unsigned seed) {
    const size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (i >= n) return;
    unsigned x = (unsigned)i * 2654435761u ^ seed;
    x ^= x >> 13;
    x *= 0x5bd1e995u;
    x ^= x >> 15;
    p[i] = (x & 0xffff) / 65536.0f;
}

int main(int argc, char **argv) {
    const int B = argc > 1 ? atoi(argv[1]) : 128, N = argc > 2 ? atoi(argv[2]) : 1000;
    const int reps = argc > 3 ? atoi(argv[3]) : 20;
    AttnGridH3 gh = attention_h3_grid<4>(B, N, 512);
    AttnGridH3 gw = attention_w64_grid(B, N, 256);
    if (argc > 4) {  // force the w64 split count
        const int nst = (N + 31) / 32, ns = atoi(argv[4]);
        gw.sps = (nst + ns - 1) / ns;
        gw.nsplit = (nst + gw.sps - 1) / gw.sps;
    }
    const size_t rows = (size_t)B * gh.Npad * CH * 2, mper = mpack_floats(N);
    const int nsm = gh.nsplit > gw.nsplit ? gh.nsplit : gw.nsplit;
    _Float16 *Q, *K, *V;
    float *M, *vexp, *op, *ml, *op2, *ml2;
    CK(hipMalloc(&Q, rows * 2));
    CK(hipMalloc(&K, rows * 2));
    CK(hipMalloc(&V, rows * 2));
    CK(hipMalloc(&M, (size_t)B * mper * 4));
    CK(hipMalloc(&vexp, (size_t)B * (gh.Npad / 32) * 4));
    CK(hipMalloc(&op, (size_t)B * nsm * gh.Npad * CH * 4));
    CK(hipMalloc(&ml, (size_t)B * nsm * gh.Npad * 2 * 4));
    CK(hipMalloc(&op2, (size_t)B * nsm * gh.Npad * CH * 4));
    CK(hipMalloc(&ml2, (size_t)B * nsm * gh.Npad * 2 * 4));
    hipLaunchKernelGGL(fill_h, dim3((rows + 255) / 256), dim3(256), 0, 0, Q, rows, 1u, 0.2f);
    hipLaunchKernelGGL(fill_h, dim3((rows + 255) / 256), dim3(256), 0, 0, K, rows, 2u, 0.2f);
    hipLaunchKernelGGL(fill_h, dim3((rows + 255) / 256), dim3(256), 0, 0, V, rows, 3u, 1.0f);
    hipLaunchKernelGGL(fill_f, dim3((B * mper + 255) / 256), dim3(256), 0, 0, M, (size_t)B * mper, 4u);
    if (getenv("BENCH_MONES")) {  // M = 1 (the M layouts out of the comparison)
        std::vector<float> ones((size_t)B * mper, 1.0f);
        CK(hipMemcpy(M, ones.data(), ones.size() * 4, hipMemcpyHostToDevice));
    }
    CK(hipMemset(vexp, 0, (size_t)B * (gh.Npad / 32) * 4));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    auto lh = [&](int ns_force) {
        AttnGridH3 g = gh;
        if (ns_force) {
            const int nst = (N + 31) / 32;
            g.sps = (nst + ns_force - 1) / ns_force;
            g.nsplit = (nst + g.sps - 1) / g.sps;
        }
        hipLaunchKernelGGL((attention_h3_kernel<4, true, true>), dim3(g.B * g.nqb * g.nsplit), dim3(256),
                           attention_h3_lds_bytes<4>(), 0, Q, K, V, vexp, M, g, op, ml);
    };
    auto lw = [&] {
        hipLaunchKernelGGL((attention_w64_kernel<true>), dim3(gw.B * gw.nqb * gw.nsplit), dim3(256), W64_LDS + W64_ST_LDS, 0, Q, K,
                           V, vexp, M, gw, op2, ml2);
    };
    auto timeit = [&](auto f) {
        for (int i = 0; i < 3; ++i) f();
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(a));
        for (int i = 0; i < reps; ++i) f();
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        return ms * 1e3 / reps;
    };
    const double flop = 4.0 * B * (double)N * N * CH;
    const double th = timeit([&] { lh(0); });
    printf("h3  B=%d N=%d nsplit=%d grid=%d: %.2f us/launch, %.1f TFLOP/s (%.3f of 833.3)\n", B, N, gh.nsplit,
           gh.B * gh.nqb * gh.nsplit, th, flop / th * 1e-6, flop / th * 1e-6 / 833.3);
    const double tw = timeit(lw);
    printf("w64 B=%d N=%d nsplit=%d grid=%d: %.2f us/launch, %.1f TFLOP/s (%.3f of 833.3)\n", B, N, gw.nsplit,
           gw.B * gw.nqb * gw.nsplit, tw, flop / tw * 1e-6, flop / tw * 1e-6 / 833.3);
#ifdef W64_STAMPS
    {  // per-region cycles of the steady-state tiles (median over the stamped waves and tiles)
        std::vector<unsigned long long> st((size_t)W64_ST_WGS * W64_NW * W64_ST_PER_WAVE);
        CK(hipMemcpyFromSymbol(st.data(), HIP_SYMBOL(g_w64_stamps), st.size() * 8, 0, hipMemcpyDeviceToHost));
        const int nt = (N + 31) / 32 / gw.nsplit;
        const char *nm[6] = {"R1 QK_A+sm2_B", "R2 PV_B+sm1_A+issue", "R3 QK_B+sm2_A", "barrier", "R4 PV_A+sm1_B", "tile"};
        for (int r = 0; r < 6; ++r) {
            std::vector<long long> d;
            for (int w = 0; w < W64_ST_WGS * W64_NW; ++w)
                for (int t = 2; t < nt - 1 && t < 39; ++t) {
                    const unsigned long long *p = &st[(size_t)w * W64_ST_PER_WAVE + 6 * t];
                    const long long v = r < 5 ? (long long)(p[r + 1] - p[r]) : (long long)(p[6] - p[0]);
                    if (p[0] && p[6]) d.push_back(v);
                }
            std::sort(d.begin(), d.end());
            if (!d.empty())
                printf("  %-22s median %lld  p10 %lld  p90 %lld cycles\n", nm[r], d[d.size() / 2], d[d.size() / 10],
                       d[d.size() * 9 / 10]);
        }
        std::vector<double> clk, span, tiles;
        for (int w = 0; w < W64_ST_WGS * W64_NW; ++w) {
            const unsigned long long *p = &st[(size_t)w * W64_ST_PER_WAVE];
            const unsigned long long c0 = p[W64_ST_PER_WAVE - 4], c1 = p[W64_ST_PER_WAVE - 3], r0 = p[W64_ST_PER_WAVE - 2],
                                     r1 = p[W64_ST_PER_WAVE - 1];
            if (r1 > r0) {
                clk.push_back((double)(c1 - c0) / (double)(r1 - r0) * 0.1);  // GHz (realtime: 100 MHz)
                span.push_back((double)(r1 - r0) * 0.01);                      // us
                if (p[6] && p[6 * (nt - 1)]) tiles.push_back((double)(p[6 * (nt - 1)] - p[6]) / (double)(c1 - c0));
            }
        }
        std::sort(clk.begin(), clk.end());
        std::sort(span.begin(), span.end());
        std::sort(tiles.begin(), tiles.end());
        if (!clk.empty())
            printf("  core: clock %.2f GHz, span %.1f us (median), steady tiles %.2f of the span\n", clk[clk.size() / 2],
                   span[span.size() / 2], tiles.empty() ? 0.0 : tiles[tiles.size() / 2]);
    }
#endif
    // bitwise comparison at the same split count
    lh(gw.nsplit);
    lw();
    CK(hipDeviceSynchronize());
    const size_t no = (size_t)B * gw.nsplit * gh.Npad * CH, nm = (size_t)B * gw.nsplit * gh.Npad * 2;
    std::vector<float> h1(no), h2(no), m1(nm), m2(nm);
    CK(hipMemcpy(h1.data(), op, no * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(h2.data(), op2, no * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(m1.data(), ml, nm * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(m2.data(), ml2, nm * 4, hipMemcpyDeviceToHost));
    size_t dO = 0, dM = 0, first = (size_t)-1;
    // rows < N only (padding rows compute on clamped operands and differ by design)
    for (size_t i = 0; i < no; ++i) {
        const size_t o = i % ((size_t)gh.Npad * CH);
        const int row = (int)(o / (32 * CH)) * 32 + (int)((o % (32 * CH)) / 4 % 64) % 32;
        if (row < N && memcmp(&h1[i], &h2[i], 4)) {
            ++dO;
            if (first == (size_t)-1) first = i;
        }
    }
    size_t dm_m = 0, dm_l = 0, firstm = (size_t)-1;
    for (size_t i = 0; i < nm; ++i)
        if ((int)(i / 2 % gh.Npad) < N && memcmp(&m1[i], &m2[i], 4)) {
            ++dM;
            (i & 1 ? dm_l : dm_m)++;
            if (firstm == (size_t)-1) firstm = i;
        }
    printf("ml: m differ %zu, l differ %zu", dm_m, dm_l);
    if (firstm != (size_t)-1) printf("; first at row %zu: m %g vs %g, l %g vs %g", firstm / 2, m1[firstm & ~1], m2[firstm & ~1], m1[firstm | 1], m2[firstm | 1]);
    printf("\n");
    printf("bitwise vs h3 at nsplit=%d: opart differ %zu of %zu, ml differ %zu of %zu%s\n", gw.nsplit, dO, no, dM, nm,
           dO + dM ? "  MISMATCH" : "  identical");
    if (first != (size_t)-1) printf("  first diff at %zu: %g vs %g\n", first, h1[first], h2[first]);
    if (getenv("BENCH_MAP")) {  // diffs per (32-row tile, channel tile t) of pair 0, split 0
        for (int rt = 0; rt < (N + 31) / 32; ++rt) {
            printf("  rows %4d:", rt * 32);
            for (int t = 0; t < 4; ++t) {
                int c = 0;
                for (int q = 0; q < 4; ++q)
                    for (int e = 0; e < 256; ++e) {
                        const size_t i = (size_t)rt * 4096 + (4 * t + q) * 256 + e;
                        c += memcmp(&h1[i], &h2[i], 4) != 0;
                    }
                printf(" t%d:%4d", t, c);
            }
            printf("\n");
        }
    }
    return dO + dM ? 2 : 0;
}
