// tools/attn_bench.hip -- A/B timing of attention_kernel_t variants in one
// process (interleaved rounds, hipEvents), outputs checked against variant 0.
// Build: hipcc -O3 --offload-arch=gfx950 -std=c++17 -ffp-contract=off -I pointdsc_amd/csrc \
//        tools/attn_bench.hip -o tools/attn_bench
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <algorithm>
#include <vector>
#include "attention.hpp"
#include "attention_h3.hpp"
#include "compat.hip"

using namespace pdsc;

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

__global__ void combine_k(const float *op, const float *ml, int N, int Npad, int ns, float *out) {
    int b = blockIdx.y, row = blockIdx.x, d = threadIdx.x;
    if (row >= N) return;
    float ms = -INFINITY;
    for (int s = 0; s < ns; ++s) ms = fmaxf(ms, ml[((size_t)(b * ns + s) * Npad + row) * 2]);
    float L = 0, a = 0;
    for (int s = 0; s < ns; ++s) {
        size_t base = (size_t)(b * ns + s) * Npad + row;
        float w = expf(ml[base * 2] - ms);
        L += w * ml[base * 2 + 1];
        a += w * op[base * CH + d];
    }
    out[((size_t)b * N + row) * CH + d] = a / L;
}

struct Variant {
    const char *name;
    void (*launch)(const float *, const float *, const float *, const float *, int, int, float *, float *, float *, hipStream_t);
};

template <int NW, int KTS, bool FE, bool XCD, int BUF = 3, bool GL = false>
void run_variant(const float *q, const float *k, const float *v, const float *M, int B, int N, float *op,
                 float *ml, float *out, hipStream_t s) {
    AttnGrid g = attention_grid<NW, KTS>(B, N, 1024);
    const int G = g.B * g.nqb * g.nsplit;
    const size_t lds = attention_lds_bytes<NW, KTS, GL>();
    auto kern = attention_kernel_t<NW, KTS, FE, XCD, BUF, GL>;
    hipLaunchKernelGGL(kern, dim3(G), dim3(NW * 64), lds, s, q, k, v, M, g, op, ml);
    CK(hipGetLastError());
    if (out) hipLaunchKernelGGL(combine_k, dim3(N, B), dim3(CH), 0, s, op, ml, N, g.Npad, g.nsplit, out);
}

static _Float16 *g_qs = nullptr;  // split layouts (allocated in main)
static float *g_mp = nullptr;     // symmetric-packed M (allocated in main)
template <int NW, bool XCD, bool PACKED = false>
void run_h3(const float *q, const float *k, const float *v, const float *M, int B, int N, float *op,
            float *ml, float *out, hipStream_t s) {
    AttnGridH3 g = attention_h3_grid<NW>(B, N, 1024);
    const size_t per = (size_t)B * g.Npad * 2 * CH;
    static bool split_done = false;  // q/k/v never change in this harness: split once
    if (!split_done) {
        const size_t n = (size_t)B * g.Npad * CH;
        hipLaunchKernelGGL(split_qkv_kernel, dim3((n + 255) / 256), dim3(256), 0, s, q, k, v, B, N, g.Npad, g.Npad,
                           g_qs, g_qs + per, g_qs + 2 * per);
        split_done = true;
    }
    const int G = g.B * g.nqb * g.nsplit;
    hipLaunchKernelGGL((attention_h3_kernel<NW, XCD, PACKED>), dim3(G), dim3(NW * 64), attention_h3_lds_bytes<NW>(), s,
                       g_qs, g_qs + per, g_qs + 2 * per, PACKED ? g_mp : M, g, op, ml);
    CK(hipGetLastError());
    if (out) hipLaunchKernelGGL(combine_k, dim3(N, B), dim3(CH), 0, s, op, ml, N, g.Npad, g.nsplit, out);
}

int main(int argc, char **argv) {
    int B = argc > 1 ? atoi(argv[1]) : 64, N = argc > 2 ? atoi(argv[2]) : 1000;
    int iters = argc > 3 ? atoi(argv[3]) : 20;
    const int Npad = round_up(N, QB);
    std::vector<Variant> V = {
        {"nw4 kt32 exp2 xcd1     ", run_variant<4, 32, true, true>},
        {"h3 nw4 xcd1            ", run_h3<4, true>},
        {"h3 nw4 xcd1 packedM    ", run_h3<4, true, true>},
        {"h3 nw4 xcd0 packedM    ", run_h3<4, false, true>},
    };
    size_t nq = (size_t)B * Npad * CH;
    std::vector<float> hq(nq * 3, 0.f), hp((size_t)B * N * 6);
    srand(1);
    auto rnd = [] { return (float)rand() / RAND_MAX; };
    for (int b = 0; b < B; ++b)
        for (int i = 0; i < N; ++i)
            for (int c = 0; c < CH; ++c)
                for (int t = 0; t < 3; ++t) hq[t * nq + ((size_t)b * Npad + i) * CH + c] = 2 * rnd() - 1;
    for (size_t i = 0; i < hp.size(); ++i) hp[i] = 3 * rnd();
    for (int b = 0; b < B; ++b)  // 30 % "inliers": tgt = src + noise
        for (int i = 0; i < N * 3 / 10; ++i)
            for (int c = 0; c < 3; ++c) hp[(size_t)B * N * 3 + ((size_t)b * N + i) * 3 + c] = hp[((size_t)b * N + i) * 3 + c] + 0.01f * rnd();
    float *dq, *dp, *dM, *dop, *dml, *dout, *dref, *dsd;
    AttnGrid gmax = attention_grid<4, 32>(B, N, 1024);
    size_t opn = (size_t)B * 64 * Npad * CH;  // generous: nsplit <= 64
    CK(hipMalloc(&dq, nq * 3 * 4)); CK(hipMalloc(&dp, hp.size() * 4)); CK(hipMalloc(&dM, (size_t)B * N * N * 4));
    CK(hipMalloc(&dop, opn * 4)); CK(hipMalloc(&dml, (size_t)B * 64 * Npad * 2 * 4));
    CK(hipMalloc(&g_qs, (size_t)3 * B * Npad * 2 * CH * 2));
    CK(hipMalloc(&dout, (size_t)B * N * CH * 4)); CK(hipMalloc(&dref, (size_t)B * N * CH * 4)); CK(hipMalloc(&dsd, 4));
    float sd = 0.1f;
    CK(hipMemcpy(dq, hq.data(), nq * 3 * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(dp, hp.data(), hp.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(dsd, &sd, 4, hipMemcpyHostToDevice));
    CK(launch_compat(dp, dp + (size_t)B * N * 3, B, N, dsd, dM, 0));
    CK(hipMalloc(&g_mp, (size_t)B * mpack_floats(N) * 4));
    CK(launch_compat_packed(dp, dp + (size_t)B * N * 3, B, N, dsd, g_mp, 0));
    const float *Q = dq, *K = dq + nq, *Vv = dq + 2 * nq;
    // correctness vs variant 0
    V[0].launch(Q, K, Vv, dM, B, N, dop, dml, dref, 0);
    std::vector<float> ref((size_t)B * N * CH), out(ref.size());
    CK(hipMemcpy(ref.data(), dref, ref.size() * 4, hipMemcpyDeviceToHost));
    for (size_t vi = 1; vi < V.size(); ++vi) {
        V[vi].launch(Q, K, Vv, dM, B, N, dop, dml, dout, 0);
        CK(hipMemcpy(out.data(), dout, out.size() * 4, hipMemcpyDeviceToHost));
        double md = 0, mr = 0;
        for (size_t i = 0; i < out.size(); ++i) { md = fmax(md, fabs(out[i] - ref[i])); mr = fmax(mr, fabs(ref[i])); }
        printf("check %-22s max|d| %.3g (max|ref| %.3g)\n", V[vi].name, md, mr);
    }
    // fp64 CPU reference for a few rows of pair 0 (M recomputed on host)
    {
        std::vector<float> hM((size_t)N * N);
        CK(hipMemcpy(hM.data(), dM, hM.size() * 4, hipMemcpyDeviceToHost));
        for (size_t vi = 0; vi < V.size(); ++vi) {
            V[vi].launch(Q, K, Vv, dM, B, N, dop, dml, dout, 0);
            CK(hipDeviceSynchronize());
            CK(hipMemcpy(out.data(), dout, out.size() * 4, hipMemcpyDeviceToHost));
            double md = 0;
            for (int i = 0; i < N; i += N / 7) {
                std::vector<double> lg(N);
                double mx = -1e300;
                for (int j = 0; j < N; ++j) {
                    double d = 0;
                    for (int c = 0; c < CH; ++c) d += (double)hq[(size_t)i * CH + c] * hq[nq + (size_t)j * CH + c];
                    lg[j] = hM[(size_t)i * N + j] * d / sqrt(128.0);
                    mx = fmax(mx, lg[j]);
                }
                double L = 0;
                for (int j = 0; j < N; ++j) L += exp(lg[j] - mx);
                for (int c = 0; c < CH; ++c) {
                    double a = 0;
                    for (int j = 0; j < N; ++j) a += exp(lg[j] - mx) * hq[2 * nq + (size_t)j * CH + c];
                    md = fmax(md, fabs(a / L - out[(size_t)i * CH + c]));
                }
            }
            if (vi == 0) {
                AttnGrid g0 = attention_grid<4, 32>(B, N, 1024);
                std::vector<float> hml((size_t)B * g0.nsplit * Npad * 2), hop(CH);
                CK(hipMemcpy(hml.data(), dml, hml.size() * 4, hipMemcpyDeviceToHost));
                CK(hipMemcpy(hop.data(), dop, CH * 4, hipMemcpyDeviceToHost));
                printf("nsplit %d sps %d nqb %d Npad %d\n", g0.nsplit, g0.sps, g0.nqb, g0.Npad);
                for (int s2 = 0; s2 < g0.nsplit; ++s2)
                    printf("  split %d row0 m=%g l=%g\n", s2, hml[((size_t)s2 * Npad) * 2], hml[((size_t)s2 * Npad) * 2 + 1]);
                printf("  O split0 row0 %g %g %g  M00..02 %g %g %g  Q00 %g\n", hop[0], hop[1], hop[2], hM[0], hM[1], hM[2], hq[0]);
                double mx = -1e300, L = 0; std::vector<double> lg(N);
                for (int j = 0; j < N; ++j) { double d = 0; for (int c = 0; c < CH; ++c) d += (double)hq[c] * hq[nq + (size_t)j * CH + c]; lg[j] = hM[j] * d / sqrt(128.0); mx = fmax(mx, lg[j]); }
                for (int j = 0; j < N; ++j) L += exp(lg[j] - mx);
                printf("  cpu row0 max logit %g L %g\n", mx, L);
            }
            printf("cpu-ref %-22s max|d| %.3g   out[0..2] %.6f %.6f %.6f\n", V[vi].name, md, out[0], out[1], out[2]);
        }
    }
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    std::vector<std::vector<float>> t(V.size());
    for (int round = 0; round < 5; ++round)
        for (size_t vi = 0; vi < V.size(); ++vi) {
            V[vi].launch(Q, K, Vv, dM, B, N, dop, dml, nullptr, 0);
            CK(hipEventRecord(e0, 0));
            for (int i = 0; i < iters; ++i) V[vi].launch(Q, K, Vv, dM, B, N, dop, dml, nullptr, 0);
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float ms; CK(hipEventElapsedTime(&ms, e0, e1));
            t[vi].push_back(ms / iters);
        }
    // the attention kernels assume N's inputs: q/k/v of rows < N (the harness writes
    // rows < Npad) -- fine: rows >= N are masked as keys and ignored as queries
    const double flops = 4.0 * B * (double)N * N * CH;
    printf("B=%d N=%d (%.2f GFLOP/launch)\n", B, N, flops / 1e9);
    for (size_t vi = 0; vi < V.size(); ++vi) {
        std::vector<float> x = t[vi];
        std::sort(x.begin(), x.end());
        printf("%-22s median %8.1f us  min %8.1f us  %6.1f TFLOP/s\n", V[vi].name, x[2] * 1e3, x[0] * 1e3, flops / (x[2] * 1e-3) / 1e12);
    }
    return 0;
}
