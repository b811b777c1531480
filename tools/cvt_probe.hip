// Probe (diagnostics): fp32 -> fp16 rounding of v_cvt_f16_f32 (scalar) vs the
// packed conversion the compiler emits for a 2 x half build, on exact fp16 ties
// and random values.  hipcc --offload-arch=gfx950 -O3 tools/cvt_probe.hip -o /tmp/cvt_probe
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));

__global__ void probe(const float *x, int n, unsigned short *s, unsigned short *p) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (2 * i + 1 >= n) return;
    _Float16 a = (_Float16)x[2 * i], b = (_Float16)x[2 * i + 1];
    asm volatile("" : "+v"(a));
    asm volatile("" : "+v"(b));
    f16x2 pk = {(_Float16)x[2 * i], (_Float16)x[2 * i + 1]};
    asm volatile("" : "+v"(pk));
    s[2 * i] = __builtin_bit_cast(unsigned short, a);
    s[2 * i + 1] = __builtin_bit_cast(unsigned short, b);
    reinterpret_cast<unsigned int *>(p)[i] = __builtin_bit_cast(unsigned int, pk);  // one 32-bit word, no repacking
}

static unsigned short rne_half(float f) {  // reference fp32 -> fp16, round to nearest even (normal range)
    _Float16 h = (_Float16)f;              // host conversion (x86: RNE)
    unsigned short u;
    memcpy(&u, &h, 2);
    return u;
}

int main() {
    std::vector<float> x;
    for (int e = -14; e < 15; ++e)      // exact ties between consecutive fp16 normals
        for (int m = 0; m < 1024; m += 7) {
            float lo = std::ldexp(1.0f + m / 1024.0f, e), hi = std::ldexp(1.0f + (m + 1) / 1024.0f, e);
            x.push_back(0.5f * (lo + hi));
            x.push_back(-0.5f * (lo + hi));
        }
    srand(1);
    for (int i = 0; i < 20000; ++i) x.push_back((rand() / (float)RAND_MAX - 0.5f) * 8.0f);
    if (x.size() & 1) x.push_back(0.0f);
    const int n = (int)x.size();
    float *dx;
    unsigned short *ds, *dp;
    hipMalloc(&dx, n * 4);
    hipMalloc(&ds, n * 2);
    hipMalloc(&dp, n * 2);
    hipMemcpy(dx, x.data(), n * 4, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(probe, dim3((n / 2 + 255) / 256), dim3(256), 0, 0, dx, n, ds, dp);
    std::vector<unsigned short> s(n), p(n);
    hipMemcpy(s.data(), ds, n * 2, hipMemcpyDeviceToHost);
    hipMemcpy(p.data(), dp, n * 2, hipMemcpyDeviceToHost);
    int ms = 0, mp = 0, msp = 0, ties = 0;
    for (int i = 0; i < n; ++i) {
        const unsigned short r = rne_half(x[i]);
        const bool tie = i < n - 20000;
        ties += tie;
        if (s[i] != r) { if (ms < 4) printf("scalar != RNE: x=%.10g s=%04x rne=%04x tie=%d\n", x[i], s[i], r, tie); ++ms; }
        if (p[i] != r) { if (mp < 4) printf("packed != RNE: x=%.10g p=%04x rne=%04x tie=%d\n", x[i], p[i], r, tie); ++mp; }
        msp += s[i] != p[i];
    }
    printf("values %d (exact ties %d): scalar!=RNE %d, packed!=RNE %d, scalar!=packed %d\n", n, ties, ms, mp, msp);
    return 0;
}
