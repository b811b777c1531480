// tools/split_probe.hip -- checks split2 (attention_h3.hpp: v_cvt_pk_f16_f32 + v_fma_mixlo/mixhi)
// against the reference split hi = f16(x), lo = f16(x - hi) on 131072 values incl.
// fp16 ties, subnormal and large magnitudes (diagnostics; run on the GPU box).
// Build: hipcc --offload-arch=gfx950 -O3 tools/split_probe.hip -o /tmp/split_probe
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstring>
#include <cstdio>
#include <cstdlib>
__global__ void k(const float* x, uint32_t* hi, uint32_t* lo) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    float x0 = x[2*i], x1 = x[2*i+1];
    uint32_t h, l;
    asm("v_cvt_pk_f16_f32 %0, %1, %2" : "=v"(h) : "v"(x0), "v"(x1));
    asm("v_fma_mixlo_f16 %0, %1, 1.0, -%2 op_sel_hi:[0,0,1]" : "=v"(l) : "v"(x0), "v"(h));
    asm("v_fma_mixhi_f16 %0, %1, 1.0, -%2 op_sel:[0,0,1] op_sel_hi:[0,0,1]" : "+v"(l) : "v"(x1), "v"(h));
    hi[i] = h; lo[i] = l;
}
int main() {
    const int n = 1 << 16;
    float* hx = (float*)malloc(n * 8); for (int i = 0; i < 2*n; ++i) { unsigned u = i * 2654435761u; u ^= u >> 13; float f = ((u & 0xffffff) / 16777216.0f - 0.5f) * 8.0f; if (i % 7 == 0) f = (float)(_Float16)f + 0.000244140625f * ((i % 3) - 1); if (i % 5 == 1) f *= 1e-5f; if (i % 5 == 2) f *= 3e-8f; if (i % 5 == 3) f *= 1e4f; hx[i] = f; }
    float* dx; uint32_t *dh, *dl; hipMalloc(&dx, n*8); hipMalloc(&dh, n*4); hipMalloc(&dl, n*4);
    hipMemcpy(dx, hx, n*8, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k, dim3(n/256), dim3(256), 0, 0, dx, dh, dl); printf("launch: %s sync: %s\n", hipGetErrorString(hipGetLastError()), hipGetErrorString(hipDeviceSynchronize()));
    uint32_t* h = (uint32_t*)malloc(n*4); uint32_t* l = (uint32_t*)malloc(n*4);
    hipMemcpy(h, dh, n*4, hipMemcpyDeviceToHost); hipMemcpy(l, dl, n*4, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int i = 0; i < n; ++i) for (int e = 0; e < 2; ++e) {
        float x = hx[2*i+e]; _Float16 rh = (_Float16)x; _Float16 rl = (_Float16)(x - (float)rh);
        uint16_t gh = (h[i] >> (16*e)) & 0xffff, gl = (l[i] >> (16*e)) & 0xffff;
        uint16_t eh, el; memcpy(&eh, &rh, 2); memcpy(&el, &rl, 2);
        if (gh != eh || gl != el) { if (bad < 5) printf("x=%.9g hi %04x/%04x lo %04x/%04x\n", x, gh, eh, gl, el); ++bad; }
    }
    printf("mismatches %d of %d\n", bad, 2*n);
}
