/*
 * oracle/exact.c -- TEST INFRASTRUCTURE ONLY (the CPU oracle's bit-exact part).
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load
 * this library, and only as the checker / CPU baseline.  The product path
 * (pointdsc_amd/) never links or calls it.
 *
 * These are the elementwise pieces of the reference hot path whose results
 * must be reproduced bit-for-bit, restated in C because numpy has no fmaf:
 *
 *   pairwise distance  models/PointDSC.py:151-152  torch.norm(p_i - p_j, dim=-1)
 *       torch-CPU fp32 evaluates it as sqrtf(fmaf(dz,dz,fmaf(dy,dy,dx*dx)))
 *       (verified bit-exact against the reference-generated goldens in
 *       tests/test_oracle.py).
 *   compatibility      models/PointDSC.py:152-153
 *       M_ij = max(0, 1 - (ds_ij - dt_ij)^2 / (sigma_d * sigma_d))
 *   NMS local maxima   models/PointDSC.py:213-216
 *       lm_i = AND_j ( c_i >= c_j  OR  ds_ij >= R )
 *
 * Build: make -C oracle   (gcc -O2 -ffp-contract=off; no -ffast-math)
 */
#include <math.h>
#include <stdint.h>

static inline float pdist3(const float *a, const float *b) {
    float dx = a[0] - b[0], dy = a[1] - b[1], dz = a[2] - b[2];
    return sqrtf(fmaf(dz, dz, fmaf(dy, dy, dx * dx)));
}

/* M [N*N] row-major; src, tgt [N*3]. */
void oracle_compat(const float *src, const float *tgt, int64_t n, float sigma_d, float *M) {
    const float s2 = sigma_d * sigma_d;
    for (int64_t i = 0; i < n; ++i) {
        for (int64_t j = 0; j < n; ++j) {
            float d = pdist3(src + 3 * i, src + 3 * j) - pdist3(tgt + 3 * i, tgt + 3 * j);
            float m = 1.0f - (d * d) / s2;
            M[i * n + j] = m > 0.0f ? m : 0.0f;
        }
    }
}

/* src distance matrix (models/PointDSC.py:151). */
void oracle_src_dist(const float *src, int64_t n, float *D) {
    for (int64_t i = 0; i < n; ++i)
        for (int64_t j = 0; j < n; ++j) D[i * n + j] = pdist3(src + 3 * i, src + 3 * j);
}

/* lm [N] in {0,1}; conf [N]. */
void oracle_local_max(const float *src, const float *conf, int64_t n, float radius, float *lm) {
    for (int64_t i = 0; i < n; ++i) {
        int ok = 1;
        for (int64_t j = 0; j < n && ok; ++j)
            ok = (conf[i] >= conf[j]) || (pdist3(src + 3 * i, src + 3 * j) >= radius);
        lm[i] = ok ? 1.0f : 0.0f;
    }
}
