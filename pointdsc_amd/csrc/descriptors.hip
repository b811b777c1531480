// descriptors.hip -- SURVEY 8(f) row 4: the descriptor stage that
// demo_registration.py:37-44 and misc/cal_fpfh.py:7-36 run through open3d,
// rebuilt on the GPU (open3d is not a dependency here; its published
// algorithms are restated, parity against open3d itself is unpinned):
//
//   PLY reader       binary_little_endian / ascii vertex x, y, z (host code)
//   voxel grid       open3d VoxelDownSample: index = floor((p - (min - v/2)) / v)
//                    in fp64, per-voxel mean of points (and of normals, then
//                    normalised); output in ascending voxel-key order (open3d's
//                    is its hash map's iteration order)
//   radius kNN       KDTreeSearchParamHybrid(radius, max_nn): the max_nn nearest
//                    points within radius, ascending (d^2, index), the query
//                    itself first; a uniform grid of radius-sized cells, one
//                    wave per query (27 cells, a d^2 histogram picks the
//                    threshold, the survivors are bitonic-sorted in LDS)
//   normals          EstimateNormals: covariance of the neighbourhood from fp64
//                    cumulants, eigenvector of the smallest eigenvalue (Jacobi);
//                    < 3 neighbours or a zero covariance -> (0, 0, 1); sign:
//                    towards a viewpoint (default: the cloud's centroid, which
//                    moves with the cloud, so normals are rigid-motion covariant)
//   SPFH / FPFH      ComputeFPFHFeature: pair features (alpha, phi, theta) of the
//                    Darboux frame in fp64, 3 x 11 bins of 100 / (k - 1), then
//                    FPFH_i = SPFH_i + (100 / sum) * sum_k SPFH_k / d_k^2 per
//                    group, accumulated in neighbour order like the reference
//
// Everything is independent per point (HBM/latency-bound gathers, fp64 VALU);
// the sorts are hipCUB radix sorts of 63-bit cell keys.
#include <hipcub/hipcub.hpp>

#include <cctype>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "pdsc_common.hpp"
#include "pdsc_internal.hpp"

namespace pdsc {

typedef unsigned long long u64;
constexpr int KEY_BITS = 21;
constexpr long long KEY_MAX = (1LL << KEY_BITS) - 1;

PDSC_DEV u64 pack_key(long long ix, long long iy, long long iz) {
    return ((u64)ix << (2 * KEY_BITS)) | ((u64)iy << KEY_BITS) | (u64)iz;
}

// ------------------------------------------------------------ cloud statistics
// min / max (fp32, exact) and the fp64 coordinate sum, two-stage, fixed order.
constexpr int ST_BLOCKS = 256;

__global__ __launch_bounds__(256) void cloud_stats_partial_kernel(const float *__restrict__ p, int n,
                                                                  float *__restrict__ pmn, float *__restrict__ pmx,
                                                                  double *__restrict__ psum) {
    __shared__ float smn[4][3], smx[4][3];
    __shared__ double ssum[4][3];
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    float mn[3] = {INFINITY, INFINITY, INFINITY}, mx[3] = {-INFINITY, -INFINITY, -INFINITY};
    double sm[3] = {0.0, 0.0, 0.0};
    for (int i = blockIdx.x * 256 + tid; i < n; i += gridDim.x * 256)
        for (int c = 0; c < 3; ++c) {
            const float v = p[3 * (size_t)i + c];
            mn[c] = fminf(mn[c], v);
            mx[c] = fmaxf(mx[c], v);
            sm[c] += (double)v;
        }
    for (int c = 0; c < 3; ++c) {
        for (int o = 32; o > 0; o >>= 1) {
            mn[c] = fminf(mn[c], __shfl_xor(mn[c], o));
            mx[c] = fmaxf(mx[c], __shfl_xor(mx[c], o));
            sm[c] += __shfl_xor(sm[c], o);
        }
        if (lane == 0) {
            smn[wave][c] = mn[c];
            smx[wave][c] = mx[c];
            ssum[wave][c] = sm[c];
        }
    }
    __syncthreads();
    if (tid < 3) {
        float a = smn[0][tid], b = smx[0][tid];
        double s = ssum[0][tid];
        for (int w = 1; w < 4; ++w) {
            a = fminf(a, smn[w][tid]);
            b = fmaxf(b, smx[w][tid]);
            s += ssum[w][tid];
        }
        pmn[blockIdx.x * 3 + tid] = a;
        pmx[blockIdx.x * 3 + tid] = b;
        psum[blockIdx.x * 3 + tid] = s;
    }
}

__global__ void cloud_stats_final_kernel(const float *__restrict__ pmn, const float *__restrict__ pmx,
                                         const double *__restrict__ psum, int nb, int n, CloudStats *st) {
    const int c = threadIdx.x;
    if (c >= 3) return;
    float a = INFINITY, b = -INFINITY;
    double s = 0.0;
    for (int i = 0; i < nb; ++i) {
        a = fminf(a, pmn[3 * i + c]);
        b = fmaxf(b, pmx[3 * i + c]);
        s += psum[3 * i + c];
    }
    st->mn[c] = a;
    st->mx[c] = b;
    st->centroid[c] = s / (double)n;
}

// --------------------------------------------------------------- cell keys
// q = floor(((double)p - ((double)min - half)) / cell) per axis (open3d's voxel
// index with half = voxel / 2; the neighbour grid with half = 0).
PDSC_DEV bool cell_of(const float *p, const CloudStats *st, double cell, double half, long long q[3]) {
    bool ok = true;
    for (int c = 0; c < 3; ++c) {
        const double o = (double)st->mn[c] - half;
        const double r = ((double)p[c] - o) / cell;
        long long v = (long long)floor(r);
        if (!(v >= 0 && v <= KEY_MAX)) {
            ok = false;
            v = v < 0 ? 0 : KEY_MAX;
        }
        q[c] = v;
    }
    return ok;
}

__global__ void cell_key_kernel(const float *__restrict__ p, int n, const CloudStats *st, double cell, double half,
                                u64 *__restrict__ key, int *__restrict__ idx, int *__restrict__ err) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    long long q[3];
    if (!cell_of(p + 3 * (size_t)i, st, cell, half, q)) err[0] = 1;  // extent / cell >= 2^21
    key[i] = pack_key(q[0], q[1], q[2]);
    idx[i] = i;
}

// ------------------------------------------------------------- radius kNN
constexpr int KNN_WPB = 4;      // waves (queries) per workgroup
constexpr int KNN_BINS = 1024;  // d^2 / r^2 histogram
constexpr int KNN_CAP = 1024;   // survivors sorted in LDS per query

PDSC_DEV int find_cell(const u64 *__restrict__ ukey, int nr, u64 k) {
    int lo = 0, hi = nr;
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (ukey[mid] < k)
            lo = mid + 1;
        else
            hi = mid;
    }
    return (lo < nr && ukey[lo] == k) ? lo : -1;
}

PDSC_DEV double dist2_d(const float *a, const float *b) {
    const double dx = (double)b[0] - (double)a[0], dy = (double)b[1] - (double)a[1], dz = (double)b[2] - (double)a[2];
    return dx * dx + dy * dy + dz * dz;
}

PDSC_DEV int knn_bin(double d2, double r2) {
    const int b = (int)(d2 / r2 * KNN_BINS);
    return b < KNN_BINS ? (b < 0 ? 0 : b) : KNN_BINS - 1;
}

// One wave per query.  Lanes 0..26 own the 27 cells around the query's cell;
// pass 1 histograms d^2 of every point within the radius, pass 2 keeps the
// bins up to the one where the count reaches K, and a bitonic sort of the
// survivors by (d^2, index) -- the query first -- gives the K nearest.
__global__ __launch_bounds__(KNN_WPB * 64) void radius_knn_kernel(const float *__restrict__ pts, int n,
                                                                   const CloudStats *st, double cell, GridView g,
                                                                   double r2, int K, int *__restrict__ nbr,
                                                                   double *__restrict__ d2o, int *__restrict__ cnt,
                                                                   int *__restrict__ err) {
    __shared__ int hist[KNN_WPB][KNN_BINS];
    __shared__ double bd[KNN_WPB][KNN_CAP];
    __shared__ int bi[KNN_WPB][KNN_CAP];
    __shared__ int nc[KNN_WPB];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int q = blockIdx.x * KNN_WPB + wave;
    if (q >= n) return;  // wave-uniform; no workgroup barriers below
    const float *pq = pts + 3 * (size_t)q;
    long long c0[3];
    cell_of(pq, st, cell, 0.0, c0);
    const int nr = *g.nruns;
    int cs = 0, cc = 0;
    if (lane < 27) {
        const long long x = c0[0] + lane % 3 - 1, y = c0[1] + (lane / 3) % 3 - 1, z = c0[2] + lane / 9 - 1;
        if (x >= 0 && y >= 0 && z >= 0 && x <= KEY_MAX && y <= KEY_MAX && z <= KEY_MAX) {
            const int u = find_cell(g.ukey, nr, pack_key(x, y, z));
            if (u >= 0) {
                cs = g.ustart[u];
                cc = g.ucount[u];
            }
        }
    }
    int *h = hist[wave];
    for (int b = lane; b < KNN_BINS; b += 64) h[b] = 0;
    __builtin_amdgcn_wave_barrier();
    for (int c = 0; c < 27; ++c) {
        const int s = __shfl(cs, c), m = __shfl(cc, c);
        for (int j = lane; j < m; j += 64) {
            const double d2 = dist2_d(pq, pts + 3 * (size_t)g.sidx[s + j]);
            if (d2 <= r2) atomicAdd(&h[knn_bin(d2, r2)], 1);
        }
    }
    __builtin_amdgcn_wave_barrier();
    // the threshold bin: lane l owns bins 16 l .. 16 l + 15
    int loc = 0;
    for (int b = 0; b < 16; ++b) loc += h[16 * lane + b];
    int incl = loc;
    for (int o = 1; o < 64; o <<= 1) {
        const int t = __shfl_up(incl, o);
        if (lane >= o) incl += t;
    }
    const int total = __shfl(incl, 63);
    int bstar = KNN_BINS - 1;
    if (total > K) {
        // first lane whose inclusive count reaches K, then the bin inside it
        const unsigned long long reach = __ballot(incl >= K);
        const int l = __builtin_ctzll(reach);
        int run = __shfl(incl - loc, l);
        int bb = 16 * l;
        for (int b = 0; b < 16; ++b) {  // wave-uniform walk over lane l's 16 bins
            run += h[16 * l + b];
            if (run >= K) {
                bb = 16 * l + b;
                break;
            }
        }
        bstar = bb;
    }
    if (lane == 0) nc[wave] = 0;
    __builtin_amdgcn_wave_barrier();
    double *sd = bd[wave];
    int *si = bi[wave];
    for (int c = 0; c < 27; ++c) {
        const int s = __shfl(cs, c), m = __shfl(cc, c);
        for (int j = lane; j < m; j += 64) {
            const int pi = g.sidx[s + j];
            const double d2 = dist2_d(pq, pts + 3 * (size_t)pi);
            if (d2 <= r2 && knn_bin(d2, r2) <= bstar) {
                const int slot = atomicAdd(&nc[wave], 1);
                if (slot < KNN_CAP) {
                    sd[slot] = pi == q ? -1.0 : d2;  // the query itself sorts first
                    si[slot] = pi;
                }
            }
        }
    }
    __builtin_amdgcn_wave_barrier();
    int m = nc[wave];
    if (m > KNN_CAP) {
        if (lane == 0) err[1] = 1;
        m = KNN_CAP;
    }
    int P = 2;
    while (P < m) P <<= 1;
    for (int t = m + lane; t < P; t += 64) {
        sd[t] = INFINITY;
        si[t] = 0x7fffffff;
    }
    __builtin_amdgcn_wave_barrier();
    for (int k = 2; k <= P; k <<= 1)
        for (int j = k >> 1; j > 0; j >>= 1) {
            for (int t = lane; t < P / 2; t += 64) {
                const int i = (t / j) * 2 * j + (t % j), l = i + j;
                const double di = sd[i], dl = sd[l];
                const int ii = si[i], il = si[l];
                const bool gt = di > dl || (di == dl && ii > il);
                if (gt == ((i & k) == 0)) {
                    sd[i] = dl;
                    sd[l] = di;
                    si[i] = il;
                    si[l] = ii;
                }
            }
            __builtin_amdgcn_wave_barrier();
        }
    const int kk = min(K, min(total, m));
    if (lane == 0) cnt[q] = kk;
    for (int t = lane; t < K; t += 64) {
        nbr[(size_t)q * K + t] = t < kk ? si[t] : -1;
        if (d2o) d2o[(size_t)q * K + t] = t < kk ? fmax(sd[t], 0.0) : 0.0;
    }
}

// ----------------------------------------------------------------- normals
// open3d 0.9.0's FastEigen3x3 (EstimateNormals.cpp; `fast_normal_computation`,
// true by default in estimate_normals): the eigenvalues of the symmetric 3x3 A
// in closed form (largest l0, middle l1, smallest l2; Wikipedia "Eigenvalue
// algorithm", 3x3 symmetric) and the smallest one's eigenvector as
// (A - l0 I)(A - l1 I) e0 -- Cayley-Hamilton: that column lies in the l2
// eigenspace -- normalised, or 0 when it vanishes.  In exact arithmetic it is
// (l2 - l0)(l2 - l1)(v2 . e0) v2, so the sign open3d returns makes n_x >= 0.
// Every operation in open3d's order (Eigen's 3x3 determinant and product as
// sums left to right; the library builds without fma contraction, as does this
// file: -ffp-contract=off).
// Eigen's normalized(): v / sqrt(squaredNorm), unchanged when that is 0.
PDSC_DEV double o3d_normalize(D3 &v) {
    const double z = (v.x * v.x + v.y * v.y) + v.z * v.z;
    if (z > 0) {
        const double n = sqrt(z);
        v = d3(v.x / n, v.y / n, v.z / n);
    }
    return z;
}
PDSC_DEV D3 o3d09_fast_eigen3x3(double a00, double a11, double a22, double a01, double a02, double a12) {
    const double p1 = a01 * a01 + a02 * a02 + a12 * a12;
    double l0, l1, l2;
    if (p1 == 0.0) {
        l2 = fmin(a00, fmin(a11, a22));
        l0 = fmax(a00, fmax(a11, a22));
        l1 = ((a00 + a11) + a22) - l0 - l2;  // A.trace() - l0 - l2
    } else {
        const double q = ((a00 + a11) + a22) / 3.0;
        const double d0 = a00 - q, d1 = a11 - q, d2 = a22 - q;
        const double p2 = ((d0 * d0 + d1 * d1) + d2 * d2) + 2 * p1;
        const double p = sqrt(p2 / 6.0);
        const double ip = 1.0 / p;  // B = (1 / p) (A - q I)
        const double b00 = ip * d0, b11 = ip * d1, b22 = ip * d2, b01 = ip * a01, b02 = ip * a02, b12 = ip * a12;
        // Eigen's 3x3 determinant: m00 (m11 m22 - m12 m21) - m10 (m01 m22 - m02 m21) + m20 (m01 m12 - m02 m11)
        const double det = (b00 * (b11 * b22 - b12 * b12) - b01 * (b01 * b22 - b02 * b12)) + b02 * (b01 * b12 - b02 * b11);
        const double r = det / 2.0;
        double phi;
        if (r <= -1)
            phi = M_PI / 3.0;
        else if (r >= 1)
            phi = 0.0;
        else
            phi = acos(r) / 3.0;
        l0 = q + 2.0 * p * cos(phi);
        l2 = q + 2.0 * p * cos(phi + 2.0 * M_PI / 3.0);
        l1 = q * 3.0 - l0 - l2;
    }
    // (A - l0 I) (A.col(0) - (l1, 0, 0))
    const double c0 = a00 - l1, c1 = a01, c2 = a02;
    const double m00 = a00 - l0, m11 = a11 - l0, m22 = a22 - l0;
    D3 v = d3((m00 * c0 + a01 * c1) + a02 * c2, (a01 * c0 + m11 * c1) + a12 * c2, (a02 * c0 + a12 * c1) + m22 * c2);
    if (o3d_normalize(v) == 0.0) return d3(0, 0, 0);
    return v;
}

// orient: PDSC_NORMALS_OPEN3D (the eigenvector's own sign, as open3d 0.9 leaves
// it on a cloud without normals), _VIEWPOINT (towards viewpoint), _CENTROID
// (towards the cloud's centroid)
__global__ void normals_kernel(const float *__restrict__ pts, int n, const int *__restrict__ nbr,
                               const int *__restrict__ cnt, int K, const CloudStats *st, int orient,
                               const float *__restrict__ viewpoint, float *__restrict__ nrm) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const int c = cnt[i];
    D3 nv = d3(0, 0, 1);
    if (c >= 3) {
        // open3d ComputeNormal: cumulants of (x, y, z, xx, xy, xz, yy, yz, zz) / k
        double s0 = 0, s1 = 0, s2 = 0, s3 = 0, s4 = 0, s5 = 0, s6 = 0, s7 = 0, s8 = 0;
        for (int t = 0; t < c; ++t) {
            const float *p = pts + 3 * (size_t)nbr[(size_t)i * K + t];
            const double x = p[0], y = p[1], z = p[2];
            s0 += x;
            s1 += y;
            s2 += z;
            s3 += x * x;
            s4 += x * y;
            s5 += x * z;
            s6 += y * y;
            s7 += y * z;
            s8 += z * z;
        }
        const double inv = (double)c;
        s0 /= inv, s1 /= inv, s2 /= inv, s3 /= inv, s4 /= inv, s5 /= inv, s6 /= inv, s7 /= inv, s8 /= inv;
        const double a00 = s3 - s0 * s0, a11 = s6 - s1 * s1, a22 = s8 - s2 * s2;
        const double a01 = s4 - s0 * s1, a02 = s5 - s0 * s2, a12 = s7 - s1 * s2;
        const D3 v = o3d09_fast_eigen3x3(a00, a11, a22, a01, a02, a12);
        if (v.x != 0.0 || v.y != 0.0 || v.z != 0.0) nv = v;  // a zero vector -> (0, 0, 1) (EstimateNormals)
    }
    if (orient != PDSC_NORMALS_OPEN3D) {
        const float *p = pts + 3 * (size_t)i;
        const bool vpt = orient == PDSC_NORMALS_VIEWPOINT;
        const double vx = vpt ? (double)viewpoint[0] : st->centroid[0];
        const double vy = vpt ? (double)viewpoint[1] : st->centroid[1];
        const double vz = vpt ? (double)viewpoint[2] : st->centroid[2];
        if (nv.x * (vx - p[0]) + nv.y * (vy - p[1]) + nv.z * (vz - p[2]) < 0) nv = d3(-nv.x, -nv.y, -nv.z);
    }
    nrm[3 * (size_t)i + 0] = (float)nv.x;
    nrm[3 * (size_t)i + 1] = (float)nv.y;
    nrm[3 * (size_t)i + 2] = (float)nv.z;
}

// ---------------------------------------------------------- voxel downsample
// One thread per occupied voxel, its points in ascending original index (the
// radix sort is stable): the fp64 sums in open3d's insertion order.
__global__ void voxel_reduce_kernel(const float *__restrict__ pts, const float *__restrict__ nrm, GridView g,
                                    float *__restrict__ opts, float *__restrict__ onrm, int *__restrict__ count) {
    const int v = blockIdx.x * 256 + threadIdx.x;
    const int nr = *g.nruns;
    if (v == 0) count[0] = nr;
    if (v >= nr) return;
    const int s = g.ustart[v], m = g.ucount[v];
    double px = 0, py = 0, pz = 0, nx = 0, ny = 0, nz = 0;
    for (int t = 0; t < m; ++t) {
        const int i = g.sidx[s + t];
        px += pts[3 * (size_t)i];
        py += pts[3 * (size_t)i + 1];
        pz += pts[3 * (size_t)i + 2];
        if (nrm) {
            nx += nrm[3 * (size_t)i];
            ny += nrm[3 * (size_t)i + 1];
            nz += nrm[3 * (size_t)i + 2];
        }
    }
    const double dm = (double)m;
    opts[3 * (size_t)v] = (float)(px / dm);
    opts[3 * (size_t)v + 1] = (float)(py / dm);
    opts[3 * (size_t)v + 2] = (float)(pz / dm);
    if (nrm && onrm) {
        D3 a = d3(nx, ny, nz);  // open3d: normal_.normalized() of the sum (a zero sum stays 0)
        o3d_normalize(a);
        onrm[3 * (size_t)v] = (float)a.x;
        onrm[3 * (size_t)v + 1] = (float)a.y;
        onrm[3 * (size_t)v + 2] = (float)a.z;
    }
}

// ------------------------------------------------------------ SPFH / FPFH
PDSC_DEV D3 ld3(const float *p) { return d3(p[0], p[1], p[2]); }
PDSC_DEV D3 sub3(const D3 &a, const D3 &b) { return d3(a.x - b.x, a.y - b.y, a.z - b.z); }

// (alpha, phi, theta) of the Darboux frame (open3d ComputePairFeatures, PCL's
// computePairFeatures); all zero for coincident points or a degenerate frame.
PDSC_DEV void pair_features(D3 p1, D3 n1, D3 p2, D3 n2, double &f0, double &f1, double &f2) {
    f0 = f1 = f2 = 0.0;
    D3 dp = sub3(p2, p1);
    const double f3 = sqrt(dp.x * dp.x + dp.y * dp.y + dp.z * dp.z);
    if (f3 == 0.0) return;
    D3 a = n1, b = n2;
    const double angle1 = dot3(a, dp) / f3, angle2 = dot3(b, dp) / f3;
    double theta;
    if (acos(fabs(angle1)) > acos(fabs(angle2))) {
        a = n2;
        b = n1;
        dp = d3(-dp.x, -dp.y, -dp.z);
        theta = -angle2;
    } else {
        theta = angle1;
    }
    D3 v = cross3(dp, a);
    const double vn = sqrt(v.x * v.x + v.y * v.y + v.z * v.z);
    if (vn == 0.0) return;
    v = d3(v.x / vn, v.y / vn, v.z / vn);
    const D3 w = cross3(a, v);
    f2 = theta;
    f1 = dot3(v, b);
    f0 = atan2(dot3(w, b), dot3(a, b));
}

PDSC_DEV int fpfh_bin(double x) {  // (int)floor(...) clamped to [0, 10]
    int h = (int)floor(x);
    return h < 0 ? 0 : (h > 10 ? 10 : h);
}

// One wave per point: lanes take neighbours 1 + lane and 65 + lane (K <= 128);
// bin counts by ballot, then lane b sums 100 / (k - 1) count_b times.
__global__ __launch_bounds__(256) void spfh_kernel(const float *__restrict__ pts, const float *__restrict__ nrm,
                                                   int n, const int *__restrict__ nbr, const int *__restrict__ cnt,
                                                   int K, double *__restrict__ spfh) {
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int i = blockIdx.x * 4 + wave;
    if (i >= n) return;
    const int c = cnt[i];
    double *row = spfh + (size_t)i * 33;
    if (c <= 1) {
        if (lane < 33) row[lane] = 0.0;
        return;
    }
    const D3 p1 = ld3(pts + 3 * (size_t)i), n1 = ld3(nrm + 3 * (size_t)i);
    int hb[2][3];
    for (int r = 0; r < 2; ++r) {
        const int k = 1 + lane + 64 * r;
        hb[r][0] = hb[r][1] = hb[r][2] = -1;
        if (k < c) {
            const int j = nbr[(size_t)i * K + k];
            double f0, f1, f2;
            pair_features(p1, n1, ld3(pts + 3 * (size_t)j), ld3(nrm + 3 * (size_t)j), f0, f1, f2);
            hb[r][0] = fpfh_bin(11 * (f0 + M_PI) / (2.0 * M_PI));
            hb[r][1] = fpfh_bin(11 * (f1 + 1.0) * 0.5);
            hb[r][2] = fpfh_bin(11 * (f2 + 1.0) * 0.5);
        }
    }
    int mine = 0;
#pragma unroll
    for (int g = 0; g < 3; ++g)
#pragma unroll
        for (int b = 0; b < 11; ++b) {
            const int cb = __popcll(__ballot(hb[0][g] == b)) + __popcll(__ballot(hb[1][g] == b));
            if (lane == 11 * g + b) mine = cb;
        }
    if (lane < 33) {
        const double incr = 100.0 / (double)(c - 1);
        double v = 0.0;
        for (int t = 0; t < mine; ++t) v += incr;
        row[lane] = v;
    }
}

// One wave per point: lane j < 33 accumulates its bin over the neighbours in
// order; lanes 33..35 accumulate the three group sums in (k, bin) order.
__global__ __launch_bounds__(256) void fpfh_kernel(int n, const int *__restrict__ nbr, const int *__restrict__ cnt,
                                                   const double *__restrict__ d2, int K,
                                                   const double *__restrict__ spfh, double *__restrict__ out,
                                                   float *__restrict__ outn) {
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int i = blockIdx.x * 4 + wave;
    if (i >= n) return;
    const int c = cnt[i];
    double f = 0.0, gs = 0.0;
    if (c > 1) {
        for (int k = 1; k < c; ++k) {
            const double dist = d2[(size_t)i * K + k];
            if (dist == 0.0) continue;
            const double *sr = spfh + (size_t)nbr[(size_t)i * K + k] * 33;
            if (lane < 33) f += sr[lane] / dist;
            if (lane >= 33 && lane < 36)
                for (int b = 0; b < 11; ++b) gs += sr[11 * (lane - 33) + b] / dist;
        }
    }
    double s = __shfl(gs, 33 + (lane < 33 ? lane / 11 : 0));
    if (s != 0.0) s = 100.0 / s;
    double v = 0.0;
    if (c > 1 && lane < 33) v = f * s + spfh[(size_t)i * 33 + lane];
    if (lane < 33) out[(size_t)i * 33 + lane] = v;
    if (outn) {  // demo_registration.py:42: f / (||f|| + 1e-6)
        double ss = lane < 33 ? v * v : 0.0;
        for (int o = 32; o > 0; o >>= 1) ss += __shfl_xor(ss, o);
        if (lane < 33) outn[(size_t)i * 33 + lane] = (float)(v / (sqrt(ss) + 1e-6));
    }
}

// ------------------------------------------------------------------ launchers
size_t grid_workspace_bytes(int n) {
    size_t a = 0, b = 0, c = 0;
    (void)hipcub::DeviceRadixSort::SortPairs(nullptr, a, (const u64 *)nullptr, (u64 *)nullptr, (const int *)nullptr,
                                             (int *)nullptr, n, 0, 3 * KEY_BITS);
    (void)hipcub::DeviceRunLengthEncode::Encode(nullptr, b, (const u64 *)nullptr, (u64 *)nullptr, (int *)nullptr,
                                                (int *)nullptr, n);
    (void)hipcub::DeviceScan::ExclusiveSum(nullptr, c, (const int *)nullptr, (int *)nullptr, n);
    const size_t cub = std::max(a, std::max(b, c));
    const size_t nn = (size_t)std::max(n, 1);
    return align_bytes(ST_BLOCKS * 3 * (2 * sizeof(float) + sizeof(double))) + align_bytes(sizeof(CloudStats)) +
           3 * align_bytes(nn * sizeof(u64)) + 5 * align_bytes(nn * sizeof(int)) + align_bytes(4 * sizeof(int)) +
           align_bytes(cub);
}

hipError_t build_grid(const float *pts, int n, double cell, double half, void *ws, GridBufs &G, hipStream_t s) {
    char *w = static_cast<char *>(ws);
    auto take = [&](size_t bytes) {
        char *p = w;
        w += align_bytes(bytes);
        return p;
    };
    const size_t nn = (size_t)std::max(n, 1);
    float *pmn = reinterpret_cast<float *>(take(ST_BLOCKS * 3 * (2 * sizeof(float) + sizeof(double))));
    float *pmx = pmn + ST_BLOCKS * 3;
    double *psum = reinterpret_cast<double *>(pmx + ST_BLOCKS * 3);
    G.st = reinterpret_cast<CloudStats *>(take(sizeof(CloudStats)));
    u64 *key = reinterpret_cast<u64 *>(take(nn * sizeof(u64)));
    G.view.skey = reinterpret_cast<u64 *>(take(nn * sizeof(u64)));
    G.view.ukey = reinterpret_cast<u64 *>(take(nn * sizeof(u64)));
    int *idx = reinterpret_cast<int *>(take(nn * sizeof(int)));
    G.view.sidx = reinterpret_cast<int *>(take(nn * sizeof(int)));
    G.view.ustart = reinterpret_cast<int *>(take(nn * sizeof(int)));
    G.view.ucount = reinterpret_cast<int *>(take(nn * sizeof(int)));
    take(nn * sizeof(int));  // reserved
    int *flags = reinterpret_cast<int *>(take(4 * sizeof(int)));
    G.view.nruns = flags;
    G.err = flags + 1;  // [0] range, [1] kNN capacity
    size_t cub = 0, a = 0, b = 0, c = 0;
    (void)hipcub::DeviceRadixSort::SortPairs(nullptr, a, (const u64 *)nullptr, (u64 *)nullptr, (const int *)nullptr,
                                             (int *)nullptr, n, 0, 3 * KEY_BITS);
    (void)hipcub::DeviceRunLengthEncode::Encode(nullptr, b, (const u64 *)nullptr, (u64 *)nullptr, (int *)nullptr,
                                                (int *)nullptr, n);
    (void)hipcub::DeviceScan::ExclusiveSum(nullptr, c, (const int *)nullptr, (int *)nullptr, n);
    cub = std::max(a, std::max(b, c));
    void *tmp = take(cub);
    hipError_t e;
    if ((e = hipMemsetAsync(flags, 0, 4 * sizeof(int), s)) != hipSuccess) return e;
    if ((e = hipMemsetAsync(G.view.ucount, 0, nn * sizeof(int), s)) != hipSuccess) return e;
    hipLaunchKernelGGL(cloud_stats_partial_kernel, dim3(ST_BLOCKS), dim3(256), 0, s, pts, n, pmn, pmx, psum);
    hipLaunchKernelGGL(cloud_stats_final_kernel, dim3(1), dim3(64), 0, s, pmn, pmx, psum, ST_BLOCKS, n, G.st);
    hipLaunchKernelGGL(cell_key_kernel, dim3((n + 255) / 256), dim3(256), 0, s, pts, n, G.st, cell, half, key, idx,
                       G.err);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    size_t tb = a;
    if ((e = hipcub::DeviceRadixSort::SortPairs(tmp, tb, key, G.view.skey, idx, G.view.sidx, n, 0, 3 * KEY_BITS, s)) !=
        hipSuccess)
        return e;
    tb = b;
    if ((e = hipcub::DeviceRunLengthEncode::Encode(tmp, tb, G.view.skey, G.view.ukey, G.view.ucount, G.view.nruns, n,
                                                   s)) != hipSuccess)
        return e;
    tb = c;
    return hipcub::DeviceScan::ExclusiveSum(tmp, tb, G.view.ucount, G.view.ustart, n, s);
}

hipError_t launch_radius_knn(const float *pts, int n, const GridBufs &G, double radius, int K, int *nbr, double *d2,
                             int *cnt, hipStream_t s) {
    hipLaunchKernelGGL(radius_knn_kernel, dim3((n + KNN_WPB - 1) / KNN_WPB), dim3(KNN_WPB * 64), 0, s, pts, n, G.st,
                       radius, G.view, radius * radius, K, nbr, d2, cnt, G.err);
    return hipGetLastError();
}

hipError_t launch_normals(const float *pts, int n, const int *nbr, const int *cnt, int K, const GridBufs &G,
                          int orient, const float *viewpoint, float *nrm, hipStream_t s) {
    hipLaunchKernelGGL(normals_kernel, dim3((n + 255) / 256), dim3(256), 0, s, pts, n, nbr, cnt, K, G.st, orient,
                       viewpoint, nrm);
    return hipGetLastError();
}

hipError_t launch_voxel_reduce(const float *pts, const float *nrm, int n, const GridBufs &G, float *opts, float *onrm,
                               int *count, hipStream_t s) {
    hipLaunchKernelGGL(voxel_reduce_kernel, dim3((n + 255) / 256), dim3(256), 0, s, pts, nrm, G.view, opts, onrm,
                       count);
    return hipGetLastError();
}

hipError_t launch_fpfh(const float *pts, const float *nrm, int n, const int *nbr, const int *cnt, const double *d2,
                       int K, double *spfh, double *out, float *outn, hipStream_t s) {
    hipLaunchKernelGGL(spfh_kernel, dim3((n + 3) / 4), dim3(256), 0, s, pts, nrm, n, nbr, cnt, K, spfh);
    hipLaunchKernelGGL(fpfh_kernel, dim3((n + 3) / 4), dim3(256), 0, s, n, nbr, cnt, d2, K, spfh, out, outn);
    return hipGetLastError();
}

// ------------------------------------------------------------- PLY (host)
// The vertex element's x, y, z of a binary_little_endian or ascii PLY (what
// open3d.io.read_point_cloud reads for the demo's clouds).  Elements before
// the vertex element must have fixed-size rows (no list properties).
static int ply_type_size(const std::string &t) {
    if (t == "char" || t == "uchar" || t == "int8" || t == "uint8") return 1;
    if (t == "short" || t == "ushort" || t == "int16" || t == "uint16") return 2;
    if (t == "int" || t == "uint" || t == "int32" || t == "uint32" || t == "float" || t == "float32") return 4;
    if (t == "double" || t == "float64") return 8;
    return 0;
}

static double ply_value(const unsigned char *p, const std::string &t) {
    if (t == "float" || t == "float32") {
        float v;
        memcpy(&v, p, 4);
        return v;
    }
    if (t == "double" || t == "float64") {
        double v;
        memcpy(&v, p, 8);
        return v;
    }
    if (t == "char" || t == "int8") return (double)*(const signed char *)p;
    if (t == "uchar" || t == "uint8") return (double)*p;
    if (t == "short" || t == "int16") {
        int16_t v;
        memcpy(&v, p, 2);
        return v;
    }
    if (t == "ushort" || t == "uint16") {
        uint16_t v;
        memcpy(&v, p, 2);
        return v;
    }
    if (t == "int" || t == "int32") {
        int32_t v;
        memcpy(&v, p, 4);
        return v;
    }
    uint32_t v;
    memcpy(&v, p, 4);
    return v;
}

int ply_read_xyz(const char *path, float *xyz, int64_t capacity, int64_t *n_out, std::string &err) {
    FILE *f = fopen(path, "rb");
    if (!f) {
        err = std::string("cannot open ") + path;
        return 1;
    }
    struct Prop {
        std::string type, name;
        bool list;
    };
    struct Elem {
        std::string name;
        int64_t count;
        std::vector<Prop> props;
    };
    std::vector<Elem> elems;
    std::string format;
    char line[4096];
    if (!fgets(line, sizeof line, f) || strncmp(line, "ply", 3) != 0) {
        fclose(f);
        err = "not a PLY file";
        return 1;
    }
    bool done = false;
    while (fgets(line, sizeof line, f)) {
        char a[256] = {0}, b[256] = {0}, c[256] = {0}, d[256] = {0}, e[256] = {0};
        const int k = sscanf(line, "%255s %255s %255s %255s %255s", a, b, c, d, e);
        if (k <= 0) continue;
        if (!strcmp(a, "format")) format = b;
        else if (!strcmp(a, "element") && k >= 3) elems.push_back({b, atoll(c), {}});
        else if (!strcmp(a, "property") && !elems.empty()) {
            if (!strcmp(b, "list")) elems.back().props.push_back({d, e, true});
            else elems.back().props.push_back({b, c, false});
        } else if (!strcmp(a, "end_header")) {
            done = true;
            break;
        }
    }
    if (!done) {
        fclose(f);
        err = "no end_header";
        return 1;
    }
    const bool ascii = format == "ascii";
    if (!ascii && format != "binary_little_endian") {
        fclose(f);
        err = "unsupported PLY format " + format;
        return 1;
    }
    for (const Elem &el : elems) {
        if (el.name != "vertex") {  // skip a preceding element (fixed-size rows only)
            size_t row = 0;
            for (const Prop &p : el.props) {
                if (p.list || !ply_type_size(p.type)) {
                    fclose(f);
                    err = "element '" + el.name + "' before vertex has list/unknown properties";
                    return 1;
                }
                row += ply_type_size(p.type);
            }
            if (ascii) {
                for (int64_t r = 0; r < el.count; ++r)
                    if (!fgets(line, sizeof line, f)) break;
            } else if (fseek(f, (long)(row * el.count), SEEK_CUR) != 0) {
                fclose(f);
                err = "truncated file";
                return 1;
            }
            continue;
        }
        int ix = -1, iy = -1, iz = -1;
        std::vector<size_t> off;
        size_t row = 0;
        for (size_t q = 0; q < el.props.size(); ++q) {
            const Prop &p = el.props[q];
            if (p.list || !ply_type_size(p.type)) {
                fclose(f);
                err = "vertex element has list/unknown properties";
                return 1;
            }
            off.push_back(row);
            row += ply_type_size(p.type);
            if (p.name == "x") ix = (int)q;
            if (p.name == "y") iy = (int)q;
            if (p.name == "z") iz = (int)q;
        }
        if (ix < 0 || iy < 0 || iz < 0) {
            fclose(f);
            err = "vertex element has no x/y/z";
            return 1;
        }
        *n_out = el.count;
        if (!xyz) {
            fclose(f);
            return 0;
        }
        if (capacity < el.count) {
            fclose(f);
            err = "capacity too small";
            return 1;
        }
        if (ascii) {
            std::vector<double> vals(el.props.size());
            for (int64_t r = 0; r < el.count; ++r) {
                for (size_t q = 0; q < vals.size(); ++q)
                    if (fscanf(f, "%lf", &vals[q]) != 1) {
                        fclose(f);
                        err = "truncated ascii vertex data";
                        return 1;
                    }
                xyz[3 * r] = (float)vals[ix];
                xyz[3 * r + 1] = (float)vals[iy];
                xyz[3 * r + 2] = (float)vals[iz];
            }
        } else {
            std::vector<unsigned char> buf(row * (size_t)std::min<int64_t>(el.count, 65536));
            for (int64_t r0 = 0; r0 < el.count; r0 += 65536) {
                const int64_t m = std::min<int64_t>(65536, el.count - r0);
                if (fread(buf.data(), row, (size_t)m, f) != (size_t)m) {
                    fclose(f);
                    err = "truncated binary vertex data";
                    return 1;
                }
                for (int64_t r = 0; r < m; ++r) {
                    const unsigned char *p = buf.data() + r * row;
                    xyz[3 * (r0 + r)] = (float)ply_value(p + off[ix], el.props[ix].type);
                    xyz[3 * (r0 + r) + 1] = (float)ply_value(p + off[iy], el.props[iy].type);
                    xyz[3 * (r0 + r) + 2] = (float)ply_value(p + off[iz], el.props[iz].type);
                }
            }
        }
        fclose(f);
        return 0;
    }
    fclose(f);
    err = "no vertex element";
    return 1;
}

}  // namespace pdsc
