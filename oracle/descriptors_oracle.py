"""CPU restatement of the descriptor stage -- TEST INFRASTRUCTURE ONLY.

Only tests/ may import this module; the product path (pointdsc_amd/
descriptors.py over libpdsc.so) never does.

What it restates: the open3d calls of demo_registration.py:37-44 and
misc/cal_fpfh.py:7-36 -- VoxelDownSample, EstimateNormals and
ComputeFPFHFeature with KDTreeSearchParamHybrid(radius, max_nn) -- from
open3d's published algorithms (open3d 0.x, not installed here and not
vendored in the reference: PARITY UNPINNED against open3d itself).  The
restatement fixes the choices open3d leaves to its containers (hash-map
voxel order -> ascending voxel key; nanoflann tie order -> ascending
(d^2, index), the query first) exactly as include/pdsc.h documents them, and
evaluates every sum in the same order as the kernels, so index outputs are
compared bit-exactly and floating outputs to the last few ulps.  Normals:
open3d 0.9.0's (environment.yml:76) EstimateNormals with its default
fast_normal_computation -- FastEigen3x3, whose eigenvector
(A - l0 I)(A - l1 I) e0 carries the sign n_x >= 0 -- optionally flipped
towards a viewpoint or the centroid.
"""
import numpy as np

KEY_BITS = 21


def voxel_keys(pts, cell, half):
    """floor(((double)p - ((double)min - half)) / cell) per axis, packed like the kernels."""
    p = np.asarray(pts, np.float32).astype(np.float64)
    o = p.min(0) - half
    q = np.floor((p - o) / cell).astype(np.int64)
    if (q < 0).any() or (q >= (1 << KEY_BITS)).any():
        raise ValueError("extent / cell >= 2^21")
    return (q[:, 0] << (2 * KEY_BITS)) | (q[:, 1] << KEY_BITS) | q[:, 2]


def _seq_group_sum(vals, start, count):
    """Per-group sums of rows vals[start[g] : start[g] + count[g]], added in row order."""
    out = np.zeros((len(start),) + vals.shape[1:], np.float64)
    for j in range(int(count.max()) if len(count) else 0):
        m = count > j
        out[m] += vals[start[m] + j]
    return out


def voxel_down_sample(pts, voxel_size, normals=None):
    """VoxelDownSample: (points [m,3] fp32, normals [m,3] fp32 | None, voxel keys [m])."""
    v = float(np.float32(voxel_size))
    key = voxel_keys(pts, v, 0.5 * v)
    order = np.argsort(key, kind="stable")
    uk, start, count = np.unique(key[order], return_index=True, return_counts=True)
    p = np.asarray(pts, np.float32).astype(np.float64)[order]
    out = (_seq_group_sum(p, start, count) / count[:, None]).astype(np.float32)
    on = None
    if normals is not None:
        # AccumulatedPoint::GetAverageNormal: the SUM, normalized() (v / sqrt(squaredNorm), 0 stays 0)
        a = _seq_group_sum(np.asarray(normals, np.float32).astype(np.float64)[order], start, count)
        on = _normalized(a).astype(np.float32)
    return out, on, uk


def _normalized(v):
    """Eigen's normalized() row-wise: v / sqrt((x x + y y) + z z); zero rows unchanged."""
    z = (v[:, 0] * v[:, 0] + v[:, 1] * v[:, 1]) + v[:, 2] * v[:, 2]
    n = np.sqrt(np.where(z > 0, z, 1.0))
    return np.where(z[:, None] > 0, v / n[:, None], v)


def fast_eigen3x3(C):
    """open3d 0.9.0 FastEigen3x3 (geometry/EstimateNormals.cpp) on [n,3,3] fp64:
    eigenvalues in closed form (l0 >= l1 >= l2), the eigenvector of l2 as
    (A - l0 I)(A - l1 I) e0 normalised, 0 where it vanishes -- each operation in
    the order of the kernel (pointdsc_amd/csrc/descriptors.hip)."""
    a00, a11, a22 = C[:, 0, 0], C[:, 1, 1], C[:, 2, 2]
    a01, a02, a12 = C[:, 0, 1], C[:, 0, 2], C[:, 1, 2]
    p1 = a01 * a01 + a02 * a02 + a12 * a12
    diag = p1 == 0.0
    with np.errstate(all="ignore"):
        q = ((a00 + a11) + a22) / 3.0
        d0, d1, d2 = a00 - q, a11 - q, a22 - q
        p = np.sqrt((((d0 * d0 + d1 * d1) + d2 * d2) + 2 * p1) / 6.0)
        ip = 1.0 / p
        b00, b11, b22, b01, b02, b12 = ip * d0, ip * d1, ip * d2, ip * a01, ip * a02, ip * a12
        det = (b00 * (b11 * b22 - b12 * b12) - b01 * (b01 * b22 - b02 * b12)) + b02 * (b01 * b12 - b02 * b11)
        r = det / 2.0
        phi = np.where(r <= -1, np.pi / 3.0, np.where(r >= 1, 0.0, np.arccos(np.clip(r, -1, 1)) / 3.0))
        l0 = q + 2.0 * p * np.cos(phi)
        l2 = q + 2.0 * p * np.cos(phi + 2.0 * np.pi / 3.0)
        l1 = q * 3.0 - l0 - l2
    dl2 = np.minimum(a00, np.minimum(a11, a22))
    dl0 = np.maximum(a00, np.maximum(a11, a22))
    dl1 = ((a00 + a11) + a22) - dl0 - dl2
    l0, l1 = np.where(diag, dl0, l0), np.where(diag, dl1, l1)
    c0, c1, c2 = a00 - l1, a01, a02
    m00, m11, m22 = a00 - l0, a11 - l0, a22 - l0
    v = np.stack([(m00 * c0 + a01 * c1) + a02 * c2, (a01 * c0 + m11 * c1) + a12 * c2,
                  (a02 * c0 + a12 * c1) + m22 * c2], 1)
    return _normalized(v)


def _d2(q, p):
    d = p.astype(np.float64) - q.astype(np.float64)
    return d[..., 0] * d[..., 0] + d[..., 1] * d[..., 1] + d[..., 2] * d[..., 2]


def radius_knn(pts, radius, max_nn, chunk=256, queries=None):
    """KDTreeSearchParamHybrid: (nbr [q,K] int32, dist2 [q,K] fp64, count [q]) for
    the points `queries` (default: every point) of the cloud."""
    p = np.asarray(pts, np.float32)
    qidx = np.arange(len(p)) if queries is None else np.asarray(queries, np.int64)
    n = len(qidx)
    r = float(np.float32(radius))
    r2 = r * r
    K = int(max_nn)
    nbr = np.full((n, K), -1, np.int32)
    d2o = np.zeros((n, K), np.float64)
    cnt = np.zeros(n, np.int32)
    tree = None
    if tree is None and len(p) > 20000:
        from scipy.spatial import cKDTree
        tree = cKDTree(p.astype(np.float64))
    for q0 in range(0, n, chunk):
        rows = np.arange(q0, min(n, q0 + chunk))
        qs = qidx[rows]
        if tree is None:
            D = _d2(p[qs, None, :], p[None, :, :])
            cand = [np.nonzero(D[i] <= r2)[0] for i in range(len(qs))]
            dl = [D[i, c] for i, c in enumerate(cand)]
        else:
            cand = [np.asarray(c, np.int64) for c in tree.query_ball_point(p[qs].astype(np.float64), r * (1 + 1e-9))]
            dl = []
            for i, c in zip(qs, cand):
                d = _d2(p[i], p[c])
                keep = d <= r2
                cand[len(dl)] = c[keep]
                dl.append(d[keep])
        for row, i, c, d in zip(rows, qs, cand, dl):
            key = np.where(c == i, -1.0, d)
            o = np.lexsort((c, key))[:K]
            nbr[row, :len(o)] = c[o]
            d2o[row, :len(o)] = np.maximum(key[o], 0.0)
            cnt[row] = len(o)
    return nbr, d2o, cnt


def estimate_normals(pts, radius, max_nn=30, viewpoint=None, queries=None, orient=None):
    """EstimateNormals as open3d 0.9 computes it (fast_eigen3x3 of the fp64
    cumulant covariance; (0,0,1) under 3 neighbours or for a zero vector), with
    open3d's sign (orient 'open3d', the default without a viewpoint), or flipped
    towards `viewpoint` ('viewpoint') or the cloud's centroid ('centroid').
    Returns (normals fp32 [q,3], eigenvalues [q,3] ascending) for the points
    `queries` (default: all)."""
    cloud = np.asarray(pts, np.float32)
    if orient is None:
        orient = "viewpoint" if viewpoint is not None else "open3d"
    qidx = np.arange(len(cloud)) if queries is None else np.asarray(queries, np.int64)
    nbr, _, cnt = radius_knn(cloud, radius, max_nn, queries=qidx)
    p = cloud[qidx]
    n = len(p)
    s = np.zeros((n, 9), np.float64)
    for t in range(int(max_nn)):
        m = cnt > t
        x = cloud[np.where(m, nbr[:, t], 0)].astype(np.float64)
        terms = np.stack([x[:, 0], x[:, 1], x[:, 2], x[:, 0] * x[:, 0], x[:, 0] * x[:, 1], x[:, 0] * x[:, 2],
                          x[:, 1] * x[:, 1], x[:, 1] * x[:, 2], x[:, 2] * x[:, 2]], 1)
        s[m] += terms[m]
    s /= np.maximum(cnt, 1)[:, None].astype(np.float64)
    C = np.empty((n, 3, 3))
    C[:, 0, 0] = s[:, 3] - s[:, 0] * s[:, 0]
    C[:, 1, 1] = s[:, 6] - s[:, 1] * s[:, 1]
    C[:, 2, 2] = s[:, 8] - s[:, 2] * s[:, 2]
    C[:, 0, 1] = C[:, 1, 0] = s[:, 4] - s[:, 0] * s[:, 1]
    C[:, 0, 2] = C[:, 2, 0] = s[:, 5] - s[:, 0] * s[:, 2]
    C[:, 1, 2] = C[:, 2, 1] = s[:, 7] - s[:, 1] * s[:, 2]
    w = np.linalg.eigvalsh(C)
    nv = fast_eigen3x3(C)
    zero = (cnt < 3) | np.all(nv == 0, 1)
    nv[zero] = (0.0, 0.0, 1.0)
    if orient != "open3d":
        vp = cloud.astype(np.float64).mean(0) if orient == "centroid" else np.asarray(viewpoint, np.float64)
        flip = np.sum(nv * (vp - p.astype(np.float64)), 1) < 0
        nv[flip] *= -1
    return nv.astype(np.float32), w


def pair_features(p1, n1, p2, n2):
    """open3d ComputePairFeatures (PCL computePairFeatures), vectorised: (f0, f1, f2)."""
    dp = p2 - p1
    f3 = np.sqrt(dp[:, 0] * dp[:, 0] + dp[:, 1] * dp[:, 1] + dp[:, 2] * dp[:, 2])
    ok = f3 != 0
    f3s = np.where(ok, f3, 1.0)

    def dot(a, b):
        return a[:, 0] * b[:, 0] + a[:, 1] * b[:, 1] + a[:, 2] * b[:, 2]

    a1 = dot(n1, dp) / f3s
    a2 = dot(n2, dp) / f3s
    swap = np.arccos(np.abs(a1)) > np.arccos(np.abs(a2))
    a = np.where(swap[:, None], n2, n1)
    b = np.where(swap[:, None], n1, n2)
    dpp = np.where(swap[:, None], -dp, dp)
    theta = np.where(swap, -a2, a1)
    v = np.cross(dpp, a)
    vn = np.sqrt(v[:, 0] * v[:, 0] + v[:, 1] * v[:, 1] + v[:, 2] * v[:, 2])
    ok &= vn != 0
    v = v / np.where(vn != 0, vn, 1.0)[:, None]
    w = np.cross(a, v)
    f1 = dot(v, b)
    f0 = np.arctan2(dot(w, b), dot(a, b))
    z = np.zeros_like(f0)
    return np.where(ok, f0, z), np.where(ok, f1, z), np.where(ok, theta, z)


def _bin(x):
    return np.clip(np.floor(x), 0, 10).astype(np.int64)


def compute_fpfh(pts, normals, radius, max_nn=100):
    """ComputeFPFHFeature: (fpfh [n,33] fp64, normalised fp32 [n,33])."""
    p = np.asarray(pts, np.float32).astype(np.float64)
    nr = np.asarray(normals, np.float32).astype(np.float64)
    nbr, d2, cnt = radius_knn(pts, radius, max_nn)
    n, K = nbr.shape
    counts = np.zeros((n, 33), np.int64)
    for k in range(1, K):
        m = cnt > k
        if not m.any():
            continue
        i = np.nonzero(m)[0]
        j = nbr[i, k]
        f0, f1, f2 = pair_features(p[i], nr[i], p[j], nr[j])
        counts[i, _bin(11 * (f0 + np.pi) / (2.0 * np.pi))] += 1
        counts[i, 11 + _bin(11 * (f1 + 1.0) * 0.5)] += 1
        counts[i, 22 + _bin(11 * (f2 + 1.0) * 0.5)] += 1
    incr = 100.0 / np.maximum(cnt - 1, 1).astype(np.float64)
    spfh = np.zeros((n, 33), np.float64)
    for t in range(int(counts.max()) if counts.size else 0):
        spfh += np.where(counts > t, incr[:, None], 0.0)
    spfh[cnt <= 1] = 0.0
    f = np.zeros((n, 33), np.float64)
    gs = np.zeros((n, 3), np.float64)
    for k in range(1, K):
        m = (cnt > k) & (d2[:, k] != 0.0)
        if not m.any():
            continue
        val = spfh[np.where(m, nbr[:, k], 0)] / np.where(m, d2[:, k], 1.0)[:, None]
        val[~m] = 0.0
        f += val
        for g in range(3):
            for b in range(11):
                gs[:, g] += val[:, 11 * g + b]
    s = np.where(gs != 0, 100.0 / np.where(gs != 0, gs, 1.0), gs)
    out = f * np.repeat(s, 11, axis=1) + spfh
    out[cnt <= 1] = 0.0
    nrm = np.sqrt((out * out).sum(1, keepdims=True))
    return out, (out / (nrm + 1e-6)).astype(np.float32)
