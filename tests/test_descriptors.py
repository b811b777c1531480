"""SURVEY.md §8(f) row 4 on the CPU: the PLY reader of libpdsc (host code) on the
reference's demo clouds (tests/golden/demo_data: demo_data/cloud_bin_{0,1}.ply
of the reference, data files) and on synthetic PLY variants, and the
descriptor oracle's own invariants (it is the checker of the GPU tests)."""
import os
import struct

import numpy as np
import pytest

from conftest import GOLDEN
from oracle import descriptors_oracle as DO

DEMO = os.path.join(GOLDEN, "demo_data")


def _raw_xyz(path):
    raw = open(path, "rb").read()
    h = raw.index(b"end_header\n") + len(b"end_header\n")
    n = int([ln for ln in raw[:h].decode().splitlines() if ln.startswith("element vertex")][0].split()[2])
    return np.frombuffer(raw[h:h + 12 * n], dtype="<f4").reshape(n, 3)


@pytest.mark.parametrize("name,n", [("cloud_bin_0.ply", 258342), ("cloud_bin_1.ply", 268977)])
def test_ply_demo_clouds(name, n):
    from pointdsc_amd.descriptors import read_ply
    p = read_ply(os.path.join(DEMO, name))
    assert p.shape == (n, 3) and p.dtype == np.float32
    assert np.array_equal(p, _raw_xyz(os.path.join(DEMO, name)))


def test_ply_variants(tmp_path):
    """ascii; binary with double x/y/z, extra properties and a fixed-size element
    before the vertices; errors for big-endian, list properties and missing files."""
    from pointdsc_amd.descriptors import read_ply
    rng = np.random.RandomState(0)
    xyz = rng.randn(17, 3)
    a = tmp_path / "a.ply"
    a.write_text("ply\nformat ascii 1.0\nelement vertex 17\nproperty float x\nproperty float y\n"
                 "property float z\nproperty uchar red\nend_header\n" +
                 "".join(f"{x:.9g} {y:.9g} {z:.9g} 7\n" for x, y, z in xyz))
    assert np.allclose(read_ply(str(a)), xyz.astype(np.float32), atol=1e-6)
    b = tmp_path / "b.ply"
    hdr = ("ply\nformat binary_little_endian 1.0\nelement camera 2\nproperty float fx\nproperty short id\n"
           "element vertex 17\nproperty uchar flag\nproperty double x\nproperty double y\nproperty double z\n"
           "property int label\nend_header\n").encode()
    body = b"".join(struct.pack("<fh", 1.0, i) for i in range(2))
    body += b"".join(struct.pack("<Bdddi", 1, x, y, z, 5) for x, y, z in xyz)
    b.write_bytes(hdr + body)
    assert np.array_equal(read_ply(str(b)), xyz.astype(np.float32))
    c = tmp_path / "c.ply"
    c.write_bytes(hdr.replace(b"binary_little_endian", b"binary_big_endian") + body)
    with pytest.raises(RuntimeError, match="unsupported PLY format"):
        read_ply(str(c))
    d = tmp_path / "d.ply"
    d.write_bytes(b"ply\nformat binary_little_endian 1.0\nelement face 1\nproperty list uchar int vertex_indices\n"
                  b"element vertex 1\nproperty float x\nproperty float y\nproperty float z\nend_header\n")
    with pytest.raises(RuntimeError, match="list"):
        read_ply(str(d))
    with pytest.raises(RuntimeError, match="cannot open"):
        read_ply(str(tmp_path / "missing.ply"))


def _rigid(seed):
    rng = np.random.RandomState(seed)
    q = rng.randn(4)
    q /= np.linalg.norm(q)
    w, x, y, z = q
    R = np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
                  [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
                  [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)]])
    return R, rng.uniform(-1, 1, 3)


def test_oracle_voxel_matches_loop():
    rng = np.random.RandomState(3)
    p = (rng.rand(400, 3) * 2).astype(np.float32)
    out, _, keys = DO.voxel_down_sample(p, 0.3)
    mn = p.astype(np.float64).min(0) - 0.5 * float(np.float32(0.3))
    groups = {}
    for i, x in enumerate(p.astype(np.float64)):
        groups.setdefault(tuple(np.floor((x - mn) / float(np.float32(0.3))).astype(int)), []).append(x)
    assert len(groups) == len(out)
    ref = np.array([np.sum(groups[k], 0) / len(groups[k]) for k in sorted(groups)], np.float32)
    np.testing.assert_allclose(out, ref, atol=1e-6)


def test_oracle_pair_features_and_fpfh_rigid_invariance():
    """FPFH with centroid-oriented normals does not change under a rigid motion
    (the property the demo's self-registration test relies on)."""
    rng = np.random.RandomState(5)
    u, v = rng.rand(2, 600)
    p = np.stack([u, v, 0.2 * np.sin(3 * u) * np.cos(2 * v)], 1).astype(np.float32)
    R, t = _rigid(1)
    q = (p.astype(np.float64) @ R.T + t).astype(np.float32)
    n1, _ = DO.estimate_normals(p, 0.1, 30, orient="centroid")
    n2, _ = DO.estimate_normals(q, 0.1, 30, orient="centroid")
    np.testing.assert_allclose(n1.astype(np.float64) @ R.T, n2, atol=1e-4)
    f1, _ = DO.compute_fpfh(p, n1, 0.25, 100)
    f2, _ = DO.compute_fpfh(q, n2, 0.25, 100)
    rows_equal = np.mean(np.abs(f1 - f2).max(1) < 1e-3)
    assert rows_equal > 0.95, rows_equal
    a0, a1, a2 = DO.pair_features(np.zeros((1, 3)), np.array([[0, 0, 1.0]]), np.array([[1.0, 0, 0]]),
                                  np.array([[0, 0, 1.0]]))
    assert abs(a0[0]) < 1e-15 and abs(a1[0]) < 1e-15 and abs(a2[0]) < 1e-15


def test_oracle_open3d_fast_eigen_sign():
    """open3d 0.9's FastEigen3x3 (the normals of its default estimate_normals):
    the smallest-eigenvalue eigenvector up to fp64 rounding, its sign n_x >= 0
    (it is (l2 - l0)(l2 - l1)(v2 . e0) v2 before normalisation); a diagonal
    covariance whose smallest entry is not a00 gives the zero vector, which
    EstimateNormals replaces by (0, 0, 1)."""
    rng = np.random.RandomState(9)
    A = rng.randn(500, 3, 3)
    C = A @ A.transpose(0, 2, 1)
    v = DO.fast_eigen3x3(C)
    w, V = np.linalg.eigh(C)
    assert np.all(np.abs(np.sum(v * V[:, :, 0], 1)) > 1 - 1e-9)
    assert np.all(v[:, 0] >= 0)
    D = np.zeros((2, 3, 3))
    D[0] = np.diag([0.5, 2.0, 3.0])  # smallest a00: e0 itself
    D[1] = np.diag([3.0, 0.5, 2.0])  # smallest a11: (A - l0)(A - l1) e0 = 0
    v = DO.fast_eigen3x3(D)
    np.testing.assert_array_equal(v[0], [1.0, 0.0, 0.0])
    np.testing.assert_array_equal(v[1], [0.0, 0.0, 0.0])
    # on a noisy plane through the origin with normal along -x the estimate is along +x
    u = rng.rand(400, 2)
    p = np.stack([1e-3 * rng.randn(400), u[:, 0], u[:, 1]], 1).astype(np.float32)
    n, _ = DO.estimate_normals(p, 0.2, 30)
    assert np.mean(n[:, 0] > 0.99) > 0.95
