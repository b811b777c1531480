import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a HIP device (MI355X); run with -m gpu")
    config.addinivalue_line("markers", "slow: long-running CPU test")


def golden_names():
    return sorted(f[:-4] for f in os.listdir(GOLDEN) if f.endswith(".npz") and not f.startswith("weights_"))


def load_golden(name):
    with np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def golden_state_dict(g):
    """The exact state dict a golden case was generated with (see tools/gen_goldens.py)."""
    from pointdsc_amd.synthetic import trained_state_dict
    return trained_state_dict(str(g["preset"]), int(g["num_layers"]), float(g["cls_bias_shift"]),
                              float(g["cls_scale"]))


def golden_hparams(g):
    return dict(num_layers=int(g["num_layers"]), inlier_threshold=float(g["inlier_threshold"]),
                nms_radius=float(g["nms_radius"]), num_iterations=10, ratio=0.1, k=40)


def assert_close_scaled(actual, desired, rel=5e-5):
    """|actual - desired| <= rel * max|desired| elementwise (fp32 encoder
    outputs: the error of a 12-layer fp32 network scales with the feature
    magnitude, not with each element)."""
    actual, desired = np.asarray(actual, np.float64), np.asarray(desired, np.float64)
    scale = max(np.abs(desired).max(), 1e-30)
    err = np.abs(actual - desired).max()
    assert err <= rel * scale, f"max |diff| {err:.3g} > {rel:g} * {scale:.3g}"


def assert_seeds_equivalent(ours, ref, scores, tol=0.0):
    """Seed lists agree up to the order of (near-)tied scores.

    torch's argsort orders equal scores arbitrarily; the build
    breaks ties by ascending index.  Position by position the scores must agree
    within ``tol``, and the sets may differ only among scores within ``tol`` of
    the last seed's score."""
    ours, ref = np.asarray(ours, np.int64), np.asarray(ref, np.int64)
    assert ours.shape == ref.shape
    so, sr = scores[ours], scores[ref]
    assert np.all(np.abs(so - sr) <= tol), np.nonzero(np.abs(so - sr) > tol)
    diff = set(ours.tolist()) ^ set(ref.tolist())
    if diff:
        edge = sr[-1]
        assert all(abs(scores[i] - edge) <= tol for i in diff), diff


def assert_knn_equivalent(ours, ref, normed, seeds, eps=2e-6):
    """kNN rows agree up to near-equal distances: sorted by distance, the i-th
    neighbour of both lists is at the same distance within ``eps`` (so order
    swaps and boundary exchanges are allowed only between near-ties)."""
    f = np.asarray(normed, np.float64)
    for r, s in enumerate(np.asarray(seeds)):
        d = 2.0 - 2.0 * (f[s] @ f.T)
        do, dr = np.sort(d[ours[r]]), np.sort(d[ref[r]])
        assert np.all(np.abs(do - dr) <= eps), (r, np.max(np.abs(do - dr)))


@pytest.fixture(scope="session")
def gpu_device():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return torch.device("cuda:0")
