"""Synthetic scan-pair correspondences and release-shape random weights.

Shared by the golden-vector generator (tools/gen_goldens.py), the tests and
bench.py so that every consumer regenerates byte-identical inputs from a seed.
Both generators use ``numpy.random.RandomState`` (a frozen stream).

Input recipe (SURVEY.md §8 d): ``src ~ U[0, extent]^3``; a random ground-truth
rotation (uniform axis, angle ``U[0, pi)``) and translation
``U[-1, 1] * extent / 3``; a fraction ``inlier_ratio`` of the correspondences
are inliers ``tgt = R src + t + N(0, (0.1 tau)^2)``, the rest are outliers
``tgt ~ U[0, extent]^3``.  ``corr_pos = [src, tgt] - mean`` exactly as the
reference's loaders build it (``datasets/ThreeDMatch.py:316-319``,
``demo_registration.py:107-108``).
"""
from __future__ import annotations

import math
from collections import OrderedDict

import numpy as np

# Named configurations (SURVEY.md §5 "Config / flags").
PRESETS = {
    # snapshot/PointDSC_3DMatch_release/config.json
    "3dmatch": dict(extent=3.0, sigma_d=0.10, inlier_threshold=0.10, nms_radius=0.10),
    # snapshot/PointDSC_KITTI_release/config.json + evaluation/test_KITTI.py:211-216
    "kitti": dict(extent=60.0, sigma_d=1.2, inlier_threshold=0.6, nms_radius=0.6),
}


def random_rotation(rng: np.random.RandomState) -> np.ndarray:
    axis = rng.normal(size=3)
    axis /= np.linalg.norm(axis)
    angle = rng.uniform(0.0, math.pi)
    kx = np.array([[0, -axis[2], axis[1]], [axis[2], 0, -axis[0]], [-axis[1], axis[0], 0]])
    return np.eye(3) + math.sin(angle) * kx + (1 - math.cos(angle)) * (kx @ kx)


def synthetic_pair(num_corr: int, seed: int, preset: str = "3dmatch",
                   inlier_ratio: float = 0.3):
    """One scan pair of ``num_corr`` putative correspondences.

    Returns a dict of float32 arrays: ``corr_pos [N,6]``, ``src_keypts [N,3]``,
    ``tgt_keypts [N,3]``, ``gt_trans [4,4]``, ``gt_labels [N]``.
    """
    p = PRESETS[preset]
    ext, tau = p["extent"], p["inlier_threshold"]
    rng = np.random.RandomState(seed)
    src = rng.uniform(0.0, ext, size=(num_corr, 3))
    R = random_rotation(rng)
    t = rng.uniform(-1.0, 1.0, size=3) * ext / 3.0
    n_in = int(round(num_corr * inlier_ratio))
    perm = rng.permutation(num_corr)
    inl = np.zeros(num_corr, dtype=bool)
    inl[perm[:n_in]] = True
    tgt = src @ R.T + t + rng.normal(0.0, 0.1 * tau, size=(num_corr, 3))
    out = ~inl
    tgt[out] = rng.uniform(0.0, ext, size=(int(out.sum()), 3))
    gt = np.eye(4)
    gt[:3, :3], gt[:3, 3] = R, t
    src32, tgt32 = src.astype(np.float32), tgt.astype(np.float32)
    corr_pos = np.concatenate([src32, tgt32], axis=-1)
    corr_pos = corr_pos - corr_pos.mean(0)
    return {
        "corr_pos": corr_pos.astype(np.float32),
        "src_keypts": src32,
        "tgt_keypts": tgt32,
        "gt_trans": gt.astype(np.float32),
        "gt_labels": inl.astype(np.float32),
    }


def synthetic_batch(num_pairs: int, num_corr: int, seed: int, preset: str = "3dmatch",
                    inlier_ratio: float = 0.3):
    """``num_pairs`` independent pairs stacked on a leading batch axis."""
    pairs = [synthetic_pair(num_corr, seed * 100003 + i, preset, inlier_ratio)
             for i in range(num_pairs)]
    return {k: np.stack([p[k] for p in pairs]) for k in pairs[0]}


def state_dict_keys(num_layers: int):
    """Parameter/buffer names of ``models/PointDSC.py:81-121`` in state_dict order."""
    keys = ["sigma", "sigma_spat"]
    bn = ["weight", "bias", "running_mean", "running_var", "num_batches_tracked"]
    for i in range(num_layers):
        p = f"encoder.blocks.PointCN_layer_{i}"
        keys += [f"{p}.0.weight", f"{p}.0.bias"] + [f"{p}.1.{b}" for b in bn]
        p = f"encoder.blocks.NonLocal_layer_{i}"
        keys += [f"{p}.fc_message.0.weight", f"{p}.fc_message.0.bias"]
        keys += [f"{p}.fc_message.1.{b}" for b in bn]
        keys += [f"{p}.fc_message.3.weight", f"{p}.fc_message.3.bias"]
        keys += [f"{p}.fc_message.4.{b}" for b in bn]
        keys += [f"{p}.fc_message.6.weight", f"{p}.fc_message.6.bias"]
        for q in ("q", "k", "v"):
            keys += [f"{p}.projection_{q}.weight", f"{p}.projection_{q}.bias"]
    keys += ["encoder.layer0.weight", "encoder.layer0.bias"]
    for j in (0, 2, 4):
        keys += [f"classification.{j}.weight", f"classification.{j}.bias"]
    return keys


def synthetic_state_dict(num_layers: int = 12, num_channels: int = 128, in_dim: int = 6,
                         seed: int = 0, sigma: float = 1.0, sigma_d: float = 0.10,
                         cls_bias: float = 10.0) -> "OrderedDict[str, np.ndarray]":
    """Random weights with the reference's shapes (numpy float32).

    Conv weights are xavier-normal (the reference's own init,
    ``models/PointDSC.py:116-121``); BatchNorm affine and running statistics are
    randomised so that eval-mode BN is not the identity; the classifier's last
    bias is ``cls_bias`` so that seed confidences are positive and the NMS/argsort
    of ``pick_seeds`` is tie-free (SURVEY.md §7 "Tie semantics").
    """
    rng = np.random.RandomState(seed)
    C, H = num_channels, num_channels // 2
    sd = OrderedDict()

    def conv(name, cout, cin):
        std = math.sqrt(2.0 / (cin + cout))
        sd[name + ".weight"] = (rng.normal(0, std, size=(cout, cin, 1))).astype(np.float32)
        sd[name + ".bias"] = rng.uniform(-0.1, 0.1, size=cout).astype(np.float32)

    def bn(name, c):
        sd[name + ".weight"] = rng.uniform(0.8, 1.2, size=c).astype(np.float32)
        sd[name + ".bias"] = rng.normal(0, 0.1, size=c).astype(np.float32)
        sd[name + ".running_mean"] = rng.normal(0, 0.1, size=c).astype(np.float32)
        sd[name + ".running_var"] = rng.uniform(0.5, 2.0, size=c).astype(np.float32)
        sd[name + ".num_batches_tracked"] = np.array(1000, dtype=np.int64)

    sd["sigma"] = np.array([sigma], dtype=np.float32)
    sd["sigma_spat"] = np.array([sigma_d], dtype=np.float32)
    for i in range(num_layers):
        p = f"encoder.blocks.PointCN_layer_{i}"
        conv(p + ".0", C, C)
        bn(p + ".1", C)
        p = f"encoder.blocks.NonLocal_layer_{i}"
        conv(p + ".fc_message.0", H, C)
        bn(p + ".fc_message.1", H)
        conv(p + ".fc_message.3", H, H)
        bn(p + ".fc_message.4", H)
        conv(p + ".fc_message.6", C, H)
        for q in ("q", "k", "v"):
            conv(f"{p}.projection_{q}", C, C)
    conv("encoder.layer0", C, in_dim)
    conv("classification.0", 32, C)
    conv("classification.2", 32, 32)
    conv("classification.4", 1, 32)
    sd["classification.4.bias"][:] = cls_bias
    assert list(sd.keys()) == state_dict_keys(num_layers)
    return sd


# bench.py's classifier rescale (shift, scale) of the trained stand-in weights: the
# unscaled logits of the bench pairs reach -460 and are all negative on some pairs,
# where pick_seeds' ranking (models/PointDSC.py:216-217) is decided by the order of
# tied zero scores -- arbitrary in torch's argsort.  logit / 32 + 15
# lies in [0.6, 16] on all 128 bench pairs (tests/golden/bench_3dmatch_1k_tf.npz):
# the same NMS and seed order wherever the unscaled ranking is tie-free.
BENCH_CLS = (15.0, 2.0 ** -5)


def trained_weights_path(preset: str = "3dmatch") -> str:
    """The synthetic stand-in checkpoint trained by tools/train_synthetic.py."""
    import os
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    return os.path.join(root, "tests", "golden", f"weights_{preset}.npz")


def trained_state_dict(preset: str = "3dmatch", num_layers: int = 12, cls_bias_shift: float = 0.0,
                       cls_scale: float = 1.0) -> "OrderedDict[str, np.ndarray]":
    """Trained synthetic weights (numpy), truncated to ``num_layers`` encoder
    layers.  The classifier's last layer becomes ``cls_scale * (w h + b) +
    cls_bias_shift`` (``cls_scale`` a power of two, so the rescale is exact);
    golden cases use it to make every seed score positive and distinct."""
    with np.load(trained_weights_path(preset), allow_pickle=False) as z:
        full = {k: z[k] for k in z.files}
    sd = OrderedDict()
    for key in state_dict_keys(num_layers):
        sd[key] = full[key].copy()
    sc = np.float32(cls_scale)
    sd["classification.4.weight"] = (sd["classification.4.weight"] * sc).astype(np.float32)
    sd["classification.4.bias"] = (sd["classification.4.bias"] * sc + np.float32(cls_bias_shift)).astype(np.float32)
    return sd
