"""Pin the CPU oracle (oracle/) against golden vectors produced by the reference
itself (tools/gen_goldens.py ran /root/reference/models/PointDSC.py).  CPU only."""
import hashlib

import numpy as np
import pytest

from conftest import (assert_close_scaled, assert_knn_equivalent, assert_rigid, assert_seeds_equivalent,
                      assert_seeds_near_ties, golden_hparams, golden_names, golden_state_dict, load_golden, seed_H_rank)
from oracle import pdsc_oracle as O

NAMES = golden_names()
FAST = [n for n in NAMES if len(load_golden(n)["src_keypts"]) <= 1000]


def _digest(sd):
    h = hashlib.sha256()
    for k, v in sd.items():
        h.update(k.encode())
        h.update(np.ascontiguousarray(v).tobytes())
    return h.hexdigest()


@pytest.mark.parametrize("name", NAMES)
def test_weights_regenerate(name):
    g = load_golden(name)
    assert _digest(golden_state_dict(g)) == str(g["weights_sha256"])


@pytest.mark.parametrize("name", [n for n in NAMES if "M" in load_golden(n)])
def test_compat_bit_exact(name):
    g = load_golden(name)
    M = O.compat(g["src_keypts"], g["tgt_keypts"], float(np.float32(g["sigma_d"])))
    assert np.array_equal(M, g["M"])  # bit-exact (models/PointDSC.py:150-153)


@pytest.mark.parametrize("name", NAMES)
def test_compat_checksums(name):
    g = load_golden(name)
    M = O.compat(g["src_keypts"], g["tgt_keypts"], float(np.float32(g["sigma_d"])))
    assert np.array_equal(np.diagonal(M), g["M_diag"])
    np.testing.assert_allclose(M.astype(np.float64).sum(-1), g["M_row_sums"], rtol=1e-12, atol=1e-9)


@pytest.mark.parametrize("name", FAST)
def test_stages_isolated(name):
    """Each stage fed with the reference's own inputs for that stage."""
    g = load_golden(name)
    sd = golden_state_dict(g)
    src, tgt = g["src_keypts"], g["tgt_keypts"]
    tau = float(g["inlier_threshold"])
    # a1-a4
    M = O.compat(src, tgt, float(np.float32(g["sigma_d"])))
    feat = O.encoder(g["corr_pos"], M, sd, int(g["num_layers"]))
    assert_close_scaled(feat, g["corr_features"])
    np.testing.assert_allclose(O.classify(feat, sd), g["confidence"], rtol=1e-5, atol=1e-3)
    # a5 from the reference confidences
    seeds, lm = O.pick_seeds(src, g["confidence"], float(g["nms_radius"]), len(g["seeds"]))
    assert np.array_equal(lm, g["is_local_max"])
    assert_seeds_equivalent(seeds, g["seeds"], g["confidence"] * lm)
    # a6 from the reference features
    normed = O.normalize(g["corr_features"])
    knn = O.knn_seed_rows(normed, g["seeds"], g["knn_idx"].shape[1])
    assert_knn_equivalent(knn, g["knn_idx"], normed, g["seeds"])
    # a7-a8 from the reference kNN
    T = O.local_consistency(normed, src, tgt, g["knn_idx"], float(sd["sigma"][0]), float(sd["sigma_spat"][0]))
    if "T" in g:
        np.testing.assert_allclose(T, g["T"], atol=5e-5)
    v, _ = O.power_iteration(T)
    np.testing.assert_allclose(v, g["leading_eig"], atol=1e-5)
    # a9 from the reference weights
    ve = g["leading_eig"]
    w = (ve / (ve.sum(-1, keepdims=True) + np.float32(1e-6))).astype(np.float32)
    seed_trans = O.rigid_transform_3d(src[g["knn_idx"]], tgt[g["knn_idx"]], w)
    ok = seed_H_rank(g) > 1e-5  # rank(H) < 2: the rotation is LAPACK's arbitrary pick (properties only)
    np.testing.assert_allclose(seed_trans[ok], g["seed_trans"][ok], atol=1e-4)
    for s in np.nonzero(~ok)[0]:
        assert_rigid(seed_trans[s], src[g["knn_idx"][s]].astype(np.float64), tgt[g["knn_idx"][s]].astype(np.float64),
                     w[s])
    # a10 from the reference hypotheses
    fitness, best, labels = O.verify(g["seed_trans"], src, tgt, tau)
    assert np.array_equal(fitness, g["seed_fitness"])  # from the reference's own hypotheses: all seeds
    np.testing.assert_allclose(g["seed_trans"][best], g["trans_pre_refine"], atol=0)
    assert np.array_equal(labels, g["final_labels"])
    # a11 from the reference pre-refinement pose
    final, hist = O.post_refinement(g["trans_pre_refine"], src, tgt, tau)
    assert len(hist) == len(g["refine_trans"])
    np.testing.assert_allclose(final, g["final_trans"], atol=1e-4)


@pytest.mark.parametrize("name", FAST)
def test_end_to_end(name):
    g = load_golden(name)
    out = O.forward_testing(g["corr_pos"], g["src_keypts"], g["tgt_keypts"], golden_state_dict(g),
                            **golden_hparams(g))
    assert np.array_equal(out["final_labels"], g["final_labels"])
    np.testing.assert_allclose(out["final_trans"], g["final_trans"], atol=1e-4)


@pytest.mark.slow
@pytest.mark.parametrize("name", [n for n in NAMES if n not in FAST])
def test_forward_5k(name):
    g = load_golden(name)
    out = O.forward_testing(g["corr_pos"], g["src_keypts"], g["tgt_keypts"], golden_state_dict(g),
                            record=True, **golden_hparams(g))
    tol = float(np.abs(out["confidence"] - g["confidence"]).max())
    assert tol <= 1e-3
    # seeds from our own confidences: only near-tie decisions may differ (conftest)
    assert_seeds_near_ties(out["seeds"], out["confidence"], g, tol)
    assert np.array_equal(out["final_labels"], g["final_labels"])
    np.testing.assert_allclose(out["final_trans"], g["final_trans"], atol=1e-4)


def test_power_iteration_kat():
    """Known-answer test after misc/eigen.py:9-67: power iteration on random
    symmetric non-negative matrices converges to numpy's leading eigenvector."""
    rng = np.random.RandomState(0)
    A = rng.rand(8, 20, 20).astype(np.float32)
    A = (A + A.transpose(0, 2, 1)) / 2
    v, _ = O.power_iteration(A, num_iterations=200)
    w, V = np.linalg.eigh(A.astype(np.float64))
    lead = np.abs(V[:, :, -1])
    np.testing.assert_allclose(v, lead, atol=1e-5)


def test_rigid_transform_recovers_pose():
    rng = np.random.RandomState(3)
    A = rng.rand(4, 50, 3).astype(np.float32)
    from pointdsc_amd.synthetic import random_rotation
    R = np.stack([random_rotation(rng) for _ in range(4)]).astype(np.float32)
    t = rng.rand(4, 3).astype(np.float32)
    B = np.einsum("bij,bnj->bni", R, A) + t[:, None]
    T = O.rigid_transform_3d(A, B.astype(np.float32), np.ones((4, 50), np.float32))
    np.testing.assert_allclose(T[:, :3, :3], R, atol=1e-5)
    np.testing.assert_allclose(T[:, :3, 3], t, atol=1e-5)


@pytest.mark.parametrize("name", ["train_small", "train_rel_1k", "train_kitti_1k", "train_mix"])
def test_training_forward_goldens(name):
    """The oracle's eval-mode training forward and SpectralMatchingLoss
    (models/PointDSC.py:158-191, libs/loss.py:115-139) against the reference's
    own outputs: seeds identical, logits / M rows within the fp32 noise of this
    2-layer network, the loss to fp32 resolution on the reference's M."""
    g = load_golden(name)
    sd = golden_state_dict(g)
    hp = golden_hparams(g)
    B, N = g["final_labels"].shape
    o = O.forward_training(g["corr_pos"], g["src_keypts"], g["tgt_keypts"], sd, hp["num_layers"],
                           inlier_threshold=hp["inlier_threshold"])
    Ms = o["M"]
    for b in range(B):
        assert np.array_equal(o["seeds"][b], g["seeds"][b])
        np.testing.assert_allclose(o["final_labels"][b], g["final_labels"][b], atol=1e-4)
        np.testing.assert_allclose(o["M"][b][:8], g["M_rows"][b], atol=1e-4)
        assert np.all(np.diagonal(o["M"][b]) == 0) and np.array_equal(np.diagonal(o["M"][b]), g["M_diag"][b])
        np.testing.assert_allclose(o["final_trans"][b], g["final_trans"][b], atol=1e-4)
    for balanced, key in ((True, "sm_loss_balanced"), (False, "sm_loss_mse")):
        np.testing.assert_allclose(O.spectral_matching_loss(np.stack(Ms), g["gt_labels"], balanced), g[key],
                                   rtol=2e-5)
        if "M" in g:
            np.testing.assert_allclose(O.spectral_matching_loss(g["M"], g["gt_labels"], balanced), g[key], rtol=2e-6)


@pytest.mark.parametrize("tag", ["bench_3dmatch_1k_tf", "bench_3dmatch_1k"])
def test_bench_pairs_golden(tag):
    """The oracle on bench.py's own pairs vs the reference's outputs on them
    (tools/gen_goldens.py run_bench): labels bit-exact and poses within 1e-4 on
    every pair whose seed ranking is tie-free (all 128 with the bench's rescaled
    classifier; the raw weights leave some pairs' seeds to tied zero scores)."""
    from pointdsc_amd.synthetic import BENCH_CLS, synthetic_pair, trained_state_dict
    g = load_golden(tag)
    sd = trained_state_dict(str(g["preset"]), 12, *(BENCH_CLS if tag.endswith("_tf") else ()))
    tied = g["n_nonpositive_seed_scores"] > 0
    for i in list(range(6)) + [int(np.nonzero(tied)[0][0])] if tied.any() else range(8):
        p = synthetic_pair(int(g["num_corr"]), int(g["pair_seed_base"]) + i, str(g["preset"]))
        r = O.forward_testing(p["corr_pos"], p["src_keypts"], p["tgt_keypts"], sd, num_layers=12)
        assert np.array_equal(r["final_labels"].astype(np.uint8), g["final_labels"][i]), i
        if not tied[i]:
            np.testing.assert_allclose(r["final_trans"], g["final_trans"][i], atol=1e-4, err_msg=str(i))
