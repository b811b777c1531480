#!/usr/bin/env python3
"""Generate golden vectors from the *reference* PointDSC (this container only).

Runs ``/root/reference/models/PointDSC.py`` unchanged (CPU, eval, no_grad,
one torch thread) on synthetic inputs from ``pointdsc_amd.synthetic``, records the hot path's intermediates by wrapping
the reference's own functions, and writes small ``.npz`` fixtures (data only:
inputs, expected outputs) under ``tests/golden/``.  Weights: the trained
synthetic stand-in checkpoint (``tools/train_synthetic.py`` ->
``tests/golden/weights_<preset>.npz``) truncated to ``num_layers`` with the
classifier's last layer rescaled by a power of two and shifted so every logit
lies in [1, ~33] (positive, finely resolved seed scores); scale, shift and a
sha256 of the exact state dict are stored.  The reference never leaves this
container.

Usage:  PYTHONDONTWRITEBYTECODE=1 python tools/gen_goldens.py [case ...]
"""
import hashlib
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from pointdsc_amd.synthetic import PRESETS, synthetic_pair, trained_state_dict  # noqa: E402

REF = "/root/reference"

# name: (num_layers, N, preset, pair seed, inlier ratio, store_M, store_T)
CASES = {
    "small_3dm":    (2, 256, "3dmatch", 11, 0.3, True, True),
    "small_kitti":  (2, 300, "kitti", 12, 0.3, True, True),
    "tiny_k":       (2, 30, "3dmatch", 13, 0.3, True, True),     # k = N-1 = 29 < 40, N % 4 != 0
    "tiny_out":     (2, 64, "3dmatch", 14, 0.0, True, True),     # all outliers
    "rel_1k":       (12, 1000, "3dmatch", 21, 0.3, False, True),
    "rel_1k_kitti": (12, 1000, "kitti", 22, 0.3, False, False),
    "odd_777":      (12, 777, "3dmatch", 25, 0.2, False, False),
    "rel_5k":       (12, 5000, "3dmatch", 23, 0.3, False, False),
    "rel_5k_lo":    (12, 5000, "3dmatch", 24, 0.06, False, False),  # FPFH-like inlier ratio
    "rel_5k_kitti": (12, 5000, "kitti", 26, 0.3, False, False),     # BASELINE configs[4] shape
    # rank-deficient neighbourhoods: 60 copies of one inlier correspondence and
    # 60 collinear inliers (rigid_transform_3d's H of rank 0 / 1, common.py:7-45)
    "degen_1k":     (12, 1000, "3dmatch", 27, 0.3, False, False),
    "out_5k":       (12, 5000, "3dmatch", 28, 0.0, False, False),   # all outliers at full size
    # evaluation/test_KITTI.py:151 builds up to num_node=12000 correspondences
    "kitti_12k":    (12, 12000, "kitti", 29, 0.3, False, False),
}

# cases whose inputs are edited after synthetic_pair (name -> function(pair) -> pair)
def _degenerate(pair):
    src, tgt, gt = pair["src_keypts"].copy(), pair["tgt_keypts"].copy(), pair["gt_trans"].astype(np.float64)
    inl = np.nonzero(pair["gt_labels"] > 0)[0]
    dup, line = inl[1:61], inl[61:121]
    src[dup], tgt[dup] = src[inl[0]], tgt[inl[0]]                  # duplicates of inlier inl[0]
    p0, d = src[inl[0]].astype(np.float64), np.array([0.6, -0.3, 0.74])
    pts = p0 + np.linspace(-0.8, 0.8, len(line))[:, None] * d / np.linalg.norm(d)
    src[line] = pts.astype(np.float32)                             # collinear inliers
    tgt[line] = (pts @ gt[:3, :3].T + gt[:3, 3]).astype(np.float32)
    corr = np.concatenate([src, tgt], axis=-1)
    return dict(pair, src_keypts=src, tgt_keypts=tgt, corr_pos=(corr - corr.mean(0)).astype(np.float32))


MUTATE = {"degen_1k": _degenerate}

# layer-0 inputs wider than corr_pos (datasets/ThreeDMatch.py:303-315): name -> in_dim.
# 9: [src, tgt, src - tgt] (src, tgt centred here); 70: centred [src, tgt] + both 32-d
# descriptors (FCGF's width: 6 + 2 x 32).  The descriptors are synthetic FCGF-like
# unit vectors; an inlier's target descriptor is its source descriptor plus noise,
# renormalised, an outlier's an independent draw.  layer0: the trained [128, 6]
# columns for corr_pos, seeded random columns for the rest.
WIDE = {"wide9_1k": 9, "wide70_1k": 70}
CASES["wide9_1k"] = (12, 1000, "3dmatch", 33, 0.3, False, False)
CASES["wide70_1k"] = (12, 1000, "3dmatch", 32, 0.3, False, False)


def _unit_rows(x):
    return x / np.linalg.norm(x, axis=1, keepdims=True)


def wide_inputs(pair, in_dim, seed):
    """The reference's layer-0 input for in_dim 9 / 70 (ThreeDMatch.py:308-315)."""
    src, tgt = pair["src_keypts"], pair["tgt_keypts"]
    if in_dim == 9:  # (src, tgt centred as the 6 / 70 branches do: the trained columns' distribution)
        c = np.concatenate([src, tgt], axis=-1)
        return np.concatenate([c - c.mean(0), src - tgt], axis=-1).astype(np.float32), {}
    rng = np.random.RandomState(seed + 1000)
    n = src.shape[0]
    sdesc = _unit_rows(rng.randn(n, 32))
    tdesc = _unit_rows(rng.randn(n, 32))
    inl = pair["gt_labels"] > 0
    tdesc[inl] = _unit_rows(sdesc[inl] + rng.normal(0.0, 0.1, size=sdesc[inl].shape))
    sdesc, tdesc = sdesc.astype(np.float32), tdesc.astype(np.float32)
    corr_pos = np.concatenate([src, tgt], axis=-1)
    corr_pos = corr_pos - corr_pos.mean(0)
    return np.concatenate([corr_pos, sdesc, tdesc], axis=-1).astype(np.float32), dict(src_desc=sdesc, tgt_desc=tdesc)


def wide_layer0(sd_np, in_dim, seed):
    """layer0 [128, in_dim, 1]: the trained corr_pos columns, seeded random others."""
    rng = np.random.RandomState(seed + 2000)
    w6 = sd_np["encoder.layer0.weight"]
    extra = rng.randn(w6.shape[0], in_dim - 6, 1) / np.sqrt(in_dim)
    if in_dim == 9:  # src - tgt is metres-scale for outliers: keep the trained columns dominant
        extra = extra * 0.1
    return np.concatenate([w6, extra.astype(np.float32)], axis=1).astype(np.float32)
STORE_FEATURES_MAX_N = 5000  # larger cases keep the logits, not the [N, 128] features


def weights_digest(sd):
    h = hashlib.sha256()
    for k, v in sd.items():
        h.update(k.encode())
        h.update(np.ascontiguousarray(v).tobytes())
    return h.hexdigest()


def run_case(name):
    L, N, preset, pseed, ratio, store_M, store_T = CASES[name]
    C = 128
    import torch
    sys.path.insert(0, REF)
    import models.PointDSC as refmod

    torch.set_num_threads(1 if N <= 5000 else os.cpu_count())
    p = PRESETS[preset]
    pair = synthetic_pair(N, pseed, preset, ratio)
    if name in MUTATE:
        pair = MUTATE[name](pair)
    in_dim, extra_out = WIDE.get(name, 6), {}
    if in_dim != 6:
        wide_corr, extra_out = wide_inputs(pair, in_dim, pseed)
        pair = dict(pair, corr_pos=wide_corr)
    sd_np = trained_state_dict(preset, L)
    if in_dim != 6:
        l0w = wide_layer0(sd_np, in_dim, pseed)
        sd_np["encoder.layer0.weight"] = l0w
    # ctor exactly as evaluation/test_3DMatch.py:215-224 / test_KITTI.py:280-290
    model = refmod.PointDSC(in_dim=in_dim, num_layers=L, num_channels=C, num_iterations=10,
                            ratio=0.1, inlier_threshold=p["inlier_threshold"],
                            sigma_d=p["sigma_d"], k=40, nms_radius=p["nms_radius"])
    model.load_state_dict({k: torch.from_numpy(v) for k, v in sd_np.items()}, strict=True)
    model.eval()
    with torch.no_grad():  # classifier shift so that min logit >= 1 on this pair
        x = {k: torch.from_numpy(pair[k])[None] for k in ("corr_pos", "src_keypts", "tgt_keypts")}
        sdist = torch.norm(x["src_keypts"][:, :, None] - x["src_keypts"][:, None], dim=-1)
        tdist = torch.norm(x["tgt_keypts"][:, :, None] - x["tgt_keypts"][:, None], dim=-1)
        Mc = torch.clamp(1.0 - (sdist - tdist) ** 2 / model.sigma_spat ** 2, min=0)
        logits = model.classification(model.encoder(x["corr_pos"].permute(0, 2, 1), Mc))
        lo, hi = logits.min().item(), logits.max().item()
    m = max(0, int(np.ceil(np.log2(max(abs(lo), abs(hi), 1e-3) / 16.0))))
    scale = float(2.0 ** -m)
    shift = float(np.ceil(max(0.0, 1.0 - lo * scale)))
    sd_np = trained_state_dict(preset, L, shift, scale)
    if in_dim != 6:
        sd_np["encoder.layer0.weight"] = l0w
        extra_out["layer0_weight"] = l0w
    model.load_state_dict({k: torch.from_numpy(v) for k, v in sd_np.items()}, strict=True)

    rec = {"rigid_calls": []}
    orig_knn, orig_rigid = refmod.knn, refmod.rigid_transform_3d

    def knn_wrap(x, k, ignore_self=False, normalized=True):
        idx = orig_knn(x, k, ignore_self=ignore_self, normalized=normalized)
        rec["knn_full"] = idx.clone()
        return idx

    def rigid_wrap(A, B, weights=None, weight_threshold=0):
        out = orig_rigid(A, B, weights, weight_threshold)
        rec["rigid_calls"].append(out.clone())
        return out

    refmod.knn, refmod.rigid_transform_3d = knn_wrap, rigid_wrap
    o_pick, o_eig, o_seed = model.pick_seeds, model.cal_leading_eigenvector, model.cal_seed_trans

    def pick_wrap(dists, scores, R, max_num):
        s = o_pick(dists, scores, R, max_num)
        rec["seeds"] = s.clone()
        rel = (scores.T >= scores) | (dists[0] >= R)
        rec["is_local_max"] = rel.min(-1)[0].float().clone()
        return s

    def eig_wrap(M, method="power"):
        rec["T"] = M.clone()
        out = o_eig(M, method)
        rec["leading_eig"] = out.clone()
        return out

    def seed_wrap(*a):
        out = o_seed(*a)
        rec["seed_out"] = [t.clone() for t in out]
        return out

    model.pick_seeds, model.cal_leading_eigenvector, model.cal_seed_trans = pick_wrap, eig_wrap, seed_wrap
    hooks = [model.encoder.register_forward_hook(lambda m, i, o: rec.__setitem__("enc", o.clone())),
             model.classification.register_forward_hook(lambda m, i, o: rec.__setitem__("conf", o.clone()))]

    data = {k: torch.from_numpy(pair[k])[None] for k in ("corr_pos", "src_keypts", "tgt_keypts")}
    data["testing"] = True
    with torch.no_grad():
        res = model(data)
        src = data["src_keypts"]
        tgt = data["tgt_keypts"]
        sd = torch.norm(src[:, :, None, :] - src[:, None, :, :], dim=-1)
        M = torch.clamp(1.0 - (sd - torch.norm(tgt[:, :, None, :] - tgt[:, None, :, :], dim=-1)) ** 2
                        / model.sigma_spat ** 2, min=0)
    for h in hooks:
        h.remove()
    refmod.knn, refmod.rigid_transform_3d = orig_knn, orig_rigid

    seeds = rec["seeds"][0].numpy().astype(np.int64)
    seed_trans, fitness, trans0, labels0 = [t.numpy() for t in rec["seed_out"]]
    out = dict(
        num_layers=L, num_channels=C, preset=preset, pair_seed=pseed, cls_bias_shift=shift, cls_scale=scale,
        inlier_ratio=ratio, weights_sha256=weights_digest(sd_np),
        sigma_d=p["sigma_d"], inlier_threshold=p["inlier_threshold"], nms_radius=p["nms_radius"],
        corr_pos=pair["corr_pos"], src_keypts=pair["src_keypts"], tgt_keypts=pair["tgt_keypts"],
        gt_trans=pair["gt_trans"], gt_labels=pair["gt_labels"],
        corr_features=rec["enc"][0].numpy().T.copy() if N <= STORE_FEATURES_MAX_N else np.zeros((0, C), np.float32),
        confidence=rec["conf"][0, 0].numpy(),                   # [N]
        is_local_max=rec["is_local_max"].numpy(),               # [N]
        seeds=seeds,                                            # [S]
        knn_idx=rec["knn_full"][0].numpy()[seeds].astype(np.int64),   # [S, k]
        leading_eig=rec["leading_eig"].numpy(),                 # [S, k]
        seed_trans=seed_trans[0], seed_fitness=fitness[0],
        trans_pre_refine=trans0[0], final_labels=res["final_labels"][0].numpy(),
        final_trans=res["final_trans"][0].numpy(),
        refine_trans=np.stack([t[0].numpy() for t in rec["rigid_calls"][1:]])
        if len(rec["rigid_calls"]) > 1 else np.zeros((0, 4, 4), np.float32),
        M_row_sums=M[0].double().sum(-1).numpy(), M_diag=torch.diagonal(M[0]).numpy(),
        in_dim=in_dim, **extra_out,
    )
    if store_M:
        out["M"] = M[0].numpy()
    if store_T:
        out["T"] = rec["T"].numpy()
    assert np.array_equal(labels0[0], out["final_labels"])
    # tie-freeness of the seed ranking: seeds have positive, distinct scores
    sc = (out["confidence"] * out["is_local_max"])[seeds]
    out["seed_score_min_gap"] = float(np.min(-np.diff(sc))) if len(sc) > 1 else 1.0
    out["seed_score_min"] = float(sc.min())
    path = os.path.join(REPO, "tests", "golden", f"{name}.npz")
    np.savez_compressed(path, **out)
    print(f"{name}: N={N} S={len(seeds)} refine_iters={len(out['refine_trans'])} "
          f"min_gap={out['seed_score_min_gap']:.3g} min_score={out['seed_score_min']:.3g} "
          f"labels={int(out['final_labels'].sum())} -> {os.path.relpath(path, REPO)} "
          f"({os.path.getsize(path) / 1e3:.0f} kB)")


def run_training(name, L, N, B, preset, pseed, ratio):
    """The reference's TRAINING-mode forward (no 'testing' key, models/PointDSC.py:158-163,
    176, 182, 189-191) on B pairs at once, plus SpectralMatchingLoss (libs/loss.py:115-139),
    balanced and not, against the pairs' ground-truth labels."""
    import torch
    sys.path.insert(0, REF)
    import models.PointDSC as refmod
    from libs.loss import SpectralMatchingLoss
    torch.set_num_threads(1)
    p = PRESETS[preset]
    ratios = ratio if isinstance(ratio, tuple) else (ratio,) * B
    pairs = [synthetic_pair(N, pseed * 1000 + b, preset, ratios[b]) for b in range(B)]
    sd_np = trained_state_dict(preset, L, 10.0, 1.0)  # classifier shift: distinct positive logits
    model = refmod.PointDSC(in_dim=6, num_layers=L, num_channels=128, num_iterations=10, ratio=0.1,
                            inlier_threshold=p["inlier_threshold"], sigma_d=p["sigma_d"], k=40,
                            nms_radius=p["nms_radius"])
    model.load_state_dict({k: torch.from_numpy(v) for k, v in sd_np.items()}, strict=True)
    model.eval()
    rec = {}
    o_seed = model.cal_seed_trans

    def seed_wrap(seeds, *a):
        rec["seeds"] = seeds.clone()
        out = o_seed(seeds, *a)
        rec["seed_out"] = [t.clone() for t in out]
        return out

    model.cal_seed_trans = seed_wrap
    data = {k: torch.from_numpy(np.stack([q[k] for q in pairs])) for k in ("corr_pos", "src_keypts", "tgt_keypts")}
    gt = torch.from_numpy(np.stack([q["gt_labels"] for q in pairs]))
    with torch.no_grad():
        res = model(data)
        loss_b = SpectralMatchingLoss(balanced=True)(res["M"], gt).item()
        loss_u = SpectralMatchingLoss(balanced=False)(res["M"], gt).item()
    M = res["M"].numpy()
    out = dict(num_layers=L, preset=preset, pair_seed=pseed, inlier_ratio=np.array(ratios), weights_sha256=weights_digest(sd_np),
               cls_bias_shift=10.0, cls_scale=1.0, sigma_d=p["sigma_d"], inlier_threshold=p["inlier_threshold"],
               nms_radius=p["nms_radius"],
               corr_pos=data["corr_pos"].numpy(), src_keypts=data["src_keypts"].numpy(),
               tgt_keypts=data["tgt_keypts"].numpy(), gt_labels=gt.numpy(),
               final_trans=res["final_trans"].numpy(), final_labels=res["final_labels"].numpy(),
               seeds=rec["seeds"].numpy().astype(np.int64), seed_fitness=rec["seed_out"][1].numpy(),
               M_row_sums=M.astype(np.float64).sum(-1), M_diag=np.diagonal(M, axis1=1, axis2=2).copy(),
               M_rows=M[:, :8].copy(), sm_loss_balanced=loss_b, sm_loss_mse=loss_u)
    if N <= 300:
        out["M"] = M
    path = os.path.join(REPO, "tests", "golden", f"train_{name}.npz")
    np.savez_compressed(path, **out)
    print(f"train_{name}: B={B} N={N} L={L} loss balanced {loss_b:.6g} mse {loss_u:.6g} -> "
          f"{os.path.relpath(path, REPO)} ({os.path.getsize(path) / 1e3:.0f} kB)")


def run_bench(preset="3dmatch", P=128, N=1000, shift=0.0, scale=1.0):
    """The reference's testing forward on bench.py's own headline pairs: pair g
    seeded 1000*100003+g (bench.py), N=1000, the UNSHIFTED trained synthetic
    weights (classifier shift/scale as trained_state_dict; bench.py's tie-free
    variant BENCH_CLS = (15, 2^-5) puts every logit of these pairs in [0.6, 16]).
    Stores per pair: final_trans, final_labels, confidence, is_local_max, seeds
    and the seed-ranking tie margins (seed scores are conf * is_local_max,
    models/PointDSC.py:216-217: with negative logits the zero scores of
    non-maxima tie), so the GPU tests can tell a genuine pose
    error from a tie the reference breaks arbitrarily."""
    import torch
    sys.path.insert(0, REF)
    import models.PointDSC as refmod
    torch.set_num_threads(os.cpu_count())
    p = PRESETS[preset]
    sd_np = trained_state_dict(preset, 12, shift, scale)
    model = refmod.PointDSC(in_dim=6, num_layers=12, num_channels=128, num_iterations=10, ratio=0.1,
                            inlier_threshold=p["inlier_threshold"], sigma_d=p["sigma_d"], k=40,
                            nms_radius=p["nms_radius"])
    model.load_state_dict({k: torch.from_numpy(v) for k, v in sd_np.items()}, strict=True)
    model.eval()
    rec = {}
    o_pick = model.pick_seeds

    def pick_wrap(dists, scores, R, max_num):
        s = o_pick(dists, scores, R, max_num)
        rec["seeds"] = s.clone()
        rec["is_local_max"] = ((scores.T >= scores) | (dists[0] >= R)).min(-1)[0].float().clone()
        return s

    model.pick_seeds = pick_wrap
    hook = model.classification.register_forward_hook(lambda m, i, o: rec.__setitem__("conf", o.clone()))
    keys = ("final_trans", "final_labels", "confidence", "is_local_max", "seeds")
    out = {k: [] for k in keys}
    for g in range(P):
        pair = synthetic_pair(N, 1000 * 100003 + g, preset)
        data = {k: torch.from_numpy(pair[k])[None] for k in ("corr_pos", "src_keypts", "tgt_keypts")}
        data["testing"] = True
        with torch.no_grad():
            res = model(data)
        out["final_trans"].append(res["final_trans"][0].numpy())
        out["final_labels"].append(res["final_labels"][0].numpy().astype(np.uint8))
        out["confidence"].append(rec["conf"][0, 0].numpy())
        out["is_local_max"].append(rec["is_local_max"].numpy().astype(np.uint8))
        out["seeds"].append(rec["seeds"][0].numpy().astype(np.int32))
    hook.remove()
    out = {k: np.stack(v) for k, v in out.items()}
    sc = out["confidence"] * out["is_local_max"]
    out["n_nonpositive_seed_scores"] = np.array([(sc[g][out["seeds"][g]] <= 0).sum() for g in range(P)])
    tag = f"bench_{preset}_{N // 1000}k" + ("_tf" if shift else "")
    path = os.path.join(REPO, "tests", "golden", f"{tag}.npz")
    np.savez_compressed(path, preset=preset, num_corr=N, pairs=P, cls_bias_shift=shift, cls_scale=scale,
                        pair_seed_base=1000 * 100003, weights_sha256=weights_digest(sd_np), **out)
    print(f"{tag}: {P} pairs, pairs with non-positive seed scores: "
          f"{int((out['n_nonpositive_seed_scores'] > 0).sum())} -> {os.path.relpath(path, REPO)} "
          f"({os.path.getsize(path) / 1e3:.0f} kB)")


TRAIN_CASES = {"small": (2, 256, 2, "3dmatch", 41, 0.3), "rel_1k": (12, 1000, 2, "3dmatch", 42, 0.3),
               "kitti_1k": (12, 1000, 1, "kitti", 43, 0.2),
               # pairs that converge after different numbers of power iterations: the
               # batch-global allclose exit (models/PointDSC.py:354) differs from a per-pair one
               "mix": (12, 400, 6, "3dmatch", 44, (0.0, 0.05, 0.3, 0.6, 0.9, 0.15))}


def run_kabsch():
    """The reference's rigid_transform_3d (models/common.py:7-45, LAPACK SVD on the
    CPU) on degenerate inputs: all-zero and negative weights (H = 0: LAPACK's
    U = V = I, so R = I), three points, coplanar points (rank-2 H: R unique),
    and rank-1 H (collinear or duplicated points: R is LAPACK's choice among a
    one-parameter family -- recorded, compared by properties only)."""
    import torch
    sys.path.insert(0, REF)
    from models.common import rigid_transform_3d
    rng = np.random.RandomState(31)
    from pointdsc_amd.synthetic import random_rotation
    cases = {}

    def add(name, A, w, kind):
        R = random_rotation(rng)
        B = (A.astype(np.float64) @ R.T + rng.uniform(-1, 1, 3)).astype(np.float32)
        with torch.no_grad():
            T = rigid_transform_3d(torch.from_numpy(A)[None], torch.from_numpy(B)[None],
                                   torch.from_numpy(w)[None]).numpy()[0]
        cases[name] = (A, B, w, T, kind)

    n = 40
    A = rng.rand(n, 3).astype(np.float32)
    add("zero_weights", A, np.zeros(n, np.float32), "pinned")
    add("negative_weights", A, -rng.rand(n).astype(np.float32), "pinned")
    add("three_points", rng.rand(3, 3).astype(np.float32), rng.rand(3).astype(np.float32), "pinned")
    P = rng.rand(n, 3).astype(np.float32)
    P[:, 2] = 0.5
    add("coplanar", P, rng.rand(n).astype(np.float32), "pinned")
    L = (rng.rand(1, 3) + np.linspace(0, 1, n)[:, None] * np.array([[0.3, -0.5, 0.8]])).astype(np.float32)
    add("collinear", L, rng.rand(n).astype(np.float32), "properties")
    D = np.repeat(rng.rand(1, 3), n, axis=0).astype(np.float32)
    add("duplicates", D, rng.rand(n).astype(np.float32), "properties")
    out = {}
    for i, (k, (A, B, w, T, kind)) in enumerate(cases.items()):
        out[f"{k}__A"], out[f"{k}__B"], out[f"{k}__w"], out[f"{k}__T"] = A, B, w, T
        out[f"{k}__pinned"] = np.array(kind == "pinned")
    path = os.path.join(REPO, "tests", "golden", "kabsch_degenerate.npz")
    np.savez_compressed(path, **out)
    print(f"kabsch_degenerate: {len(cases)} cases -> {os.path.relpath(path, REPO)}")


if __name__ == "__main__":
    names = sys.argv[1:] or list(CASES) + ["kabsch"] + ["train_" + t for t in TRAIN_CASES]
    for n in names:
        if n == "kabsch":
            run_kabsch()
        elif n.startswith("bench_"):  # bench_<preset>[_tf]: the bench's weights [tie-free variant]
            from pointdsc_amd.synthetic import BENCH_CLS
            parts = n.split("_")
            run_bench(parts[1], **(dict(shift=BENCH_CLS[0], scale=BENCH_CLS[1]) if parts[-1] == "tf" else {}))
        elif n.startswith("train_"):
            run_training(n[6:], *TRAIN_CASES[n[6:]])
        else:
            run_case(n)
