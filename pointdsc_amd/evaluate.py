"""Registration evaluation harness, sharded over GPUs.

Per-pair statistics rows with the columns of evaluation/test_3DMatch.py:90-101
(and test_KITTI.py:118-129, whose column 11 is the ICP time instead of the
scene index):

  0 success  1 RE (deg)  2 TE (cm)  3 input inlier #  4 input inlier ratio
  5 output inlier #  6 precision  7 recall  8 f1  9 model time  10 data time
  11 scene index

RE/TE/success follow libs/loss.py:12-59 (TransformationLoss; thresholds
re_thre/te_thre from config.py:111-129: 15 deg / 30 cm for 3DMatch, 5 deg /
60 cm for KITTI); precision/recall/f1 follow libs/loss.py:62-111
(ClassificationLoss on pred_labels > 0, sklearn's zero_division=0 result).
All statistics of a batch are computed at once on the device the poses live
on; they are O(N) per pair and not on the hot path.

Aggregation follows test_3DMatch.py:138-176: per-scene means (RE/TE over the
successful pairs only), the mean over scenes, and the all-pair means.  Across
ranks the rows are all-gathered (pointdsc_amd.dist.gather_rows) so the
all-pair means are exact; the reference's KITTI driver instead all-reduces
per-rank averages (test_KITTI.py:169-185), which weighs ranks equally.
"""
import math

import numpy as np
import torch

COLUMNS = ["success", "re_deg", "te_cm", "input_inliers", "input_inlier_ratio", "output_inliers",
           "precision", "recall", "f1", "model_time", "data_time", "scene"]
THRESHOLDS = {"3dmatch": (15.0, 30.0), "kitti": (5.0, 60.0)}  # (re_thre deg, te_thre cm)


def pair_stats(trans, gt_trans, pred_labels, gt_labels, re_thre=15.0, te_thre=30.0, counts=None):
    """[B, 9] float64 rows (columns 0-8) for a batch of B pairs.

    trans, gt_trans [B,4,4]; pred_labels, gt_labels [B,N] (0/1); counts: each
    pair's correspondences when the batch is ragged (labels zero-padded past
    them), else every pair has N."""
    trans, gt_trans = trans.float(), gt_trans.float()
    R, t = trans[:, :3, :3], trans[:, :3, 3]
    gR, gt_t = gt_trans[:, :3, :3], gt_trans[:, :3, 3]
    # libs/loss.py:44-49: acos(clamp((tr(R^T R_gt) - 1)/2)) in deg, |t - t_gt| in cm
    tr = torch.diagonal(R.transpose(1, 2) @ gR, dim1=1, dim2=2).sum(-1)
    re = torch.acos(torch.clamp((tr - 1) / 2.0, min=-1, max=1)) * 180 / np.pi
    te = torch.sqrt(torch.sum((t - gt_t) ** 2, dim=-1)) * 100
    success = ((te < te_thre) & (re < re_thre)).double()
    gt = gt_labels > 0
    pred = pred_labels > 0
    n_in = gt.sum(-1).double()
    tp = (gt & pred).sum(-1).double()
    n_pred = pred.sum(-1).double()
    precision = torch.where(n_pred > 0, tp / n_pred.clamp(min=1), torch.zeros_like(tp))
    recall = torch.where(n_in > 0, tp / n_in.clamp(min=1), torch.zeros_like(tp))
    denom = precision + recall
    f1 = torch.where(denom > 0, 2 * precision * recall / denom.clamp(min=1e-300), torch.zeros_like(tp))
    if counts is None:
        ratio = gt_labels.float().mean(-1).double()  # torch.mean of the 0/1 labels
    else:
        # the same fp32 sum / count the unpadded mean computes
        ratio = (n_in.float() / torch.as_tensor(counts, dtype=torch.float32, device=n_in.device)).double()
    return torch.stack([success, re.double(), te.double(), n_in, ratio, tp, precision, recall, f1], dim=1)


def _mean_success_only(stats, col):
    ok = stats[:, 0] == 1
    return float(stats[ok, col].mean()) if ok.any() else math.nan


def aggregate(stats, n_scenes=None):
    """Scene-level and all-pair summaries of [P, 12] rows (numpy float64),
    as test_3DMatch.py:141-176 logs them."""
    stats = np.asarray(stats, dtype=np.float64)
    out = {"pairs": int(stats.shape[0])}
    scenes = sorted(set(stats[:, 11].astype(int).tolist())) if n_scenes is None else list(range(n_scenes))
    vals = []
    for s in scenes:
        st = stats[stats[:, 11].astype(int) == s]
        if len(st) == 0:
            continue
        v = st.mean(0)
        v[1], v[2] = _mean_success_only(st, 1), _mean_success_only(st, 2)
        vals.append(v)
    if vals:
        avg = np.stack(vals).mean(0)
        out["scene_mean"] = {c: float(avg[i]) for i, c in enumerate(COLUMNS[:11])}
    allp = stats.mean(0)
    out["all_pairs"] = {c: float(allp[i]) for i, c in enumerate(COLUMNS[:11])}
    out["all_pairs"]["re_deg"] = _mean_success_only(stats, 1)
    out["all_pairs"]["te_cm"] = _mean_success_only(stats, 2)
    return out


def report_lines(stats, n_scenes=None):
    """The summary lines evaluation/test_3DMatch.py:141-176 logs, from [P, 12] rows:
    per scene, the mean over scenes and the all-pair means (same wording and
    rounding, so the logs of the two builds diff line by line)."""
    stats = np.asarray(stats, dtype=np.float64)
    scenes = sorted(set(stats[:, 11].astype(int).tolist())) if n_scenes is None else list(range(n_scenes))
    lines, vals = [], []
    for i, s in enumerate(scenes):
        st = stats[stats[:, 11].astype(int) == s]
        if len(st) == 0:
            continue
        v = st.mean(0)
        v[1], v[2] = _mean_success_only(st, 1), _mean_success_only(st, 2)
        vals.append(v)
        lines.append(f"Scene {i}th: Reg Recall={v[0] * 100:.2f}%  Mean RE={v[1]:.2f}  Mean TE={v[2]:.2f}  "
                     f"Mean Precision={v[6] * 100:.2f}%  Mean Recall={v[7] * 100:.2f}%  Mean F1={v[8] * 100:.2f}%")
    if vals:
        a = np.stack(vals).mean(0)
        lines += [f"All {len(vals)} scenes, Mean Reg Recall={a[0] * 100:.2f}%, Mean Re={a[1]:.2f}, Mean Te={a[2]:.2f}",
                  f"\tInput:  Mean Inlier Num={a[3]:.2f}(ratio={a[4] * 100:.2f}%)",
                  f"\tOutput: Mean Inlier Num={a[5]:.2f}(precision={a[6] * 100:.2f}%, recall={a[7] * 100:.2f}%, "
                  f"f1={a[8] * 100:.2f}%)",
                  f"\tMean model time: {a[9]:.2f}s, Mean data time: {a[10]:.2f}s"]
    p = stats.mean(0)
    ok = stats[:, 0] == 1
    c = stats[ok].mean(0) if ok.any() else np.full(stats.shape[1], np.nan)
    lines += ["*" * 40,
              f"All {stats.shape[0]} pairs, Mean Reg Recall={p[0] * 100:.2f}%, Mean Re={c[1]:.2f}, Mean Te={c[2]:.2f}",
              f"\tInput:  Mean Inlier Num={p[3]:.2f}(ratio={p[4] * 100:.2f}%)",
              f"\tOutput: Mean Inlier Num={p[5]:.2f}(precision={p[6] * 100:.2f}%, recall={p[7] * 100:.2f}%, "
              f"f1={p[8] * 100:.2f}%)",
              f"\tMean model time: {p[9]:.2f}s, Mean data time: {p[10]:.2f}s"]
    return lines


def save_outputs(stats, log_path=None, npy_path=None, n_scenes=None):
    """The driver's outputs (test_3DMatch.py:238-241): the summary log and, with
    --save_npy, the [P, 12] float64 stats matrix (np.save, no pickle)."""
    if log_path:
        with open(log_path, "w") as f:
            f.write("\n".join(report_lines(stats, n_scenes)) + "\n")
    if npy_path:
        np.save(npy_path, np.asarray(stats, dtype=np.float64), allow_pickle=False)


def pair_sizes(n_pairs, num_corr, seed=0):
    """Per-pair correspondence counts: num_corr for every pair, or, for a (lo, hi)
    range, pair i's count drawn from U{lo..hi} by its own seed (so every rank
    and every batching of the job sees the same sizes) -- the varying N of the
    reference's evaluation sets (datasets/ThreeDMatch.py:268-290)."""
    if isinstance(num_corr, int):
        return [num_corr] * n_pairs
    lo, hi = (int(x) for x in num_corr)
    return [int(np.random.RandomState(seed * 100003 + i + 7).randint(lo, hi + 1)) for i in range(n_pairs)]


def evaluate_synthetic(model, n_pairs, num_corr, preset="3dmatch", batch=16, seed=0, device=None,
                       inlier_ratio=0.3):
    """Sharded evaluation over n_pairs synthetic pairs: rank r evaluates pairs
    r, r+W, ... in batches through the batched forward (the ragged forward,
    PointDSC.forward_list, when num_corr is a (lo, hi) range of sizes), then the
    [n_pairs, 12] stats matrix is all-gathered.  Returns (stats numpy, summary dict)."""
    import time
    from . import dist, kernels
    from .synthetic import synthetic_pair
    rank, W = dist.world()
    mine = dist.shard_indices(n_pairs, rank, W)
    sizes = pair_sizes(n_pairs, num_corr, seed)
    re_thre, te_thre = THRESHOLDS[preset]
    rows = []
    for b0 in range(0, len(mine), batch):
        idx = mine[b0:b0 + batch]
        t0 = time.perf_counter()
        ps = [synthetic_pair(sizes[i], seed * 100003 + i, preset=preset, inlier_ratio=inlier_ratio) for i in idx]
        counts = [sizes[i] for i in idx]
        ragged = len(set(counts)) > 1
        if ragged:
            corr, src, tgt, gtL = (kernels.pad_pairs([torch.from_numpy(p[k][:, None] if p[k].ndim == 1 else p[k])
                                                      for p in ps])[0].to(device)
                                   for k in ("corr_pos", "src_keypts", "tgt_keypts", "gt_labels"))
            gtL = gtL[..., 0]
            gtT = torch.from_numpy(np.stack([p["gt_trans"] for p in ps])).to(device)
        else:
            corr, src, tgt, gtT, gtL = (torch.from_numpy(np.stack([p[k] for p in ps])).to(device)
                                        for k in ("corr_pos", "src_keypts", "tgt_keypts", "gt_trans", "gt_labels"))
        if device is not None and device.type == "cuda":
            torch.cuda.synchronize(device)
        t_data = (time.perf_counter() - t0) / len(idx)
        t0 = time.perf_counter()
        if ragged:
            T, L = model.forward_padded(corr, src, tgt, counts)
        else:
            T, L = model.forward_batched(corr, src, tgt)
        if device is not None and device.type == "cuda":
            torch.cuda.synchronize(device)
        t_model = (time.perf_counter() - t0) / len(idx)
        st = pair_stats(T, gtT, L, gtL, re_thre, te_thre, counts if ragged else None).cpu()
        extra = torch.tensor([[t_model, t_data, 0.0]], dtype=torch.float64).expand(len(idx), 3)
        rows.append(torch.cat([st, extra], dim=1))
    mine_rows = torch.cat(rows) if rows else torch.zeros((0, 12), dtype=torch.float64)
    grp = torch.distributed.is_available() and torch.distributed.is_initialized()
    gdev = device if (grp and device is not None and device.type == "cuda") else None
    allrows = dist.gather_rows(mine_rows, n_pairs, device=gdev).cpu().numpy()
    return allrows, aggregate(allrows)


def main():
    """torchrun entry: python -m torch.distributed.run --nproc-per-node W
    -m pointdsc_amd.evaluate --pairs 256 --num-corr 1000"""
    import argparse
    import json
    import os
    import torch.distributed as tdist
    from .PointDSC import PointDSC
    from .synthetic import PRESETS, trained_state_dict
    ap = argparse.ArgumentParser()
    ap.add_argument("--pairs", type=int, default=64)
    ap.add_argument("--num-corr", default="1000", help="N, or LO:HI for per-pair sizes in that range (ragged batches)")
    ap.add_argument("--preset", default="3dmatch", choices=list(PRESETS))
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--inlier-ratio", type=float, default=0.3)
    ap.add_argument("--log", default=None, help="write the test_3DMatch.py-style summary log here")
    ap.add_argument("--save-npy", default=None, help="np.save the [P, 12] per-pair stats here")
    a = ap.parse_args()
    W = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    grp = W > 1 or "RANK" in os.environ  # launched by torchrun: RCCL even for one rank
    if grp:
        tdist.init_process_group("nccl", init_method="env://")
    p = PRESETS[a.preset]
    m = PointDSC(num_layers=12, inlier_threshold=p["inlier_threshold"], sigma_d=p["sigma_d"],
                 nms_radius=p["nms_radius"])
    m.load_state_dict({k: torch.from_numpy(v) for k, v in trained_state_dict(a.preset).items()})
    m = m.to(dev).eval()
    nc = tuple(int(x) for x in a.num_corr.split(":")) if ":" in a.num_corr else int(a.num_corr)
    stats, summary = evaluate_synthetic(m, a.pairs, nc, a.preset, a.batch, device=dev,
                                        inlier_ratio=a.inlier_ratio)
    if not tdist.is_initialized() or tdist.get_rank() == 0:
        save_outputs(stats, a.log, a.save_npy)
        print(json.dumps(summary))
    if grp:
        tdist.destroy_process_group()


if __name__ == "__main__":
    main()
