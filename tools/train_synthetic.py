#!/usr/bin/env python3
"""Train a synthetic stand-in for the release checkpoints (this container only).

The release weights (``snapshot/*/models/model_best.pkl``) are not in the
reference tree (``.MISSING_LARGE_BLOBS``).  Random weights make the
12-layer SCNonlocal encoder collapse every correspondence onto one feature
(mean cosine 0.999 at N=1000), so seeds and kNN become tie-dominated and no
fixture could pin the hot path.  This script trains the *reference* module
(``/root/reference/models/PointDSC.py``, training-mode forward) for a few
hundred Adam steps on synthetic pairs (``pointdsc_amd.synthetic``) with the
reference's losses restated: balanced BCE on the confidence logits
(``libs/loss.py:66-112``) + spectral-matching loss on M (``libs/loss.py:115-139``).
Output: ``tests/golden/weights_<preset>.npz`` (a fixture: data only).
Consumers that need tie-free seed scores rescale/shift the classifier's last
layer themselves (``pointdsc_amd.synthetic.trained_state_dict``).

Usage: PYTHONDONTWRITEBYTECODE=1 python tools/train_synthetic.py {3dmatch,kitti} [iters]
"""
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from pointdsc_amd.synthetic import PRESETS, synthetic_pair, synthetic_state_dict  # noqa: E402


def main(preset="3dmatch", iters=400, N=500, bs=4):
    import torch
    import torch.nn as nn
    sys.path.insert(0, "/root/reference")
    import models.PointDSC as refmod

    torch.manual_seed(0)
    torch.set_num_threads(8)
    p = PRESETS[preset]
    model = refmod.PointDSC(in_dim=6, num_layers=12, num_channels=128, num_iterations=10,
                            ratio=0.1, inlier_threshold=p["inlier_threshold"],
                            sigma_d=p["sigma_d"], k=40, nms_radius=p["nms_radius"])
    init = synthetic_state_dict(12, 128, seed=7, sigma_d=p["sigma_d"], cls_bias=0.0)
    model.load_state_dict({k: torch.from_numpy(v) for k, v in init.items()})
    opt = torch.optim.Adam([q for q in model.parameters() if q.requires_grad], lr=1e-3)
    rng = np.random.RandomState(1234)
    model.train()
    t0 = time.time()
    for it in range(iters):
        pairs = [synthetic_pair(N, int(rng.randint(1 << 30)), preset, float(rng.uniform(0.05, 0.5)))
                 for _ in range(bs)]
        data = {k: torch.from_numpy(np.stack([q[k] for q in pairs]))
                for k in ("corr_pos", "src_keypts", "tgt_keypts")}
        gt = torch.from_numpy(np.stack([q["gt_labels"] for q in pairs]))
        res = model(data)
        logits = res["final_labels"]
        num_pos = torch.relu(gt.sum() - 1) + 1
        num_neg = torch.relu((1 - gt).sum() - 1) + 1
        cls = nn.BCEWithLogitsLoss(pos_weight=num_neg / num_pos)(logits, gt)
        gM = ((gt[:, None, :] + gt[:, :, None]) == 2).float()
        gM = gM * (1 - torch.eye(N))[None]
        M = res["M"]
        smp = ((M - 1) ** 2 * gM).sum((-1, -2)) / (torch.relu(gM.sum((-1, -2)) - 1) + 1)
        smn = (M ** 2 * (1 - gM)).sum((-1, -2)) / (torch.relu((1 - gM).sum((-1, -2)) - 1) + 1)
        loss = cls + (0.5 * smp + 0.5 * smn).mean()
        opt.zero_grad()
        loss.backward()
        if all(torch.isfinite(q.grad).all() for q in model.parameters() if q.grad is not None):
            opt.step()
        if it % 25 == 0 or it == iters - 1:
            with torch.no_grad():
                acc = ((logits > 0).float() == gt).float().mean()
            print(f"[{preset}] it {it:4d} loss {loss.item():.4f} cls {cls.item():.4f} "
                  f"acc {acc.item():.3f} t {time.time() - t0:.0f}s", flush=True)
    model.eval()
    sd = {k: v.detach().numpy().copy() for k, v in model.state_dict().items()}
    out = os.path.join(REPO, "tests", "golden", f"weights_{preset}.npz")
    np.savez_compressed(out, **sd)
    print(f"wrote {out}")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "3dmatch",
         int(sys.argv[2]) if len(sys.argv) > 2 else 400)
