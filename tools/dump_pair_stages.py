#!/usr/bin/env python3
"""Stage-by-stage HIP outputs for chosen bench pairs (GPU box), to localise a
pose difference against the oracle (compare with tools/bench_parity.py here).

Runs the batched forward (debug: confidence, seeds) at the bench shape, then
the per-stage C entries on the chosen pairs: encoder (normed), seed kNN, NSM
weights, seed hypotheses, post-refinement.

Usage:  python tools/dump_pair_stages.py OUT.npz PAIR [PAIR ...] [--precision h3] [--unscaled]
"""
import argparse
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("out")
    ap.add_argument("pairs", type=int, nargs="+")
    ap.add_argument("--precision", default="h3")
    ap.add_argument("--unscaled", action="store_true")
    a = ap.parse_args()
    from pointdsc_amd import kernels
    from pointdsc_amd.PointDSC import PointDSC
    from pointdsc_amd.synthetic import BENCH_CLS, PRESETS, synthetic_pair, trained_state_dict
    p = PRESETS["3dmatch"]
    dev = torch.device("cuda:0")
    m = PointDSC(in_dim=6, num_layers=12, num_channels=128, num_iterations=10, ratio=0.1,
                 inlier_threshold=p["inlier_threshold"], sigma_d=p["sigma_d"], k=40, nms_radius=p["nms_radius"],
                 precision=a.precision)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in
                       trained_state_dict("3dmatch", 12, *(() if a.unscaled else BENCH_CLS)).items()})
    m = m.to(dev).eval()
    cfg, packed = m.pdsc_config(), m.packed_weights()
    ps = [synthetic_pair(1000, 1000 * 100003 + g) for g in range(128)]
    data = {k: torch.from_numpy(np.stack([q[k] for q in ps])).to(dev) for k in ("corr_pos", "src_keypts", "tgt_keypts")}
    T, L, conf, seeds = kernels.forward_testing(cfg, packed, data["corr_pos"], data["src_keypts"], data["tgt_keypts"],
                                                debug=True)
    out = {"pairs": np.array(a.pairs)}
    for i in a.pairs:
        c, s, t = (data[k][i:i + 1] for k in ("corr_pos", "src_keypts", "tgt_keypts"))
        sd_ = m.sigma_spat.detach()
        M = kernels.compat(s, t, sd_)
        feat, normed, conf1 = kernels.encoder(cfg, packed, c, M)
        sd1 = seeds[i:i + 1].contiguous()
        knn = kernels.seed_knn(normed, sd1, 40, a.precision)
        w, it = kernels.nsm_weights(normed, s, t, knn, 10, m.sigma.detach(), sd_, a.precision)
        st, fit, best, tr0, lab = kernels.seed_hypotheses(s, t, knn, w, p["inlier_threshold"])
        trf = kernels.post_refine(tr0, s, t, 0.10)
        for k, v in dict(T=T[i], L=L[i], conf=conf[i], seeds=seeds[i], feat=feat[0], normed=normed[0], conf1=conf1[0],
                         knn=knn[0], w=w[0], iters=it, seed_trans=st[0], fitness=fit[0], best=best, tr0=tr0[0],
                         lab=lab[0], trf=trf[0]).items():
            out[f"{k}_{i}"] = v.cpu().numpy()
    np.savez_compressed(a.out, **out)


if __name__ == "__main__":
    main()
