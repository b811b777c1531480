#!/usr/bin/env python3
"""Dump the HIP path's outputs on bench.py's own headline pairs (GPU box).

The bench's 128 pairs (N=1000, pair g seeded 1000*100003+g, trained synthetic
weights) through both precision modes, with the debug outputs (confidence,
seeds).  The npz is compared against the reference here (tools/bench_parity.py).

Usage:  python tools/dump_bench_pairs.py OUT.npz [--pairs 128] [--num-corr 1000] [--preset 3dmatch]
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
    ap.add_argument("--pairs", type=int, default=128)
    ap.add_argument("--num-corr", type=int, default=1000)
    ap.add_argument("--preset", default="3dmatch")
    ap.add_argument("--unscaled", action="store_true", help="the raw trained weights (tied seed scores)")
    a = ap.parse_args()
    from pointdsc_amd import kernels
    from pointdsc_amd.PointDSC import PointDSC
    from pointdsc_amd.synthetic import BENCH_CLS, PRESETS, synthetic_pair, trained_state_dict
    p = PRESETS[a.preset]
    dev = torch.device("cuda:0")
    model = PointDSC(in_dim=6, num_layers=12, num_channels=128, num_iterations=10, ratio=0.1,
                     inlier_threshold=p["inlier_threshold"], sigma_d=p["sigma_d"], k=40, nms_radius=p["nms_radius"])
    model.load_state_dict({k: torch.from_numpy(v) for k, v in trained_state_dict(a.preset, 12, *(() if a.unscaled else BENCH_CLS)).items()})
    model = model.to(dev).eval()
    ps = [synthetic_pair(a.num_corr, 1000 * 100003 + g, a.preset) for g in range(a.pairs)]
    data = {k: np.stack([q[k] for q in ps]) for k in ps[0]}
    corr, src, tgt = (torch.from_numpy(data[k]).to(dev) for k in ("corr_pos", "src_keypts", "tgt_keypts"))
    out = {}
    for prec in ("h3", "f32"):
        model.precision = prec
        tr, lab, conf, seeds = kernels.forward_testing(model.pdsc_config(), model.packed_weights(), corr, src, tgt,
                                                       debug=True)
        torch.cuda.synchronize()
        out[f"{prec}_trans"], out[f"{prec}_labels"] = tr.cpu().numpy(), lab.cpu().numpy()
        out[f"{prec}_conf"], out[f"{prec}_seeds"] = conf.cpu().numpy(), seeds.cpu().numpy()
    d = np.abs(out["h3_trans"] - out["f32_trans"]).reshape(a.pairs, -1).max(1)
    print("max pose diff h3 vs f32:", float(d.max()), "at pair", int(d.argmax()),
          "| pairs > 1e-4:", np.nonzero(d > 1e-4)[0].tolist())
    np.savez_compressed(a.out, **out)


if __name__ == "__main__":
    main()
