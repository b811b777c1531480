#!/usr/bin/env python3
"""Dump the HIP encoder's features / logits on one golden case (diagnostics).
Usage: python tools/dump_encoder.py <golden> <out.npz> [h3|f32]"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from conftest import golden_hparams, golden_state_dict, load_golden  # noqa: E402


def main():
    from pointdsc_amd import kernels
    from pointdsc_amd.PointDSC import PointDSC
    name, out = sys.argv[1], sys.argv[2]
    prec = sys.argv[3] if len(sys.argv) > 3 else "h3"
    g = load_golden(name)
    hp = golden_hparams(g)
    dev = torch.device("cuda:0")
    m = PointDSC(num_layers=hp["num_layers"], inlier_threshold=hp["inlier_threshold"], sigma_d=float(g["sigma_d"]),
                 nms_radius=hp["nms_radius"], precision=prec)
    m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in golden_state_dict(g).items()})
    m = m.to(dev).eval()
    corr, src, tgt = (torch.from_numpy(g[k][None]).to(dev) for k in ("corr_pos", "src_keypts", "tgt_keypts"))
    M = kernels.compat(src, tgt, m.sigma_spat)
    feat, normed, conf = kernels.encoder(m.pdsc_config(), m.packed_weights(), corr, M)
    np.savez(out, feat=feat[0].cpu().numpy(), conf=conf[0].cpu().numpy())


if __name__ == "__main__":
    main()
