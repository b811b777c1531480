"""Diagnostic: encoder feature / logit error against fp64, as a multiple of the
case's fp32 envelope, for single pairs and 40-pair batches (the pw / pw2 plans).
Run on the GPU box with the plan knobs (PDSC_FUSE, PDSC_PW2, ...) in the env."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
from conftest import fp32_envelope, golden_hparams, golden_names, golden_state_dict, load_golden  # noqa: E402


def main():
    from pointdsc_amd import kernels
    from pointdsc_amd.PointDSC import PointDSC
    dev = torch.device("cuda:0")
    names = sys.argv[1:] or golden_names()
    for name in names:
        g = load_golden(name)
        hp = golden_hparams(g)
        m = PointDSC(in_dim=hp["in_dim"], num_layers=hp["num_layers"], num_channels=128, num_iterations=10,
                     ratio=0.1, inlier_threshold=hp["inlier_threshold"], sigma_d=float(g["sigma_d"]), k=40,
                     nms_radius=hp["nms_radius"])
        m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in golden_state_dict(g).items()})
        m = m.to(dev).eval()
        e_f, e_c, f64, c64, mx = fp32_envelope(g, golden_state_dict(g), dev)
        for B in (1, 40):
            rep = lambda a: torch.from_numpy(np.ascontiguousarray(np.repeat(a[None], B, 0))).to(dev, torch.float32)
            corr, src, tgt = rep(g["corr_pos"]), rep(g["src_keypts"]), rep(g["tgt_keypts"])
            M = kernels.compat(src, tgt, m.sigma_spat)
            feat, _, conf = kernels.encoder(m.pdsc_config(), m.packed_weights(), corr, M)
            of = np.abs(feat[0].double().cpu().numpy() - f64).max() / mx
            oc = np.abs(conf[0].double().cpu().numpy() - c64).max()
            print(f"{name:14s} B={B:2d} in_dim={hp['in_dim']:2d} feat {of:.3g} ({of / e_f:.2f}x env {e_f:.3g}) "
                  f"logit {oc:.3g} ({oc / e_c:.2f}x env {e_c:.3g})", flush=True)


if __name__ == "__main__":
    main()
