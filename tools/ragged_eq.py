"""Diagnostic: uniform forward vs the ragged entry with every count N, per B
(prints bitwise equality and the largest pose difference per stage output)."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))


def main():
    from pointdsc_amd import kernels
    from pointdsc_amd.PointDSC import PointDSC
    from pointdsc_amd.synthetic import BENCH_CLS, PRESETS, synthetic_batch, trained_state_dict
    dev = torch.device("cuda:0")
    p = PRESETS["3dmatch"]
    m = PointDSC(in_dim=6, num_layers=12, num_channels=128, num_iterations=10, ratio=0.1,
                 inlier_threshold=p["inlier_threshold"], sigma_d=p["sigma_d"], k=40, nms_radius=p["nms_radius"])
    m.load_state_dict({k: torch.from_numpy(v) for k, v in trained_state_dict("3dmatch", 12, *BENCH_CLS).items()})
    m = m.to(dev).eval()
    for B in (24, 64, 65, 128):
        d = synthetic_batch(B, 1000, seed=83)
        c, s, t = (torch.from_numpy(d[k]).to(dev) for k in ("corr_pos", "src_keypts", "tgt_keypts"))
        u = kernels.forward_stages(m.pdsc_config(), m.packed_weights(), c, s, t, check_range=False)
        T, L, st = kernels.forward_ragged(m.pdsc_config(), m.packed_weights(), c, s, t, [1000] * B, debug=True,
                                          check_range=False)
        r = dict(st, final_trans=T, final_labels=L)
        out = []
        for k in ("conf", "seeds", "knn", "weights", "final_trans", "final_labels"):
            a, b = u[k], r[k]
            eq = torch.equal(a, b)
            diff = (a.float() - b.float()).abs().max().item()
            npairs = int((a.float() - b.float()).abs().flatten(1).max(1).values.gt(0).sum().item())
            out.append(f"{k} eq={eq} maxdiff={diff:.3g} pairs={npairs}")
        print(f"B={B}: " + " | ".join(out), flush=True)


if __name__ == "__main__":
    main()
