"""Bitwise equality of two library builds (diagnostic): every stage output of
the testing forward (kernels.forward_stages) for a few (B, N) shapes.
  PDSC_LIB_VARIANT=old python tools/variant_bits.py dump gpurun_out/old.npz
  python tools/variant_bits.py cmp gpurun_out/old.npz     (product library)
AB_SHAPES="128x1000,8x5000,1x1000" picks the shapes; both precisions run."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))


def stages():
    from pointdsc_amd import kernels
    from pointdsc_amd.PointDSC import PointDSC
    from pointdsc_amd.synthetic import BENCH_CLS, PRESETS, synthetic_batch, trained_state_dict
    dev = torch.device("cuda:0")
    p = PRESETS["3dmatch"]
    m = PointDSC(in_dim=6, num_layers=12, num_channels=128, num_iterations=10, ratio=0.1,
                 inlier_threshold=p["inlier_threshold"], sigma_d=p["sigma_d"], k=40, nms_radius=p["nms_radius"])
    m.load_state_dict({k: torch.from_numpy(v) for k, v in trained_state_dict("3dmatch", 12, *BENCH_CLS).items()})
    m = m.to(dev).eval()
    shapes = [(128, 1000), (8, 5000), (1, 1000)]
    if os.environ.get("AB_SHAPES"):
        shapes = [tuple(int(v) for v in x.split("x")) for x in os.environ["AB_SHAPES"].split(",")]
    res = {}
    for B, N in shapes:
        d = synthetic_batch(B, N, seed=11)
        c, s, t = (torch.from_numpy(d[k]).to(dev) for k in ("corr_pos", "src_keypts", "tgt_keypts"))
        for prec in ("h3", "f32"):
            out = kernels.forward_stages(m.pdsc_config(prec), m.packed_weights(prec), c, s, t, check_range=False)
            for k, v in out.items():
                res[f"{B}x{N}_{prec}_{k}"] = v.cpu().numpy()
    return res


def main():
    mode, path = sys.argv[1], sys.argv[2]
    res = stages()
    if mode == "dump":
        np.savez(path, **res)
        print(f"dumped {len(res)} arrays to {path}")
        return 0
    ref = np.load(path)
    bad = [k for k in res if k not in ref or res[k].tobytes() != ref[k].tobytes()]
    print(f"compared {len(res)} arrays: {len(bad)} differ {bad[:12]}")
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
