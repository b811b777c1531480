"""A single-pair testing forward (bs = 1, the reference drivers' call shape),
run REPS times eagerly through ForwardPlan on a synthetic pair of N
correspondences -- the program tools/single_pair_timeline.sh profiles (kernel
trace) to get the per-launch timeline of one forward."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    from pointdsc_amd import kernels
    from pointdsc_amd.PointDSC import PointDSC
    from pointdsc_amd.synthetic import BENCH_CLS, PRESETS, synthetic_batch, trained_state_dict
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    dev = torch.device("cuda:0")
    p = PRESETS["3dmatch"]
    m = PointDSC(in_dim=6, num_layers=12, num_channels=128, num_iterations=10, ratio=0.1,
                 inlier_threshold=p["inlier_threshold"], sigma_d=p["sigma_d"], k=40, nms_radius=p["nms_radius"])
    m.load_state_dict({k: torch.from_numpy(v) for k, v in trained_state_dict("3dmatch", 12, *BENCH_CLS).items()})
    m = m.to(dev).eval()
    d = synthetic_batch(1, N, seed=7000)
    c, s, t = (torch.from_numpy(d[k]).to(dev) for k in ("corr_pos", "src_keypts", "tgt_keypts"))
    plan = kernels.ForwardPlan(m.pdsc_config(), m.packed_weights(), 1, N, dev)
    for _ in range(reps):
        plan.run(c, s, t)
    torch.cuda.synchronize()
    print(f"single pair N={N}: {reps} forwards", flush=True)


if __name__ == "__main__":
    main()
