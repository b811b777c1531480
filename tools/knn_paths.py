"""Which knn_select path each seed row takes in a single-pair testing forward
(diagnostic; needs the -DKNN_DIAG variant build: make -C pointdsc_amd/csrc
variant V=knndiag VFLAGS=-DKNN_DIAG, run with PDSC_LIB_VARIANT=knndiag).
Usage: python tools/knn_paths.py N [seed]"""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))


def main():
    from pointdsc_amd import _lib, kernels
    from pointdsc_amd.PointDSC import PointDSC
    from pointdsc_amd.synthetic import BENCH_CLS, PRESETS, synthetic_batch, trained_state_dict
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 5000
    seed = int(sys.argv[2]) if len(sys.argv) > 2 else 7000
    B = int(sys.argv[3]) if len(sys.argv) > 3 else 1
    dev = torch.device("cuda:0")
    p = PRESETS["3dmatch"]
    m = PointDSC(in_dim=6, num_layers=12, num_channels=128, num_iterations=10, ratio=0.1,
                 inlier_threshold=p["inlier_threshold"], sigma_d=p["sigma_d"], k=40, nms_radius=p["nms_radius"])
    m.load_state_dict({k: torch.from_numpy(v) for k, v in trained_state_dict("3dmatch", 12, *BENCH_CLS).items()})
    m = m.to(dev).eval()
    d = synthetic_batch(B, N, seed=seed)
    c, s, t = (torch.from_numpy(d[k]).to(dev) for k in ("corr_pos", "src_keypts", "tgt_keypts"))
    L = _lib.load()
    fn = L.pdsc_diag_knn_paths
    fn.argtypes, fn.restype = [ctypes.c_void_p, ctypes.c_int], ctypes.c_int
    buf = (ctypes.c_uint * 8)()
    plan = kernels.ForwardPlan(m.pdsc_config(), m.packed_weights(), B, N, dev)
    plan.run(c, s, t)
    torch.cuda.synchronize()
    fn(buf, 1)
    plan.run(c, s, t)
    torch.cuda.synchronize()
    fn(buf, 1)
    names = ["bitonic", "readlane", "radix_fallback", "hist_passes", "small_bin"]
    print(f"B={B} N={N} seed={seed} S={int(N * 0.1)} per forward:", {n: buf[i] for i, n in enumerate(names)}, flush=True)


if __name__ == "__main__":
    main()
