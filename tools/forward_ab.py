"""A/B timing of the batched testing forward (diagnostic): ms per forward for a
few (B, N) shapes in THIS process (plan knobs such as PDSC_OVERLAP come from
the environment; AB_SHAPES="8x5000,1x1000" picks the shapes).
Usage: python tools/forward_ab.py [reps]"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))


def main():
    from pointdsc_amd import kernels
    from pointdsc_amd.PointDSC import PointDSC
    from pointdsc_amd.synthetic import BENCH_CLS, PRESETS, synthetic_batch, trained_state_dict
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    dev = torch.device("cuda:0")
    p = PRESETS["3dmatch"]
    m = PointDSC(in_dim=6, num_layers=12, num_channels=128, num_iterations=10, ratio=0.1,
                 inlier_threshold=p["inlier_threshold"], sigma_d=p["sigma_d"], k=40, nms_radius=p["nms_radius"])
    m.load_state_dict({k: torch.from_numpy(v) for k, v in trained_state_dict("3dmatch", 12, *BENCH_CLS).items()})
    m = m.to(dev).eval()
    out = []
    shapes = [(128, 1000), (8, 5000), (1, 1000)]
    if os.environ.get("AB_SHAPES"):
        shapes = [tuple(int(v) for v in x.split("x")) for x in os.environ["AB_SHAPES"].split(",")]
    for B, N in shapes:
        d = synthetic_batch(B, N, seed=7)
        c, s, t = (torch.from_numpy(d[k]).to(dev) for k in ("corr_pos", "src_keypts", "tgt_keypts"))
        plan = kernels.ForwardPlan(m.pdsc_config(), m.packed_weights(), B, N, dev)
        for _ in range(3):
            plan.run(c, s, t)
        torch.cuda.synchronize(dev)
        if os.environ.get("AB_EVENTS") == "att":  # bench.py's per-attention-launch events on every forward
            import ctypes
            from pointdsc_amd import _lib
            hip = ctypes.CDLL("libamdhip64.so")
            n = reps * 12
            st, sp = (ctypes.c_void_p * n)(), (ctypes.c_void_p * n)()
            for arr in (st, sp):
                for i in range(n):
                    e = ctypes.c_void_p()
                    hip.hipEventCreate(ctypes.byref(e))
                    arr[i] = e.value
            cnt = ctypes.c_int32(0)
            _lib.load().pdsc_attention_timing(st, sp, n, ctypes.byref(cnt))
        t0 = time.perf_counter()
        for _ in range(reps):
            plan.run(c, s, t)
        torch.cuda.synchronize(dev)
        if os.environ.get("AB_EVENTS") == "att":
            _lib.load().pdsc_attention_timing(None, None, 0, None)
        out.append(f"{B}x{N}: {(time.perf_counter() - t0) / reps * 1e3:.3f} ms")
    print(os.environ.get("AB_TAG", ""), " | ".join(out), flush=True)


if __name__ == "__main__":
    main()
