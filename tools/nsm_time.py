#!/usr/bin/env python3
"""Device time of the standalone NSM entry (nsm_seed + nsm_finish) on random
unit features, k = 40, 10 iterations, for A/B of nsm_seed variants
(PDSC_LIB_VARIANT).  Usage: python tools/nsm_time.py [reps]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from pointdsc_amd import kernels
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 50
    dev = torch.device("cuda:0")
    out = []
    for B, N in ((128, 1000), (8, 5000), (1, 1000)):
        S, k = int(0.1 * N), 40
        g = torch.Generator().manual_seed(3)
        f = torch.randn((B, N, 128), generator=g)
        f = (f / f.norm(dim=-1, keepdim=True)).to(dev)
        src = torch.rand((B, N, 3), generator=g).to(dev)
        tgt = (src.cpu() + 0.01 * torch.randn((B, N, 3), generator=g)).to(dev)
        knn = torch.randint(0, N, (B, S, k), generator=g, dtype=torch.int32).to(dev)
        sig, sd = torch.tensor([1.0], device=dev), torch.tensor([0.1], device=dev)
        for _ in range(3):
            kernels.nsm_weights(f, src, tgt, knn, 10, sig, sd)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            kernels.nsm_weights(f, src, tgt, knn, 10, sig, sd)
        e1.record()
        torch.cuda.synchronize()
        out.append(f"{B}x{N}: {e0.elapsed_time(e1) / reps * 1e3:.1f} us")
    print(os.environ.get("PDSC_LIB_VARIANT", "-"), " | ".join(out), flush=True)


if __name__ == "__main__":
    main()
