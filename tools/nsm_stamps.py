#!/usr/bin/env python3
"""Where nsm_seed_kernel's waves spend their time: s_memtime stamps of the
diagnostic build (make -C pointdsc_amd/csrc variant V=stamps VFLAGS=-DATT_STAMPS)
of 64 evenly spaced workgroups, through the standalone NSM entry on random
unit features (k = 40, 10 iterations).  Segments: knn row load issue, P gather,
Gram (gathers + MFMA + LDS triangle), T = F o S, power iteration.
Usage: PDSC_LIB_VARIANT=stamps python tools/nsm_stamps.py [--pairs 128] [--num-corr 1000]"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
ST_PER_WAVE, ST_WGS = 256, 64


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pairs", type=int, default=128)
    ap.add_argument("--num-corr", type=int, default=1000)
    a = ap.parse_args()
    from pointdsc_amd import _lib, kernels
    dev = torch.device("cuda:0")
    B, N, k = a.pairs, a.num_corr, 40
    S = int(0.1 * N)
    g = torch.Generator().manual_seed(3)
    f = torch.randn((B, N, 128), generator=g)
    f = (f / f.norm(dim=-1, keepdim=True)).to(dev)
    src = torch.rand((B, N, 3), generator=g).to(dev)
    tgt = (src.cpu() + 0.01 * torch.randn((B, N, 3), generator=g)).to(dev)
    knn = torch.randint(0, N, (B, S, k), generator=g, dtype=torch.int32).to(dev)
    sig, sd = torch.tensor([1.0], device=dev), torch.tensor([0.1], device=dev)
    L = _lib.load()
    for _ in range(3):
        kernels.nsm_weights(f, src, tgt, knn, 10, sig, sd)
    torch.cuda.synchronize()
    assert L.pdsc_diag_nsm_stamps_clear() == 0
    kernels.nsm_weights(f, src, tgt, knn, 10, sig, sd)
    torch.cuda.synchronize()
    buf = np.zeros(ST_WGS * 4 * ST_PER_WAVE, np.uint64)
    assert L.pdsc_diag_nsm_stamps(buf.ctypes.data_as(ctypes.c_void_p), ctypes.c_size_t(buf.nbytes)) == 0
    st = buf.reshape(ST_WGS * 4, ST_PER_WAVE).astype(np.int64)
    st = st[(st[:, 0] > 0) & (st[:, 5] > 0) & (st[:, 17] > 0)]
    ghz = np.median((st[:, 5] - st[:, 0]) / (st[:, 17] - st[:, 16]) * 0.1)
    names = ["issue", "P gather", "Gram", "T build", "power iteration"]
    seg = {n: float(np.mean(st[:, i + 1] - st[:, i]) / ghz / 1e3) for i, n in enumerate(names)}
    r0 = st[:, 16].min()
    rep = {"pairs": B, "num_corr": N, "waves": int(st.shape[0]), "clock_ghz": float(ghz),
           "wave_us_mean": float(np.mean(st[:, 17] - st[:, 16]) / 100.0),
           "launch_span_us": float((st[:, 17].max() - r0) / 100.0),
           "start_us_pctl": [float(np.percentile((st[:, 16] - r0) / 100.0, q)) for q in (0, 25, 50, 75, 100)],
           "end_us_pctl": [float(np.percentile((st[:, 17] - r0) / 100.0, q)) for q in (0, 25, 50, 75, 90, 100)],
           "segments_us": seg}
    print(json.dumps(rep, indent=1))


if __name__ == "__main__":
    main()
