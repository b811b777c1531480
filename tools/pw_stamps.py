#!/usr/bin/env python3
"""Where a small batch's pointwise-chain launch (pw_mid_kernel) and split-K
attention launch (attention_h3_kernel) spend their time: s_memtime stamps of
the diagnostic build (make -C pointdsc_amd/csrc variant V=stamps VFLAGS=-DATT_STAMPS).
Runs B pairs of N (default a single N = 1000 pair) and reads the stamps of the
last pw_mid and attention launches of one forward (every 16th workgroup).
Usage: PDSC_LIB_VARIANT=stamps python tools/pw_stamps.py [--pairs 1] [--num-corr 1000]"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
ST_PER_WAVE, ST_WGS = 256, 64


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pairs", type=int, default=1)
    ap.add_argument("--num-corr", type=int, default=1000)
    a = ap.parse_args()
    from pointdsc_amd import _lib, kernels
    from pointdsc_amd.PointDSC import PointDSC
    from pointdsc_amd.synthetic import BENCH_CLS, PRESETS, synthetic_batch, trained_state_dict
    dev = torch.device("cuda:0")
    p = PRESETS["3dmatch"]
    model = PointDSC(in_dim=6, num_layers=12, num_channels=128, num_iterations=10, ratio=0.1,
                     inlier_threshold=p["inlier_threshold"], sigma_d=p["sigma_d"], k=40, nms_radius=p["nms_radius"])
    model.load_state_dict({k: torch.from_numpy(v) for k, v in trained_state_dict("3dmatch", 12, *BENCH_CLS).items()})
    model = model.to(dev).eval()
    d = synthetic_batch(a.pairs, a.num_corr, seed=7000)
    corr, src, tgt = (torch.from_numpy(d[k]).to(dev) for k in ("corr_pos", "src_keypts", "tgt_keypts"))
    plan = kernels.ForwardPlan(model.pdsc_config(), model.packed_weights(), a.pairs, a.num_corr, dev)
    L = _lib.load()
    for _ in range(5):
        plan.run(corr, src, tgt)
    torch.cuda.synchronize()
    assert L.pdsc_diag_att_stamps_clear() == 0
    plan.run(corr, src, tgt)
    torch.cuda.synchronize()
    buf = np.zeros(ST_WGS * 4 * ST_PER_WAVE, np.uint64)
    assert L.pdsc_diag_att_stamps(buf.ctypes.data_as(ctypes.c_void_p), ctypes.c_size_t(buf.nbytes)) == 0
    st = buf.reshape(ST_WGS, 4, ST_PER_WAVE).astype(np.int64)
    rep = {}
    # wave 0 of each stamped workgroup (small-batch launches run 1-, 2- or 8-wave
    # workgroups; only waves 0-3 stamp, and wave 0 always exists)
    st = st[:, :1, :]
    pw = st[(st[:, :, 150] > 0).all(1) & (st[:, :, 159] > 0).all(1)]
    if len(pw):
        ghz = np.median((pw[:, :, 159] - pw[:, :, 150]) / (pw[:, :, 187] - pw[:, :, 186]) * 0.1)
        names = ["combine", "fc0", "fc3", "fc6", "pcn", "split+q panel", "q", "k", "v"]
        rep["pw_mid"] = {"workgroups": int(len(pw)), "clock_ghz": float(ghz),
                         "total_us": float(((pw[:, :, 187] - pw[:, :, 186]) / 100.0).mean()),
                         "phases_us": {nm: round(float(((pw[:, :, 151 + i] - pw[:, :, 150 + i]) / ghz / 1e3).mean()), 3)
                                       for i, nm in enumerate(names)}}
    at = st[(st[:, :, 160] > 0).all(1) & (st[:, :, 161] > 0).all(1)]
    if len(at):
        ghz = np.median((at[:, :, 161] - at[:, :, 160]) / (at[:, :, 185] - at[:, :, 184]) * 0.1)
        r0 = at[:, :, 184].min()
        rep["attention"] = {"workgroups": int(len(at)), "clock_ghz": float(ghz),
                            "total_us": float(((at[:, :, 185] - at[:, :, 184]) / 100.0).mean()),
                            "start_spread_us": float((at[:, :, 184].max() - r0) / 100.0),
                            "first_tile_top_us": float(((at[:, :, 1] - at[:, :, 160]) / ghz / 1e3).mean()),
                            "tile_cycles": [float((at[:, :, 1 + 6 * t + 5] - at[:, :, 1 + 6 * t]).mean()) for t in range(2)]}
    print(json.dumps(rep, indent=1))


if __name__ == "__main__":
    main()
