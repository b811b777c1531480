#!/usr/bin/env python3
"""Where a fused attention + chain launch (attn_pw2_kernel) spends its time:
s_memtime stamps of a diagnostic build (make -C pointdsc_amd/csrc variant V=stamps
VFLAGS=-DATT_STAMPS).  Runs the bench's headline batch (128 pairs x N=1000) and
reads the stamps of the last attn_pw2 launch of one forward (layer L-2): every
16th workgroup's 4 waves, per key tile (top, S ready, M + DMA waited, softmax done, PV
issued, barrier passed), then the chain phase.
Usage: PDSC_LIB_VARIANT=stamps python tools/att_stamps.py [--pairs 128] [--num-corr 1000]"""
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
    ap.add_argument("--pairs", type=int, default=128)
    ap.add_argument("--num-corr", type=int, default=1000)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    from pointdsc_amd import _lib, kernels
    from pointdsc_amd.PointDSC import PointDSC
    from pointdsc_amd.synthetic import BENCH_CLS, PRESETS, synthetic_pair, trained_state_dict
    dev = torch.device("cuda:0")
    p = PRESETS["3dmatch"]
    model = PointDSC(in_dim=6, num_layers=12, num_channels=128, num_iterations=10, ratio=0.1,
                     inlier_threshold=p["inlier_threshold"], sigma_d=p["sigma_d"], k=40, nms_radius=p["nms_radius"])
    model.load_state_dict({k: torch.from_numpy(v) for k, v in trained_state_dict("3dmatch", 12, *BENCH_CLS).items()})
    model = model.to(dev).eval()
    ps = [synthetic_pair(a.num_corr, 1000 * 100003 + g, "3dmatch") for g in range(a.pairs)]
    data = {k: np.stack([q[k] for q in ps]) for k in ps[0]}
    corr, src, tgt = (torch.from_numpy(data[k]).to(dev) for k in ("corr_pos", "src_keypts", "tgt_keypts"))
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
    ok = (st[:, :, 188] > 0) & (st[:, :, 189] > 0)
    st = st[ok.all(1)]
    cfirst = (st[:, :, 179] > 0).all(1)
    normal = ~cfirst & (st[:, :, 180] > 0).all(1)
    end_k = np.where(cfirst[:, None], 181, 180)
    tend = np.take_along_axis(st, end_k[:, :, None], 2)[:, :, 0]
    ghz = np.median((tend - st[:, :, 0]) / (st[:, :, 189] - st[:, :, 188]) * 0.1)
    r0 = st[:, :, 188].min()
    us = lambda c: c / ghz / 1e3
    rep = {"workgroups": int(st.shape[0]), "chain_first": int(cfirst.sum()), "clock_ghz": float(ghz),
           "launch_us": float((st[:, :, 189].max() - r0) / 100.0),
           "wg_real_us": [[round(float((st[i, 0, 188] - r0) / 100), 1), round(float((st[i, :, 189].max() - r0) / 100), 1)]
                          for i in np.argsort(st[:, 0, 188])]}
    if normal.any():
        n = st[normal]
        rep["normal"] = {"attention_us": float(us(n[:, :, 170] - n[:, :, 0]).mean()),
                         "glue_us": float(us(n[:, :, 171] - n[:, :, 170]).mean()),
                         "chain_us": float(us(n[:, :, 180] - n[:, :, 171]).mean()),
                         "chain_layers_us": {nm: float(us(n[:, :, b] - n[:, :, a]).mean()) for nm, a, b in
                                             [("fc0", 171, 172), ("fc3", 172, 173), ("fc6", 173, 174), ("pcn", 174, 175),
                                              ("q", 175, 176), ("k", 176, 177), ("v", 177, 178), ("tail", 178, 180)]}}
        # the chain's weight chunks (w2_layer): MFMAs, the sync (DMA wait + barrier), and
        # the gap to the next chunk (epilogues, stores, the next layer's setup)
        ch = []
        for c in range(11):
            i0, i1, i2 = 192 + 3 * c, 193 + 3 * c, 194 + 3 * c
            if not (n[:, :, i2] > 0).all():
                break
            nxt = 192 + 3 * (c + 1) if c < 10 and (n[:, :, 192 + 3 * (c + 1)] > 0).all() else 180
            ch.append({"chunk": c, "mma_us": round(float(us(n[:, :, i1] - n[:, :, i0]).mean()), 3),
                       "sync_us": round(float(us(n[:, :, i2] - n[:, :, i1]).mean()), 3),
                       "after_us": round(float(us(n[:, :, nxt] - n[:, :, i2]).mean()), 3)})
        rep["normal"]["chain_chunks"] = ch
    if cfirst.any():
        c = st[cfirst]
        rep["chain_first"] = {"chain_us": float(us(c[:, :, 179] - c[:, :, 0]).mean()),
                              "attention_us": float(us(c[:, :, 181] - c[:, :, 179]).mean())}
    nt = 23
    idx = 1 + 6 * np.arange(nt)
    names = ["mfma wait (S)", "vmcnt (M+DMA)", "softmax", "pv issue", "barrier"]
    seg = {names[k]: (st[:, :, idx + k + 1] - st[:, :, idx + k]).astype(np.float64) for k in range(5)}
    seg["loop"] = (st[:, :, idx[1:]] - st[:, :, idx[:-1] + 5]).astype(np.float64)
    rep["per_tile_cycles"] = {k: {"mean": round(float(v.mean()), 1), "p10": float(np.percentile(v, 10)),
                                  "p90": float(np.percentile(v, 90))} for k, v in seg.items()}
    rep["per_tile_cycles_first_tile"] = {k: round(float(v[:, :, 0].mean()), 1) for k, v in seg.items() if k != "loop"}
    tile = (st[:, :, idx + 5] - st[:, :, idx]).astype(np.float64)
    rep["tile_cycles_mean"] = float(tile.mean())
    print(json.dumps(rep, indent=1))
    if a.out:
        np.save(a.out, st)


if __name__ == "__main__":
    main()
