"""The stream-K form of the split path's attention (attention_w64_sk_kernel:
one round of one workgroup per CU over all (query block, key tile) pairs) against
the split grid it replaces (knob PDSC_W64_SK=0), run with -m gpu.

Both plans compute each query's softmax over the same keys; only the key ranges
of the partials (and so the fp32 order of the combine) differ.  Per shape: the
forward's logits agree within 1e-4 x (1 + max |logit|), no NaN, and the slot
count pdsc_attention_layout reports is what each plan stores (shapes where
stream-K needs more slots than the split grid, and fewer)."""
import ctypes
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

# (B, N): 8 x 5000 is the bench's N = 5000 leg; 24 x 1500 stores 3 slots where
# the split grid stores 1; 9 x 5000 zero-fills a 4th slot; 16 x 2500 a third
CASES = [(8, 5000), (24, 1500), (9, 5000), (16, 2500)]


def _dump(path):
    from pointdsc_amd import _lib, kernels
    from pointdsc_amd.PointDSC import PointDSC
    from pointdsc_amd.synthetic import BENCH_CLS, PRESETS, synthetic_batch, trained_state_dict
    dev = torch.device("cuda:0")
    p = PRESETS["3dmatch"]
    m = PointDSC(in_dim=6, num_layers=12, num_channels=128, num_iterations=10, ratio=0.1,
                 inlier_threshold=p["inlier_threshold"], sigma_d=p["sigma_d"], k=40, nms_radius=p["nms_radius"])
    m.load_state_dict({k: torch.from_numpy(v) for k, v in trained_state_dict("3dmatch", 12, *BENCH_CLS).items()})
    m = m.to(dev).eval()
    out = {}
    for i, (B, N) in enumerate(CASES):
        plan, npad, ns = ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int32()
        _lib.check(_lib.load().pdsc_encoder_plan(B, N, 0, ctypes.byref(plan)), "encoder_plan")
        _lib.check(_lib.load().pdsc_attention_layout(B, N, 0, ctypes.byref(npad), ctypes.byref(ns)), "layout")
        d = synthetic_batch(B, N, seed=300 + i)
        c, s, t = (torch.from_numpy(d[k]).to(dev) for k in ("corr_pos", "src_keypts", "tgt_keypts"))
        with torch.no_grad():
            st = kernels.forward_stages(m.pdsc_config(), m.packed_weights(), c, s, t)
        out[f"conf{i}"] = st["conf"].cpu().numpy()
        out[f"plan{i}"] = np.array([plan.value, ns.value])
    np.savez(path, **out)


def test_stream_k_matches_split_grid(gpu_device, tmp_path):
    here = os.path.dirname(os.path.abspath(__file__))
    res = {}
    for knob in ("0", "1"):
        path = tmp_path / f"sk_{knob}.npz"
        code = f"import sys; sys.path[:0] = [{here!r}, {os.path.dirname(here)!r}]; " \
               f"import test_gpu_w64_sk as t; t._dump({str(path)!r})"
        subprocess.run([sys.executable, "-c", code], env=dict(os.environ, PDSC_W64_SK=knob), check=True, timeout=300)
        res[knob] = np.load(path)
    for i, (B, N) in enumerate(CASES):
        a, b = res["0"][f"conf{i}"], res["1"][f"conf{i}"]
        assert res["0"][f"plan{i}"][0] == 2 and res["1"][f"plan{i}"][0] == 2, (B, N)  # the split path
        assert np.isfinite(a).all() and np.isfinite(b).all(), (B, N)
        err = float(np.abs(a - b).max())
        assert err <= 1e-4 * (1.0 + float(np.abs(a).max())), f"B={B} N={N}: {err:.3g}"
    ns0 = [int(res["0"][f"plan{i}"][1]) for i in range(len(CASES))]
    ns1 = [int(res["1"][f"plan{i}"][1]) for i in range(len(CASES))]
    assert ns0 == [3, 1, 4, 3] and ns1 == [3, 3, 4, 3], (ns0, ns1)
