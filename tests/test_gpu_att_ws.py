"""The tiny plan's wave-split attention (attention_h3_ws_kernel: a key split's
tiles spread over 4 waves, each wave's K and V halves refilled a tile ahead,
the waves merged through LDS into one partial) against the one-wave kernel it
replaces (knob PDSC_ATT_WS=1), run with -m gpu.

Both compute each query's softmax over the same keys; only the fp32 order in
which a split's tiles are summed differs (per-wave runs merged by 2^(m_w - m*)).
Per shape: the forward's logits agree within 1e-4 x (1 + max |logit|), no NaN,
labels equal, and poses within 1e-4 -- or, where the two summation orders
decided a seed / kNN near-tie differently, BOTH results held to the oracle by
the near-tie rule (conftest.assert_held_to_oracle), as the other cross-plan
tests do."""
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

from conftest import assert_held_to_oracle

pytestmark = pytest.mark.gpu

# single pairs whose tiny plan has splits of >= 4 key tiles (the wave-split
# kernel's rule); 1 x 1000 is the bench's single pair, 1 x 990 a ragged last tile
CASES = [(1, 1000), (1, 1024), (1, 990), (2, 500)]


def _model_sd():
    from pointdsc_amd.PointDSC import PointDSC
    from pointdsc_amd.synthetic import BENCH_CLS, PRESETS, trained_state_dict
    p = PRESETS["3dmatch"]
    m = PointDSC(in_dim=6, num_layers=12, num_channels=128, num_iterations=10, ratio=0.1,
                 inlier_threshold=p["inlier_threshold"], sigma_d=p["sigma_d"], k=40, nms_radius=p["nms_radius"])
    sd = trained_state_dict("3dmatch", 12, *BENCH_CLS)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
    return m, sd


def _data(i, B, N):
    from pointdsc_amd.synthetic import synthetic_batch
    return synthetic_batch(B, N, seed=500 + i)


def _dump(path):
    from pointdsc_amd import kernels
    dev = torch.device("cuda:0")
    m, _ = _model_sd()
    m = m.to(dev).eval()
    out = {}
    for i, (B, N) in enumerate(CASES):
        d = _data(i, B, N)
        c, s, t = (torch.from_numpy(d[k]).to(dev) for k in ("corr_pos", "src_keypts", "tgt_keypts"))
        with torch.no_grad():
            st = kernels.forward_stages(m.pdsc_config(), m.packed_weights(), c, s, t)
        for k in ("conf", "seeds", "knn", "final_trans", "final_labels"):
            out[f"{k}{i}"] = st[k].cpu().numpy()
    np.savez(path, **out)


def test_wave_split_matches_one_wave(gpu_device, tmp_path):
    here = os.path.dirname(os.path.abspath(__file__))
    res = {}
    for knob in ("1", "4"):
        path = tmp_path / f"ws_{knob}.npz"
        code = f"import sys; sys.path[:0] = [{here!r}, {os.path.dirname(here)!r}]; " \
               f"import test_gpu_att_ws as t; t._dump({str(path)!r})"
        subprocess.run([sys.executable, "-c", code], env=dict(os.environ, PDSC_ATT_WS=knob), check=True, timeout=300)
        res[knob] = np.load(path)
    _, sd = _model_sd()
    for i, (B, N) in enumerate(CASES):
        a, b = res["1"][f"conf{i}"], res["4"][f"conf{i}"]
        assert np.isfinite(a).all() and np.isfinite(b).all(), (B, N)
        err = float(np.abs(a - b).max())
        assert err <= 1e-4 * (1.0 + float(np.abs(a).max())), f"B={B} N={N}: logits {err:.3g}"
        d = _data(i, B, N)
        for p in range(B):
            what = f"B={B} N={N} pair {p}"
            assert np.array_equal(res["1"][f"final_labels{i}"][p], res["4"][f"final_labels{i}"][p]), what
            dT = float(np.abs(res["1"][f"final_trans{i}"][p] - res["4"][f"final_trans{i}"][p]).max())
            if dT <= 1e-4:
                continue
            q = {k: d[k][p] for k in ("corr_pos", "src_keypts", "tgt_keypts")}
            for knob in ("1", "4"):
                r = res[knob]
                assert_held_to_oracle(q, r[f"final_labels{i}"][p], r[f"final_trans{i}"][p], r[f"conf{i}"][p],
                                      r[f"seeds{i}"][p], r[f"knn{i}"][p], sd, f"{what} WS={knob} (dT {dT:.3g})",
                                      num_layers=12)
