"""The other forms of a5 give exactly the compare kernels' bits: the opt-in
sorted forms (seeds.hip: bitonic-sorted NMS window and seed ranking, knob
PDSC_SEED_SORT=1, measurement only) and the default select form of the ranking
(radix-selected threshold + candidate ranking, seed_select_kernel; knob
PDSC_SEED_SELECT=0 for the compare kernel): is_local_max and the seed list, on
tie-heavy scores, -0 / +0 scores, negative local maxima and duplicate points,
and ties at the threshold wider than the candidate buffer (run with -m gpu)."""
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

CASES = [(3, 1000, 100, 0.1), (2, 5000, 500, 0.1), (1, 777, 77, 0.6), (4, 64, 6, 0.05), (1, 6000, 600, 1e-3),
         (2, 3000, 300, 0.02), (1, 9000, 4000, 0.02), (2, 2000, 1999, 0.0)]


def _inputs(B, N, seed):
    rng = np.random.RandomState(seed)
    src = (rng.rand(B, N, 3) * 3).astype(np.float32)
    idx = np.arange(0, N - 1, 17)
    src[:, idx] = src[:, idx + 1]  # duplicate points
    conf = np.round(rng.randn(B, N) * 4).astype(np.float32)  # many exact ties
    conf[:, ::5] = 0.0
    conf[:, 1::11] = -0.0
    return src, conf


def _dump(path):
    from pointdsc_amd import kernels
    dev = torch.device("cuda:0")
    out = {}
    for i, (B, N, S, R) in enumerate(CASES):
        src, conf = _inputs(B, N, 100 + i)
        seeds, lm = kernels.pick_seeds(torch.from_numpy(src).to(dev), torch.from_numpy(conf).to(dev), R, S)
        out[f"seeds{i}"], out[f"lm{i}"] = seeds.cpu().numpy(), lm.cpu().numpy()
    np.savez(path, **out)


def test_seed_kernel_forms_bit_identical(gpu_device, tmp_path):
    here = os.path.dirname(os.path.abspath(__file__))
    res = {}
    for tag, env in (("full", dict(PDSC_SEED_SORT="0", PDSC_SEED_SELECT="0")), ("sort", dict(PDSC_SEED_SORT="1")),
                     ("select", dict(PDSC_SEED_SORT="0", PDSC_SEED_SELECT="1"))):
        path = tmp_path / f"seeds_{tag}.npz"
        code = f"import sys; sys.path[:0] = [{here!r}, {os.path.dirname(here)!r}]; " \
               f"import test_gpu_seed_sort as t; t._dump({str(path)!r})"
        subprocess.run([sys.executable, "-c", code], env=dict(os.environ, **env), check=True, timeout=240)
        res[tag] = np.load(path)
    for form in ("sort", "select"):
        for k in res["full"].files:
            assert np.array_equal(res["full"][k], res[form][k]), (form, k)
