"""The other forms of a5 give exactly the compare kernels' bits: the 2- and
4-rows-per-thread NMS compare (local_max_rows_kernel, 2 the default for
batches from r06; PDSC_LM_RPT=1 for the one-row local_max_kernel), the opt-in
sorted forms (seeds.hip: bitonic-sorted NMS window and seed ranking, knob
PDSC_SEED_SORT=1, measurement only) and the default select form of the ranking
(radix-selected threshold + candidate ranking, seed_select_kernel; knob
PDSC_SEED_SELECT=0 for the compare kernel): is_local_max and the seed list, on
tie-heavy scores, -0 / +0 scores, negative local maxima and duplicate points,
and ties at the threshold wider than the candidate buffer; and the forward's
two-launch select form (candidates ranked by seed_cand_rank_kernel from S > 256,
in the forward's kdist scratch) against the compare kernels, uniform and ragged
batches (run with -m gpu)."""
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

CASES = [(3, 1000, 100, 0.1), (2, 5000, 500, 0.1), (1, 777, 77, 0.6), (4, 64, 6, 0.05), (1, 6000, 600, 1e-3),
         (2, 3000, 300, 0.02), (1, 9000, 4000, 0.02), (2, 2000, 1999, 0.0),
         (130, 640, 64, 0.08)]  # (the last: >= 1024 row blocks of 64 -> the 64-row NMS kernels)


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
    for tag, env in (("full", dict(PDSC_SEED_SORT="0", PDSC_SEED_SELECT="0", PDSC_LM_RPT="1")),
                     ("sort", dict(PDSC_SEED_SORT="1")),
                     ("select", dict(PDSC_SEED_SORT="0", PDSC_SEED_SELECT="1")),
                     ("rows2", dict(PDSC_SEED_SORT="0", PDSC_SEED_SELECT="0", PDSC_LM_RPT="2")),
                     ("rows4", dict(PDSC_SEED_SORT="0", PDSC_SEED_SELECT="0", PDSC_LM_RPT="4"))):
        path = tmp_path / f"seeds_{tag}.npz"
        code = f"import sys; sys.path[:0] = [{here!r}, {os.path.dirname(here)!r}]; " \
               f"import test_gpu_seed_sort as t; t._dump({str(path)!r})"
        subprocess.run([sys.executable, "-c", code], env=dict(os.environ, **env), check=True, timeout=240)
        res[tag] = np.load(path)
    for form in ("sort", "select", "rows2", "rows4"):
        for k in res["full"].files:
            assert np.array_equal(res["full"][k], res[form][k]), (form, k)


RAGGED_SIZES = [5000, 4100, 4700, 3300, 5000, 4900, 2900, 4400]  # ragged: S = 290 .. 500


def _dump_forward(path):
    from pointdsc_amd import kernels
    from pointdsc_amd.PointDSC import PointDSC
    from pointdsc_amd.synthetic import BENCH_CLS, PRESETS, synthetic_pair, trained_state_dict
    dev = torch.device("cuda:0")
    p = PRESETS["3dmatch"]
    m = PointDSC(in_dim=6, num_layers=12, num_channels=128, num_iterations=10, ratio=0.1,
                 inlier_threshold=p["inlier_threshold"], sigma_d=p["sigma_d"], k=40, nms_radius=p["nms_radius"])
    m.load_state_dict({k: torch.from_numpy(v) for k, v in trained_state_dict("3dmatch", 12, *BENCH_CLS).items()})
    m = m.to(dev).eval()
    cfg, pk = m.pdsc_config(), m.packed_weights()
    sizes = RAGGED_SIZES
    ps = [synthetic_pair(n, 300 + i) for i, n in enumerate(sizes)]
    pu = [synthetic_pair(5000, 400 + i) for i in range(8)]
    out = {}
    with torch.no_grad():
        x = [torch.from_numpy(np.stack([q[k] for q in pu])).to(dev) for k in ("corr_pos", "src_keypts", "tgt_keypts")]
        st = kernels.forward_stages(cfg, pk, *x, check_range=False)
        out["u_seeds"], out["u_conf"] = st["seeds"].cpu().numpy(), st["conf"].cpu().numpy()
        x = []
        for k in ("corr_pos", "src_keypts", "tgt_keypts"):
            a = np.zeros((8, 5000, ps[0][k].shape[1]), np.float32)
            for b, q in enumerate(ps):
                a[b, :sizes[b]] = q[k][:sizes[b]]
            x.append(torch.from_numpy(a).to(dev))
        _, _, dbg = kernels.forward_ragged(cfg, pk, *x, sizes, debug=True, check_range=False)
        out["r_seeds"] = dbg["seeds"].cpu().numpy()
    np.savez(path, **out)


def test_forward_select_forms_bit_identical(gpu_device, tmp_path):
    here = os.path.dirname(os.path.abspath(__file__))
    res = {}
    for tag, env in (("full", dict(PDSC_SEED_SELECT="0")), ("select", dict(PDSC_SEED_SELECT="2"))):
        path = tmp_path / f"fwd_{tag}.npz"
        code = f"import sys; sys.path[:0] = [{here!r}, {os.path.dirname(here)!r}]; " \
               f"import test_gpu_seed_sort as t; t._dump_forward({str(path)!r})"
        subprocess.run([sys.executable, "-c", code], env=dict(os.environ, **env), check=True, timeout=240)
        res[tag] = np.load(path)
    assert np.array_equal(res["full"]["u_conf"], res["select"]["u_conf"])
    assert np.array_equal(res["full"]["u_seeds"], res["select"]["u_seeds"])
    for b, n in enumerate(RAGGED_SIZES):  # a ragged pair's seeds: its own int(n * ratio) slots
        S = int(n * 0.1)
        assert np.array_equal(res["full"]["r_seeds"][b, :S], res["select"]["r_seeds"][b, :S]), b
