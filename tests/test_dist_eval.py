"""SURVEY 8(e) multi-GPU sharding and 8(f) row 2 evaluation harness, on CPU.

* shard_indices: the reference's DistributedSampler(shuffle=False) split
  (evaluation/test_KITTI.py:246-251) without padding duplicates.
* gather_rows / job_throughput: world-size-2 gloo process group (the RCCL path
  on MI355X runs the same calls with device tensors).
* pair_stats: RE/TE/success of libs/loss.py:39-57 and precision/recall/F1 of
  libs/loss.py:100-112 (sklearn, the reference's own metric functions).
* aggregate: per-scene then mean-over-scenes, RE/TE over successful pairs only
  (evaluation/test_3DMatch.py:141-176)."""
import math
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from pointdsc_amd import dist as pdist
from pointdsc_amd import evaluate as ev


@pytest.mark.parametrize("n,W", [(10, 1), (10, 3), (7, 8), (0, 2), (257, 8)])
def test_shard_indices_partition(n, W):
    seen = []
    for r in range(W):
        idx = pdist.shard_indices(n, r, W)
        assert idx == list(range(r, n, W))
        assert len(idx) == pdist.shard_count(n, r, W)
        seen += idx
    assert sorted(seen) == list(range(n))
    with pytest.raises(ValueError):
        pdist.shard_indices(n, W, W)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, W, port, n, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=W)
    try:
        mine = pdist.shard_indices(n, rank, W)
        rows = torch.tensor([[10.0 * i + c for c in range(12)] for i in mine], dtype=torch.float64).reshape(-1, 12)
        out = pdist.gather_rows(rows, n)
        units, secs = pdist.job_throughput(len(mine) * 1000, 0.5 + rank)
        q.put((rank, out.numpy(), units, secs))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("n", [9, 2, 1])
def test_gather_rows_gloo_world2(n):
    W = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, W, port, n, q)) for r in range(W)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(W)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    want = np.array([[10.0 * i + c for c in range(12)] for i in range(n)])
    for rank, out, units, secs in res:
        assert np.array_equal(out, want), rank
        assert units == n * 1000 and secs == 1.5


def test_gather_rows_rejects_wrong_shard():
    with pytest.raises(ValueError):
        pdist.gather_rows(torch.zeros(3, 12), 5)  # world 1 owns all 5


def _rot(axis, deg):
    a = np.asarray(axis, float) / np.linalg.norm(axis)
    K = np.array([[0, -a[2], a[1]], [a[2], 0, -a[0]], [-a[1], a[0], 0]])
    t = np.deg2rad(deg)
    return np.eye(3) + np.sin(t) * K + (1 - np.cos(t)) * K @ K


def test_pair_stats_match_reference_metrics():
    from sklearn.metrics import f1_score, precision_score, recall_score
    rng = np.random.RandomState(0)
    B, N = 6, 200
    gt = np.tile(np.eye(4), (B, 1, 1))
    pr = np.tile(np.eye(4), (B, 1, 1))
    degs = [0.5, 10.0, 20.0, 3.0, 179.0, 0.0]
    dts = [0.01, 0.2, 0.0, 0.5, 0.0, 0.0]
    for b in range(B):
        gt[b, :3, :3] = _rot(rng.randn(3), rng.rand() * 90)
        gt[b, :3, 3] = rng.randn(3)
        pr[b, :3, :3] = _rot(rng.randn(3), degs[b]) @ gt[b, :3, :3]
        pr[b, :3, 3] = gt[b, :3, 3] + dts[b] * np.array([1.0, 0, 0])
    gl = (rng.rand(B, N) < 0.3).astype(np.float32)
    pl = (rng.rand(B, N) < 0.3).astype(np.float32)
    pl[5] = 0  # no predicted inliers: sklearn's zero_division result (0)
    st = ev.pair_stats(torch.from_numpy(pr).float(), torch.from_numpy(gt).float(), torch.from_numpy(pl),
                       torch.from_numpy(gl), 15.0, 30.0).numpy()
    for b in range(B):
        R, gR = pr[b, :3, :3].astype(np.float32), gt[b, :3, :3].astype(np.float32)
        re = math.degrees(math.acos(min(1, max(-1, (np.trace(R.T @ gR) - 1) / 2))))
        te = np.linalg.norm(pr[b, :3, 3] - gt[b, :3, 3]) * 100
        assert abs(st[b, 1] - re) < 2e-2 and abs(st[b, 2] - te) < 1e-3, b
        assert st[b, 0] == float(te < 30 and re < 15)
        assert st[b, 3] == gl[b].sum() and abs(st[b, 4] - gl[b].mean()) < 1e-6
        with np.errstate(all="ignore"):
            import warnings
            with warnings.catch_warnings():
                warnings.simplefilter("ignore")
                p = precision_score(gl[b], pl[b] > 0)
                r = recall_score(gl[b], pl[b] > 0)
                f = f1_score(gl[b], pl[b] > 0)
        assert abs(st[b, 6] - p) < 1e-12 and abs(st[b, 7] - r) < 1e-12 and abs(st[b, 8] - f) < 1e-12, b


def test_pair_stats_ragged_counts():
    """Zero-padded labels of a ragged batch: the input inlier ratio divides by each
    pair's own count; every other column is unchanged by the padding."""
    rng = np.random.RandomState(3)
    T = torch.eye(4).expand(3, 4, 4).clone()
    counts = [50, 80, 120]
    gl = torch.zeros(3, 120)
    pl = torch.zeros(3, 120)
    for b, n in enumerate(counts):
        gl[b, :n] = torch.from_numpy((rng.rand(n) < 0.3).astype(np.float32))
        pl[b, :n] = torch.from_numpy((rng.rand(n) < 0.3).astype(np.float32))
    st = ev.pair_stats(T, T, pl, gl, counts=counts).numpy()
    for b, n in enumerate(counts):
        one = ev.pair_stats(T[b:b + 1], T[b:b + 1], pl[b:b + 1, :n], gl[b:b + 1, :n]).numpy()[0]
        np.testing.assert_allclose(st[b], one, rtol=1e-12)
    assert ev.pair_sizes(4, (700, 1300)) == ev.pair_sizes(4, (700, 1300)) and ev.pair_sizes(3, 9) == [9, 9, 9]


def test_aggregate_scene_then_mean():
    rows = np.zeros((5, 12))
    rows[:, 0] = [1, 0, 1, 1, 1]        # success
    rows[:, 1] = [1.0, 99, 3.0, 5.0, 7.0]  # RE (failed pair excluded from RE/TE means)
    rows[:, 2] = [10, 999, 30, 50, 70]
    rows[:, 11] = [0, 0, 0, 1, 1]       # scenes
    out = ev.aggregate(rows)
    assert out["pairs"] == 5
    assert abs(out["all_pairs"]["success"] - 0.8) < 1e-12
    assert abs(out["all_pairs"]["re_deg"] - 4.0) < 1e-12
    # scene 0: success 2/3, RE mean over its successful pairs = 2; scene 1: 1, RE 6
    assert abs(out["scene_mean"]["success"] - (2 / 3 + 1) / 2) < 1e-12
    assert abs(out["scene_mean"]["re_deg"] - 4.0) < 1e-12
    assert abs(out["scene_mean"]["te_cm"] - 40.0) < 1e-12


def test_report_lines_and_npy(tmp_path):
    """The driver's outputs (evaluation/test_3DMatch.py:141-176, :238-241): the
    scene / all-scene / all-pair lines with the reference's wording and numbers,
    and the [P, 12] float64 stats saved without pickle."""
    rows = np.zeros((5, 12))
    rows[:, 0] = [1, 0, 1, 1, 1]
    rows[:, 1] = [1.0, 99, 3.0, 5.0, 7.0]
    rows[:, 2] = [10, 999, 30, 50, 70]
    rows[:, 6:9] = 0.5
    rows[:, 11] = [0, 0, 0, 1, 1]
    lines = ev.report_lines(rows)
    assert lines[0] == ("Scene 0th: Reg Recall=66.67%  Mean RE=2.00  Mean TE=20.00  Mean Precision=50.00%  "
                        "Mean Recall=50.00%  Mean F1=50.00%")
    assert lines[1].startswith("Scene 1th: Reg Recall=100.00%  Mean RE=6.00  Mean TE=60.00")
    assert lines[2] == "All 2 scenes, Mean Reg Recall=83.33%, Mean Re=4.00, Mean Te=40.00"
    assert "All 5 pairs, Mean Reg Recall=80.00%, Mean Re=4.00, Mean Te=40.00" in lines
    ev.save_outputs(rows, str(tmp_path / "r.log"), str(tmp_path / "r.npy"))
    assert (tmp_path / "r.log").read_text().splitlines() == lines
    back = np.load(tmp_path / "r.npy", allow_pickle=False)
    assert back.dtype == np.float64 and np.array_equal(back, rows)


@pytest.mark.gpu
def test_evaluate_synthetic_on_device(gpu_device):
    """f2 end to end on one GPU: sharded (world 1) synthetic evaluation through
    forward_batched, per-pair rows and the reference's aggregation."""
    from pointdsc_amd.PointDSC import PointDSC
    from pointdsc_amd.synthetic import trained_state_dict
    m = PointDSC(in_dim=6, num_layers=12, num_channels=128, num_iterations=10, ratio=0.1,
                 inlier_threshold=0.10, sigma_d=0.10, k=40, nms_radius=0.10)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in trained_state_dict("3dmatch", 12).items()})
    m = m.to(gpu_device).eval()
    stats, summary = ev.evaluate_synthetic(m, 12, 600, "3dmatch", batch=5, device=gpu_device)
    assert stats.shape == (12, 12)
    assert summary["pairs"] == 12
    assert summary["all_pairs"]["success"] >= 0.9  # synthetic pairs with 30 % inliers register
    assert 0.0 <= summary["all_pairs"]["f1"] <= 1.0
    # mixed sizes: the ragged forward (PointDSC.forward_list's kernel) per batch
    stats2, summary2 = ev.evaluate_synthetic(m, 12, (500, 900), "3dmatch", batch=5, device=gpu_device)
    assert stats2.shape == (12, 12) and summary2["all_pairs"]["success"] >= 0.9
    assert np.all((stats2[:, 4] > 0.2) & (stats2[:, 4] < 0.4))  # input inlier ratio over each pair's own N
