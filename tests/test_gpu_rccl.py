"""RCCL (torch.distributed "nccl") on device tensors, on the one-GPU test box:
bench.py and the evaluation driver launched by torchrun with one rank, so the
per-pair row all-gather and the max-reduce of the timed region run through
RCCL (evaluation/test_KITTI.py:220-228, 270-272 is the reference's launch).
The N>1 paths are the same code; their rank logic is covered by the gloo tests
(test_bench_launcher.py, test_dist_eval.py)."""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _torchrun(args, timeout=300):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
           "--master-addr", "127.0.0.1", "--master-port", str(_port())] + args
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    return [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]


@pytest.mark.gpu
def test_bench_one_rank_rccl():
    out = _torchrun(["bench.py", "--gpus", "1", "--steps", "2", "--warmup", "1", "--pairs", "16",
                     "--no-cpu-baseline", "--f32-steps", "0", "--path-n", "0"])
    assert len(out) == 1
    res = out[0]
    assert res["n_gpus"] == 1 and res["pairs_gathered"] == 16 and res["value"] > 0
    assert res["synthetic_recall"] >= 0.9


@pytest.mark.gpu
def test_evaluate_one_rank_rccl():
    out = _torchrun(["-m", "pointdsc_amd.evaluate", "--pairs", "12", "--num-corr", "600", "--batch", "5"])
    assert len(out) == 1
    assert out[0]["pairs"] == 12 and out[0]["all_pairs"]["success"] >= 0.9
