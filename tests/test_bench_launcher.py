"""bench.py --gpus N launches N rank processes itself (evaluation/test_KITTI.py:220-228
spawns one process per GPU the same way) -- exercised here on CPU with gloo
through --launcher-selftest, which runs the launch, the strided pair split,
the all-gather of per-pair result rows and the max-reduce, but no forward."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(*args, timeout=240):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], cwd=ROOT, env=env,
                          capture_output=True, text=True, timeout=timeout)


def _json_lines(out):
    return [json.loads(l) for l in out.splitlines() if l.startswith("{")]


def test_launcher_world_2_gathers_every_pair():
    r = _run("--gpus", "2", "--pairs", "3", "--launcher-selftest")
    assert r.returncode == 0, r.stderr[-2000:]
    lines = _json_lines(r.stdout)
    assert len(lines) == 1, r.stdout  # rank 0 only
    out = lines[0]
    assert out["n_gpus"] == 2 and out["pairs_total"] == 6
    assert out["pair_ids"] == list(range(6))  # rows back in global pair order
    assert out["synthetic_recall"] == 1.0


def test_launcher_single_rank_runs_in_process():
    r = _run("--gpus", "1", "--pairs", "2", "--launcher-selftest")
    assert r.returncode == 0, r.stderr[-2000:]
    out = _json_lines(r.stdout)[0]
    assert out["n_gpus"] == 1 and out["pair_ids"] == [0, 1]


def test_launcher_fails_when_a_rank_fails():
    r = _run("--gpus", "2", "--pairs", "0", "--launcher-selftest")  # every rank raises (no pairs)
    assert r.returncode != 0
    assert not _json_lines(r.stdout)
