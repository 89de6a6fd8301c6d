"""`bench.py --gpus N` starts its own ranks (no external launcher): a CPU self-test with the
gloo backend in place of RCCL.  The parent process spawns N children with the torchrun
environment, every rank joins the process group, takes its contiguous share of the C4
60-min meeting's 64-window batch grid and all-gathers window logits (ts_vad/pipeline.py);
rank 0 prints ONE JSON line whose n_gpus is the process-group size."""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(*args, env=None):
    e = dict(os.environ)
    for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_PORT"):
        e.pop(k, None)
    e.update(env or {})
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), *args], capture_output=True, text=True,
                       timeout=240, env=e, cwd=REPO)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    return r, lines


@pytest.mark.parametrize("n", [2, 3])
def test_bench_spawns_ranks(n):
    r, lines = _run("--gpus", str(n), "--workload", "dist_check", "--steps", "2", "--warmup", "1")
    assert r.returncode == 0, r.stderr[-2000:]
    assert len(lines) == 1, r.stdout            # rank 0 only
    line = json.loads(lines[0])
    assert line["n_gpus"] == n
    assert line["ranks_joined"] == list(range(n))
    assert line["gather_matches_global_order"] is True
    assert line["steps"] == 2 and line["warmup"] == 1


def test_bench_single_rank_does_not_spawn():
    r, lines = _run("--gpus", "1", "--workload", "dist_check", "--steps", "1", "--warmup", "0")
    assert r.returncode == 0, r.stderr[-2000:]
    line = json.loads(lines[0])
    assert line["n_gpus"] == 1 and line["ranks_joined"] == [0]


def test_bench_default_workloads():
    """Defaults: the C2 headline at one GPU, the C4 60-min meeting when N > 1."""
    sys.path.insert(0, REPO)
    import bench
    a = bench.parse([])
    assert a.gpus == 1 and a.workload is None
    assert bench.WORKLOADS["c4"]["rs_len"] == 4 and bench.WORKLOADS["c4"]["variant"] == 0
    assert bench.WORKLOADS["c2"]["variant"] == 1


def test_failed_rank_stops_the_job():
    """A rank that dies makes the launcher stop its siblings and return the failing code
    (instead of hanging in a collective)."""
    r, _ = _run("--gpus", "2", "--workload", "dist_check", "--steps", "1", "--warmup", "0", "--batch", "0")
    assert r.returncode != 0
