"""`bench.py`'s TS-VAD strong-scaling `main()` itself at world size 2 on the CPU (gloo), with the device
operations under the pipeline replaced by the CPU oracle (tests/bench_main_standin.py): the N > 1 control
flow the driver's 8-GPU run takes -- rank setup, rank-join all-gather, timing with barriers and the
max-over-ranks reduction, TSVADPipeline's window shards and logit all-gather, rank-0-only RTTM lines and the
one JSON line -- end to end.  The 2-rank posteriors must equal the 1-rank ones bit for bit."""
import json
import os
import subprocess
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ARGS = ["--workload", "c4", "--minutes", "0.35", "--batch", "4", "--steps", "1", "--warmup", "0",
        "--no-cpu-baseline", "--no-kernel-timing", "--precision", "fp32"]


def _port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(world, out):
    port = str(_port())
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=port, OMP_NUM_THREADS="2")
        procs.append(subprocess.Popen([sys.executable, os.path.join(REPO, "tests", "bench_main_standin.py"), out,
                                       *ARGS], env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True,
                                      cwd=REPO))
    outs = []
    for p in procs:
        try:
            o, e = p.communicate(timeout=400)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
        outs.append((p.returncode, o, e))
    for rc, o, e in outs:
        assert rc == 0, e[-3000:]
    lines = [ln for ln in outs[0][1].splitlines() if ln.startswith("{")]
    assert len(lines) == 1, outs[0][1][-2000:]
    assert not any(ln.startswith("{") for _, o, _ in outs[1:] for ln in o.splitlines()), "only rank 0 prints"
    return json.loads(lines[0])


def test_bench_main_two_ranks_matches_one(tmp_path):
    d1, d2 = tmp_path / "w1", tmp_path / "w2"
    d1.mkdir()
    d2.mkdir()
    one = _run(1, str(d1))
    two = _run(2, str(d2))
    assert one["n_gpus"] == 1 and two["n_gpus"] == 2
    assert two["rccl_ranks"] == [0, 1] and two["scaling"] == "strong"
    assert two["config"]["meeting_minutes"] == one["config"]["meeting_minutes"] == 0.35
    assert two["config"]["windows"] == one["config"]["windows"]
    assert "window-shard x2" in two["config"]["parallelism"]
    for line in (one, two):
        assert line["value"] > 0 and line["ms_per_step"] > 0 and line["end_to_end"]["ms_per_step"] > 0
    p1 = np.load(d1 / "post_rank0.npy")
    for r in range(2):       # every rank holds the gathered meeting posteriors
        np.testing.assert_array_equal(np.load(d2 / f"post_rank{r}.npy"), p1)
    assert np.isfinite(p1).all()
