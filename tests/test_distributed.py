"""N>1 path on CPU (gloo, world_size 2): window sharding on the global batch grid
plus the all-gather in ts_vad/pipeline.py re-assemble exactly the single-process
window logits, and the overlap average (oracle restatement of infer.py:90-94)
over the gathered logits is bit-identical to the one-rank result."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from speaker_diarization_amd.ts_vad.pipeline import gather_windows
from speaker_diarization_amd.ts_vad.windows import plan_windows, shard_batches

N_LABELS = 25 * 60 * 7 + 13     # 7 min + a ragged tail
RS_LEN, SHIFT, BATCH, NS = 6, 1, 64, 4


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _global_logits(plan):
    g = torch.Generator().manual_seed(1234)
    return torch.randn(plan.n_win, NS, plan.chunk, generator=g)


def _worker(rank, world, port, outdir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        plan = plan_windows(N_LABELS, RS_LEN, SHIFT)
        full = _global_logits(plan)
        w0, w1 = shard_batches(plan, BATCH, world, rank)
        local = full[w0:w1].clone()          # what window_logits() computes on this rank
        got = gather_windows(local, plan, BATCH, world)
        torch.save({"got": got, "range": (w0, w1)}, os.path.join(outdir, f"r{rank}.pt"))
    finally:
        dist.destroy_process_group()


def _average(logits, plan):
    from oracle.pipeline_ref import overlap_average
    return overlap_average(logits.numpy(), plan.starts, plan.lens, plan.n_labels)


@pytest.mark.parametrize("world", [2])
def test_gloo_shard_gather_matches_single_rank(tmp_path, world):
    port = _free_port()
    mp.spawn(_worker, args=(world, port, str(tmp_path)), nprocs=world, join=True)
    plan = plan_windows(N_LABELS, RS_LEN, SHIFT)
    full = _global_logits(plan)
    ranges = []
    for r in range(world):
        d = torch.load(os.path.join(tmp_path, f"r{r}.pt"), weights_only=True)
        assert torch.equal(d["got"], full), f"rank {r} gathered logits differ"
        ranges.append(tuple(d["range"]))
    # shards tile [0, n_win) contiguously on the 64-window batch grid
    assert ranges[0][0] == 0 and ranges[-1][1] == plan.n_win
    for (a0, a1), (b0, b1) in zip(ranges, ranges[1:]):
        assert a1 == b0 and a1 % BATCH == 0
    ref = _average(full, plan)
    got = _average(torch.load(os.path.join(tmp_path, "r1.pt"), weights_only=True)["got"], plan)
    np.testing.assert_array_equal(got, ref)
