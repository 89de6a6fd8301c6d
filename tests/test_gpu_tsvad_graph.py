"""A captured + replayed TS-VAD forward equals the direct launches bit for bit (sd_tsvad_forward_graph, a
diagnostic entry point: the product path launches directly).

Round-3 history: the graph path of that time diverged from its second launch on (max 0.098 on
the posteriors) and its persistent BiLSTM reported lost co-residency.  Re-running that tree (round 4, stage
dumps) showed every stage identical except the BiLSTM output, and that replacing the BiLSTM's hipMemsetAsync
zeroing of h / c (captured as memset nodes) with a zeroing kernel made every replay bit-identical: the
memset nodes did not take effect before the next kernel node from the graph's second launch on.  Every
forward now zeroes with a kernel (zero_fill), so a caller that captures it gets no memset node.  Cases: the
C2 shape at B = 384 on two streams (fork / join inside the graph), and on one stream with the per-step
recurrence kernels (the failing configuration of round 3) in a child process (the switches are read once)."""
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

from speaker_diarization_amd import _lib
from speaker_diarization_amd.ts_vad.model import TSVADModel
from speaker_diarization_amd.weights import TSVADConfig, to_torch, tsvad_state_dict

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _direct_vs_replays(B, dev, replays=(1, 2, 3)):
    cfg = TSVADConfig.ots_vad_v1(rs_len=6)
    m = TSVADModel(cfg, device=dev, precision="bf16", max_batch=B)
    m.load_state_dict(to_torch(tsvad_state_dict(cfg, seed=779)))
    g = torch.Generator().manual_seed(5)
    x = torch.randn(B, 598, 80, generator=g).to(dev)
    ts = torch.randn(B, 4, 192, generator=g).to(dev)
    out = torch.empty(B, 4, 150, device=dev)
    m.forward(x, ts, 150, out=out)
    ref = out.clone()
    diffs = []
    for r in replays:
        out.zero_()
        _lib.call("sd_tsvad_forward_graph", m._h, _lib.ptr(x), _lib.ptr(ts), B, 598, 150, _lib.ptr(out), r, None,
                  _lib.stream_ptr(dev))
        m.status()
        diffs.append(float((out - ref).abs().max()))
    return diffs


def test_graph_replays_bit_identical_two_streams(gpu):
    assert _direct_vs_replays(384, gpu) == [0.0, 0.0, 0.0]


CHILD = r"""
import sys, torch
sys.path.insert(0, {repo!r}); sys.path.insert(0, {repo!r} + "/tests")
from test_gpu_tsvad_graph import _direct_vs_replays
print("DIFFS", _direct_vs_replays(64, torch.device("cuda", 0), (1, 2, 3, 4)))
"""


def test_graph_replays_bit_identical_one_stream_step_recurrence(gpu):
    env = dict(os.environ, SDIAR_CAM_ONE_STREAM="1", SDIAR_NO_LSTM_SEQ="1")
    r = subprocess.run([sys.executable, "-c", CHILD.format(repo=REPO)], env=env, capture_output=True, text=True,
                       timeout=110)
    assert r.returncode == 0, r.stderr[-2000:]
    assert "DIFFS [0.0, 0.0, 0.0, 0.0]" in r.stdout, r.stdout
