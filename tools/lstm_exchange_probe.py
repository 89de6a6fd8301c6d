"""The persistent LSTM's h-exchange floors (GPU box): the shipped 4-workgroup counter protocol
(sd_probe_lstm_handoff), the same 4 workgroups on data-tagged granules (sd_probe_lstm_granule: every lane polls 16
granules of 3 peers), and round 6's 2-workgroup 1-to-1 granule form (sd_probe_lstm_granule2: 8 granules of ONE
peer) -- us per step, median of 5 runs of 4000 steps each.
    python3 tools/lstm_exchange_probe.py"""
import ctypes
import statistics
import sys

import torch

sys.path.insert(0, ".")
from speaker_diarization_amd import _lib

dev = torch.device("cuda", 0)
st = _lib.stream_ptr(dev)
for name in ("sd_probe_lstm_handoff", "sd_probe_lstm_granule", "sd_probe_lstm_granule2"):
    us = ctypes.c_float()
    _lib.call(name, 200, ctypes.byref(us), st)      # warm
    runs = []
    for _ in range(5):
        _lib.call(name, 4000, ctypes.byref(us), st)
        runs.append(us.value)
    print(f"{name:24s} median {statistics.median(runs):.3f} us per step  ({', '.join('%.3f' % r for r in runs)})")
