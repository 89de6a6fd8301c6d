"""Replayed-graph memset -> kernel visibility (sd_probe_graph_memset; GPU box)."""
import ctypes
import sys

sys.path.insert(0, ".")
import torch

from speaker_diarization_amd import _lib

torch.zeros(1, device="cuda")
for fork in (0, 1):
    for n in (1 << 16, 1 << 20, 1 << 24):
        R = 6
        bad = (ctypes.c_int * R)()
        _lib.call("sd_probe_graph_memset", n, R, fork, bad, _lib.stream_ptr())
        print(f"fork={fork} n={n}: non-zero reads per replay {list(bad)}", flush=True)
