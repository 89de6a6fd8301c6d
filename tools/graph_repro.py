"""TS-VAD forward: direct launches vs hipGraph replays of the same forward, stage by stage (GPU box).
    python3 tools/graph_repro.py [B] [dot_path]
Prints max |diff| of every stage buffer (sd_tsvad_debug_buffer) and the logits after 1, 2 and 3 replays of a
freshly captured graph, against the direct forward on the same inputs."""
import ctypes
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from speaker_diarization_amd import _lib
from speaker_diarization_amd.ts_vad.model import TSVADModel
from speaker_diarization_amd.weights import TSVADConfig, to_torch, tsvad_state_dict

B = int(sys.argv[1]) if len(sys.argv) > 1 else 384
dot = sys.argv[2] if len(sys.argv) > 2 else None
dev = torch.device("cuda", 0)
cfg = TSVADConfig.ots_vad_v1(rs_len=6)
m = TSVADModel(cfg, device=dev, precision="bf16", max_batch=B)
m.load_state_dict(to_torch(tsvad_state_dict(cfg, seed=779)))
g = torch.Generator().manual_seed(5)
x = torch.randn(B, 598, 80, generator=g).to(dev)
ts = torch.randn(B, 4, 192, generator=g).to(dev)
T = 150
names = ["mix", "mixg", "X2", "H", "Y"]


def stages():
    out = []
    for i in range(5):
        p, n = ctypes.c_void_p(), ctypes.c_int64()
        _lib.call("sd_tsvad_debug_buffer", m._h, i, ctypes.byref(p), ctypes.byref(n))
        out.append((p.value, n.value))
    return out


def snapshot():
    """Copies of the stage buffers (raw device pointers -> host via hipMemcpy)."""
    import ctypes.util
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    torch.cuda.synchronize()
    res = []
    for p, n in stages():
        h = np.empty(n // 4, np.float32)
        assert hip.hipMemcpy(h.ctypes.data, p, n, 2) == 0     # hipMemcpyDeviceToHost
        res.append(h)
    return res


out = torch.empty(B, 4, T, device=dev)
m.forward(x, ts, T, out=out)
m.forward(x, ts, T, out=out)
torch.cuda.synchronize()
ref = out.cpu().numpy().copy()
ref_st = snapshot()
for reps in (1, 2, 3):
    out.zero_()
    _lib.call("sd_tsvad_forward_graph", m._h, _lib.ptr(x), _lib.ptr(ts), B, 598, T, _lib.ptr(out), reps,
              (dot.encode() if (dot and reps == 3) else None), _lib.stream_ptr(dev))
    torch.cuda.synchronize()
    got = out.cpu().numpy()
    st = snapshot()
    diffs = " ".join(f"{nm}={float(np.nanmax(np.abs(a - b))) if a.size else 0:.3g}" for nm, a, b in zip(names, st, ref_st))
    print(f"replays {reps}: logits max|diff| {float(np.nanmax(np.abs(got - ref))):.3g} nan={int(np.isnan(got).sum())} | {diffs}",
          flush=True)
try:
    m.status()
    print("status ok")
except RuntimeError as e:
    print("status:", e)
