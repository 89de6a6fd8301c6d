"""Phase split of the conformer pw2 + FFN row program (rowprog.hip program 5, the C2 line's dominant kernel) from
its stamping instantiation (sd_debug_rowprog_probe; GPU box).  One C2-shaped TS-VAD forward (ots_vad v1, B windows
of 598 fbank frames, one stream so the 6 launches run one after another); per wave, s_memtime cycles of: piece waits
(barrier), refill issue (the DMA instructions of the next piece), epilogue stores, tile loads; MFMA streaming + LayerNorms = the
rest.  Printed per 128-token tile (mean over waves).
    SDIAR_CAM_ONE_STREAM=1 python3 tools/rowprog_probe.py [B]"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from speaker_diarization_amd import _lib
from speaker_diarization_amd.ts_vad.model import TSVADModel
from speaker_diarization_amd.weights import TSVADConfig, to_torch, tsvad_state_dict

assert os.environ.get("SDIAR_CAM_ONE_STREAM"), "run with SDIAR_CAM_ONE_STREAM=1 (launches must not overlap)"
B = int(sys.argv[1]) if len(sys.argv) > 1 else 600
dev = torch.device("cuda", 0)
cfg = TSVADConfig.ots_vad_v1(rs_len=6)
m = TSVADModel(cfg, device=dev, precision="bf16", max_batch=B)
m.load_state_dict(to_torch(tsvad_state_dict(cfg, seed=777)))
g = torch.Generator().manual_seed(3)
x = torch.randn(B, 598, 80, generator=g).to(dev)
ts = torch.randn(B, 4, 192, generator=g).to(dev)
m.forward(x, ts, 150)                         # warm
torch.cuda.synchronize()
stamps = torch.zeros(256 * 8 * 8, dtype=torch.int64, device=dev)
_lib.call("sd_debug_rowprog_probe", _lib.ptr(stamps))
m.forward(x, ts, 150)
torch.cuda.synchronize()
_lib.call("sd_debug_rowprog_probe", None)
s = stamps.view(256, 8, 8).cpu().numpy().astype(np.float64)
live = s[:, 0, 5] > 0
s = s[live]
tiles = s[:, :, 5]                              # tiles this wave ran over the forward's launches
per_tile = s[:, :, :5] / tiles[:, :, None]
mean = per_tile.reshape(-1, 5).mean(0)
names = ["whole", "piece waits", "refill issue", "epilogue", "tile loads"]
print(f"B {B}: {int(live.sum())} workgroups, {tiles.mean():.1f} tiles per wave over the forward's launches")
for n, v in zip(names, mean):
    print(f"  {n:16s} {v:9.0f} cycles per tile ({100 * v / mean[0]:5.1f} %)")
rest = mean[0] - mean[1:].sum()
print(f"  {'MFMA stream + LN':16s} {rest:9.0f} cycles per tile ({100 * rest / mean[0]:5.1f} %)")
w = per_tile[:, :, 1]
print(f"  piece waits across waves: min {w.min():.0f} median {np.median(w):.0f} max {w.max():.0f}")
