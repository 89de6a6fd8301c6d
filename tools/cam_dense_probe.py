"""Phase stamps of one cam_dense launch (sd_debug_cam_dense_probe; GPU box).
    python3 tools/cam_dense_probe.py [B] [T] [cin]
Stamps (100 MHz): 0 start, 1 k-step 0 in LDS, 2 GEMM done, 3 h image done, 4 sums + conv done,
5 parts met (split), 6 gate + cross-cut taps done (or hand-over published), 7 own frames out,
8 (last part) the first part's decision known, 9 end."""
import math
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from speaker_diarization_amd import _lib

B = int(sys.argv[1]) if len(sys.argv) > 1 else 600
T = int(sys.argv[2]) if len(sys.argv) > 2 else 299
cin = int(sys.argv[3]) if len(sys.argv) > 3 else 512
dev = torch.device("cuda", 0)
ld = 1024
x = (torch.randn(B, T, ld, device=dev) * 0.5).to(torch.bfloat16)
g = torch.Generator().manual_seed(cin)
r = lambda *s: torch.randn(*s, generator=g).to(dev)
p = dict(s1=1 + 0.1 * r(cin), h1=0.1 * r(cin), wb=r(128, cin) / math.sqrt(cin), a2=1 + 0.1 * r(128),
         b2=0.1 * r(128), wl=r(32, 128, 3) / 20, bl=0.1 * r(32), w1=r(64, 128) / 11, c1=0.1 * r(64),
         w2=r(32, 64) / 8, c2=0.1 * r(32))
args = [_lib.ptr(p[k]) for k in ("s1", "h1", "wb", "a2", "b2", "wl", "bl", "w1", "c1", "w2", "c2")]
st = _lib.stream_ptr(dev)
split = (T + 15) // 16 > 10
nwg = 2 * B if split else B
stamps = torch.zeros(nwg * 16, dtype=torch.int64, device=dev)
_lib.call("sd_op_cam_dense", _lib.ptr(x), B, T, ld, cin, 2, *args, x.data_ptr() + 2 * cin, 2, st)   # warm
_lib.call("sd_debug_cam_dense_probe", _lib.ptr(stamps))
_lib.call("sd_op_cam_dense", _lib.ptr(x), B, T, ld, cin, 2, *args, x.data_ptr() + 2 * cin, 1, st)
torch.cuda.synchronize()
_lib.call("sd_debug_cam_dense_probe", None)
s = stamps.view(nwg, 16).cpu().numpy().astype(np.float64) / 100.0     # us
t0 = s[:, 0].min()
s = np.where(s > 0, s - t0, np.nan)
span = np.nanmax(s[:, 9])
print(f"B {B} T {T} cin {cin}: {nwg} workgroups, launch span {span:.1f} us")
names = ["start->kstep0", "gemm", "epilogue", "sums+conv", "arrive+meet", "gate", "own out", "decision", "handed out"]
for i, n in enumerate(names):
    d = s[:, i + 1] - s[:, i]
    d = d[~np.isnan(d)]
    if len(d):
        print(f"  {n:14s} n={len(d):5d} median {np.median(d):6.2f} p90 {np.percentile(d, 90):6.2f} us")
life = s[:, 9] - s[:, 0]
print(f"  lifetime median {np.nanmedian(life):.2f} p90 {np.nanpercentile(life, 90):.2f}")
if split:
    last = ~np.isnan(s[:, 8])
    print(f"  last arrivers {last.sum()}: lifetime median {np.nanmedian(life[last]):.2f}; first {np.nanmedian(life[~last]):.2f}")
    print(f"  hand-overs: {int((~np.isnan(s[:, 6]) & np.isnan(s[:, 5])).sum())}")
# concurrency: workgroups alive over time
ts = np.linspace(0, span, 40)
alive = [int(((s[:, 0] <= t) & (s[:, 9] > t)).sum()) for t in ts]
print("  alive:", " ".join(str(a) for a in alive))
starts = np.sort(s[:, 0])
print("  start times (us) of WG #0, 256, 511, 512, 767, 1023:", [round(float(starts[i]), 1) for i in (0, 256, 511, 512, 767, min(1023, nwg - 1)) if i < nwg])
