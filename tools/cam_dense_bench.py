"""Per-launch time of the fused CAM++ dense layer (sd_op_cam_dense) over input widths (GPU box).
    python3 tools/cam_dense_bench.py [B] [T]"""
import math
import sys

import torch

sys.path.insert(0, ".")
from speaker_diarization_amd import _lib

B = int(sys.argv[1]) if len(sys.argv) > 1 else 600
T = int(sys.argv[2]) if len(sys.argv) > 2 else 299
dev = torch.device("cuda", 0)
lib = _lib.load()
for cin in (128, 256, 512, 768, 992):
    ld = 1024
    x = (torch.randn(B, T, ld, device=dev) * 0.5).to(torch.bfloat16)
    g = torch.Generator().manual_seed(cin)
    r = lambda *s: torch.randn(*s, generator=g).to(dev)
    p = dict(s1=1 + 0.1 * r(cin), h1=0.1 * r(cin), wb=r(128, cin) / math.sqrt(cin), a2=1 + 0.1 * r(128),
             b2=0.1 * r(128), wl=r(32, 128, 3) / 20, bl=0.1 * r(32), w1=r(64, 128) / 11, c1=0.1 * r(64),
             w2=r(32, 64) / 8, c2=0.1 * r(32))
    args = [_lib.ptr(p[k]) for k in ("s1", "h1", "wb", "a2", "b2", "wl", "bl", "w1", "c1", "w2", "c2")]
    st = _lib.stream_ptr(dev)

    def run(n):
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        _lib.call("sd_op_cam_dense", _lib.ptr(x), B, T, ld, cin, 2, *args, x.data_ptr() + 2 * cin, n, st)
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1)

    run(2)
    t1 = min(run(1) for _ in range(3))
    t11 = min(run(11) for _ in range(3))
    per = (t11 - t1) / 10
    byts = 2.0 * B * T * (cin + 32) + 2.0 * 128 * cin
    print(f"B {B} T {T} cin {cin:4d}: {per * 1e3:7.1f} us/launch  {byts / per / 1e9:6.2f} TB/s", flush=True)
