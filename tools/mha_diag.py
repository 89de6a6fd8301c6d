"""Per-layout max error of mha_block against the torch restatement, per 16-token tile (diagnostic)."""
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
sys.path.insert(0, "tests")
from test_gpu_mha_block import _ref, _run  # noqa: E402

dev = torch.device("cuda", 0)
for S, T in ((1, 160), (2, 150), (3, 37)):
    g = torch.Generator().manual_seed(7)
    y = torch.randn(S, T, 384, generator=g).to(torch.bfloat16).to(dev)
    w = (torch.randn(1152, 384, generator=g) * 384 ** -0.5).to(dev)
    b = (torch.randn(1152, generator=g) * 0.1).to(dev)
    ref = _ref(y, w.to(torch.bfloat16).float(), b, None)
    for v in (1, 0, 2, 3, 4, 5, 6):
        o = _run(y, w, b, None, v)
        e = (o.float() - ref).abs().cpu().numpy()
        nt = (T + 15) // 16
        tiles = [int(1000 * e[:, t * 16:(t + 1) * 16].max()) for t in range(nt)]
        print(f"S {S} T {T} variant {v}: max {e.max():.3e}  per tile x1000 {tiles}")
