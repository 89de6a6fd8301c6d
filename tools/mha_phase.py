"""mha_block phase probe (GPU box, under rocprofv3 --kernel-trace --stats): the C2 shape (2400 sequences x 150
tokens) through the shipped layout and the probe variants 8 (no attention), 9 (no projection MFMAs) and 10
(neither); their kernel times split the launch into prologue + weight stream + barriers, projection MFMAs and
attention.  Outputs of the probes are meaningless."""
import sys

import torch

sys.path.insert(0, ".")
sys.path.insert(0, "tests")
from test_gpu_mha_block import _run  # noqa: E402

dev = torch.device("cuda", 0)
g = torch.Generator().manual_seed(7)
S, T = 2400, 150
y = torch.randn(S, T, 384, generator=g).to(torch.bfloat16).to(dev)
w = (torch.randn(1152, 384, generator=g) * 384 ** -0.5).to(dev)
b = (torch.randn(1152, generator=g) * 0.1).to(dev)
for v in (0, 8, 9, 10):
    for _ in range(5):
        _run(y, w, b, None, v)
torch.cuda.synchronize()
print("done")
