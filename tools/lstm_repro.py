"""Repeat the C2 TS-VAD step and report any lost LSTM co-residency (diagnostic, GPU box)."""
import sys
import time
sys.path.insert(0, '.')
import bench
import torch
a = bench.parse(['--steps', '3', '--warmup', '1', '--no-cpu-baseline', '--no-c4-ref'])
dev = torch.device('cuda', 0)
job = bench.tsvad_job(bench.WORKLOADS['c2'], a, 1, dev, 10.0)
n = int(sys.argv[1]) if len(sys.argv) > 1 else 12
fails = 0
import numpy as np
out = sys.argv[2] if len(sys.argv) > 2 else None
for i in range(n):
    t = time.perf_counter()
    try:
        post = job['step']()
        if out and i == n - 1:
            np.save(out, post.cpu().numpy())
        torch.cuda.synchronize()
        print(f'step {i} ok {1e3 * (time.perf_counter() - t):.1f} ms', flush=True)
    except Exception as e:
        fails += 1
        print(f'step {i} FAIL {1e3 * (time.perf_counter() - t):.1f} ms: {e}', flush=True)
print('fails', fails)
