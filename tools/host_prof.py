"""Host-side cProfile of the C2 bench step (GPU box): where the wall time outside the GPU span goes."""
import cProfile, pstats, sys, time, types
sys.path.insert(0, '.')
import bench, torch
a = bench.parse(['--steps', '3', '--warmup', '1', '--no-cpu-baseline', '--no-c4-ref'])
dev = torch.device('cuda', 0)
job = bench.tsvad_job(bench.WORKLOADS['c2'], a, 1, dev, 10.0)
for _ in range(2): job['step']()
torch.cuda.synchronize()
t = time.perf_counter()
for _ in range(3): job['step']()
torch.cuda.synchronize()
print('step ms', (time.perf_counter() - t) / 3 * 1e3)
pr = cProfile.Profile()
pr.enable()
for _ in range(3): job['step']()
torch.cuda.synchronize()
pr.disable()
pstats.Stats(pr).sort_stats('cumulative').print_stats(35)
