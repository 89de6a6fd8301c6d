"""Host enqueue time of the C2 step (GPU box): how long the host takes to hand the step's launches to the two
slice streams, against the step's GPU time.  If the enqueue of slice A takes milliseconds, slice B's first
kernel starts that late on its stream (the r05 timeline's ~5.6 ms stream-1 start)."""
import sys, time
sys.path.insert(0, '.')
import bench, torch
a = bench.parse(['--steps', '3', '--warmup', '1', '--no-cpu-baseline', '--no-c4-ref'])
dev = torch.device('cuda', 0)
job = bench.tsvad_job(bench.WORKLOADS[sys.argv[1] if len(sys.argv) > 1 else 'c2'], a, 1, dev, 10.0)
pipe = job['pipe']
for _ in range(3): job['step']()
torch.cuda.synchronize()
enq, tot = [], []
for _ in range(10):
    plan = pipe.plan(job['n_lab'])
    t0 = time.perf_counter()
    pipe.average(pipe.window_logits(job['wav'], job['ts'], plan, check=False), plan)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    enq.append((t1 - t0) * 1e3); tot.append((t2 - t0) * 1e3)
enq.sort(); tot.sort()
print(f"enqueue ms median {enq[5]:.3f} min {enq[0]:.3f} | step wall ms median {tot[5]:.3f}")
