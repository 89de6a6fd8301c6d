"""One rank of `bench.py`'s TS-VAD `main()` with the REAL HIP forward, every rank on cuda:0 (one leased GPU),
the process group on gloo (RCCL refuses two ranks on one device).  tests/test_gpu_two_rank.py starts the ranks.

Test infrastructure: only the backend and the device choice differ from the driver's N-GPU run.  Everything
else is the shipped path -- bench.main's rank setup, rank-join gather, barrier + max-over-ranks timing, each
rank's own 25-GB workspace handle, its two-stream window slices (>= 384 windows per device call), its shard of
the wav (fbank of its own span), the logit all-gather (gloo: staged through host memory by
ts_vad/pipeline.gather_windows), the rank-0 RTTM lines and the JSON line.  Each rank saves the posteriors of
its last step to <out>/post_rank<r>.npy.

    RANK=.. WORLD_SIZE=.. MASTER_ADDR=127.0.0.1 MASTER_PORT=.. python tests/bench_main_gpu_ranks.py OUT [bench args]
"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import bench  # noqa: E402

LAST = {}


def gloo_on_one_gpu(backend="nccl"):
    import torch
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    torch.cuda.set_device(0)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("gloo")
    return world, rank, torch.device("cuda", 0)


if __name__ == "__main__":
    out_dir = sys.argv[1]
    bench.dist_setup = gloo_on_one_gpu
    _job = bench.tsvad_job

    def job(*args, **kw):
        j = _job(*args, **kw)
        step = j["step"]

        def keep():
            LAST["post"] = step()
            return LAST["post"]
        j["step"] = keep
        return j
    bench.tsvad_job = job
    a = bench.parse(sys.argv[2:])
    bench.main(a, bench.WORKLOADS[a.workload])
    np.save(os.path.join(out_dir, f"post_rank{os.environ.get('RANK', '0')}.npy"), LAST["post"].cpu().numpy())
