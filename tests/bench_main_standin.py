"""One rank of `bench.py`'s TS-VAD `main()` on the CPU (tests/test_bench_main_gloo.py starts the ranks).

Test infrastructure, never a product path: the process group is gloo instead of RCCL, and the four device
operations under the pipeline are replaced by the CPU oracle (per-window fbank + TS-VAD forward of each
reference batch, oracle/pipeline_ref.py; sigmoid + ordered overlap mean; the RTTM writer).  Everything
else is the shipped code: bench.main's rank setup, rank-join all-gather, barrier + max-over-ranks timing,
end-to-end timing with the RTTM lines on rank 0 only and its JSON line, and TSVADPipeline.posteriors'
window sharding (shard_batches) and logit all-gather (gather_windows).  Each rank saves the posteriors of
its last step to <out>/post_rank<r>.npy for the test to compare across world sizes.

    RANK=.. WORLD_SIZE=.. MASTER_ADDR=127.0.0.1 MASTER_PORT=.. python tests/bench_main_standin.py OUT [bench args]
"""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import bench  # noqa: E402
from oracle.pipeline_ref import overlap_average, window_batches  # noqa: E402
from oracle.postprocess_ref import rttm_lines  # noqa: E402
from oracle.tsvad_ref import tsvad_forward  # noqa: E402
from speaker_diarization_amd.synth import make_meeting, speaker_embeddings  # noqa: E402
from speaker_diarization_amd.ts_vad import postprocess  # noqa: E402
from speaker_diarization_amd.ts_vad.pipeline import TSVADPipeline  # noqa: E402
from speaker_diarization_amd.weights import TSVADConfig, to_torch, tsvad_state_dict  # noqa: E402


class _ModelShape:
    """What TSVADPipeline reads from its model."""

    def __init__(self, cfg, max_batch):
        self.cfg, self.max_batch = cfg, max_batch
        self.device = torch.device("cpu")
        self.max_num_speaker = cfg.max_num_speaker


class OraclePipeline(TSVADPipeline):
    """TSVADPipeline with window_logits / average computed by the oracle; posteriors() (shard + gather)
    is the product method, unchanged."""

    def __init__(self, sd, cfg, batch_size):
        super().__init__(_ModelShape(cfg, batch_size), segment_shift=1, batch_size=batch_size)
        self.sd = sd

    @torch.no_grad()
    def window_logits(self, wav, ts, plan, w0=0, w1=None, out=None, check=True):
        w1 = plan.n_win if w1 is None else w1
        out = torch.zeros(w1 - w0, self.model.max_num_speaker, plan.chunk)
        windows = [(int(plan.starts[i]), int(plan.ends[i])) for i in range(w0, w1)]
        for b0, ws, ref, tsb, L in window_batches(wav.numpy(), ts.numpy(), windows, self.batch_size,
                                                  self.cfg.sample_rate, self.cfg.label_rate):
            out[b0:b0 + len(ws), :, :L] = tsvad_forward(self.sd, self.cfg, ref, tsb, L)
        return out

    @staticmethod
    def average(logits, plan):
        return torch.from_numpy(overlap_average(logits.numpy(), plan.starts, plan.lens, plan.n_labels))


LAST = {}


def standin_job(wl, a, world, dev, total_min):
    cfg = TSVADConfig(rs_len=wl["rs_len"]) if wl["variant"] == 0 else TSVADConfig.ots_vad_v1(rs_len=wl["rs_len"])
    sd_np = tsvad_state_dict(cfg, seed=777)
    pipe = OraclePipeline(to_torch(sd_np), cfg, a.batch)
    meeting = make_meeting(total_min * 60.0, n_spk=4, seed=777)
    ts_np = speaker_embeddings(4, seed=777)
    job = dict(cfg=cfg, sd_np=sd_np, model=None, pipe=pipe, meeting=meeting, ts_np=ts_np,
               wav=torch.from_numpy(meeting.wav), ts=torch.from_numpy(ts_np), n_lab=meeting.labels.shape[1],
               frames=meeting.wav.size // 160)

    def step():
        LAST["post"] = pipe.posteriors(job["wav"], job["ts"], job["n_lab"])
        return LAST["post"]
    job["step"] = step
    return job


if __name__ == "__main__":
    out_dir = sys.argv[1]
    torch.set_num_threads(2)
    _setup = bench.dist_setup
    bench.dist_setup = lambda backend="nccl": _setup("gloo")
    bench.tsvad_job = standin_job
    postprocess.posteriors_to_rttm_gpu = lambda keys, p: rttm_lines({k: p[i].numpy() for i, k in enumerate(keys)})
    a = bench.parse(sys.argv[2:])
    bench.main(a, bench.WORKLOADS[a.workload])
    np.save(os.path.join(out_dir, f"post_rank{os.environ.get('RANK', '0')}.npy"), LAST["post"].numpy())
