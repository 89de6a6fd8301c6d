"""The N>1 product path on the HIP kernels, simulated in one process.

For every rank of world sizes 2/3/8 the real per-rank work runs on the GPU: the
sub-span `kaldi_fbank(wav[s0:s1])` and `window_logits(w0, w1)` of the rank's
contiguous batch range (`shard_batches`, the 64-window grid of
ts_vad_dataset.py:242-271 + infer.py:232-238).  The shards concatenated in
`gather_windows` order must equal the one-rank window logits bit for bit, and
so must the overlap-averaged posteriors (the "bit-identical to 1 GPU when the
averaging order is fixed" promise of §8(e)).  The EEND-EDA chunk shard
(`chunk_activities` over `shard_chunks` ranges, infer_eda.py:99-113) is checked
the same way.
"""
import numpy as np
import pytest
import torch

from speaker_diarization_amd.synth import make_meeting, speaker_embeddings
from speaker_diarization_amd.ts_vad.model import TSVADModel
from speaker_diarization_amd.ts_vad.pipeline import TSVADPipeline
from speaker_diarization_amd.ts_vad.windows import shard_batches
from speaker_diarization_amd.weights import TSVADConfig, to_torch, tsvad_state_dict

pytestmark = pytest.mark.gpu

MINUTES = 7.0            # C4 shape (rs_len 4, shift 1), ~420 windows, ragged tail
WORLDS = (2, 3, 8)


@pytest.fixture(scope="module")
def c4_meeting():
    m = make_meeting(MINUTES * 60.0 + 1.37, n_spk=4, seed=4242)
    return m, speaker_embeddings(4, seed=4242)


@pytest.mark.parametrize("precision", ["bf16", "fp32"])
def test_tsvad_window_shards_bit_identical(gpu, c4_meeting, precision):
    meeting, ts_np = c4_meeting
    cfg = TSVADConfig(rs_len=4)
    model = TSVADModel(cfg, device=gpu, precision=precision, max_batch=128)
    model.load_state_dict(to_torch(tsvad_state_dict(cfg, seed=777)))
    pipe = TSVADPipeline(model, segment_shift=1, batch_size=64)
    wav = torch.from_numpy(meeting.wav).to(gpu)
    ts = torch.from_numpy(ts_np).to(gpu)
    n_lab = meeting.labels.shape[1]
    plan = pipe.plan(n_lab)
    full = pipe.window_logits(wav, ts, plan)
    ref_post = pipe.average(full, plan)
    for world in WORLDS:
        parts = []
        for rank in range(world):
            w0, w1 = shard_batches(plan, 64, world, rank)
            # each rank only holds its audio span: pass exactly the samples it reads
            parts.append(pipe.window_logits(wav, ts, plan, w0, w1))
        got = torch.cat(parts, 0)
        assert got.shape == full.shape
        diff = (got - full).abs().max().item()
        assert torch.equal(got, full), f"world {world}: shard logits differ by {diff}"
        post = pipe.average(got, plan)
        assert torch.equal(torch.nan_to_num(post, 7.0), torch.nan_to_num(ref_post, 7.0)), f"world {world}"


def test_tsvad_rank_reads_only_its_span(gpu, c4_meeting):
    """A rank handed only its audio span (wav[s0:s1]) computes the same logits as with the
    whole meeting in HBM: the sub-span fbank is frame-aligned (640 samples per label frame)."""
    meeting, ts_np = c4_meeting
    cfg = TSVADConfig(rs_len=4)
    model = TSVADModel(cfg, device=gpu, precision="bf16", max_batch=64)
    model.load_state_dict(to_torch(tsvad_state_dict(cfg, seed=777)))
    pipe = TSVADPipeline(model, segment_shift=1, batch_size=64)
    wav = torch.from_numpy(meeting.wav).to(gpu)
    ts = torch.from_numpy(ts_np).to(gpu)
    plan = pipe.plan(meeting.labels.shape[1])
    w0, w1 = shard_batches(plan, 64, 3, 1)
    spl = plan.samples_per_label
    s0, s1 = int(plan.starts[w0]) * spl, int(plan.ends[w1 - 1]) * spl
    # a buffer that is zero outside the rank's span: must not change the rank's logits
    only = torch.zeros_like(wav)
    only[s0:s1] = wav[s0:s1]
    a = pipe.window_logits(wav, ts, plan, w0, w1)
    b = pipe.window_logits(only, ts, plan, w0, w1)
    assert torch.equal(a, b)


@pytest.mark.parametrize("world", WORLDS)
@pytest.mark.parametrize("seconds,max_seqs", [(15 * 60.0 + 3.3, 8), (53 * 60.0 + 20.3, 16)])
def test_eda_chunk_shards_bit_identical(gpu, world, seconds, max_seqs):
    """9003 frames (4 x 2000 + 1003) and 32003 frames (16 equal chunks + a 3-frame tail): with 16
    chunks the one-rank forward batches M = 32 000 rows, a rank of world 2 / 4 / 8 M = 16 000 /
    8 000 / 4 000 — any GEMM choice that depended on the batched M (e.g. a split-K count) would
    change the fp32 summation and show here."""
    from speaker_diarization_amd.eend_eda.infer import (EdaInferArgs, chunk_activities, gen_chunk_indices,
                                                        recording_features, shard_chunks)
    from speaker_diarization_amd.eend_eda.models import EendEdaModel
    from speaker_diarization_amd.weights import EDAConfig, eda_state_dict
    meeting = make_meeting(seconds, n_spk=3, seed=99)
    torch.manual_seed(777)
    m = EendEdaModel(n_speakers=3, in_size=345, n_heads=4, n_units=256, n_layers=2, device=gpu,
                     precision="bf16", max_seqs=max_seqs, max_frames=2000)
    m.load_state_dict(to_torch(eda_state_dict(EDAConfig(model_type="EendEda", n_speakers=3, n_layers=2),
                                              seed=5)))
    args = EdaInferArgs(num_speakers=None)
    wav = torch.from_numpy(meeting.wav.astype(np.float32)).to(gpu)
    feats = recording_features(m, wav, args)
    chunks = list(gen_chunk_indices(feats.shape[0], args.chunk_size))
    perms = [torch.randperm(e - s, generator=torch.Generator().manual_seed(i)) for i, (s, e) in enumerate(chunks)]
    acts, probs = chunk_activities(m, feats, args, perms)
    got_a, got_p = [], []
    for rank in range(world):
        c0, c1 = shard_chunks(len(chunks), world, rank)
        a, p = chunk_activities(m, feats, args, perms, c0, c1)
        got_a.extend(a)
        got_p.append(p)
    assert len(got_a) == len(acts)
    for x, y in zip(got_a, acts):
        assert torch.equal(x, y)
    assert torch.equal(torch.cat(got_p), probs)
