"""Chunk-streaming TS-VAD on the GPU (libsdiar sd_tsvad_stream_*) vs the reference goldens and
the CPU oracle.  Tolerances: fp32 1e-3 absolute (north_star); bf16 1 % of the logit range
(bf16 operands carry 8 mantissa bits, and this model's logits reach |8|, four times the offline
TS-VAD's, whose bf16 bound is 2e-2 absolute)."""
import os

import numpy as np
import pytest
import torch

from make_golden import TSVAD_STREAM_CASES, tsvad_stream_inputs
from speaker_diarization_amd.ts_vad.streaming import TSVADStreamingModel
from speaker_diarization_amd.weights import TSVADStreamingConfig, to_torch, tsvad_streaming_state_dict

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")


@pytest.mark.parametrize("precision", ["fp32", "bf16"])
@pytest.mark.parametrize("name", list(TSVAD_STREAM_CASES))
def test_stream_matches_reference(gpu, name, precision):
    T_lab, dcs, left, T_fb, iseed, wseed = TSVAD_STREAM_CASES[name]
    m = TSVADStreamingModel(TSVADStreamingConfig(), device=gpu, precision=precision, max_labels=128)
    m.load_state_dict(to_torch(tsvad_streaming_state_dict(TSVADStreamingConfig(), seed=wseed)))
    xs, ts = tsvad_stream_inputs(T_fb, iseed)
    y = m.forward_chunk_by_chunk_temp1(torch.from_numpy(xs), torch.from_numpy(ts), torch.zeros(1, 4, T_lab),
                                       decoding_chunk_size=dcs, num_decoding_left_chunks=left).cpu().numpy()
    g = np.load(os.path.join(GOLD, name + ".npz"))["logits"]
    err = np.abs(y - g).max()
    print(f"{name} {precision}: max|logit diff| = {err:.3e} (max|logit| {np.abs(g).max():.2f})")
    assert err < (1e-3 if precision == "fp32" else 1e-2 * max(1.0, float(np.abs(g).max())))


def test_stream_long_window_vs_oracle(gpu):
    """A 16 s window (400 label frames, 16 chunks of 25) through the long-sequence attention
    kernel (T > 256) vs the oracle's literal chunk loop, with a 4-chunk left context."""
    from oracle.tsvad_stream_ref import forward_chunk_by_chunk
    sd = tsvad_streaming_state_dict(TSVADStreamingConfig(), seed=71)
    xs, ts = tsvad_stream_inputs(1600, 72)
    m = TSVADStreamingModel(device=gpu, precision="fp32", max_labels=400).load_state_dict(to_torch(sd))
    for left in (-1, 4):
        y = m.forward_chunk_by_chunk(torch.from_numpy(xs), torch.from_numpy(ts), 400, 25, left).cpu().numpy()
        with torch.no_grad():
            ref = forward_chunk_by_chunk(to_torch(sd), torch.from_numpy(xs), torch.from_numpy(ts), 400, 25, left).numpy()
        assert np.abs(y - ref).max() < 1e-3, left


def test_stream_errors(gpu):
    sd = to_torch(tsvad_streaming_state_dict(TSVADStreamingConfig(), seed=3))
    m = TSVADStreamingModel(device=gpu, precision="fp32", max_labels=64).load_state_dict(sd)
    xs, ts = tsvad_stream_inputs(200, 4)
    with pytest.raises(ValueError):
        m.forward_chunk_by_chunk(torch.from_numpy(xs), torch.from_numpy(ts), 100, 25)   # > max_labels
    with pytest.raises(AssertionError):
        m.forward_chunk_by_chunk(torch.from_numpy(xs), torch.from_numpy(ts), 50, 0)     # chunk size 0 (model.py assert)
    bad = dict(sd)
    bad.pop("fc.bias")
    with pytest.raises(RuntimeError, match="fc.bias"):
        TSVADStreamingModel(device=gpu, max_labels=64).load_state_dict(bad)


@pytest.mark.parametrize("T_lab,dcs,left", [(250, 25, -1), (100, 25, 1), (70, 25, -1), (64, 10, 0)])
def test_stream_windows_batch(gpu, T_lab, dcs, left):
    """forward_windows over B windows == forward_chunk_by_chunk on each window alone (with and
    without a partial last chunk), and window 0 vs the oracle's chunk loop."""
    from oracle.tsvad_stream_ref import forward_chunk_by_chunk
    sd = tsvad_streaming_state_dict(TSVADStreamingConfig(), seed=91)
    B = 3
    m = TSVADStreamingModel(device=gpu, precision="fp32", max_labels=T_lab, max_windows=B).load_state_dict(to_torch(sd))
    xs = np.stack([tsvad_stream_inputs(4 * T_lab, 100 + b)[0][0] for b in range(B)])
    ts = np.stack([tsvad_stream_inputs(4 * T_lab, 100 + b)[1][0] for b in range(B)])
    y = m.forward_windows(torch.from_numpy(xs).to(gpu), torch.from_numpy(ts), T_lab, dcs, left).cpu().numpy()
    for b in range(B):
        yb = m.forward_chunk_by_chunk(torch.from_numpy(xs[b:b + 1]), torch.from_numpy(ts[b:b + 1]), T_lab, dcs,
                                      left).cpu().numpy()
        assert np.abs(y[b:b + 1] - yb).max() < 1e-5, b
    with torch.no_grad():
        ref = forward_chunk_by_chunk(to_torch(sd), torch.from_numpy(xs[:1]), torch.from_numpy(ts[:1]), T_lab, dcs,
                                     left).numpy()
    assert np.abs(y[:1] - ref).max() < 1e-3


@pytest.mark.parametrize("T_lab,dcs", [(26, 25), (51, 5), (12, 1)])
def test_stream_one_label_chunks_vs_oracle(gpu, T_lab, dcs):
    """Chunks of a single label frame (4 fbank frames -> CAM++ 2 -> speech_down_or_up 1), as the
    last chunk of every window with n_labels % chunk == 1 and every chunk at chunk size 1."""
    from oracle.tsvad_stream_ref import forward_chunk_by_chunk
    sd = tsvad_streaming_state_dict(TSVADStreamingConfig(), seed=93)
    xs, ts = tsvad_stream_inputs(4 * T_lab, 94)
    m = TSVADStreamingModel(device=gpu, precision="fp32", max_labels=64).load_state_dict(to_torch(sd))
    y = m.forward_chunk_by_chunk(torch.from_numpy(xs), torch.from_numpy(ts), T_lab, dcs).cpu().numpy()
    with torch.no_grad():
        ref = forward_chunk_by_chunk(to_torch(sd), torch.from_numpy(xs), torch.from_numpy(ts), T_lab, dcs).numpy()
    assert np.abs(y - ref).max() < 1e-3


@pytest.mark.parametrize("precision", ["fp32", "bf16"])
def test_streaming_pipeline_ragged_meeting_vs_oracle(gpu, precision):
    """StreamingWindowDecoder inside TSVADPipeline on a meeting with n_labels % 25 != 0: every
    window (the shrinking tail windows included) must equal the reference recipe's decode of that
    window alone (batch 1, its own length: oracle chunk loop on the window's fbank + CMN)."""
    from oracle.fbank_ref import window_fbank
    from oracle.tsvad_stream_ref import forward_chunk_by_chunk
    from speaker_diarization_amd.synth import make_meeting, speaker_embeddings
    from speaker_diarization_amd.ts_vad.pipeline import TSVADPipeline
    from speaker_diarization_amd.ts_vad.streaming import StreamingWindowDecoder
    meeting = make_meeting(40.0 + 13 * 0.04 + 0.01, n_spk=4, seed=95)
    n_lab = meeting.wav.size // 640
    assert n_lab % 25 == 13
    sd = tsvad_streaming_state_dict(TSVADStreamingConfig(), seed=96)
    m = TSVADStreamingModel(device=gpu, precision=precision, max_labels=250, max_windows=16).load_state_dict(
        to_torch(sd))
    pipe = TSVADPipeline(StreamingWindowDecoder(m, 25, -1), segment_shift=1, batch_size=64)
    assert pipe.batch_size == 1
    ts = speaker_embeddings(4, seed=96)
    wav = torch.from_numpy(meeting.wav).to(gpu)
    plan = pipe.plan(n_lab)
    lg = pipe.window_logits(wav, torch.from_numpy(ts).to(gpu), plan).cpu().numpy()
    spl = plan.samples_per_label
    check = [0, 7] + list(range(plan.n_win - 11, plan.n_win))
    tol = 1e-3 if precision == "fp32" else 8e-2
    for w in check:
        s, e = int(plan.starts[w]), int(plan.ends[w])
        f = torch.from_numpy(window_fbank(meeting.wav[s * spl:e * spl]))[None]
        with torch.no_grad():
            ref = forward_chunk_by_chunk(to_torch(sd), f, torch.from_numpy(ts)[None], e - s, 25, -1).numpy()[0]
        err = np.abs(lg[w, :, : e - s] - ref).max()
        assert err < tol, (w, e - s, err)
