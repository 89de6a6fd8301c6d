"""Streaming FS-EEND (sd_fseend_stream_*: K/V histories + hipGraph replay) against the
whole-recording test() path, the CPU oracle and the reference golden vector.

The reference has no streaming entry point: it recomputes OnlineTransformerDADiarization.test()
(fs_eend.py:79-96) over the whole recording.  With its causal masks (mask_delay 0 in every
shipped config) the concatenated stream output must equal that forward.  Tolerances: fp32
1e-3 (north_star), bf16 3e-2; graph replay vs direct launches: bit-identical."""
import os

import numpy as np
import pytest
import torch

from oracle import fseend_ref
from speaker_diarization_amd._lib import SdiarError
from speaker_diarization_amd.fs_eend.model import OnlineTransformerDADiarization
from speaker_diarization_amd.weights import FSEENDConfig, fseend_state_dict, to_torch
from tests.golden.make_golden import FSEEND_CASES, eda_inputs

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")
FP32_ATOL = 1e-3
BF16_ATOL = 3e-2


def _model(wseed, precision="fp32", max_frames=2048, delay=0):
    m = OnlineTransformerDADiarization(n_speakers=None, in_size=345, n_units=256, n_heads=4, enc_n_layers=4,
                                       dec_n_layers=2, dropout=0.1, has_mask=True, max_seqlen=10000,
                                       dec_dim_feedforward=2048, conv_delay=9, mask_delay=delay,
                                       precision=precision, max_seqs=1, max_frames=max_frames, max_nspks=6)
    m.load_state_dict(to_torch(fseend_state_dict(FSEENDConfig(mask_delay=delay), seed=wseed)))
    return m


def _stream_all(m, x, chunk, C=6, use_graph=True, pieces=None):
    s = m.stream(chunk=chunk, max_frames=x.shape[0] + 64, max_nspks=C, use_graph=use_graph)
    outs = []
    if pieces is None:
        pieces = [chunk] * (x.shape[0] // chunk + 1)
    i = 0
    for p in pieces:
        if i >= x.shape[0]:
            break
        outs.append(s.push(x[i : i + p]))
        i += p
    if i < x.shape[0]:
        outs.append(s.push(x[i:]))
    outs.append(s.flush())
    return torch.cat(outs, 0), s


@pytest.mark.parametrize("chunk", [1, 4, 7, 32])
def test_stream_matches_test_fp32(gpu, chunk):
    T = 157
    m = _model(801)
    x = torch.from_numpy(eda_inputs([T], seed=81)[0]).to(gpu)
    ref, _, _ = m.test([x], [T], max_nspks=6)
    out, _ = _stream_all(m, x, chunk)
    assert out.shape == (T, 6)
    np.testing.assert_allclose(out.cpu().numpy(), ref[0].cpu().numpy(), atol=FP32_ATOL)


def test_stream_matches_oracle_and_golden(gpu):
    lens, C, delay, iseed, wseed = FSEEND_CASES["fseend_T240"]
    g = dict(np.load(os.path.join(GOLD, "fseend_T240.npz")))
    m = _model(wseed)
    xs = eda_inputs(lens, seed=iseed)
    out, _ = _stream_all(m, torch.from_numpy(xs[0]).to(gpu), 5, C=C)
    np.testing.assert_allclose(out.cpu().numpy(), g["out"], atol=FP32_ATOL)
    sd = to_torch(fseend_state_dict(FSEENDConfig(), seed=wseed))
    ro, _, _ = fseend_ref.fseend_test(sd, FSEENDConfig(), [torch.from_numpy(xs[0])], lens, C)
    np.testing.assert_allclose(out.cpu().numpy(), ro[0].numpy(), atol=FP32_ATOL)


@pytest.mark.parametrize("chunk", [1, 3])      # 1: the fused slot block (stream_slot_block), 3: three launches
@pytest.mark.parametrize("precision", ["fp32", "bf16"])
def test_graph_replay_is_bit_identical(gpu, precision, chunk):
    T = 120
    m = _model(802, precision)
    x = torch.from_numpy(eda_inputs([T], seed=82)[0]).to(gpu)
    a, _ = _stream_all(m, x, chunk, use_graph=True)
    b, _ = _stream_all(m, x, chunk, use_graph=False)
    assert torch.equal(a, b)


def test_stream_bf16_vs_test(gpu):
    T = 300
    m = _model(803, "bf16")
    x = torch.from_numpy(eda_inputs([T], seed=83)[0]).to(gpu)
    ref, _, _ = m.test([x], [T], max_nspks=6)
    out, _ = _stream_all(m, x, 8)
    np.testing.assert_allclose(out.cpu().numpy(), ref[0].cpu().numpy(), atol=BF16_ATOL)
    sd = to_torch(fseend_state_dict(FSEENDConfig(), seed=803))
    ro, _, _ = fseend_ref.fseend_test(sd, FSEENDConfig(), [x.cpu()], [T], 6)
    np.testing.assert_allclose(out.cpu().numpy(), ro[0].numpy(), atol=BF16_ATOL)


def test_stream_long_many_key_tiles(gpu):
    """T = 1100 frames: several 256-key attention blocks and ragged last tiles."""
    T = 1100
    m = _model(804, max_frames=T)
    x = torch.from_numpy(eda_inputs([T], seed=84)[0]).to(gpu)
    ref, _, _ = m.test([x], [T], max_nspks=6)
    out, _ = _stream_all(m, x, 16)
    np.testing.assert_allclose(out.cpu().numpy(), ref[0].cpu().numpy(), atol=FP32_ATOL)


@pytest.mark.parametrize("chunk", [1, 3])
def test_merge_counters_wrap_to_zero(gpu, chunk):
    """The decode attention's and the slot block's last-arriver counters: a wrapping increment
    that is back at 0 after every launch, here with a block count that does not divide 2^32 (1164 frames ->
    5 blocks per (slot, head)), across graph replays and a reset; the scores stay those of test()."""
    T = 1100
    m = _model(804, max_frames=T)
    x = torch.from_numpy(eda_inputs([T], seed=84)[0]).to(gpu)
    ref, _, _ = m.test([x], [T], max_nspks=6)
    s = m.stream(chunk=chunk, max_frames=T + 64, max_nspks=6, use_graph=True)
    assert (s.debug_counters() == 0).all()
    for rep in range(2):
        outs = []
        for i in range(0, T, chunk):
            outs.append(s.push(x[i : i + chunk]))
            if (i // chunk) % 97 == 5:
                c = s.debug_counters()
                assert c.size == 6 * 4 + 1 and (c == 0).all(), c
        outs.append(s.flush())
        assert (s.debug_counters() == 0).all()
        np.testing.assert_allclose(torch.cat(outs).cpu().numpy(), ref[0].cpu().numpy(), atol=FP32_ATOL)
        s.reset()


@pytest.mark.parametrize("T", [1, 5, 9, 10, 28])
def test_short_recordings_flush(gpu, T):
    """Shorter than the 9-frame look-ahead: every score comes out of flush()."""
    m = _model(805, max_frames=64)
    x = torch.from_numpy(eda_inputs([T], seed=85 + T)[0]).to(gpu)
    ref, _, _ = m.test([x], [T], max_nspks=6)
    out, _ = _stream_all(m, x, 4)
    np.testing.assert_allclose(out.cpu().numpy(), ref[0].cpu().numpy(), atol=FP32_ATOL)


def test_ragged_pushes_and_reset(gpu):
    T = 90
    m = _model(806)
    x = torch.from_numpy(eda_inputs([T], seed=86)[0]).to(gpu)
    ref, _, _ = m.test([x], [T], max_nspks=6)
    s = m.stream(chunk=4, max_frames=256)
    for _ in range(2):   # second pass after reset() reuses the histories and captured graphs
        outs, i = [], 0
        for p in [1, 6, 13, 2, 30, 11, 27]:
            outs.append(s.push(x[i : i + p]))
            i += p
        outs.append(s.flush())
        out = torch.cat(outs)
        np.testing.assert_allclose(out.cpu().numpy(), ref[0].cpu().numpy(), atol=FP32_ATOL)
        s.reset()


def test_stream_errors(gpu):
    m = _model(807, max_frames=64)
    with pytest.raises(ValueError):
        m.stream(chunk=33)
    with pytest.raises(ValueError):
        m.stream(chunk=4, max_nspks=7)
    s = m.stream(chunk=4, max_frames=8)
    x = torch.from_numpy(eda_inputs([20], seed=87)[0]).to(gpu)
    s.push(x[:8])
    with pytest.raises(ValueError, match="max_frames"):
        s.push(x[8:12])
    s2 = m.stream(chunk=4, max_frames=64)
    s2.push(x[:4])
    s2.flush()
    with pytest.raises(SdiarError, match="ended"):
        s2.push(x[4:8])
    md = _model(808, max_frames=64, delay=2)
    with pytest.raises(ValueError, match="mask_delay"):
        md.stream(chunk=4)


# ----------------------------------------------------------------------------- audio in (latency mode)
def _wav8k(seconds, seed, extra=0):
    from speaker_diarization_amd.synth import make_meeting
    w = make_meeting(seconds, n_spk=3, seed=seed, sample_rate=8000).wav.astype(np.float32)
    return w[: int(seconds * 8000) + extra] if extra >= 0 else w[: int(seconds * 8000) + extra]


def _audio_stream(m, wav, chunk, pieces, precision_graph=True):
    s = m.stream(chunk=chunk, max_frames=wav.size // 800 + 64, use_graph=precision_graph).set_audio()
    x = torch.from_numpy(wav).cuda()
    outs, i, k = [], 0, 0
    while i < wav.size:
        p = pieces[k % len(pieces)]
        outs.append(s.push_audio(x[i : i + p]))
        i += p
        k += 1
    outs.append(s.flush())
    return torch.cat(outs, 0), s


def _whole(m, wav):
    from speaker_diarization_amd.feature import eend_features
    f = eend_features(torch.from_numpy(wav).cuda(), 8000, 200, 80, "logmel23", 7, 10, ld=m.in_ld)
    out, _, _ = m.test_device(f[None], [f.shape[0]], 6, want_emb=False, want_attractors=False)
    return out[0]


@pytest.mark.parametrize("seconds,extra,chunk", [(30.0, 0, 1), (30.0, 37, 4), (12.0, -80 * 3, 7), (25.0, 5, 32)])
def test_audio_stream_matches_test_fp32(gpu, seconds, extra, chunk):
    """80 ms pushes (640 samples at 8 kHz) of raw audio == eend_features(whole wav) + test(): lengths
    with and without the multiple-of-hop last-frame drop (feature.py:176-184), chunks 1..32."""
    wav = _wav8k(seconds, 90 + chunk, extra)
    m = _model(811, max_frames=wav.size // 800 + 64)
    ref = _whole(m, wav)
    out, _ = _audio_stream(m, wav, chunk, [640])
    assert out.shape == ref.shape, (out.shape, ref.shape)
    np.testing.assert_allclose(out.cpu().numpy(), ref.cpu().numpy(), atol=FP32_ATOL)


def test_audio_stream_matches_oracle(gpu):
    """Against the CPU oracle end to end: the restated librosa frontend (fp64) + fs_eend.py test()."""
    from oracle import eend_ref
    wav = _wav8k(20.0, 95, 13)
    m = _model(812, max_frames=400)
    out, _ = _audio_stream(m, wav, 2, [640, 17, 1300])
    Y = eend_ref.features(wav.astype(np.float64), 8000, 200, 80, 7, 10, "logmel23")
    sd = to_torch(fseend_state_dict(FSEENDConfig(), seed=812))
    ro, _, _ = fseend_ref.fseend_test(sd, FSEENDConfig(), [torch.from_numpy(np.ascontiguousarray(Y, np.float32))],
                                      [len(Y)], 6)
    assert out.shape[0] == len(Y)
    np.testing.assert_allclose(out.cpu().numpy(), ro[0].numpy(), atol=FP32_ATOL)


def test_audio_stream_bf16_graph_and_ragged(gpu):
    """bf16, chunk 1: graph replay == direct launches bit for bit, ragged pushes == 80 ms pushes bit for
    bit (the frontend rows do not depend on how the audio was cut), and both == test() within bf16."""
    wav = _wav8k(24.0, 97, 3)
    m = _model(813, "bf16", max_frames=400)
    a, _ = _audio_stream(m, wav, 1, [640])
    b, _ = _audio_stream(m, wav, 1, [640], precision_graph=False)
    c, _ = _audio_stream(m, wav, 1, [1, 799, 5000, 64, 640 * 7 + 3])
    assert torch.equal(a, b) and torch.equal(a, c)
    np.testing.assert_allclose(a.cpu().numpy(), _whole(m, wav).cpu().numpy(), atol=BF16_ATOL)


@pytest.mark.parametrize("n", [200, 500, 800, 881, 1600])
def test_audio_stream_short_inputs(gpu, n):
    """Shorter than one model frame's look-ahead: everything comes out of flush()."""
    wav = _wav8k(1.0, 99, 0)[:n]
    m = _model(814, max_frames=64)
    out, _ = _audio_stream(m, wav, 4, [640])
    np.testing.assert_allclose(out.cpu().numpy(), _whole(m, wav).cpu().numpy(), atol=FP32_ATOL)


def test_audio_stream_reset_modes_and_errors(gpu):
    wav = _wav8k(6.0, 98, 0)
    m = _model(815, max_frames=128)
    ref = _whole(m, wav).cpu().numpy()
    s = m.stream(chunk=3, max_frames=128)
    with pytest.raises(RuntimeError, match="set_audio"):
        s.push_audio(torch.zeros(10))
    for _ in range(2):
        s.set_audio()
        outs = [s.push_audio(torch.from_numpy(wav[i : i + 640]).cuda()) for i in range(0, wav.size, 640)]
        np.testing.assert_allclose(torch.cat(outs + [s.flush()]).cpu().numpy(), ref, atol=FP32_ATOL)
        with pytest.raises(SdiarError, match="ended"):
            s.push_audio(torch.zeros(10).cuda())
        s.reset()
    # back to feature rows after reset: same scores from the whole-recording features
    from speaker_diarization_amd.feature import eend_features
    f = eend_features(torch.from_numpy(wav).cuda(), 8000, 200, 80, "logmel23", 7, 10)[:, :345]
    np.testing.assert_allclose(torch.cat([s.push(f), s.flush()]).cpu().numpy(), ref, atol=FP32_ATOL)
    s.reset()
    s.set_audio()
    with pytest.raises(SdiarError, match="audio"):
        s._push_rows(f[:3])
