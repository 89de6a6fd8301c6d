"""Oracle pinning: CPU restatement vs reference golden vectors (tests/golden)."""
import numpy as np
import pytest
import torch

from make_golden import TSVAD_CASES, TSVAD_DYN_CASES, TSVAD_NAN_CASES, tsvad_case_inputs, tsvad_inputs
from oracle import fbank_ref
from oracle.tsvad_ref import speech_encoder_out, tsvad_forward
from speaker_diarization_amd.weights import TSVADConfig, tsvad_state_dict, to_torch
from speaker_diarization_amd import frontend


def _cfg(variant, rs):
    return TSVADConfig(rs_len=rs) if variant == 0 else TSVADConfig.ots_vad_v1(rs_len=rs)


@pytest.mark.parametrize("name", list(TSVAD_CASES))
def test_tsvad_oracle_matches_reference(name):
    v, rs, B, T, nl, iseed, wseed = TSVAD_CASES[name]
    g = np.load(f"{__file__.rsplit('/', 1)[0]}/golden/{name}.npz")
    cfg = _cfg(v, rs)
    sd = to_torch(tsvad_state_dict(cfg, seed=wseed))
    x, ts = tsvad_inputs(B, T, nl, seed=iseed)
    out = tsvad_forward(sd, cfg, torch.from_numpy(x), torch.from_numpy(ts), nl).numpy()
    np.testing.assert_allclose(out, g["logits"], atol=2e-5, rtol=1e-5)
    enc = speech_encoder_out(sd, torch.from_numpy(x)).numpy()
    np.testing.assert_allclose(enc, g["speech_enc"], atol=1e-5, rtol=1e-5)


@pytest.mark.parametrize("name", list(TSVAD_DYN_CASES))
def test_tsvad_oracle_dynamic_variant_matches_reference(name):
    """The 'dynamic' weight variant (weights.dynamic_weights: centred / scaled gsp_fc and BiLSTM input, fc x4) on
    windows of the bench meeting, pinned by the reference run (make_golden.py TSVAD_DYN_CASES); the fixture
    holds the window fbanks.  The logits move with the frame (std across frames 0.6-1.1, vs 0.03-0.3 plain)."""
    v, rs = TSVAD_DYN_CASES[name][:2]
    g = np.load(f"{__file__.rsplit('/', 1)[0]}/golden/{name}.npz")
    cfg = _cfg(v, rs)
    sd = to_torch(tsvad_state_dict(cfg, seed=777, dynamic=True))
    out = tsvad_forward(sd, cfg, torch.from_numpy(g["ref_speech"]), torch.from_numpy(g["ts"]), int(g["n_label"])).numpy()
    np.testing.assert_allclose(out, g["logits"], atol=5e-5, rtol=1e-5)
    assert g["logits"].std(axis=-1).mean() > 0.5


@pytest.mark.parametrize("name", list(TSVAD_NAN_CASES))
def test_tsvad_oracle_nan_bypass_matches_reference(name):
    """BatchNorm1D (model.py:161-171): one NaN fbank value in window w -> the reference skips the wrapped
    BatchNorm for EVERY window of the batch and window w's logits are NaN.  The oracle restates it and is
    pinned by the reference run on that input (make_golden.py TSVAD_NAN_CASES)."""
    (v, rs, B, T, nl, iseed, wseed), x, ts = tsvad_case_inputs(name)
    g = np.load(f"{__file__.rsplit('/', 1)[0]}/golden/{name}.npz")
    cfg = _cfg(v, rs)
    sd = to_torch(tsvad_state_dict(cfg, seed=wseed))
    out = tsvad_forward(sd, cfg, torch.from_numpy(x), torch.from_numpy(ts), nl).numpy()
    bad = TSVAD_NAN_CASES[name][1]
    assert np.isnan(g["logits"][bad]).all() and np.isnan(out[bad]).all()
    keep = [i for i in range(B) if i != bad]
    np.testing.assert_allclose(out[keep], g["logits"][keep], atol=2e-5, rtol=1e-5)
    # the bypass is real: the finite windows differ from the same windows in a batch without the NaN
    base = np.load(f"{__file__.rsplit('/', 1)[0]}/golden/{TSVAD_NAN_CASES[name][0]}.npz")["logits"]
    assert np.abs(base[keep] - g["logits"][keep]).max() > 1e-3


def test_tsvad_golden_shapes():
    for name, (v, rs, B, T, nl, *_r) in TSVAD_CASES.items():
        g = np.load(f"{__file__.rsplit('/', 1)[0]}/golden/{name}.npz")
        assert g["logits"].shape == (B, 4, nl)
        assert int(g["variant"]) == v and int(g["T_fb"]) == T


def test_fbank_frame_count_and_banks():
    # kaldi snip_edges: 1 + (N - 400) // 160: 4 s -> 398, 6 s -> 598
    assert frontend.num_frames(64000) == 398 and frontend.num_frames(96000) == 598
    assert frontend.num_frames(399) == 0 and frontend.num_frames(400) == 1
    f = fbank_ref.fbank(np.zeros(64000, np.float32) + 0.01)
    assert f.shape == (398, 80)
    a = fbank_ref.mel_banks()
    b = frontend.kaldi_mel_banks(80)
    assert a.shape == b.shape == (80, 257)
    np.testing.assert_allclose(a, b, atol=2e-5)
    assert (a[:, -1] == 0).all() and (a.sum(1) > 0).all()
    # triangles: each bank peaks below 1 and is contiguous
    for row in a:
        nz = np.flatnonzero(row)
        assert nz.size and (np.diff(nz) == 1).all() and row.max() <= 1.0


def test_fbank_matches_direct_dft():
    rng = np.random.default_rng(0)
    wav = (rng.standard_normal(2000) * 0.1).astype(np.float32)
    f = fbank_ref.fbank(wav)
    # frame 3 by a literal DFT of the kaldi-processed frame
    x = wav[3 * 160: 3 * 160 + 400].astype(np.float64) * 32768
    x = x - x.mean()
    x = x - 0.97 * np.concatenate([x[:1], x[:-1]])
    x = x * (0.54 - 0.46 * np.cos(2 * np.pi * np.arange(400) / 399))
    n = np.arange(512)
    k = np.arange(257)[:, None]
    X = (np.pad(x, (0, 112))[None, :] * np.exp(-2j * np.pi * k * n / 512)).sum(1)
    e = (np.abs(X) ** 2) @ fbank_ref.mel_banks().T
    np.testing.assert_allclose(f[3], np.log(np.maximum(e, np.finfo(np.float32).eps)), rtol=1e-5, atol=1e-4)


def test_window_fbank_is_meeting_fbank_slice():
    """Frames of a window starting at label frame s are meeting frames 4s.. (the
    reuse the MI355X frontend relies on)."""
    rng = np.random.default_rng(1)
    wav = (rng.standard_normal(16000 * 8) * 0.1).astype(np.float32)
    full = fbank_ref.fbank(wav)
    s, e = 50, 150   # label frames, 640 samples each
    win = fbank_ref.fbank(wav[s * 640: e * 640])
    np.testing.assert_allclose(win, full[4 * s: 4 * s + win.shape[0]], rtol=1e-6, atol=1e-5)
