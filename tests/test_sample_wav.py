"""The real-speech fixture (tests/golden/sample_wav.npz: pyannote's 30-s, 16 kHz, 2-speaker sample.wav and its
RTTM, made by make_sample_fixture.py) and the CPU oracles' frontends on it: the kaldi fbank restatement
(oracle/fbank_ref.py, ts_vad_dataset.py:29-56) and the EEND STFT / logmel23_mn / splice restatement
(oracle/eend_ref.py, feature.py:64-184).  Both stay parity-unpinned against torchaudio / librosa (absent here);
the GPU kernels are held to them on this signal in test_gpu_real_speech.py."""
import os

import numpy as np

from oracle import eend_ref, fbank_ref
from speaker_diarization_amd.der import md_eval, read_rttm

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def sample():
    z = np.load(os.path.join(GOLD, "sample_wav.npz"))
    return z["pcm16"].astype(np.float32) / 32768.0, str(z["rttm"])


def test_fixture_is_the_30s_16k_sample():
    wav, rttm = sample()
    assert wav.shape == (480000,) and np.abs(wav).max() < 1.0 and np.abs(wav).std() > 1e-3
    data = read_rttm(rttm.splitlines())
    assert len(data) == 1 and len(next(iter(data.values())).speakers) == 2
    # the md-eval restatement scores the reference against itself as perfect, with and without a collar
    for collar in (0.0, 0.25):
        assert md_eval(rttm.splitlines(), rttm.splitlines(), collar=collar).der == 0.0


def test_oracle_frontends_on_real_speech():
    wav, _ = sample()
    f = fbank_ref.fbank(wav)                                   # hamming, x 2^15, dither 0
    assert f.shape == (1 + (480000 - 400) // 160, 80) and np.isfinite(f).all()
    # speech has structure the synthetic pulse trains lack: a wide per-bin dynamic range
    assert (f.max(0) - f.min(0)).min() > 5.0
    y = eend_ref.features(wav[::2].astype(np.float64), 8000, 200, 80, 7, 10, "logmel23")
    assert y.shape == (len(range(0, 1 + 240000 // 80 - (240000 % 80 == 0), 10)), 345) and np.isfinite(y).all()
