"""Frontend kernels on REAL speech (tests/golden/sample_wav.npz: pyannote's 30-s, 16 kHz, 2-speaker
sample.wav) against the CPU oracles, where every other frontend case runs synthetic pulse trains:
 - kaldi fbank (fbank.hip; ts_vad_dataset.py:29-56, hamming, x 2^15) over the whole file, the TS-VAD
   pipeline's per-window CMN slices (ts_vad_dataset.py:55) and the embedding extractor's povey fbank
   (generate_chunk_..._for_diarization.py:307-331) vs oracle/fbank_ref.py;
 - the EEND frontend (eend.hip: feature.stft + logmel23 / logmel23_mn + splice + subsample,
   feature.py:64-184) at 8 kHz (the file decimated by 2, as data) vs oracle/eend_ref.py.
Bounds are the synthetic cases' (fp32 fbank 2e-3 abs + 1e-4 rel; fp64 STFT path 1e-5).  The oracles are
parity-unpinned against torchaudio 2.5.1 / librosa 0.10.2 (absent here)."""
import os

import numpy as np
import pytest
import torch

from oracle import eend_ref, fbank_ref
from speaker_diarization_amd import frontend
from speaker_diarization_amd.feature import eend_features
from speaker_diarization_amd.ts_vad.embedding import kaldi_fbank_povey

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")


def _wav():
    return np.load(os.path.join(GOLD, "sample_wav.npz"))["pcm16"].astype(np.float32) / 32768.0


def test_kaldi_fbank_real_speech(gpu):
    wav = _wav()
    ref = fbank_ref.fbank(wav)
    out = frontend.kaldi_fbank(torch.from_numpy(wav).to(gpu)).cpu().numpy()
    assert out.shape == ref.shape
    np.testing.assert_allclose(out, ref, atol=2e-3, rtol=1e-4)


def test_window_cmn_real_speech(gpu):
    """The pipeline's windows (one fbank pass, window slices, per-window mean removal) == the reference's
    per-window FBank(mean_nor=True) of each window's own samples (6-s windows, 1-s shift)."""
    wav = _wav()
    feats = frontend.kaldi_fbank(torch.from_numpy(wav).to(gpu))
    starts = [0, 100, 1000, 2400]            # fbank frames = label frames x 4 (40 ms / 10 ms)
    n = 598
    st = torch.tensor(starts, dtype=torch.int32, device=gpu)
    ns = torch.tensor([n] * len(starts), dtype=torch.int32, device=gpu)
    out = frontend.window_cmn(feats, st, ns, n).cpu().numpy()
    for i, s in enumerate(starts):
        ref = fbank_ref.window_fbank(wav[s * 160:s * 160 + 96000])
        assert ref.shape == (n, 80)
        np.testing.assert_allclose(out[i], ref, atol=2e-3, rtol=1e-4)


def test_povey_fbank_real_speech(gpu):
    wav = _wav()[:16000 * 6]
    ref = fbank_ref.fbank(wav, scale=1.0, window="povey")
    out = kaldi_fbank_povey(torch.from_numpy(wav).to(gpu)).cpu().numpy()
    np.testing.assert_allclose(out, ref, atol=2e-3, rtol=1e-4)


@pytest.mark.parametrize("transform", ["logmel23", "logmel23_mn"])
def test_eend_frontend_real_speech(gpu, transform):
    wav8 = _wav()[::2].astype(np.float64)
    ref = eend_ref.features(wav8, 8000, 200, 80, 7, 10, transform)
    got = eend_features(torch.from_numpy(wav8.astype(np.float32)).to(gpu), 8000, 200, 80, transform, 7, 10)
    got = got.cpu().numpy()[:, :345]
    assert got.shape == ref.shape
    np.testing.assert_allclose(got, ref, atol=1e-5, rtol=0)
