"""Hashes of the GPU Kaldi fbank and the EEND STFT log-mel features of fixed signals (A/B bit identity across
launch shapes)."""
import hashlib
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from speaker_diarization_amd import frontend  # noqa: E402
from speaker_diarization_amd.feature import eend_features  # noqa: E402

rng = np.random.default_rng(7)
for n in (16000 * 600 + 77, 16000 * 3 + 5):
    wav = torch.from_numpy((rng.standard_normal(n) * 0.1).astype(np.float32)).cuda()
    out = frontend.kaldi_fbank(wav).cpu().numpy()
    print("fbank", n, out.shape, hashlib.sha256(out.tobytes()).hexdigest()[:16], flush=True)
for n, sr, fs, fsh in ((16000 * 600 + 77, 16000, 400, 160), (8000 * 600 + 31, 8000, 200, 80), (16000 * 3 + 5, 16000, 400, 160)):
    wav = torch.from_numpy((rng.standard_normal(n) * 0.1).astype(np.float32)).cuda()
    out = eend_features(wav, sr, fs, fsh).cpu().numpy()
    print("eend", n, sr, out.shape, hashlib.sha256(out.tobytes()).hexdigest()[:16], flush=True)
