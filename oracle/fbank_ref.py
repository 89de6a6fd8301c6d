"""Kaldi fbank restated in numpy (float64) — oracle.

Restates torchaudio.compliance.kaldi.fbank (torchaudio 2.5.1, pinned by the
reference requirements; NOT installed here -> parity unpinned) for the call in
egs/alimeeting/ts_vad2/ts_vad_dataset.py:39-52: num_mel_bins=80, 16 kHz,
dither (0 here), window_type="hamming", use_energy=False, defaults otherwise
(frame 25 ms / shift 10 ms, snip_edges, remove_dc_offset, preemphasis 0.97,
round_to_power_of_two -> 512, use_power, use_log_fbank, low_freq 20,
high_freq 0 -> Nyquist).  Checked by invariants in tests/test_oracle.py.
"""
from __future__ import annotations

import math

import numpy as np


def mel_banks(n_mels=80, sr=16000.0, n_fft=512, low=20.0, high=0.0):
    """kaldi get_mel_banks (HTK mel 1127 ln(1 + f/700)), padded to n_fft/2+1 columns."""
    if high <= 0:
        high += sr / 2
    mel = lambda f: 1127.0 * np.log1p(np.asarray(f, np.float64) / 700.0)
    lo, hi = mel(low), mel(high)
    d = (hi - lo) / (n_mels + 1)
    b = np.arange(n_mels)[:, None]
    left, center, right = lo + b * d, lo + (b + 1) * d, lo + (b + 2) * d
    m = mel(sr / n_fft * np.arange(n_fft // 2))[None, :]
    w = np.maximum(0.0, np.minimum((m - left) / (center - left), (right - m) / (right - center)))
    return np.pad(w, ((0, 0), (0, 1)))


def fbank(wav, n_mels=80, sr=16000, scale=float(1 << 15), dither=0.0, rng=None, window="hamming"):
    """wav: (N,) float in [-1, 1) -> (1 + (N-400)//160, n_mels) float32.
    window "povey" (kaldi's default, hann^0.85) is the embedding extractor's
    (generate_chunk_speaker_embedding_from_modelscope_for_diarization.py:326-327)."""
    x = np.asarray(wav, np.float64) * scale
    fl, fs, nfft = 400, 160, 512
    if len(x) < fl:
        return np.zeros((0, n_mels), np.float32)
    nf = 1 + (len(x) - fl) // fs
    idx = np.arange(nf)[:, None] * fs + np.arange(fl)[None, :]
    fr = x[idx]
    if dither != 0.0:
        fr = fr + (rng or np.random.default_rng()).standard_normal(fr.shape) * dither
    fr = fr - fr.mean(axis=1, keepdims=True)
    prev = np.concatenate([fr[:, :1], fr[:, :-1]], axis=1)
    fr = fr - 0.97 * prev
    cw = np.cos(2 * math.pi * np.arange(fl) / (fl - 1))
    if window == "hamming":
        win = 0.54 - 0.46 * cw
    elif window == "povey":
        win = (0.5 - 0.5 * cw) ** 0.85
    else:
        raise ValueError(f"Invalid window type {window}")
    fr = fr * win
    spec = np.abs(np.fft.rfft(fr, n=nfft, axis=1)) ** 2
    e = spec @ mel_banks(n_mels, sr, nfft).T
    return np.log(np.maximum(e, np.finfo(np.float32).eps)).astype(np.float32)


def embed_fbank(wav_slice, n_mels=80):
    """FBank(80, mean_nor=True)(wav) of the embedding extractor
    (generate_chunk_..._for_diarization.py:307-331): povey window, dither 0, no 2^15 scale."""
    f = fbank(wav_slice, n_mels, scale=1.0, window="povey")
    return (f - f.mean(axis=0, keepdims=True)).astype(np.float32)


def window_fbank(wav_slice, n_mels=80):
    """FBank(80, mean_nor=True)(wav) of one window (ts_vad_dataset.py:39-56)."""
    f = fbank(wav_slice, n_mels)
    return (f - f.mean(axis=0, keepdims=True)).astype(np.float32)
