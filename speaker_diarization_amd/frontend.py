"""Feature frontends on the MI355X path.

kaldi_fbank(): FBank.__call__ of egs/alimeeting/ts_vad2/ts_vad_dataset.py:29-56
(torchaudio.compliance.kaldi.fbank, 80 HTK mel bins, hamming, use_energy=False)
computed by the HIP kernel over a whole recording; window_cmn() slices per-window
frames, subtracts the per-window mean (mean_nor=True) and zero-pads to the batch
maximum like TSVADDataset.collater (ts_vad_dataset.py:664-701).
"""
from __future__ import annotations

import math
from functools import lru_cache

import numpy as np

from . import _lib

FRAME_LEN = 400   # 25 ms @ 16 kHz
FRAME_SHIFT = 160  # 10 ms
NFFT = 512


def num_frames(n_samples: int) -> int:
    """Kaldi snip_edges frame count: 1 + (N - 400) // 160 (0 if N < 400)."""
    if n_samples < FRAME_LEN:
        return 0
    return 1 + (n_samples - FRAME_LEN) // FRAME_SHIFT


@lru_cache(maxsize=8)
def kaldi_mel_banks(n_mels: int = 80, sample_rate: float = 16000.0, low_freq: float = 20.0,
                    high_freq: float = 0.0) -> np.ndarray:
    """HTK-mel triangular banks (n_mels, 257), float32, last column zero — the
    kaldi `get_mel_banks` construction (vtln_warp 1.0) as used by kaldi.fbank."""
    num_fft_bins = NFFT // 2
    nyquist = 0.5 * sample_rate
    if high_freq <= 0.0:
        high_freq += nyquist
    fft_bin_width = np.float32(sample_rate / NFFT)
    mel_lo = 1127.0 * math.log(1.0 + low_freq / 700.0)
    mel_hi = 1127.0 * math.log(1.0 + high_freq / 700.0)
    delta = (mel_hi - mel_lo) / (n_mels + 1)
    b = np.arange(n_mels, dtype=np.float32)[:, None]
    left = (np.float32(mel_lo) + b * np.float32(delta)).astype(np.float32)
    center = (np.float32(mel_lo) + (b + 1.0) * np.float32(delta)).astype(np.float32)
    right = (np.float32(mel_lo) + (b + 2.0) * np.float32(delta)).astype(np.float32)
    f = (fft_bin_width * np.arange(num_fft_bins, dtype=np.float32)).astype(np.float32)
    mel = (np.float32(1127.0) * np.log1p(f / np.float32(700.0))).astype(np.float32)[None, :]
    up = (mel - left) / (center - left)
    down = (right - mel) / (right - center)
    banks = np.maximum(np.float32(0.0), np.minimum(up, down)).astype(np.float32)
    return np.pad(banks, ((0, 0), (0, 1)))


_fb_cache: dict = {}


def _mel_device(n_mels: int, device):
    import torch
    key = (n_mels, str(device))
    if key not in _fb_cache:
        _fb_cache[key] = torch.from_numpy(kaldi_mel_banks(n_mels)).to(device)
    return _fb_cache[key]


def kaldi_fbank(wav, n_mels: int = 80, scale: float = float(1 << 15), out=None):
    """wav: 1-D float32 CUDA tensor in [-1, 1) -> (n_frames, n_mels) log-mel (dither 0)."""
    import torch
    assert wav.is_cuda and wav.dtype == torch.float32 and wav.dim() == 1
    n = num_frames(wav.numel())
    if out is None:
        out = torch.empty(n, n_mels, device=wav.device, dtype=torch.float32)
    fb = _mel_device(n_mels, wav.device)
    _lib.call("sd_fbank_kaldi", _lib.ptr(wav.contiguous()), wav.numel(), scale, n, _lib.ptr(fb), n_mels,
              _lib.ptr(out), _lib.stream_ptr(wav.device))
    return out


def window_cmn(feats, win_start, win_n, T_out: int, out=None):
    """feats (F, n_mels) CUDA; win_start/win_n int32 CUDA (n_win) -> (n_win, T_out, n_mels)."""
    import torch
    n_win = win_start.numel()
    n_mels = feats.shape[1]
    if out is None:
        out = torch.empty(n_win, T_out, n_mels, device=feats.device, dtype=torch.float32)
    _lib.call("sd_window_cmn", _lib.ptr(feats), n_mels, _lib.ptr(win_start), _lib.ptr(win_n), n_win, T_out,
              _lib.ptr(out), _lib.stream_ptr(feats.device))
    return out
