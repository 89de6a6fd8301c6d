"""speaker_diarization/feature.py on the MI355X path (EEND / EEND-EDA / FS-EEND frontend).

`eend_features(wav)` = feature.stft -> feature.transform -> feature.splice ->
[::subsampling] (eend_eda/infer_eda.py:94-98) as one HIP pipeline over a
recording already in HBM: centred float64 STFT + Slaney log-mel per frame,
per-recording mean (logmel23_mn), splice/subsample into 352-wide f32 rows that
the EDA input GEMM reads directly.  Only the mel basis (librosa.filters.mel,
a constant) is built on the host.
"""
from __future__ import annotations

from functools import lru_cache

import numpy as np

from . import _lib

TRANSFORMS = {"logmel23_mn": 1, "logmel23": 0}


def get_input_dim(frame_size: int, context_size: int, transform_type: str) -> int:
    """feature.get_input_dim (feature.py:10-21)."""
    if transform_type.startswith("logmel23"):
        dim = 23
    else:
        fft_size = 1 << (frame_size - 1).bit_length()
        dim = fft_size // 2 + 1
    return (2 * context_size + 1) * dim


def stft_num_frames(n_samples: int, frame_shift: int) -> int:
    """Frames of feature.stft: librosa centred frames 1 + N // hop, minus the
    last one when N % hop == 0 (feature.py:176-184, _count_frames :187-192)."""
    n = 1 + n_samples // frame_shift
    return n - 1 if n_samples % frame_shift == 0 else n


def _hz_to_mel(f: np.ndarray) -> np.ndarray:
    f_sp, min_log_hz = 200.0 / 3, 1000.0
    min_log_mel, logstep = min_log_hz / f_sp, np.log(6.4) / 27.0
    lin = f / f_sp
    return np.where(f >= min_log_hz, min_log_mel + np.log(np.maximum(f, min_log_hz) / min_log_hz) / logstep, lin)


def _mel_to_hz(m: np.ndarray) -> np.ndarray:
    f_sp, min_log_hz = 200.0 / 3, 1000.0
    min_log_mel, logstep = min_log_hz / f_sp, np.log(6.4) / 27.0
    return np.where(m >= min_log_mel, min_log_hz * np.exp(logstep * (m - min_log_mel)), f_sp * m)


@lru_cache(maxsize=8)
def slaney_mel(sample_rate: int, n_fft: int, n_mels: int = 23) -> np.ndarray:
    """librosa.filters.mel(sr, n_fft, n_mels) with its defaults (fmin 0, fmax sr/2,
    Slaney scale, area normalisation, float32): (n_mels, 1 + n_fft // 2)."""
    n_bins = 1 + n_fft // 2
    freqs = np.arange(n_bins) * (1.0 / (n_fft * (1.0 / sample_rate)))   # np.fft.rfftfreq(n_fft, 1/sr)
    edges = _mel_to_hz(np.linspace(_hz_to_mel(np.float64(0.0)), _hz_to_mel(np.float64(sample_rate / 2.0)),
                                   n_mels + 2))
    width = np.diff(edges)
    w = np.zeros((n_mels, n_bins), dtype=np.float32)
    for i in range(n_mels):
        rise = (freqs - edges[i]) / width[i]
        fall = (edges[i + 2] - freqs) / width[i + 1]
        w[i] = np.maximum(0.0, np.minimum(rise, fall))
    w *= (2.0 / (edges[2:] - edges[:-2]))[:, None]
    return w


_mel_cache: dict = {}


def _mel_device(sample_rate: int, n_fft: int, device):
    import torch
    key = (sample_rate, n_fft, str(device))
    if key not in _mel_cache:
        _mel_cache[key] = torch.from_numpy(slaney_mel(sample_rate, n_fft)).to(device)
    return _mel_cache[key]


def eend_features(wav, sample_rate: int = 16000, frame_size: int = 400, frame_shift: int = 160,
                  transform_type: str = "logmel23_mn", context_size: int = 7, subsampling: int = 10,
                  ld: int = 352, out=None):
    """wav: 1-D float32 CUDA tensor (soundfile-scaled samples) -> (ceil(F/subsampling), ld)
    f32 CUDA features; columns [(2c+1)*23, ld) are zero."""
    import torch
    if transform_type not in TRANSFORMS:
        raise ValueError("Unknown transform_type: %s" % transform_type)
    assert wav.is_cuda and wav.dtype == torch.float32 and wav.dim() == 1
    n_frames = stft_num_frames(wav.numel(), frame_shift)
    if n_frames < 1:
        raise ValueError("recording shorter than one STFT frame")
    n_fft = 1 << (frame_size - 1).bit_length()
    n_out = -(-n_frames // subsampling)
    width = (2 * context_size + 1) * 23
    if ld < width:
        raise ValueError(f"ld {ld} < spliced width {width}")
    if out is None:
        out = torch.empty(n_out, ld, device=wav.device, dtype=torch.float32)
    work = torch.empty(n_frames * 23 + 23, device=wav.device, dtype=torch.float64)
    fb = _mel_device(sample_rate, n_fft, wav.device)
    _lib.call("sd_eend_features", _lib.ptr(wav.contiguous()), wav.numel(), frame_size, frame_shift, n_frames,
              _lib.ptr(fb), 23, TRANSFORMS[transform_type], context_size, subsampling, _lib.ptr(work),
              _lib.ptr(out), ld, _lib.stream_ptr(wav.device))
    return out
