"""Deterministic synthetic multi-speaker meetings (no datasets offline).

Follows the structure of speaker_diarization/bin/random_mixture.py:101-145:
per speaker a sequence of utterances separated by exponential silences
(sil_scale 2 s), overlaps allowed.  Utterances are speaker-specific glottal
pulse trains through two formant resonators, normalised to -26 dBFS.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List

import numpy as np
from scipy import signal


@dataclass
class Meeting:
    wav: np.ndarray          # (n_samples,) float32
    labels: np.ndarray       # (n_spk, n_labels) {0,1} at label_rate
    segments: list           # [(spk, start_s, end_s)]
    sample_rate: int
    label_rate: int
    name: str

    def rttm_lines(self) -> List[str]:
        out = []
        for spk, s, e in sorted(self.segments, key=lambda x: (x[1], x[0])):
            out.append(f"SPEAKER {self.name} 1 {s:.3f} {e - s:.3f} <NA> <NA> {spk + 1} <NA> <NA>\n")
        return out


def make_meeting(duration_s: float, n_spk: int = 4, sample_rate: int = 16000, label_rate: int = 25,
                 seed: int = 777, sil_scale: float = 2.0, name: str = "meeting") -> Meeting:
    rng = np.random.default_rng(seed)
    n = int(round(duration_s * sample_rate))
    wav = np.zeros(n, np.float64)
    n_lab = n // (sample_rate // label_rate)
    labels = np.zeros((n_spk, n_lab), np.float32)
    segs = []
    for spk in range(n_spk):
        f0 = rng.uniform(90, 240)
        formants = (rng.uniform(400, 900), rng.uniform(1100, 2400))
        t = rng.exponential(sil_scale) * 0.5 + spk * 0.7
        while t < duration_s:
            dur = rng.uniform(0.8, 4.0)
            e = min(duration_s, t + dur)
            a, b = int(t * sample_rate), int(e * sample_rate)
            if b - a > sample_rate // 10:
                m = b - a
                tt = np.arange(m) / sample_rate
                vib = 1 + 0.03 * np.sin(2 * np.pi * rng.uniform(3, 6) * tt)
                phase = np.cumsum(f0 * vib / sample_rate)
                src = (np.diff(np.floor(phase), prepend=0.0) > 0).astype(np.float64)
                src += 0.05 * rng.standard_normal(m)
                y = src
                for fc in formants:
                    r = 0.97
                    w = 2 * np.pi * fc / sample_rate
                    y = signal.lfilter([1.0], [1.0, -2 * r * np.cos(w), r * r], y)
                env = np.minimum(1.0, np.minimum(tt, tt[-1] - tt) / 0.02 + 1e-3)
                y = y * env
                rms = np.sqrt(np.mean(y ** 2)) + 1e-12
                y *= (10 ** (-26 / 20)) / rms
                wav[a:b] += y
                la, lb = int(t * label_rate), int(np.ceil(e * label_rate))
                labels[spk, la:min(lb, n_lab)] = 1
                segs.append((spk, t, e))
            t = e + rng.exponential(sil_scale)
    wav = np.clip(wav, -1.0, 1.0 - 2 ** -15).astype(np.float32)
    return Meeting(wav, labels, segs, sample_rate, label_rate, name)


def speaker_embeddings(n_spk: int, dim: int = 192, seed: int = 777) -> np.ndarray:
    """Stand-in target-speaker embeddings (the .pt files of load_ts_embed are not available)."""
    return np.random.default_rng(seed + 1).standard_normal((n_spk, dim)).astype(np.float32)
