"""EEND activities -> RTTM on the GPU (speaker_diarization/bin/make_rttm.py:20-42).

The reference thresholds T_hat (T, n_spk) with ``> threshold``, median-filters the
0/1 decisions per speaker column (scipy.signal.medfilt, zero padded), and writes
one line per run of ones with ``{:7.2f}`` start / duration in seconds
(frames x frame_shift x subsampling / sampling_rate).  A median of 0/1 decisions
equals the decision on the median of the values (order statistics commute with a
monotone threshold, and the zero padding maps to "silence" for thresholds >= 0),
so the device path filters the activities first and then thresholds:
``sd_postprocess_segments`` with the strict-threshold flag and no run-length
filters.  The host only formats the lines.
"""
from __future__ import annotations

import os
from typing import Iterable, List, Tuple

import numpy as np

from .ts_vad.postprocess import segments_gpu

FMT = "SPEAKER {:s} 1 {:7.2f} {:7.2f} <NA> <NA> {:s} <NA> <NA>"


def session_lines(session: str, t_hat, threshold: float = 0.5, frame_shift: int = 256, subsampling: int = 1,
                  median: int = 1, sampling_rate: int = 16000) -> List[str]:
    """RTTM lines of one session; t_hat: (T, n_spk) CUDA (or CPU) float tensor."""
    import torch
    if threshold < 0:
        raise ValueError("threshold must be >= 0 for the filter-then-threshold identity")
    t = torch.as_tensor(t_hat)
    if not t.is_cuda:
        raise ValueError("make_rttm: activities must be on the HIP device")
    post = t.t().contiguous().float()                     # (n_spk, T)
    n_spk, T = post.shape
    if T == 0:
        return []
    beg, end, cnt = segments_gpu(post, med_filter=median, thresholds=(threshold,), min_silence=0.0,
                                 min_speech=0.0, strict=True)
    lines = []
    for spk in range(n_spk):
        for s, e in zip(beg[spk, 0, :cnt[spk, 0]], end[spk, 0, :cnt[spk, 0]]):
            lines.append(FMT.format(session, int(s) * frame_shift * subsampling / sampling_rate,
                                    int(e - s) * frame_shift * subsampling / sampling_rate,
                                    session + "_" + str(spk)))
    return lines


def make_rttm(sessions: Iterable[Tuple[str, object]], out_rttm_file: str = None, **kw) -> List[str]:
    """sessions: (session, T_hat) pairs in any order; written sorted by session name as the
    reference sorts its h5 file list (make_rttm.py:22-27)."""
    lines = []
    for session, t_hat in sorted(sessions, key=lambda x: x[0]):
        lines.extend(session_lines(session, t_hat, **kw))
    if out_rttm_file is not None:
        os.makedirs(os.path.dirname(out_rttm_file) or ".", exist_ok=True)
        with open(out_rttm_file, "w") as f:
            f.writelines(line + "\n" for line in lines)
    return lines
