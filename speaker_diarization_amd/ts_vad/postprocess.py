"""Posteriors -> RTTM (ts_vad2/infer.py:27-163), host side.

Per (meeting, speaker): frame posteriors (already overlap-averaged on the GPU)
-> scipy.signal.medfilt(21) -> for each threshold: fill silences <= min_silence,
drop speech <= min_speech -> RTTM segments.  Keeps the reference's formatting
and its start-time convention (a segment after a silence starts at
(i-1)*frame_len, infer.py:103-120).
"""
from __future__ import annotations

import os
import subprocess
from typing import Dict, Iterable, List

import numpy as np
from scipy import signal

from .. import der as der_mod

THRESHOLDS = (0.2, 0.3, 0.35, 0.4, 0.45, 0.5, 0.55, 0.6, 0.7, 0.8)


def _runs(mask: np.ndarray):
    """(value, length) runs of a boolean array."""
    if mask.size == 0:
        return []
    idx = np.flatnonzero(np.diff(mask.astype(np.int8))) + 1
    bounds = np.concatenate([[0], idx, [mask.size]])
    return [(bool(mask[a]), int(b - a)) for a, b in zip(bounds[:-1], bounds[1:])]


def change_zeros_to_ones(inputs, min_silence, threshold, frame_len):
    """infer.py:27-47: silence runs <= min_silence//frame_len frames become speech
    (including a trailing run)."""
    thr = int(min_silence // frame_len)
    act = np.asarray(inputs) >= threshold
    out = []
    for v, n in _runs(act):
        out.extend([1] * n if v or n <= thr else [0] * n)
    return out


def change_ones_to_zeros(inputs, min_speech, threshold, frame_len):
    """infer.py:50-70: speech runs <= min_speech//frame_len frames become silence."""
    thr = int(min_speech // frame_len)
    act = np.asarray(inputs) >= threshold
    out = []
    for v, n in _runs(act):
        out.extend([1] * n if (v and n > thr) else [0] * n)
    return out


def segments_to_rttm(name: str, speaker_id: str, labels: Iterable[int], frame_len: float) -> List[str]:
    """The segment loop of infer.py:100-130 verbatim in behaviour."""
    lines = []
    start, duration = 0, 0
    for i, label in enumerate(labels):
        if label == 1:
            duration += frame_len
        else:
            if duration != 0:
                lines.append("SPEAKER " + str(name) + " 1 %.3f" % (start) + " %.3f " % (duration)
                             + "<NA> <NA> " + str(speaker_id) + " <NA> <NA>\n")
                duration = 0
            start = i * frame_len
    if duration != 0:
        lines.append("SPEAKER " + str(name) + " 1 %.3f" % (start) + " %.3f " % (duration)
                     + "<NA> <NA> " + str(speaker_id) + " <NA> <NA>\n")
    return lines


def posteriors_to_rttm(post: Dict[str, np.ndarray], label_rate: int = 25, med_filter: int = 21,
                       min_silence: float = 0.32, min_speech: float = 0.0,
                       thresholds=THRESHOLDS) -> Dict[float, List[str]]:
    """post: {"<meeting>-<speaker_id>": (n_frames,) float32 averaged posteriors}."""
    frame_len = 1 / label_rate
    out = {t: [] for t in thresholds}
    for key, p in post.items():
        speaker_id = key.split("-")[-1]
        name = key[: -len(speaker_id) - 1]
        labels = signal.medfilt(np.asarray(p, dtype=np.float32), med_filter)
        for thr in thresholds:
            lt = change_zeros_to_ones(labels, min_silence, thr, frame_len)
            lt = change_ones_to_zeros(lt, min_speech, thr, frame_len)
            out[thr].extend(segments_to_rttm(name, speaker_id, lt, frame_len))
    return out


def run_lengths_frames(min_len: float, frame_len: float) -> int:
    """The recipe's int(min_len // frame_len) (e.g. 0.32 // 0.04 == 8.0)."""
    return int(min_len // frame_len)


def segments_gpu(post, med_filter: int = 21, thresholds=THRESHOLDS, min_silence: float = 0.32,
                 min_speech: float = 0.0, label_rate: int = 25, strict: bool = False):
    """Device half of posteriors_to_rttm: post (rows, T) CUDA float32 -> per
    (row, threshold) speech runs.  Returns host arrays (begin, end, count) shaped
    (rows, n_thr, cap), (rows, n_thr, cap), (rows, n_thr).  strict: speech iff
    x > threshold (EEND make_rttm) instead of x >= threshold (TS-VAD)."""
    import torch
    from .. import _lib
    post = post.contiguous().float()
    rows, T = post.shape
    frame_len = 1 / label_rate
    cap = max(1, (T + 1) // 2)
    thr = np.asarray(thresholds, dtype=np.float32)
    dev = post.device
    beg = torch.empty(rows, len(thr), cap, dtype=torch.int32, device=dev)
    end = torch.empty_like(beg)
    cnt = torch.empty(rows, len(thr), dtype=torch.int32, device=dev)
    _lib.call("sd_postprocess_segments", _lib.ptr(post), rows, T, med_filter, thr.ctypes.data, len(thr),
              run_lengths_frames(min_silence, frame_len), run_lengths_frames(min_speech, frame_len), cap,
              _lib.ptr(beg), _lib.ptr(end), _lib.ptr(cnt), int(strict), _lib.stream_ptr(dev))
    return beg.cpu().numpy(), end.cpu().numpy(), cnt.cpu().numpy()


def posteriors_to_rttm_gpu(keys: List[str], post, label_rate: int = 25, med_filter: int = 21,
                           min_silence: float = 0.32, min_speech: float = 0.0,
                           thresholds=THRESHOLDS) -> Dict[float, List[str]]:
    """posteriors_to_rttm with the filtering on the GPU.  keys[i] names row i of
    post ("<meeting>-<speaker_id>"); lines come out in the same order and format."""
    beg, end, cnt = segments_gpu(post, med_filter, thresholds, min_silence, min_speech, label_rate)
    frame_len = 1 / label_rate
    T = post.shape[1]
    # infer.py accumulates `duration += frame_len` frame by frame; keep its float sums.
    acc = [0] * (T + 1)
    for n in range(1, T + 1):
        acc[n] = acc[n - 1] + frame_len
    out = {t: [] for t in thresholds}
    for r, key in enumerate(keys):
        speaker_id = key.split("-")[-1]
        name = key[: -len(speaker_id) - 1]
        for j, thr in enumerate(thresholds):
            lines = out[thr]
            for s, e in zip(beg[r, j, :cnt[r, j]], end[r, j, :cnt[r, j]]):
                # A run starting at s > 0 is written from the preceding silent frame (infer.py:119).
                start = (int(s) - 1) * frame_len if s > 0 else 0
                lines.append("SPEAKER " + str(name) + " 1 %.3f" % (start) + " %.3f " % (acc[int(e - s)])
                             + "<NA> <NA> " + str(speaker_id) + " <NA> <NA>\n")
    return out


def write_rttms(rttms: Dict[float, List[str]], rttm_path: str):
    os.makedirs(os.path.dirname(rttm_path) or ".", exist_ok=True)
    for thr, lines in rttms.items():
        with open(f"{rttm_path}_{thr}", "w") as f:
            f.writelines(lines)


def md_eval(ref_rttm, sys_rttm, collar: float = 0.25, sctk_tool_path: str = None):
    """DER/MS/FA/SC in percent for one system RTTM, infer.py:136-151.

    Scored by speaker_diarization_amd.der (md-eval's diarization scoring restated,
    pinned to md-eval's output in tests/test_der.py).  Passing sctk_tool_path
    runs the SCTK perl script instead, exactly as the recipe does."""
    if sctk_tool_path is None:
        st = der_mod.md_eval(ref_rttm, sys_rttm, collar=collar)
        return dict(DER=round(st.der, 2), MS=round(st.ms, 2), FA=round(st.fa, 2), SC=round(st.sc, 2))
    out = subprocess.check_output(["perl", f"{sctk_tool_path}/src/md-eval/md-eval.pl", f"-c {collar}",
                                   "-s %s" % sys_rttm, f"-r {ref_rttm}"]).decode()
    d, ms, fa, sc = (float(x) for x in out.strip().split("/")[:4])
    return dict(DER=d, MS=ms, FA=fa, SC=sc)


def score_thresholds(rttms: Dict[float, List[str]], ref_rttm, collar: float = 0.25) -> Dict[float, dict]:
    """The per-threshold DER table infer.py:134-163 prints (no files written)."""
    ref = der_mod.read_rttm(ref_rttm) if not isinstance(ref_rttm, dict) else ref_rttm
    return {thr: md_eval(ref, der_mod.read_rttm(lines), collar) for thr, lines in rttms.items()}
