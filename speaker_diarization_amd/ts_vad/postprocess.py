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


def write_rttms(rttms: Dict[float, List[str]], rttm_path: str):
    os.makedirs(os.path.dirname(rttm_path) or ".", exist_ok=True)
    for thr, lines in rttms.items():
        with open(f"{rttm_path}_{thr}", "w") as f:
            f.writelines(lines)


def md_eval(sctk_tool_path: str, ref_rttm: str, sys_rttm: str, collar: float = 0.25):
    """Score with the recipes' md-eval.pl (prints DER/MS/FA/SC), infer.py:136-151."""
    out = subprocess.check_output(["perl", f"{sctk_tool_path}/src/md-eval/md-eval.pl", f"-c {collar}",
                                   "-s %s" % sys_rttm, f"-r {ref_rttm}"]).decode()
    der, ms, fa, sc = (float(x) for x in out.strip().split("/")[:4])
    return dict(DER=der, MS=ms, FA=fa, SC=sc)
