"""ts_vad2/infer.py postprocess restated literally — test oracle only.

TEST INFRASTRUCTURE: imported by tests/ only, never by the product path.
Follows infer.py:27-70 (change_zeros_to_ones / change_ones_to_zeros, element
loops) and infer.py:72-130 (np.mean over window predictions, medfilt, per
threshold filters, RTTM line loop) on float32 posteriors, element by element,
with numpy's scalar semantics (np.float32 element vs Python float threshold).
"""
from __future__ import annotations

import numpy as np
from scipy import signal

THRESHOLDS = (0.2, 0.3, 0.35, 0.4, 0.45, 0.5, 0.55, 0.6, 0.7, 0.8)


def change_zeros_to_ones(inputs, min_silence, threshold, frame_len):
    """infer.py:27-47."""
    res, num_0 = [], 0
    thr = int(min_silence // frame_len)
    for i in inputs:
        if i >= threshold:
            if num_0 != 0:
                res.extend(([0] if num_0 > thr else [1]) * num_0)
                num_0 = 0
            res.append(1)
        else:
            num_0 += 1
    res.extend(([0] if num_0 > thr else [1]) * num_0)
    return res


def change_ones_to_zeros(inputs, min_speech, threshold, frame_len):
    """infer.py:50-70."""
    res, num_1 = [], 0
    thr = int(min_speech // frame_len)
    for i in inputs:
        if i < threshold:
            if num_1 != 0:
                res.extend(([1] if num_1 > thr else [0]) * num_1)
                num_1 = 0
            res.append(0)
        else:
            num_1 += 1
    res.extend(([1] if num_1 > thr else [0]) * num_1)
    return res


def rttm_lines(post, label_rate=25, med_filter=21, min_silence=0.32, min_speech=0.0, thresholds=THRESHOLDS):
    """post: {"<meeting>-<speaker>": (T,) float32 averaged posteriors} ->
    {threshold: [RTTM lines]} in the order infer.py:83-130 writes them."""
    frame_len = 1 / label_rate
    out = {t: [] for t in thresholds}
    for filename, p in post.items():
        speaker_id = filename.split("-")[-1]
        name = filename[: -len(speaker_id) - 1]
        labels = signal.medfilt(list(np.asarray(p, dtype=np.float32)), med_filter)
        for threshold in thresholds:
            lt = change_zeros_to_ones(labels, min_silence, threshold, frame_len)
            lt = change_ones_to_zeros(lt, min_speech, threshold, frame_len)
            start, duration = 0, 0
            for i, label in enumerate(lt):
                if label == 1:
                    duration += frame_len
                else:
                    if duration != 0:
                        out[threshold].append("SPEAKER " + str(name) + " 1 %.3f" % (start) + " %.3f " % (duration)
                                              + "<NA> <NA> " + str(speaker_id) + " <NA> <NA>\n")
                        duration = 0
                    start = i * frame_len
            if duration != 0:
                out[threshold].append("SPEAKER " + str(name) + " 1 %.3f" % (start) + " %.3f " % (duration)
                                      + "<NA> <NA> " + str(speaker_id) + " <NA> <NA>\n")
    return out


def eend_rttm_lines(session, t_hat, threshold=0.5, frame_shift=256, subsampling=1, median=1, sampling_rate=16000):
    """speaker_diarization/bin/make_rttm.py:27-42 for one session's T_hat (T, n_spk)."""
    lines = []
    a = np.where(np.asarray(t_hat, dtype=np.float32) > threshold, 1, 0)
    if median > 1:
        a = signal.medfilt(a, (median, 1))
    for spkid, frames in enumerate(a.T):
        frames = np.pad(frames, (1, 1), "constant")
        changes, = np.where(np.diff(frames, axis=0) != 0)
        fmt = "SPEAKER {:s} 1 {:7.2f} {:7.2f} <NA> <NA> {:s} <NA> <NA>"
        for s, e in zip(changes[::2], changes[1::2]):
            lines.append(fmt.format(session, s * frame_shift * subsampling / sampling_rate,
                                    (e - s) * frame_shift * subsampling / sampling_rate,
                                    session + "_" + str(spkid)))
    return lines
