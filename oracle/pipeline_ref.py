"""Reference TS-VAD inference loop restated on CPU — oracle / cpu_baseline.

Follows ts_vad2/infer.py:216-285 + TSVADDataset (ts_vad_dataset.py:242-271,
325-421, 664-751) + TSVADModel.infer (model.py:923-970) + postprocess's frame
averaging (infer.py:90-94): per window, fbank of the window's audio slice with
per-window CMN, batches of consecutive windows zero-padded to the batch max,
model forward, sigmoid, res_dict[name-spk][start+t].append(p), np.mean.
"""
from __future__ import annotations

from collections import defaultdict

import numpy as np
import torch

from .fbank_ref import window_fbank
from .tsvad_ref import tsvad_forward


def plan(n_labels, rs_len, shift, label_rate=25):
    dis, chunk = label_rate * shift, label_rate * rs_len
    out = []
    for start in range(0, n_labels, dis):
        end = start + chunk if start + chunk < n_labels else n_labels
        if end - start > 0:
            out.append((start, end))
    return out


def window_batches(wav, ts, windows, batch_size, sample_rate=16000, label_rate=25):
    spl = sample_rate // label_rate
    for b0 in range(0, len(windows), batch_size):
        ws = windows[b0:b0 + batch_size]
        feats = []
        for s, e in ws:
            seg = wav[s * spl: e * spl]
            if len(seg) < (e - s) * spl:   # load_rs zero-pads short reads (:355-359)
                seg = np.pad(seg, (0, (e - s) * spl - len(seg)))
            feats.append(window_fbank(seg))
        T = max(f.shape[0] for f in feats)
        L = max(e - s for s, e in ws)
        ref = np.zeros((len(ws), T, feats[0].shape[1]), np.float32)
        for i, f in enumerate(feats):
            ref[i, : f.shape[0]] = f
        yield b0, ws, torch.from_numpy(ref), torch.from_numpy(np.repeat(ts[None], len(ws), 0)), L


@torch.no_grad()
def meeting_posteriors(sd, cfg, wav, ts, n_labels, shift=1, batch_size=64, n_real=None, max_windows=None):
    """Returns (NS, n_labels) float32 posteriors (NaN where no window covers a frame)."""
    windows = plan(n_labels, cfg.rs_len, shift, cfg.label_rate)
    if max_windows is not None:
        windows = windows[:max_windows]
    ns = cfg.max_num_speaker
    n_real = ns if n_real is None else n_real
    res = defaultdict(lambda: defaultdict(list))
    for b0, ws, ref, tsb, L in window_batches(wav, ts, windows, batch_size, cfg.sample_rate, cfg.label_rate):
        prob = torch.sigmoid(tsvad_forward(sd, cfg, ref, tsb, L)).numpy()
        for b, (s, e) in enumerate(ws):
            for t in range(e - s):
                for i in range(n_real):
                    res[i][s + t].append(prob[b, i, t])
    out = np.full((ns, n_labels), np.nan, np.float32)
    for i in range(n_real):
        for t, v in res[i].items():
            out[i, t] = np.mean(v)
    return out


def overlap_average(logits, starts, lens, n_labels):
    """(n_win, NS, chunk) logits -> (NS, n_labels): sigmoid (model.py:945-946), then
    the per-frame np.mean over covering windows in window order (infer.py:90-94)."""
    prob = torch.sigmoid(torch.from_numpy(np.ascontiguousarray(logits, np.float32))).numpy()
    ns = prob.shape[1]
    res = [defaultdict(list) for _ in range(ns)]
    for w, (s, l) in enumerate(zip(starts, lens)):
        for t in range(int(l)):
            for i in range(ns):
                res[i][int(s) + t].append(prob[w, i, t])
    out = np.full((ns, n_labels), np.nan, np.float32)
    for i in range(ns):
        for t, v in res[i].items():
            out[i, t] = np.mean(v)
    return out
