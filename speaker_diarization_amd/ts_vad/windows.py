"""Inference windowing of a meeting (TSVADDataset.load_data_and_label,
ts_vad2/ts_vad_dataset.py:242-271, is_train=False) and batch/shard planning."""
from __future__ import annotations

from dataclasses import dataclass
from typing import List, Tuple

import numpy as np

from ..frontend import FRAME_LEN, FRAME_SHIFT


@dataclass
class WindowPlan:
    starts: np.ndarray        # label-frame start of each window
    ends: np.ndarray          # label-frame end (exclusive)
    n_labels: int             # label frames of the meeting
    label_rate: int = 25
    sample_rate: int = 16000
    rs_len: int = 4
    segment_shift: int = 1

    @property
    def n_win(self) -> int:
        return len(self.starts)

    @property
    def lens(self) -> np.ndarray:
        return self.ends - self.starts

    @property
    def dis(self) -> int:
        return self.label_rate * self.segment_shift

    @property
    def chunk(self) -> int:
        return self.label_rate * self.rs_len

    @property
    def samples_per_label(self) -> int:
        return self.sample_rate // self.label_rate   # load_rs: 640 samples / label frame

    @property
    def fbank_start(self) -> np.ndarray:
        """First meeting-level fbank frame of each window (640 / 160 = 4 per label frame)."""
        return self.starts * (self.samples_per_label // FRAME_SHIFT)

    @property
    def fbank_n(self) -> np.ndarray:
        """Kaldi snip_edges frame count of each window's samples (frontend.num_frames, vectorised and computed
        once per plan: the per-window Python loop ran on every batch of every step, ~1 ms of host time between
        two C2 steps)."""
        n = self.__dict__.get("_fbank_n")
        if n is None:
            ns = self.lens * self.samples_per_label
            n = np.where(ns < FRAME_LEN, 0, 1 + (ns - FRAME_LEN) // FRAME_SHIFT).astype(np.int64)
            self.__dict__["_fbank_n"] = n
        return n

    def batches(self, batch_size: int) -> List[Tuple[int, int]]:
        """Consecutive windows in dataset order (DataLoader shuffle=False, infer.py:232-238)."""
        return [(s, min(self.n_win, s + batch_size)) for s in range(0, self.n_win, batch_size)]


def plan_windows(n_labels: int, rs_len: int, segment_shift: int, label_rate: int = 25,
                 sample_rate: int = 16000) -> WindowPlan:
    dis = int(label_rate * segment_shift)
    chunk = int(label_rate * rs_len)
    starts, ends = [], []
    for start in range(0, n_labels, dis):
        end = start + chunk if start + chunk < n_labels else n_labels
        if end - start > 0:   # short_ratio = 0 at inference
            starts.append(start)
            ends.append(end)
    return WindowPlan(np.asarray(starts, np.int64), np.asarray(ends, np.int64), n_labels, label_rate,
                      sample_rate, rs_len, segment_shift)


def shard_batches(plan: WindowPlan, batch_size: int, world: int, rank: int) -> Tuple[int, int]:
    """Contiguous window range of `rank`, cut on the global batch grid so every
    batch (and hence every tail-window zero pad) is identical for
    any world size -> posteriors bit-identical to one GPU."""
    batches = plan.batches(batch_size)
    nb = len(batches)
    per, rem = divmod(nb, world)
    b0 = rank * per + min(rank, rem)
    b1 = b0 + per + (1 if rank < rem else 0)
    if b0 >= b1:
        return (0, 0)
    return (batches[b0][0], batches[b1 - 1][1])
