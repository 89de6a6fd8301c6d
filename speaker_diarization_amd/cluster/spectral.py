"""Spectral-clustering first pass of the SSND / TS-VAD pipeline (host code).

Behaviour follows egs/alimeeting/spectral_cluster/spectral_clusterer.py (cluster(), :35-89) and
egs/alimeeting/umap_cluster/make_rttm.py (:34-88) of the reference — algorithm by Xu Xiang,
Copyright (c) 2022, Apache License 2.0 — which turn the sub-segment CAM++ embeddings of a recording
into the initial speaker labels and RTTM that prepare_rttm_for_ts_vad.sh feeds to TS-VAD / SSND.

This is an independent formulation of that algorithm, not a transcription:
  * the pruned affinity is built directly as a 0/1 rank mask: after pruning, an entry's value only
    depends on its rank in its row (the n lowest -> 0, the rest -> 1), so the cosine values are used
    once, for the per-row ranks, and the symmetrised mask, its zero diagonal and the Laplacian
    D - A come out of one pass (`SpectralClusterer.laplacian`);
  * the run merge of make_rttm is vectorised: after every sub-segment the reference's open segment
    ends at that sub-segment's end, so a boundary falls between consecutive sub-segments exactly
    where there is a gap or the label changes, and the cut point is the gap edges or the midpoint
    of the overlap (`merge_segments`).
Label identity with the reference needs the same numerics where they matter: numpy's default
(quicksort) argsort per row for the ranks, scipy.linalg.eigh, the eigen-gap count and sklearn's
k_means(k, random_state=None, n_init=10) consuming numpy's global RNG — tests/test_cluster.py checks
labels and RTTM text against reference-run goldens.  The work is O(m^2 log m + m^3) in the number m
of sub-segments of ONE recording, host work as in the reference.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import scipy.linalg

Segment = Tuple[str, float, float, str]


@dataclass
class SpectralClusterer:
    p: float = 0.01                 # pruning fraction for recordings of >= 1000 sub-segments
    min_num_spks: int = 1
    max_num_spks: int = 20

    def keep_per_row(self, m: int) -> int:
        """How many of a row's highest affinities survive pruning (m - n in the reference)."""
        n_low = max(m - 10, 2) if m < 1000 else int((1.0 - self.p) * m)
        return m - n_low

    def laplacian(self, emb: np.ndarray) -> np.ndarray:
        """Unnormalised graph Laplacian of the pruned, symmetrised cosine affinity."""
        unit = emb / np.linalg.norm(emb, axis=1, keepdims=True)
        cos = 0.5 * (1.0 + unit @ unit.T)
        m = cos.shape[0]
        keep = self.keep_per_row(m)
        top = np.argsort(cos, axis=1)[:, m - keep:]        # row-wise ranks (numpy's default sort)
        mask = np.zeros_like(cos)
        np.put_along_axis(mask, top, 1.0, axis=1)
        aff = 0.5 * (mask + mask.T)
        np.fill_diagonal(aff, 0.0)
        return np.diag(aff.sum(axis=1)) - aff               # entries are >= 0: |A| = A

    def embed(self, lap: np.ndarray, num_spks: Optional[int]) -> np.ndarray:
        """Eigenvectors of the k smallest eigenvalues; k from the largest gap unless given."""
        vals, vecs = scipy.linalg.eigh(lap)
        if num_spks is None:
            num_spks = int(np.argmax(np.diff(vals[: self.max_num_spks + 1]))) + 1
        return vecs[:, : max(num_spks, self.min_num_spks)]

    def labels(self, emb, num_spks: Optional[int] = None, random_state=None):
        if len(emb) <= 2:
            return [0] * len(emb)
        from sklearn.cluster._kmeans import k_means
        spec = self.embed(self.laplacian(np.array(emb)), num_spks)
        return k_means(spec, spec.shape[1], random_state=random_state, n_init=10)[1]


def cluster(embeddings, p: float = 0.01, num_spks=None, min_num_spks: int = 1, max_num_spks: int = 20,
            random_state=None):
    """spectral_clusterer.cluster's call surface: (m, E) sub-segment embeddings -> m labels."""
    return SpectralClusterer(p, min_num_spks, max_num_spks).labels(embeddings, num_spks, random_state)


def read_labels(lines: Sequence[str], frame_shift: int = 10) -> Dict[str, List[Tuple[float, float, str]]]:
    """'<utt>-<begin_ms>-<end_ms>-<begin_frame>-<end_frame> <label>' lines -> per recording (in first-seen
    order) the sub-segments' (begin s, end s, label)."""
    out: Dict[str, List[Tuple[float, float, str]]] = {}
    for line in lines:
        name, label = line.split()
        utt, seg_ms, _, f0, f1 = name.split("-")
        base = int(seg_ms)
        out.setdefault(utt, []).append(((base + int(f0) * frame_shift) / 1000.0,
                                        (base + int(f1) * frame_shift) / 1000.0, label))
    return out


def _merge_one(utt: str, subs: List[Tuple[float, float, str]]) -> List[Segment]:
    b = np.array([s[0] for s in subs])
    e = np.array([s[1] for s in subs])
    lab = np.array([s[2] for s in subs], dtype=object)
    prev_end, nxt = e[:-1], b[1:]
    gap = nxt > prev_end
    cut = gap | (lab[1:] != lab[:-1])
    idx = np.nonzero(cut)[0]                               # boundary between sub-segments i and i + 1
    mid = (nxt[idx] + prev_end[idx]) / 2.0                 # overlap with a new label: split at the midpoint
    close = np.where(gap[idx], prev_end[idx], mid)
    open_ = np.where(gap[idx], nxt[idx], mid)
    begins = np.concatenate([b[:1], open_])
    ends = np.concatenate([close, e[-1:]])
    labels = np.concatenate([lab[:1], lab[idx + 1]])
    return [(utt, float(x), float(y), str(la)) for x, y, la in zip(begins, ends, labels)]


def merge_segments(utt_to_subseg_labels: Dict[str, list]) -> List[Segment]:
    """Consecutive same-label sub-segments that touch or overlap become one segment; a gap always
    closes the segment; an overlap between different labels is split at its midpoint."""
    out: List[Segment] = []
    for utt, subs in utt_to_subseg_labels.items():
        if subs:
            out.extend(_merge_one(utt, subs))
    return out


def rttm_lines(merged: Sequence[Segment], channel: int = 1) -> List[str]:
    """RTTM SPEAKER lines as make_rttm prints them (3-decimal onset and duration)."""
    return [f"SPEAKER {utt} {channel} {b:.3f} {e - b:.3f} <NA> <NA> {la} <NA> <NA>" for utt, b, e, la in merged]
