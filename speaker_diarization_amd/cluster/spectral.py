"""Spectral-clustering first pass of the SSND / TS-VAD pipeline (host code).

Restates egs/alimeeting/spectral_cluster/spectral_clusterer.py (cluster(), :35-89: cosine
affinity, per-row top-p pruning, unnormalised Laplacian, eigen-gap speaker count, k-means on the
spectral embeddings) and make_rttm.py (read_labels / merge_segments / RTTM lines, :34-88), which
turn the sub-segment CAM++ embeddings of a recording into the initial speaker labels and RTTM that
prepare_rttm_for_ts_vad.sh feeds to TS-VAD / SSND.  The work is O(m^2 log m + m^3) in the number
m of sub-segments of ONE recording (a few hundred to a few thousand): a LAPACK eigensolve and a
k-means on the host, as in the reference ("can follow as host
code").  k-means keeps the reference's `random_state=None` default, i.e. numpy's global RNG.
"""
from __future__ import annotations

from collections import OrderedDict
from typing import Dict, List, Sequence, Tuple

import numpy as np
import scipy.linalg


def cosine_similarity(M: np.ndarray) -> np.ndarray:
    """:37-39 — 0.5 (1 + cos) on L2-normalised rows."""
    M = M / np.linalg.norm(M, axis=1, keepdims=True)
    return 0.5 * (1.0 + np.dot(M, M.T))


def prune(M: np.ndarray, p: float) -> np.ndarray:
    """:41-52 — per row, the n smallest affinities -> 0, the rest -> 1 (n = max(m-10, 2) below
    1000 rows, else (1-p) m), then symmetrised.  Modifies M like the reference."""
    m = M.shape[0]
    n = max(m - 10, 2) if m < 1000 else int((1.0 - p) * m)
    order = np.argsort(M, axis=1, kind="quicksort")   # np.argsort default, row by row in the reference
    rows = np.arange(m)[:, None]
    M[rows, order[:, :n]] = 0.0
    M[rows, order[:, n:]] = 1.0
    return 0.5 * (M + M.T)


def laplacian(M: np.ndarray) -> np.ndarray:
    """:54-57 — zero diagonal, L = D - M with D the absolute row sums."""
    M[np.diag_indices(M.shape[0])] = 0.0
    D = np.diag(np.sum(np.abs(M), axis=1))
    return D - M


def spectral(M: np.ndarray, num_spks, min_num_spks: int, max_num_spks: int) -> np.ndarray:
    """:59-64 — eigenvectors of the smallest eigenvalues; the count from the largest eigen-gap."""
    eig_values, eig_vectors = scipy.linalg.eigh(M)
    num_spks = num_spks if num_spks is not None else np.argmax(np.diff(eig_values[:max_num_spks + 1])) + 1
    num_spks = max(num_spks, min_num_spks)
    return eig_vectors[:, :num_spks]


def kmeans(data: np.ndarray, random_state=None) -> np.ndarray:
    """:66-70 — sklearn k_means, k = number of spectral dimensions, n_init 10."""
    from sklearn.cluster._kmeans import k_means
    _, labels, _ = k_means(data, data.shape[1], random_state=random_state, n_init=10)
    return labels


def cluster(embeddings, p: float = 0.01, num_spks=None, min_num_spks: int = 1, max_num_spks: int = 20,
            random_state=None):
    """spectral_clusterer.cluster (:35-89): (m, E) sub-segment embeddings -> m labels."""
    if len(embeddings) <= 2:
        return [0] * len(embeddings)
    sim = cosine_similarity(np.array(embeddings))
    lap = laplacian(prune(sim, p))
    return kmeans(spectral(lap, num_spks, min_num_spks, max_num_spks), random_state)


def read_labels(lines: Sequence[str], frame_shift: int = 10) -> "OrderedDict[str, List[Tuple[float, float, str]]]":
    """make_rttm.read_labels (:34-46): '<utt>-<begin_ms>-<end_ms>-<begin_fr>-<end_fr> <label>' lines."""
    out: "OrderedDict[str, list]" = OrderedDict()
    for line in lines:
        subseg, label = line.strip().split()
        utt, begin_ms, end_ms, begin_frames, end_frames = subseg.split("-")
        begin = (int(begin_ms) + int(begin_frames) * frame_shift) / 1000.0
        end = (int(begin_ms) + int(end_frames) * frame_shift) / 1000.0
        out.setdefault(utt, []).append((begin, end, label))
    return out


def merge_segments(utt_to_subseg_labels: Dict[str, list]) -> List[Tuple[str, float, float, str]]:
    """make_rttm.merge_segments (:49-73): consecutive same-label sub-segments merge; overlapping
    different-label ones split at the midpoint of the overlap."""
    merged = []
    for utt, subs in utt_to_subseg_labels.items():
        if len(subs) == 0:
            continue
        begin, end, label = subs[0]
        e = end
        for b, e, la in subs[1:]:
            if b <= end and la == label:
                end = e
            elif b > end:
                merged.append((utt, begin, end, label))
                begin, end, label = b, e, la
            elif b <= end and la != label:
                pivot = (b + end) / 2.0
                merged.append((utt, begin, pivot, label))
                begin, end, label = pivot, e, la
            else:
                raise ValueError
        merged.append((utt, begin, e, label))
    return merged


def rttm_lines(merged, channel: int = 1) -> List[str]:
    """make_rttm.main (:76-84) formatting."""
    spec = "SPEAKER {} {} {:.3f} {:.3f} <NA> <NA> {} <NA> <NA>"
    return [spec.format(utt, channel, b, e - b, la) for utt, b, e, la in merged]
