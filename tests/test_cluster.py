"""Spectral-clustering first pass (speaker_diarization_amd/cluster/spectral.py) vs a run of the
reference's spectral_clusterer.cluster + make_rttm (tests/golden/cluster_*.npz,
make_cluster_golden.py): identical labels and RTTM text with numpy's global RNG seeded as in the
generator (the reference's k-means uses random_state=None)."""
import os

import numpy as np
import pytest

from make_cluster_golden import CLUSTER_CASES, cluster_inputs
from speaker_diarization_amd.cluster import spectral

GOLD = os.path.join(os.path.dirname(__file__), "golden")


@pytest.mark.parametrize("name", list(CLUSTER_CASES))
def test_cluster_matches_reference(name):
    n_spk, per, dim, noise, num, seed = CLUSTER_CASES[name]
    emb, subsegs = cluster_inputs(n_spk, per, dim, noise, seed)
    np.random.seed(seed)
    labels = np.asarray(spectral.cluster(emb, num_spks=num), np.int64)
    g = np.load(os.path.join(GOLD, name + ".npz"))
    np.testing.assert_array_equal(labels, g["labels"])
    merged = spectral.merge_segments(spectral.read_labels([f"{s} {l}" for s, l in zip(subsegs, labels)]))
    assert "\n".join(spectral.rttm_lines(merged)) == str(g["rttm"])


def test_cluster_trivial_and_merge_edges():
    assert spectral.cluster(np.ones((2, 8), np.float32)) == [0, 0]
    subs = {"u": [(0.0, 1.5, "0"), (0.75, 2.25, "0"), (1.5, 3.0, "1"), (3.5, 4.0, "1")]}
    assert spectral.merge_segments(subs) == [("u", 0.0, 1.875, "0"), ("u", 1.875, 3.0, "1"), ("u", 3.5, 4.0, "1")]


def test_vectorised_merge_matches_sequential_oracle():
    """Random sub-segment streams (1.5 s windows every 0.75 s with jitter, gaps, 1-4 labels) through
    the vectorised merge and the reference's sequential loop (oracle/cluster_ref.py): identical
    segments, bit for bit."""
    from oracle.cluster_ref import merge_segments_seq
    rng = np.random.default_rng(5)
    for trial in range(300):
        subs = {}
        for u in range(int(rng.integers(1, 4))):
            n = int(rng.integers(1, 40))
            t = np.cumsum(rng.choice([0.75, 0.75, 0.75, 2.0, 0.5], size=n)) + rng.random() * 3
            lab = rng.integers(0, int(rng.integers(1, 5)), size=n)
            subs[f"rec{u}"] = [(float(a), float(a + 1.5), str(l)) for a, l in zip(t, lab)]
        assert spectral.merge_segments(subs) == merge_segments_seq(subs), trial
