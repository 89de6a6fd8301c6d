"""Spectral-clustering goldens from the reference (egs/alimeeting/spectral_cluster/
spectral_clusterer.py cluster() and make_rttm.py), imported and run here only (kaldiio stub).
numpy's global RNG is seeded before every cluster() call (the reference's k-means uses
random_state=None), so the run is reproducible.

    python tests/golden/make_cluster_golden.py
"""
import os
import sys
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF = os.environ.get("SDIAR_REFERENCE", "/root/reference")
SC = os.path.join(REF, "egs/alimeeting/spectral_cluster")

# name: (n_spk, segments per speaker, embedding dim, noise, num_spks arg, seed)
CLUSTER_CASES = {
    "cluster_3spk": (3, 40, 192, 0.35, None, 41),
    "cluster_5spk_fixed": (5, 25, 192, 0.5, 5, 42),
    "cluster_2spk_small": (2, 4, 64, 0.3, None, 43),
}


def cluster_inputs(n_spk, per, dim, noise, seed):
    rng = np.random.default_rng(seed)
    centers = rng.standard_normal((n_spk, dim))
    lab = np.repeat(np.arange(n_spk), per)
    rng.shuffle(lab)
    emb = (centers[lab] + noise * rng.standard_normal((len(lab), dim)) * np.linalg.norm(centers, axis=1).mean()
           / np.sqrt(dim)).astype(np.float32)
    # sub-segment ids utt-begin_ms-end_ms-begin_fr-end_fr: 1.5 s windows every 0.75 s
    subsegs = [f"R8001_M8004-{0:08d}-{600000:08d}-{75 * i:08d}-{75 * i + 150:08d}" for i in range(len(lab))]
    return emb, subsegs


def main():
    sys.modules["kaldiio"] = types.ModuleType("kaldiio")
    sys.path.insert(0, SC)
    import spectral_clusterer as S
    import make_rttm as R
    for name, (n_spk, per, dim, noise, num, seed) in CLUSTER_CASES.items():
        emb, subsegs = cluster_inputs(n_spk, per, dim, noise, seed)
        np.random.seed(seed)
        labels = np.asarray(S.cluster(emb, num_spks=num), np.int64)
        lines = [f"{s} {l}" for s, l in zip(subsegs, labels)]
        import tempfile
        with tempfile.NamedTemporaryFile("w", suffix=".labels", delete=False) as f:
            f.write("\n".join(lines) + "\n")
            path = f.name
        merged = R.merge_segments(R.read_labels(path))
        os.unlink(path)
        spec = "SPEAKER {} {} {:.3f} {:.3f} <NA> <NA> {} <NA> <NA>"
        rttm = [spec.format(u, 1, b, e - b, la) for u, b, e, la in merged]
        np.savez_compressed(os.path.join(HERE, f"{name}.npz"), labels=labels, rttm=np.array("\n".join(rttm)))
        print(name, np.bincount(labels), len(rttm), "RTTM lines")


if __name__ == "__main__":
    main()
