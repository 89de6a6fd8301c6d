"""Fit the TS-VAD 'probe' weight variant: seeded random weights of the reference architecture whose final
Linear (`fc`) is fitted by logistic regression to the speaker activity of a synthetic training meeting
(round-4 verdict item 4: a DER comparison that can fail).

    PYTHONPATH=. python tools/fit_probe_fc.py            # writes speaker_diarization_amd/data/probe_fc.npz

Why: with seeded random weights every track's logits sit on a near-constant plateau (C2: per-track std
0.03-0.06), so the recipe thresholds split all or nothing and a DER difference cannot move; rescaling fc
alone (tools/calibrate_spread.py) spreads them but leaves posteriors unrelated to speech, whose DER then moves
by 0.5-3.5 points under an iid 0.01 logit perturbation (any arithmetic would fail +-0.1 there).  A fitted fc
is what a trained checkpoint's last layer is: the random trunk's features (the BiLSTM output, or the
transformer output for the CAM++/transformer model) carry each synthetic speaker's pitch / formants, and a
linear read-out of them gives posteriors that follow the activity, with threshold crossings at speech
boundaries.  Only fc changes; the trunk stays the seed-777 weights.  The fit uses the fp32 CPU oracle
(oracle/tsvad_ref.py) on a training meeting (synth seed 4242) disjoint from the bench meeting (seed 777).
sklearn's LogisticRegression (lbfgs, C = 1, fixed iteration cap) per speaker track: deterministic."""
from __future__ import annotations

import os
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from oracle.pipeline_ref import plan, window_batches  # noqa: E402
from oracle.tsvad_ref import tsvad_forward  # noqa: E402
from speaker_diarization_amd.synth import make_meeting, speaker_embeddings  # noqa: E402
from speaker_diarization_amd.weights import TSVADConfig, to_torch, tsvad_state_dict  # noqa: E402

OUT = os.path.join("speaker_diarization_amd", "data", "probe_fc.npz")


def features(cfg, sd, meeting, ts, n_win, batch=16):
    X, Y = [], []
    ws = plan(meeting.labels.shape[1], cfg.rs_len, 1)[:n_win]
    for _, w, ref, tsb, L in window_batches(meeting.wav, ts, ws, batch):
        f = []
        tsvad_forward(sd, cfg, ref, tsb, L, features=f)
        h = f[0].numpy()
        for b, (s, e) in enumerate(w):
            X.append(h[b, : e - s])
            Y.append(meeting.labels[:, s:e].T)
    return np.concatenate(X).astype(np.float64), np.concatenate(Y)


def main():
    from sklearn.linear_model import LogisticRegression
    torch.set_num_threads(8)
    out = {}
    for name, cfg, n_win in (("v1_rs6", TSVADConfig.ots_vad_v1(rs_len=6), 300), ("v0_rs4", TSVADConfig(rs_len=4), 300)):
        sd = to_torch(tsvad_state_dict(cfg, seed=777))
        train = make_meeting(n_win + 2 * cfg.rs_len + 5.0, n_spk=4, seed=4242)
        ts = speaker_embeddings(4, seed=777)
        X, Y = features(cfg, sd, train, ts, n_win)
        mu, sig = X.mean(0), X.std(0) + 1e-6
        Z = (X - mu) / sig
        W = np.zeros((4, X.shape[1]))
        b = np.zeros(4)
        for s in range(4):
            clf = LogisticRegression(C=1.0, max_iter=500, tol=1e-6).fit(Z, Y[:, s])
            # back to the unstandardised features: w' = w / sig, b' = b - w'.mu
            W[s] = clf.coef_[0] / sig
            b[s] = clf.intercept_[0] - W[s] @ mu
            acc = ((Z @ clf.coef_[0] + clf.intercept_[0] > 0) == (Y[:, s] > 0.5)).mean()
            print(f"{name} speaker {s}: train frame accuracy {acc:.3f} (active {Y[:, s].mean():.3f})")
        out[f"{name}_weight"] = W.astype(np.float32)
        out[f"{name}_bias"] = b.astype(np.float32)
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    np.savez(OUT, **out)
    print("wrote", OUT)


if __name__ == "__main__":
    main()
