"""Calibrate the 'spread' TS-VAD weight variant (round-4 verdict item 4: a DER check that can fail).

    PYTHONPATH=. python tests/golden/calibrate_spread.py [--windows 48]

Seeded random weights put every track's logits on a near-constant plateau (C2: per-track std 0.03-0.06
around offsets -0.23..0.26), so every recipe threshold either splits nothing or everything and the DER
difference between two posterior sets cannot move.  The variant rescales only the final Linear (`fc`):
    logit'_s = k_s (logit_s - mean_s),   k_s = SPREAD_STD / std_s
i.e. fc.weight[s] *= k_s, fc.bias[s] = k_s (fc.bias[s] - mean_s), with mean_s / std_s measured here by the
CPU oracle (fp32) over the first windows of the bench's synthetic meeting (speaker_diarization_amd.synth,
seed 777).  Every other weight, and the architecture, stay the reference's.  Prints the constants that
speaker_diarization_amd/weights.py SPREAD_FC holds."""
from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from oracle.pipeline_ref import plan, window_batches  # noqa: E402
from oracle.tsvad_ref import tsvad_forward  # noqa: E402
from speaker_diarization_amd.synth import make_meeting, speaker_embeddings  # noqa: E402
from speaker_diarization_amd.weights import TSVADConfig, to_torch, tsvad_state_dict  # noqa: E402


def stats(cfg, windows):
    sd = to_torch(tsvad_state_dict(cfg, seed=777))
    m = make_meeting(max(120.0, windows + 2 * cfg.rs_len), n_spk=4, seed=777)
    ts = speaker_embeddings(4, seed=777)
    ws = plan(m.labels.shape[1], cfg.rs_len, 1)[:windows]
    lg = []
    for _, w, ref, tsb, L in window_batches(m.wav, ts, ws, 16):
        out = tsvad_forward(sd, cfg, ref, tsb, L).numpy()
        for b, (s, e) in enumerate(w):
            lg.append(out[b, :, : e - s])
    lg = np.concatenate(lg, axis=1)
    return lg.mean(axis=1).astype(np.float64), lg.std(axis=1).astype(np.float64)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--windows", type=int, default=48)
    a = ap.parse_args()
    torch.set_num_threads(8)
    out = {}
    for name, cfg in (("v1_rs6", TSVADConfig.ots_vad_v1(rs_len=6)), ("v0_rs4", TSVADConfig(rs_len=4))):
        mean, std = stats(cfg, a.windows)
        out[name] = {"mean": [round(float(x), 6) for x in mean], "std": [round(float(x), 6) for x in std]}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
