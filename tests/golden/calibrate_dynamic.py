"""Calibrate the 'dynamic' TS-VAD weight variant (round-5 verdict item 1: a bf16 DER check that can fail on
weights whose activations have a realistic dynamic range).

    PYTHONPATH=. python tests/golden/calibrate_dynamic.py [--windows 48]

Seeded random weights keep almost all of every activation's energy in a frame-constant part: on C2 (ots_vad
v1) the pooled statistics that carry the whole mix signal into the conformer (GSP: per-frame mean / std over the
192 speech_down channels, model.py:689-696) vary by ~10 % across frames, the conformer output's frame-varying
part is ~0.15 of its magnitude, and the BiLSTM output moves by 0.05, so the logits sit on a plateau
(std 0.03-0.06).  The 'spread' variant rescaled only fc, by 120-240x; this variant instead centres and scales
two layers upstream with the fp32 CPU oracle and leaves fc at a gain of DYN_FC_GAIN (<= 4):

  v1 (C2):  gsp_fc   W' = W diag(G_GSP / sigma_s),  b' = b - W (G_GSP mu_s / sigma_s)
                     -> the mix input is the unit-variance, zero-mean frame statistic (mu_s, sigma_s: mean / std
                        of the two statistics over the calibration frames)
            BiLSTM   W_ih' = G_IH W_ih,  b_ih' = b_ih - (G_IH - 1) W_ih xbar
                     -> the gates keep their operating point and swing G_IH times further with the frame
                        (xbar: mean conformer output over the calibration frames, 4 x 384)
            fc       W' = k W,  b' = k (b - mean_s)          (mean_s: logit mean of track s after the above)
  v0 (C4):  fc       W' = k W,  b' = k (b - mean_s)

Every other weight and the architecture stay the reference's.  Writes speaker_diarization_amd/weights_dynamic.npz
(read by weights.dynamic_weights) and prints the resulting statistics: pre-fc feature std across frames, logit
std, and the fraction of frame posteriors in [0.2, 0.8]."""
from __future__ import annotations

import argparse
import os
import sys

import numpy as np
import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from oracle import tsvad_ref as R  # noqa: E402
from oracle.pipeline_ref import plan, window_batches  # noqa: E402
from speaker_diarization_amd import weights as W  # noqa: E402
from speaker_diarization_amd.synth import make_meeting, speaker_embeddings  # noqa: E402


def _windows(cfg, n):
    m = make_meeting(600.0, n_spk=4, seed=777)          # the bench / DER-test meeting
    ts = speaker_embeddings(4, seed=777)
    ws = plan(m.labels.shape[1], cfg.rs_len, 1)[:n]
    return list(window_batches(m.wav, ts, ws, 16))


def _valid(out, w):
    return torch.cat([out[b, :, : e - s] for b, (s, e) in enumerate(w)], 1)    # (NS, frames)


@torch.no_grad()
def calibrate_v1(n):
    cfg = W.TSVADConfig.ots_vad_v1(rs_len=6)
    sd = W.to_torch(W.tsvad_state_dict(cfg, seed=777))
    batches = _windows(cfg, n)
    trunk = [(R.speech_encoder_out(sd, ref), tsb, L, w) for _, w, ref, tsb, L in batches]

    def stats(x):
        return torch.cat([x.mean(dim=1, keepdim=True), x.std(dim=1, keepdim=True)], 1).permute(0, 2, 1)

    s_all = torch.cat([stats(x)[:, :L].reshape(-1, 2) for x, _, L, _ in trunk]).double()
    mu, sg = s_all.mean(0), s_all.std(0)
    c = {"v1_stat_mean": mu.numpy(), "v1_stat_std": sg.numpy()}
    sd = W.to_torch(W.dynamic_weights(W.tsvad_state_dict(cfg, seed=777), cfg, c, stage=1))
    conf = []
    for x, tsb, L, w in trunk:
        mix = F.linear(stats(x), sd["gsp_fc.weight"], sd["gsp_fc.bias"])[:, :L]
        B, T, _ = mix.shape
        conf.append(torch.cat([R.conformer(torch.cat((tsb[:, i, None, :].expand(B, T, -1), mix), 2),
                                           torch.full((B,), T), sd, "single_backend.") for i in range(4)], -1))
    c["v1_conformer_mean"] = torch.cat([q.reshape(-1, q.shape[-1]) for q in conf]).double().mean(0).numpy()
    sd = W.to_torch(W.dynamic_weights(W.tsvad_state_dict(cfg, seed=777), cfg, c, stage=2))
    hs, lg = [], []
    for q, (x, tsb, L, w) in zip(conf, trunk):
        h, _ = R.lstm(q, sd, "multi_backend.", bidirectional=True)
        hs.append(h.reshape(-1, h.shape[-1]))
        lg.append(_valid(F.linear(h, sd["fc.weight"], sd["fc.bias"]).transpose(1, 2), w))
    lg = torch.cat(lg, 1).double()
    c["v1_logit_mean"] = lg.mean(1).numpy()
    hs = torch.cat(hs)
    print(f"v1: stat mean {mu.numpy().round(5)} std {sg.numpy().round(5)}; BiLSTM out (pre-fc) std across frames "
          f"{hs.std(0).mean():.3f}, |h| {hs.abs().mean():.3f}")
    return c, lg


@torch.no_grad()
def calibrate_v0(n):
    cfg = W.TSVADConfig(rs_len=4)
    sd = W.to_torch(W.tsvad_state_dict(cfg, seed=777))
    lg = torch.cat([_valid(R.tsvad_forward(sd, cfg, ref, tsb, L), w) for _, w, ref, tsb, L in _windows(cfg, n)],
                   1).double()
    return {"v0_logit_mean": lg.mean(1).numpy()}, lg


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--windows", type=int, default=48)
    a = ap.parse_args()
    torch.set_num_threads(min(16, os.cpu_count() or 8))
    c1, lg1 = calibrate_v1(a.windows)
    c0, lg0 = calibrate_v0(a.windows)
    c = {**c1, **c0}
    path = os.path.join("speaker_diarization_amd", "weights_dynamic.npz")
    np.savez(path, **{k: np.asarray(v, np.float64) for k, v in c.items()})
    k = W.DYN_FC_GAIN
    for name, lg, mean in (("v1", lg1, c["v1_logit_mean"]), ("v0", lg0, c["v0_logit_mean"])):
        z = k * (lg - torch.from_numpy(mean)[:, None])
        p = torch.sigmoid(z)
        print(f"{name}: logit std per track (fc gain {k}) {z.std(1).numpy().round(3)}; frame posteriors in "
              f"[0.2, 0.8]: {float(((p > .2) & (p < .8)).double().mean()):.2f}")
    print("wrote", path)


if __name__ == "__main__":
    main()
