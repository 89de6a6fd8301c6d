"""TEST INFRASTRUCTURE (CPU): how much of a DER difference bf16 arithmetic alone makes on a TS-VAD weight variant,
and which stage makes it (round-6 evidence for DESIGN.md §3, verdict item 1).

    python tests/bf16_der_emulation.py [variant 0|1] [n_windows] [weights: plain|spread|dynamic ...]

The fp32 CPU oracle (oracle/pipeline_ref.py) is run twice on the first n windows of the bench meeting: once as
is, once with every Linear / Conv operand (input and weight) and every Linear / Conv output rounded to bf16 --
the storage and operand precision of the product's bf16 mode (fp32 accumulation, fp32 elementwise work,
fp32 residual streams).  On the plain weights this proxy reproduces the GPU's measured bf16 posterior error
(1.05e-3 here vs 1.17e-3 on the MI355X C2 line), so its DER differences say what bf16 as a number format
does to a weight variant, independent of any kernel.  With --attribute, the rounding is applied to one stage at a
time (CAM++ trunk + speech_down, gsp_fc, conformer stack, BiLSTM + fc)."""
from __future__ import annotations

import contextlib
import os
import sys
import time

import numpy as np
import torch
import torch.nn.functional as F
from scipy import signal

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle.pipeline_ref import meeting_posteriors  # noqa: E402
from oracle.postprocess_ref import THRESHOLDS, rttm_lines  # noqa: E402
from speaker_diarization_amd import der as der_mod  # noqa: E402
from speaker_diarization_amd.synth import make_meeting, speaker_embeddings  # noqa: E402
from speaker_diarization_amd.weights import TSVADConfig, to_torch, tsvad_state_dict  # noqa: E402

_ORIG = {n: getattr(F, n) for n in ("linear", "conv1d", "conv2d")}
STAGES = {"trunk": ("speech_encoder", "speech_down"), "gsp": ("gsp",), "conformer": ("single_backend",),
          "lstm+fc": ("multi_backend", "fc")}


def _r(t):
    return None if t is None else t.bfloat16().float()


@contextlib.contextmanager
def bf16_rounding(weight_ptrs=None):
    """Round operands and outputs of F.linear / conv1d / conv2d to bf16 (only for the given weights if set)."""
    def wrap(f):
        def g(x, w, b=None, *a, **k):
            if weight_ptrs is not None and w.data_ptr() not in weight_ptrs:
                return f(x, w, b, *a, **k)
            return _r(f(_r(x), _r(w), b, *a, **k))
        return g
    for n, f in _ORIG.items():
        setattr(F, n, wrap(f))
    try:
        yield
    finally:
        for n, f in _ORIG.items():
            setattr(F, n, f)


def der_table(m, post, n_win):
    keys = [f"{m.name}-{i + 1}" for i in range(4)]
    ref = der_mod.read_rttm([f"SPEAKER {m.name} 1 {s:.3f} {min(e, n_win) - s:.3f} <NA> <NA> {k + 1} <NA> <NA>\n"
                             for k, s, e in sorted(m.segments, key=lambda x: (x[1], x[0])) if s < n_win])
    rt = rttm_lines({k: post[i] for i, k in enumerate(keys)})
    return {t: der_mod.md_eval(ref, der_mod.read_rttm(rt[t]), collar=0.25).der for t in THRESHOLDS}


def crossings(p, thr=0.5):
    """Threshold crossings of the medfilt(21) posteriors (ts_vad2/infer.py:96), summed over tracks."""
    return int(sum(np.abs(np.diff((signal.medfilt(q.astype(np.float64), 21) > thr).astype(int))).sum() for q in p))


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    variant = int(args[0]) if args else 1
    n_win = int(args[1]) if len(args) > 1 else 60
    names = args[2:] or ["plain", "dynamic"]
    torch.set_num_threads(min(16, os.cpu_count() or 8))
    cfg = TSVADConfig.ots_vad_v1(rs_len=6) if variant == 1 else TSVADConfig(rs_len=4)
    m = make_meeting(600.0, n_spk=4, seed=777)
    ts = speaker_embeddings(4, seed=777)

    def post(sd):
        return np.ascontiguousarray(meeting_posteriors(sd, cfg, m.wav, ts, m.labels.shape[1], batch_size=64,
                                                       max_windows=n_win)[:, :n_win * 25])

    for name in names:
        sd = to_torch(tsvad_state_dict(cfg, seed=777, spread=name == "spread", dynamic=name == "dynamic"))
        t0 = time.time()
        p32 = post(sd)
        d32 = der_table(m, p32, n_win)
        runs = [("all stages", None)]
        if "--attribute" in sys.argv:
            runs += [(s, {v.data_ptr() for k, v in sd.items() if k.startswith(pre)}) for s, pre in STAGES.items()]
        print(f"{name} v{variant}, {n_win} windows: posteriors in [0.2, 0.8] {float(((p32 > .2) & (p32 < .8)).mean()):.2f}, "
              f"medfilt crossings at 0.5: {crossings(p32)}; fp32 DER {[round(d32[t], 2) for t in THRESHOLDS]}")
        for label, ptrs in runs:
            with bf16_rounding(ptrs):
                p16 = post(sd)
            d16 = der_table(m, p16, n_win)
            dd = [round(d16[t] - d32[t], 2) for t in THRESHOLDS]
            print(f"  bf16 {label:10s}: max|dp| {np.abs(p32 - p16).max():.2e} mean {np.abs(p32 - p16).mean():.2e}; "
                  f"dDER {dd} (max {max(map(abs, dd)):.2f})  [{time.time() - t0:.0f} s]", flush=True)


if __name__ == "__main__":
    main()
