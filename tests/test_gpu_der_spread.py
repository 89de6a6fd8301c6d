"""DER parity that can fail (round-4 verdict item 4): the TS-VAD meeting pipeline on the 'spread' weight
variant (weights.py spread_fc: the seeded reference-architecture weights with only the final Linear rescaled
per track, so the posteriors of the bench meeting cross every recipe threshold instead of sitting on a
plateau), scored by the md-eval restatement (speaker_diarization_amd/der.py, collar 0.25,
ts_vad2/infer.py:134-163) for the GPU path and for the fp32 CPU oracle (oracle/pipeline_ref.py) on the same
span of the same meeting.

fp32 mode: |DER(GPU) - DER(oracle)| <= 0.1 at every recipe threshold (north_star's +-0.1), on a table with
no threshold at DER 100 on both sides.  bf16 mode is reported beside it (printed: DER table, raw and
medfilt(21) decision flips).  On the seeded weights the bf16 path's logit error (~4e-3) is ~10 % of the
logits' own variation across frames (std 0.03-0.06 per track), and the rescale multiplies both by k ~ 120-240;
an iid 0.01 logit perturbation alone moves this DER by 0.5-3.5 points.  bf16 on this variant
therefore measures that sensitivity and is recorded, not bounded; bf16 parity is held on the plain weights
(test_gpu_tsvad.py)."""
import numpy as np
import pytest
import torch

from oracle.pipeline_ref import meeting_posteriors
from oracle.postprocess_ref import rttm_lines
from speaker_diarization_amd import der as der_mod
from speaker_diarization_amd.synth import make_meeting, speaker_embeddings
from speaker_diarization_amd.ts_vad.model import TSVADModel
from speaker_diarization_amd.ts_vad.pipeline import TSVADPipeline
from speaker_diarization_amd.ts_vad.postprocess import THRESHOLDS, posteriors_to_rttm_gpu
from speaker_diarization_amd.weights import TSVADConfig, to_torch, tsvad_state_dict

pytestmark = pytest.mark.gpu
N_WIN = 90          # windows (= seconds of meeting) scored


def _case(variant):
    cfg = TSVADConfig.ots_vad_v1(rs_len=6) if variant == 1 else TSVADConfig(rs_len=4)
    sd = to_torch(tsvad_state_dict(cfg, seed=777, spread=True))
    m = make_meeting(600.0, n_spk=4, seed=777)        # the bench meeting (the calibration's)
    keep = (N_WIN + cfg.rs_len) * 16000               # windows starting before N_WIN s are whole in it
    ts = speaker_embeddings(4, seed=777)
    return cfg, sd, m, m.wav[:keep], ts


def _der_table(m, post):
    keys = [f"{m.name}-{i + 1}" for i in range(4)]
    ref = der_mod.read_rttm([f"SPEAKER {m.name} 1 {s:.3f} {min(e, N_WIN) - s:.3f} <NA> <NA> {k + 1} <NA> <NA>\n"
                             for k, s, e in sorted(m.segments, key=lambda x: (x[1], x[0])) if s < N_WIN])
    if isinstance(post, np.ndarray):
        rt = rttm_lines({k: post[i] for i, k in enumerate(keys)})
    else:
        rt = posteriors_to_rttm_gpu(keys, post)
    return {t: der_mod.md_eval(ref, der_mod.read_rttm(rt[t]), collar=0.25).der for t in THRESHOLDS}


@pytest.fixture(scope="module", params=[1, 0], ids=["c2_v1", "c4_v0"])
def spread_case(request):
    variant = request.param
    torch.set_num_threads(16)
    cfg, sd, m, wav, ts = _case(variant)
    T = N_WIN * 25
    cpu = meeting_posteriors(sd, cfg, m.wav, ts, m.labels.shape[1], batch_size=64, max_windows=N_WIN)[:, :T]
    return variant, cfg, sd, m, wav, ts, cpu, _der_table(m, np.ascontiguousarray(cpu))


@pytest.mark.parametrize("precision", ["fp32", "bf16"])
def test_der_spread_variant(gpu, spread_case, precision):
    variant, cfg, sd, m, wav, ts, cpu, der_cpu = spread_case
    T = N_WIN * 25
    model = TSVADModel(cfg, device=gpu, precision=precision, max_batch=64)
    model.load_state_dict(sd)
    pipe = TSVADPipeline(model, segment_shift=1, batch_size=64)
    n_lab = wav.size // 640
    post = pipe.posteriors(torch.from_numpy(wav).to(gpu), torch.from_numpy(ts).to(gpu), n_lab)[:, :T].contiguous()
    der_gpu = _der_table(m, post)
    g = post.cpu().numpy()
    flips = {t: int(((g > t) != (cpu > t)).sum()) for t in THRESHOLDS}
    print(f"variant {variant} {precision}: max|post diff| {np.abs(g - cpu).max():.3e}")
    print("  DER gpu / oracle:", {t: (round(der_gpu[t], 2), round(der_cpu[t], 2)) for t in THRESHOLDS})
    print("  raw flips:", flips)
    # the table is not degenerate: every threshold has a DER below 100 on the reference side or ours
    assert all(min(der_gpu[t], der_cpu[t]) < 100.0 for t in THRESHOLDS)
    assert len({round(v, 1) for v in der_cpu.values()}) >= 5, der_cpu
    if precision == "fp32":
        assert np.abs(g - cpu).max() < 1e-3
        assert max(abs(der_gpu[t] - der_cpu[t]) for t in THRESHOLDS) <= 0.1
    else:
        # recorded, not bounded: the rescale multiplies the bf16 path's logit error (4e-3 on the plain weights,
        # ~10 % of the seeded weights' logit variation) by k = 8 / std ~ 120-240, so bf16 posteriors on this
        # variant measure that sensitivity, not parity (round 5, r05b: mean |diff| 0.24, DER 52-86 vs 52-98)
        assert np.isfinite(g).all()
