"""End-to-end TS-VAD parity on the MI355X path vs reference goldens and the CPU oracle."""
import numpy as np
import pytest
import torch

from make_golden import TSVAD_CASES, TSVAD_DYN_CASES, TSVAD_NAN_CASES, tsvad_case_inputs, tsvad_inputs
from speaker_diarization_amd.ts_vad.model import TSVADModel
from speaker_diarization_amd.weights import TSVADConfig, tsvad_state_dict, to_torch

pytestmark = pytest.mark.gpu

# fp32: exact-f32 MFMA, the north_star bound.  bf16: bf16 operands / fp32
# accumulate through ~70 layers; bound on the logits measured on the goldens (MI355X, round 3:
# 6.4e-3 v1 rs6, 7.0-7.4e-3 v0 rs4, 7.8e-3 for the B = 40 batch; the kernels are deterministic).
FP32_ATOL = 1e-3
BF16_ATOL = 1.5e-2


def _cfg(v, rs):
    return TSVADConfig(rs_len=rs) if v == 0 else TSVADConfig.ots_vad_v1(rs_len=rs)


_models = {}


def _model(v, rs, wseed, precision, gpu):
    key = (v, rs, wseed, precision)
    if key not in _models:
        cfg = _cfg(v, rs)
        m = TSVADModel(cfg, device=gpu, precision=precision, max_batch=8)
        m.load_state_dict(to_torch(tsvad_state_dict(cfg, seed=wseed)))
        _models[key] = m
    return _models[key]


@pytest.mark.parametrize("precision", ["fp32", "bf16", "bf16x3"])
@pytest.mark.parametrize("name", list(TSVAD_CASES))
def test_tsvad_forward_vs_reference_golden(gpu, name, precision):
    v, rs, B, T, nl, iseed, wseed = TSVAD_CASES[name]
    g = np.load(f"{__file__.rsplit('/', 1)[0]}/golden/{name}.npz")
    m = _model(v, rs, wseed, precision, gpu)
    x, ts = tsvad_inputs(B, T, nl, seed=iseed)
    labels = torch.zeros(B, 4, nl)
    out = m.forward(torch.from_numpy(x).to(gpu), torch.from_numpy(ts).to(gpu), labels).cpu().numpy()
    err = np.abs(out - g["logits"]).max()
    print(f"{name} {precision}: max|logit diff| = {err:.3e} (|logit| max {np.abs(g['logits']).max():.3f})")
    assert err < (BF16_ATOL if precision == "bf16" else FP32_ATOL)   # bf16x3: fp32-equivalent, the fp32 bound


@pytest.mark.parametrize("precision", ["fp32", "bf16", "bf16x3"])
@pytest.mark.parametrize("name", list(TSVAD_DYN_CASES))
def test_tsvad_dynamic_variant_vs_reference_golden(gpu, name, precision):
    """The 'dynamic' weight variant on the bench meeting's windows (reference run, make_golden.py
    TSVAD_DYN_CASES).  fp32: the north_star bound.  bf16: here the logits move with the frame (std 0.6-1.1) and
    the bf16 error is quoted against that motion (round 6, DESIGN §3: rms error / frame std of the logits);
    the bound is a regression guard on that ratio, not a parity claim."""
    v, rs = TSVAD_DYN_CASES[name][:2]
    g = np.load(f"{__file__.rsplit('/', 1)[0]}/golden/{name}.npz")
    cfg = _cfg(v, rs)
    m = TSVADModel(cfg, device=gpu, precision=precision, max_batch=8)
    m.load_state_dict(to_torch(tsvad_state_dict(cfg, seed=777, dynamic=True)))
    nl = int(g["n_label"])
    out = m.forward(torch.from_numpy(g["ref_speech"]).to(gpu), torch.from_numpy(g["ts"]).to(gpu), nl).cpu().numpy()
    d = out - g["logits"]
    ratio = float(np.sqrt((d ** 2).mean()) / g["logits"].std(axis=-1).mean())
    print(f"{name} {precision}: max|logit diff| {np.abs(d).max():.3e}, rms diff / frame std {ratio:.3e}")
    if precision != "bf16":     # fp32 and bf16x3 (fp32-equivalent GEMMs): the north_star bound
        assert np.abs(d).max() < FP32_ATOL
    else:
        assert ratio < 0.2


@pytest.mark.parametrize("precision", ["fp32", "bf16"])
@pytest.mark.parametrize("name", list(TSVAD_NAN_CASES))
def test_tsvad_nan_window_bypasses_batchnorm(gpu, name, precision):
    """BatchNorm1D's NaN bypass (model.py:161-171) against the reference run on a batch with one NaN (or, the
    *_inf / *_ninf cases, one +-Inf: the trunk's arithmetic turns it into NaN at the BatchNorm input, so the
    reference bypasses exactly as for NaN) fbank value: the bad window's logits are NaN, every other window matches the reference (whose BatchNorm was
    skipped for the whole batch) within the usual bound.  Then the scope: with forward_batch = 1 each window
    is its own reference batch, so the others keep their BatchNorm (== the golden without the NaN)."""
    (v, rs, B, T, nl, iseed, wseed), x, ts = tsvad_case_inputs(name)
    g = np.load(f"{__file__.rsplit('/', 1)[0]}/golden/{name}.npz")
    m = _model(v, rs, wseed, precision, gpu)
    xd, tsd = torch.from_numpy(x).to(gpu), torch.from_numpy(ts).to(gpu)
    out = m.forward(xd, tsd, nl).cpu().numpy()
    bad = TSVAD_NAN_CASES[name][1]
    keep = [i for i in range(B) if i != bad]
    assert np.isnan(out[bad]).all() and np.isfinite(out[keep]).all()
    tol = FP32_ATOL if precision == "fp32" else BF16_ATOL
    assert np.abs(out[keep] - g["logits"][keep]).max() < tol
    base = np.load(f"{__file__.rsplit('/', 1)[0]}/golden/{TSVAD_NAN_CASES[name][0]}.npz")["logits"]
    alone = m.forward(xd, tsd, nl, forward_batch=1).cpu().numpy()
    assert np.isnan(alone[bad]).all()
    assert np.abs(alone[keep] - base[keep]).max() < tol
    # a NaN in a window's target-speaker embedding poisons that window only (no BatchNorm sees it in
    # variant 1; variant 0's backend_down does, so its batch bypasses there too -- oracle)
    ts2 = ts.copy()
    ts2[keep[0], 1, 3] = np.nan
    x0 = np.nan_to_num(x, nan=0.0, posinf=0.0, neginf=0.0)
    out2 = m.forward(torch.from_numpy(x0).to(gpu), torch.from_numpy(ts2).to(gpu), nl).cpu().numpy()
    assert np.isnan(out2[keep[0]]).all()
    from oracle.tsvad_ref import tsvad_forward
    ref2 = tsvad_forward(to_torch(tsvad_state_dict(_cfg(v, rs), seed=wseed)), _cfg(v, rs),
                         torch.from_numpy(x0), torch.from_numpy(ts2), nl).numpy()
    assert np.isnan(ref2[keep[0]]).all()
    others = [i for i in range(B) if i != keep[0]]
    assert np.abs(out2[others] - ref2[others]).max() < tol


@pytest.mark.parametrize("name", ["tsvad_v0_rs4_nan", "tsvad_v0_rs4_ninf"])
def test_tsvad_nan_bypass_scope_across_device_calls(gpu, name):
    """A call wider than max_batch runs as several device forwards; the bypass scope must still be the
    reference's batch: forward_batch 0 -> the whole call (every window bypassed: the golden),
    forward_batch 2 -> windows [0, 2) and [2, 3) are separate reference batches."""
    (v, rs, B, T, nl, iseed, wseed), x, ts = tsvad_case_inputs(name)
    g = np.load(f"{__file__.rsplit('/', 1)[0]}/golden/{name}.npz")["logits"]
    base = np.load(f"{__file__.rsplit('/', 1)[0]}/golden/{TSVAD_NAN_CASES[name][0]}.npz")["logits"]
    bad = TSVAD_NAN_CASES[name][1]
    keep = [i for i in range(B) if i != bad]
    m = TSVADModel(_cfg(v, rs), device=gpu, precision="fp32", max_batch=2)
    m.load_state_dict(to_torch(tsvad_state_dict(_cfg(v, rs), seed=wseed)))
    xd, tsd = torch.from_numpy(x).to(gpu), torch.from_numpy(ts).to(gpu)
    out = m.forward(xd, tsd, nl).cpu().numpy()                       # 3 windows over device calls of 2 + 1
    assert np.isnan(out[bad]).all()
    assert np.abs(out[keep] - g[keep]).max() < FP32_ATOL
    out = m.forward(xd, tsd, nl, forward_batch=2).cpu().numpy()      # reference batches [0, 2), [2, 3)
    grp = [i for i in range(B) if i // 2 == bad // 2 and i != bad]
    other = [i for i in range(B) if i // 2 != bad // 2]
    assert np.isnan(out[bad]).all()
    if grp:
        assert np.abs(out[grp] - g[grp]).max() < FP32_ATOL
    assert np.abs(out[other] - base[other]).max() < FP32_ATOL


def test_tsvad_strict_load_errors(gpu):
    cfg = TSVADConfig()
    sd = to_torch(tsvad_state_dict(cfg, seed=1))
    sd.pop("fc.bias")
    m = TSVADModel(cfg, device=gpu, precision="fp32", max_batch=2)
    with pytest.raises(RuntimeError, match="fc.bias"):
        m.load_state_dict(sd)
    sd = to_torch(tsvad_state_dict(cfg, seed=1))
    sd["extra.weight"] = torch.zeros(3)
    m = TSVADModel(cfg, device=gpu, precision="fp32", max_batch=2)
    with pytest.raises(RuntimeError, match="extra.weight"):
        m.load_state_dict(sd)


def test_tsvad_length_assert(gpu):
    m = _model(0, 4, 777, "fp32", gpu)
    x = torch.zeros(1, 398, 80, device=gpu)
    ts = torch.zeros(1, 4, 192, device=gpu)
    with pytest.raises(AssertionError, match="diff"):
        m.forward(x, ts, torch.zeros(1, 4, 90))


@pytest.mark.parametrize("precision", ["fp32", "bf16", "bf16x3"])
@pytest.mark.parametrize("variant", [0, 1])
def test_pipeline_vs_oracle(gpu, variant, precision):
    """Meeting wav in HBM -> posteriors, vs the CPU restatement of the reference
    loop (per-window fbank + CMN, batch padding, res_dict mean)."""
    from oracle.pipeline_ref import meeting_posteriors
    from speaker_diarization_amd.synth import make_meeting, speaker_embeddings
    from speaker_diarization_amd.ts_vad.pipeline import TSVADPipeline
    rs = 4 if variant == 0 else 6
    cfg = _cfg(variant, rs)
    mt = make_meeting(23.0, n_spk=3, seed=11)
    ts = np.zeros((4, 192), np.float32)
    ts[:3] = speaker_embeddings(3, seed=11)
    n_lab = mt.labels.shape[1]
    sd = tsvad_state_dict(cfg, seed=5)
    ref = meeting_posteriors(to_torch(sd), cfg, mt.wav, ts, n_lab, shift=1, batch_size=8, n_real=3)
    m = TSVADModel(cfg, device=gpu, precision=precision, max_batch=8)
    m.load_state_dict(to_torch(sd))
    pipe = TSVADPipeline(m, segment_shift=1, batch_size=8)
    post = pipe.posteriors(torch.from_numpy(mt.wav).to(gpu), torch.from_numpy(ts).to(gpu), n_lab).cpu().numpy()
    err = np.abs(post[:3] - ref[:3]).max()
    print(f"pipeline v{variant} {precision}: max|post diff| = {err:.3e}")
    # posterior level (the bf16 product path measured 1.2e-3 / 1.4e-3 on MI355X for v1 / v0): 1e-3 fp32
    # (north_star), 3e-3 bf16 (about 2x measured); and the recipe's threshold decisions (ts_vad2/infer.py
    # thresholds) agree on >= 99 % of the frames at every threshold
    assert err < (3e-3 if precision == "bf16" else 1e-3)
    for thr in (0.2, 0.3, 0.35, 0.4, 0.45, 0.5, 0.55, 0.6, 0.7, 0.8):
        flips = int(((post[:3] > thr) != (ref[:3] > thr)).sum())
        assert flips <= 0.01 * post[:3].size, (thr, flips)


def test_tsvad_v1_large_batch_uses_wide_gemm_paths(gpu):
    """B = 40 windows x 4 speakers x 150 frames = 24000 conformer rows: the size at which the
    production GEMM paths take over (gemm_areg for the QKV / GLU-pw1 projections, the ring GEMM
    for the K = 512 FFN output, gemm_stream for the rest).  bf16 logits vs the fp32 CPU oracle."""
    from oracle.tsvad_ref import tsvad_forward
    cfg = _cfg(1, 6)
    sd = to_torch(tsvad_state_dict(cfg, seed=31))
    B = 40
    x, ts = tsvad_inputs(B, 598, 150, seed=32)
    m = TSVADModel(cfg, device=gpu, precision="bf16", max_batch=B)
    m.load_state_dict(sd)
    out = m.forward(torch.from_numpy(x).to(gpu), torch.from_numpy(ts).to(gpu), 150).cpu().numpy()
    with torch.no_grad():
        ref = tsvad_forward(sd, cfg, torch.from_numpy(x), torch.from_numpy(ts), 150).numpy()
    err = np.abs(out - ref).max()
    print(f"B={B} bf16: max|logit diff| = {err:.3e}")
    assert err < BF16_ATOL


def test_tsvad_bf16x3_two_row_tile_recurrence(gpu):
    """B = 520 windows: more than 512 BiLSTM sequences per direction, so the persistent recurrence runs two row
    tiles per group (co-residency: 4 x 2 x ceil(B / 16) workgroups must fit the CUs) -- in bf16x3 mode the
    split kernel lstm_group_bf16_kernel<2, 4, true>.  Its logits against the same forward in exact fp32 (the
    step kernel) within the fp32 bound."""
    cfg = _cfg(1, 6)
    sd = to_torch(tsvad_state_dict(cfg, seed=41))
    B = 520
    x, ts = tsvad_inputs(B, 598, 150, seed=42)
    xd, tsd = torch.from_numpy(x).to(gpu), torch.from_numpy(ts).to(gpu)
    outs = {}
    for prec in ("fp32", "bf16x3"):
        m = TSVADModel(cfg, device=gpu, precision=prec, max_batch=B)
        m.load_state_dict(sd)
        outs[prec] = m.forward(xd, tsd, 150).cpu().numpy()
        del m
        torch.cuda.empty_cache()
    err = np.abs(outs["bf16x3"] - outs["fp32"]).max()
    print(f"B={B} bf16x3 vs fp32: max|logit diff| = {err:.3e}")
    assert np.isfinite(outs["bf16x3"]).all() and err < FP32_ATOL


@pytest.mark.parametrize("variant", [0, 1])
def test_tsvad_repeated_forward_bit_identical(gpu, variant):
    """Repeated forwards on one handle (its workspaces, LSTM exchange buffers and counters reused) give
    the first call's logits bit for bit, also into a new output buffer, and the golden still holds."""
    name = "tsvad_v0_rs4" if variant == 0 else "tsvad_v1_rs6"
    v, rs, B, T, nl, iseed, wseed = TSVAD_CASES[name]
    cfg = _cfg(v, rs)
    m = TSVADModel(cfg, device=gpu, precision="bf16", max_batch=B)
    m.load_state_dict(to_torch(tsvad_state_dict(cfg, seed=wseed)))
    x, ts = tsvad_inputs(B, T, nl, seed=iseed)
    xd, tsd = torch.from_numpy(x).to(gpu), torch.from_numpy(ts).to(gpu)
    out = torch.empty(B, 4, nl, device=gpu)
    outs = []
    for _ in range(4):
        out.fill_(float("nan"))
        m.forward(xd, tsd, nl, out=out)
        outs.append(out.cpu().numpy().copy())
    for o in outs[1:]:
        np.testing.assert_array_equal(o, outs[0])
    other = torch.empty_like(out)
    m.forward(xd, tsd, nl, out=other)
    np.testing.assert_array_equal(other.cpu().numpy(), outs[0])
    g = np.load(f"{__file__.rsplit('/', 1)[0]}/golden/{name}.npz")
    assert np.abs(outs[-1] - g["logits"]).max() < BF16_ATOL


def test_tsvad_infer_res_dict_matches_reference(gpu):
    """TSVADModel.infer (model.py:923-970) -> (result, res_dict) vs the reference's own infer on
    the same seeded batch (tests/golden/tsvad_infer.npz, make_postprocess_golden.py): partial
    label lengths, absent speakers (-1 ids), two meetings.  Keys, frame keys and their insertion
    order, list lengths exact; probabilities fp32 <= 1e-5; the 0.5-thresholded DER/ACC/MI/FA/CF
    exact; the BCE loss <= 1e-5."""
    import os
    from make_postprocess_golden import INFER_CASE as c, infer_labels
    g = np.load(os.path.join(os.path.dirname(__file__), "golden", "tsvad_infer.npz"))
    cfg = TSVADConfig(rs_len=4)
    m = TSVADModel(cfg, device=gpu, precision="fp32", max_batch=c["B"])
    m.load_state_dict(to_torch(tsvad_state_dict(cfg, seed=c["wseed"])))
    x, ts = tsvad_inputs(c["B"], c["T_fb"], c["n_lab"], seed=c["iseed"])
    result, res_dict = m.infer(torch.from_numpy(x).to(gpu), torch.from_numpy(ts).to(gpu),
                               torch.from_numpy(infer_labels()), torch.tensor(c["lens"]), file_path=c["files"],
                               speaker_ids=c["spk"], start=c["starts"])
    assert list(res_dict) == [str(k) for k in g["keys"]]
    for i, k in enumerate(res_dict):
        assert list(res_dict[k]) == list(g[f"order_{i}"])
        frames = sorted(res_dict[k])
        assert [len(res_dict[k][t]) for t in frames] == list(g[f"counts_{i}"])
        vals = np.array([v for t in frames for v in res_dict[k][t]], np.float32)
        assert np.abs(vals - g[f"values_{i}"]).max() <= 1e-5
    got = np.array([result[k] for k in ("DER", "ACC", "MI", "FA", "CF")], np.float64)
    np.testing.assert_allclose(got, g["metrics"], rtol=0, atol=1e-12)
    assert abs(float(result["losses"]["diar"]) - float(g["loss"])) <= 1e-5
