"""SSND speaker-query decoders + full block inference on the MI355X path (sd_ssnd_*) vs the
reference goldens (tests/golden/ssnd_*.npz from egs/alimeeting/ssnd/ssnd_model.py) and the CPU
oracle (oracle/ssnd_ref.py).  fp32 <= 1e-3 (north_star); bf16 extractor + encoder within 3 % of
the logit range (the decoders stay fp32)."""
import os

import numpy as np
import pytest
import torch

from make_ssnd_golden import SSND_CASES, ssnd_cfg, ssnd_inputs
from speaker_diarization_amd.ssnd.model import SSNDModel
from speaker_diarization_amd.weights import ssnd_state_dict, to_torch

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")


def _model(N, wseed, gpu, precision="fp32", max_batch=4):
    cfg = ssnd_cfg(N)
    m = SSNDModel(None, max_speakers=N, vad_out_len=cfg.vad_out_len, device=gpu, precision=precision,
                  max_batch=max_batch)
    return m.load_state_dict(to_torch(ssnd_state_dict(cfg, seed=wseed))), cfg


@pytest.mark.parametrize("name", [n for n, c in SSND_CASES.items() if c[0] == "decode"])
def test_ssnd_decoders_match_reference(gpu, name):
    kind, B, T, N, iseed, wseed = SSND_CASES[name]
    m, cfg = _model(N, wseed, gpu, max_batch=2)       # B > max_batch: the wrapper splits the blocks
    enc, x, spk = (torch.from_numpy(a) for a in ssnd_inputs(kind, B, T, N, iseed, cfg))
    vad, emb = m.decode(enc.to(gpu), x.to(gpu), spk.to(gpu))
    g = np.load(os.path.join(GOLD, name + ".npz"))
    e1 = np.abs(vad.cpu().numpy() - g["vad_pred"]).max()
    e2 = np.abs(emb.cpu().numpy() - g["emb_pred"]).max()
    print(f"{name}: vad {e1:.2e} emb {e2:.2e}")
    assert e1 < 1e-3 and e2 < 1e-3


@pytest.mark.parametrize("precision", ["fp32", "bf16"])
def test_ssnd_infer_matches_reference(gpu, precision):
    kind, B, T_fb, N, iseed, wseed = SSND_CASES["ssnd_infer_n4"]
    m, cfg = _model(N, wseed, gpu, precision)
    feats, spk = (torch.from_numpy(a) for a in ssnd_inputs(kind, B, T_fb, N, iseed, cfg))
    vad, emb = m.infer(feats.to(gpu), spk.to(gpu))
    g = np.load(os.path.join(GOLD, "ssnd_infer_n4.npz"))
    e1 = np.abs(vad.cpu().numpy() - g["vad_pred"]).max()
    e2 = np.abs(emb.cpu().numpy() - g["emb_pred"]).max()
    print(f"ssnd infer {precision}: vad {e1:.2e} (range {np.abs(g['vad_pred']).max():.2f}) emb {e2:.2e}")
    if precision == "fp32":
        assert e1 < 1e-3 and e2 < 1e-3
    else:
        assert e1 < 3e-2 * max(1.0, np.abs(g["vad_pred"]).max()) and e2 < 3e-2 * max(1.0, np.abs(g["emb_pred"]).max())


def test_ssnd_offline_and_online_vs_oracle(gpu):
    """offline_diarization (:778-800) and the online block loop (:802-897) driven by the GPU infer
    equal the same host logic driven by the oracle's infer."""
    from oracle import ssnd_ref
    N, wseed = 4, 904
    m, cfg = _model(N, wseed, gpu)
    sd = to_torch(ssnd_state_dict(cfg, seed=wseed))
    rng = np.random.default_rng(5)
    blocks = [rng.standard_normal((800, 80)).astype(np.float32) for _ in range(3)]
    lab, prob = m.offline_diarization(torch.from_numpy(blocks[0]).to(gpu))
    with torch.no_grad():
        vad_ref, _ = ssnd_ref.infer(sd, cfg, torch.from_numpy(blocks[0])[None], sd["E_all"][:N][None])
    assert np.abs(prob.cpu().numpy() - torch.sigmoid(vad_ref)[0].numpy()).max() < 1e-4
    out = m.online_infer(blocks, l_c=16, l_r=4)

    class _Ref:   # the reference loop over the oracle's infer (same host code path)
        max_speakers, emb_dim, device = N, cfg.emb_dim, torch.device("cpu")
        e_pse, e_non = sd["e_pse"], sd["e_non"]

        def infer(self, feats, spk):
            with torch.no_grad():
                return ssnd_ref.infer(sd, cfg, feats.cpu(), spk.cpu())
    ref = SSNDModel.online_infer(_Ref(), blocks, l_c=16, l_r=4)
    assert sorted(out) == sorted(ref)
    for k in ref:
        assert out[k].shape == ref[k].shape and np.abs(out[k] - ref[k]).max() < 1e-4, k


def test_ssnd_strict_load_and_shape_errors(gpu):
    cfg = ssnd_cfg(4)
    sd = to_torch(ssnd_state_dict(cfg, seed=1))
    sd.pop("det_decoder.out_proj.bias")
    with pytest.raises(RuntimeError, match="det_decoder.out_proj.bias"):
        SSNDModel(None, max_speakers=4, vad_out_len=200, device=gpu).load_state_dict(sd)
    sd = to_torch(ssnd_state_dict(cfg, seed=1))
    sd["extra.weight"] = torch.zeros(3)
    with pytest.raises(RuntimeError, match="extra.weight"):
        SSNDModel(None, max_speakers=4, vad_out_len=200, device=gpu).load_state_dict(sd)
    m, _ = _model(4, 1, gpu)
    with pytest.raises(AssertionError):
        m.infer(torch.zeros(1, 800, 80, device=gpu), torch.zeros(1, 3, 256, device=gpu))   # N != max_speakers
    with pytest.raises(Exception):
        m.infer(torch.zeros(1, 400, 80, device=gpu), torch.zeros(1, 4, 256, device=gpu))   # block too short
