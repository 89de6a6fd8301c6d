"""CAM++ target-speaker embedding extractor on the GPU (libsdiar sd_campp_* / sd_fbank_kaldi_ex)
against the reference goldens and the CPU oracle.  Tolerances: fp32 1e-3 (north_star); bf16
trunk: 5e-2 absolute on unit-scale embeddings plus cosine similarity >= 0.999."""
import os

import numpy as np
import pytest
import torch

from make_golden import CAMPP_CASES, CAMPP_EXTRACT, campp_inputs, embed_wav
from oracle import fbank_ref
from oracle.tsvad_ref import campplus_embedding
from speaker_diarization_amd.ts_vad.embedding import (CAMPPlus, FBank, extract_embed, kaldi_fbank_povey,
                                                      load_ts_embed)
from speaker_diarization_amd.weights import campplus_state_dict, to_torch

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")


def _model(gpu, E, wseed, precision="fp32", **kw):
    m = CAMPPlus(feat_dim=80, embedding_size=E, device=gpu, precision=precision, **kw)
    return m.load_state_dict(to_torch(campplus_state_dict(wseed, E)))


def _cos(a, b):
    a, b = a.reshape(len(a), -1), b.reshape(len(b), -1)
    return (a * b).sum(1) / np.linalg.norm(a, axis=1) / np.linalg.norm(b, axis=1)


@pytest.mark.parametrize("precision", ["fp32", "bf16"])
@pytest.mark.parametrize("name", list(CAMPP_CASES))
def test_campp_forward_matches_reference(gpu, name, precision):
    B, T, E, iseed, wseed = CAMPP_CASES[name]
    g = np.load(os.path.join(GOLD, name + ".npz"))
    m = _model(gpu, E, wseed, precision, max_batch=B, max_frames=T)
    x = torch.from_numpy(campp_inputs(B, T, iseed)).to(gpu)
    emb = m(x).cpu().numpy()
    tout = m(x, get_time_out=True).cpu().numpy()
    assert emb.shape == (B, E) and tout.shape == (B, 512, (T - 1) // 2 + 1)
    if precision == "fp32":
        np.testing.assert_allclose(emb, g["emb"], atol=1e-3, rtol=0)
        np.testing.assert_allclose(tout[:, :, :64], g["time_out"], atol=1e-3, rtol=0)
    else:
        np.testing.assert_allclose(emb, g["emb"], atol=5e-2, rtol=0)
        assert _cos(emb, g["emb"]).min() >= 0.999
        assert _cos(tout[:, :, :64], g["time_out"]).min() >= 0.999


@pytest.mark.parametrize("precision", ["fp32", "bf16"])
def test_extract_embed_matches_reference(gpu, precision):
    secs, bs, wav_seed, wseed = CAMPP_EXTRACT["campp_extract"]
    g = np.load(os.path.join(GOLD, "campp_extract.npz"))
    m = _model(gpu, 192, wseed, precision, max_batch=bs)
    for i, s in enumerate(secs):
        got = extract_embed(embed_wav(s, wav_seed + i), m, batch_size=bs).cpu().numpy()
        assert got.shape == g[f"emb{i}"].shape
        if precision == "fp32":
            np.testing.assert_allclose(got, g[f"emb{i}"], atol=1e-3, rtol=0)
        else:
            assert _cos(got, g[f"emb{i}"]).min() >= 0.999


def test_extract_embed_long_file_matches_oracle(gpu, tmp_path):
    """A 40 s file (34 chunks, several device batches) against the oracle, then the .pt round trip
    the TS-VAD dataset reads back (mean over chunks)."""
    from oracle.tsvad_ref import extract_embed as ref_extract
    sd = campplus_state_dict(9, 192)
    wav = embed_wav(40.0, 21)
    m = CAMPPlus(device=gpu, precision="fp32", max_batch=16).load_state_dict(to_torch(sd))
    got = extract_embed(wav, m).cpu()
    with torch.no_grad():
        ref = ref_extract(to_torch(sd), wav.astype(np.float32).astype(np.float64)).numpy()
    assert got.shape == (34, 192)
    np.testing.assert_allclose(got.numpy(), ref, atol=1e-3, rtol=0)
    os.makedirs(tmp_path / "meet")
    torch.save(got, tmp_path / "meet" / "7.pt")
    ts = load_ts_embed(str(tmp_path), "meet", [7, -1, -2], 192)
    assert ts.shape == (3, 192) and (ts[1:] == 0).all()
    torch.testing.assert_close(ts[0], got.mean(0))


@pytest.mark.parametrize("n", [400, 16000 * 3 + 123, 16000 * 20])
def test_fbank_povey(gpu, n):
    rng = np.random.default_rng(n)
    wav = (rng.standard_normal(n) * 0.1).astype(np.float32)
    ref = fbank_ref.fbank(wav, scale=1.0, window="povey")
    out = kaldi_fbank_povey(torch.from_numpy(wav).to(gpu)).cpu().numpy()
    assert out.shape == ref.shape
    np.testing.assert_allclose(out, ref, atol=2e-3, rtol=1e-4)
    fe = FBank(80, sample_rate=16000, mean_nor=True)
    f = fe(torch.from_numpy(wav).to(gpu)).cpu().numpy()
    np.testing.assert_allclose(f, ref - ref.mean(0, keepdims=True), atol=2e-3, rtol=1e-4)


def test_campp_batch_split_and_errors(gpu):
    sd = campplus_state_dict(4, 192)
    m = CAMPPlus(device=gpu, precision="fp32", max_batch=2, max_frames=200).load_state_dict(to_torch(sd))
    x = torch.from_numpy(campp_inputs(5, 150, 8))
    got = m(x.to(gpu)).cpu().numpy()      # 5 > max_batch: three device calls
    with torch.no_grad():
        ref = campplus_embedding(to_torch(sd), x).numpy()
    np.testing.assert_allclose(got, ref, atol=1e-3, rtol=0)
    with pytest.raises(ValueError):
        m(torch.zeros(1, 300, 80, device=gpu))          # exceeds max_frames
    with pytest.raises(ValueError):
        m(torch.zeros(1, 100, 40, device=gpu))          # feat_dim
    bad = dict(to_torch(sd))
    bad.pop("xvector.dense.linear.weight")
    with pytest.raises(RuntimeError, match="state_dict"):
        CAMPPlus(device=gpu, max_batch=2).load_state_dict(bad)
    extra = dict(to_torch(sd))
    extra["xvector.dense.nonlinear.batchnorm.weight"] = torch.ones(192)   # affine=False has no weight
    with pytest.raises(RuntimeError, match="Unexpected"):
        CAMPPlus(device=gpu, max_batch=2).load_state_dict(extra)
