"""CAM++ embedding extractor oracle pinned to the reference (tests/golden/campp_*.npz,
made by tests/golden/make_golden.py from cam_pplus_wespeaker.CAMPPlus and the reference
extract_embed of generate_chunk_speaker_embedding_from_modelscope_for_diarization.py)."""
import os

import numpy as np
import pytest
import torch

from make_golden import CAMPP_CASES, CAMPP_EXTRACT, campp_inputs, embed_wav
from oracle import fbank_ref
from oracle.tsvad_ref import campplus_embedding, campplus_time_out, embedding_chunks, extract_embed
from speaker_diarization_amd.ts_vad import embedding as emb_mod
from speaker_diarization_amd.weights import campplus_layout, campplus_state_dict, to_torch

GOLD = os.path.join(os.path.dirname(__file__), "golden")


@pytest.mark.parametrize("name", list(CAMPP_CASES))
def test_campp_oracle_matches_reference(name):
    B, T, E, iseed, wseed = CAMPP_CASES[name]
    g = np.load(os.path.join(GOLD, name + ".npz"))
    sd = to_torch(campplus_state_dict(wseed, E))
    x = torch.from_numpy(campp_inputs(B, T, iseed))
    with torch.no_grad():
        emb = campplus_embedding(sd, x).numpy()
        tout = campplus_time_out(sd, x, pre="").numpy()
    assert emb.shape == (B, E) and tout.shape == (B, 512, (T - 1) // 2 + 1)
    np.testing.assert_allclose(emb, g["emb"], atol=2e-5, rtol=1e-5)
    np.testing.assert_allclose(tout[:, :, :64], g["time_out"], atol=2e-5, rtol=1e-5)


def test_extract_embed_oracle_matches_reference():
    secs, bs, wav_seed, wseed = CAMPP_EXTRACT["campp_extract"]
    g = np.load(os.path.join(GOLD, "campp_extract.npz"))
    sd = to_torch(campplus_state_dict(wseed, 192))
    for i, s in enumerate(secs):
        wav = embed_wav(s, wav_seed + i).astype(np.float32).astype(np.float64)   # torch.FloatTensor, :283
        with torch.no_grad():
            got = extract_embed(sd, wav, batch_size=bs).numpy()
        np.testing.assert_allclose(got, g[f"emb{i}"], atol=2e-5, rtol=1e-5)
    # the reference batched 3 + 1 chunks for the 9.5 s file and 1 for the 4 s file
    assert g["batches"].tolist() == [3, 1, 1]


@pytest.mark.parametrize("n,expect", [
    (96000, [(0, 96000)]),                       # exactly one chunk long -> whole file
    (96001, [(0, 96000)]),
    (112000, [(0, 96000)]),                      # range(0, 16000, 16000): the end-aligned chunk is dropped
    (112001, [(0, 96000), (16000, 112000)]),
    (30000, [(0, 30000)]),
])
def test_embedding_chunk_plan(n, expect):
    assert embedding_chunks(n) == expect
    assert emb_mod.embedding_chunks(n) == expect


def test_povey_fbank_matches_direct_dft():
    rng = np.random.default_rng(7)
    wav = (rng.standard_normal(2400) * 0.1).astype(np.float32)
    f = fbank_ref.fbank(wav, scale=1.0, window="povey")
    x = wav[5 * 160: 5 * 160 + 400].astype(np.float64)
    x = x - x.mean()
    x = x - 0.97 * np.concatenate([x[:1], x[:-1]])
    x = x * (0.5 - 0.5 * np.cos(2 * np.pi * np.arange(400) / 399)) ** 0.85
    n = np.arange(512)
    k = np.arange(257)[:, None]
    X = (np.pad(x, (0, 112))[None, :] * np.exp(-2j * np.pi * k * n / 512)).sum(1)
    e = (np.abs(X) ** 2) @ fbank_ref.mel_banks().T
    np.testing.assert_allclose(f[5], np.log(np.maximum(e, np.finfo(np.float32).eps)), rtol=1e-5, atol=1e-4)
    with pytest.raises(ValueError):
        fbank_ref.fbank(wav, window="blackman")


def test_embed_chunk_fbank_is_file_fbank_slice():
    """Chunk k's frames are file frames 100k.. (the reuse extract_embed relies on)."""
    wav = embed_wav(9.0, 3)
    full = fbank_ref.fbank(wav, scale=1.0, window="povey")
    for a, b in embedding_chunks(len(wav)):
        c = fbank_ref.fbank(wav[a:b], scale=1.0, window="povey")
        np.testing.assert_allclose(c, full[a // 160: a // 160 + c.shape[0]], rtol=1e-6, atol=1e-5)


def test_standalone_layout_keys():
    keys = [k for k, _, _ in campplus_layout("", 512)]
    assert keys[0] == "head.conv1.weight" and "xvector.dense.linear.weight" in keys
    assert "xvector.dense.nonlinear.batchnorm.weight" not in keys      # batchnorm_ is affine=False
    sd = campplus_state_dict(1, 512)
    assert sd["xvector.dense.linear.weight"].shape == (512, 1024, 1)
