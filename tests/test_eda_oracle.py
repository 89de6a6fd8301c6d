"""EEND-EDA oracle (oracle/eend_ref.py) against the reference goldens, plus the
host-side pieces of the drop-in that run without a GPU (RNG replay, selection,
chunk planning, Slaney mel basis)."""
import os

import numpy as np
import pytest
import torch

from oracle import eend_ref
from speaker_diarization_amd import feature
from speaker_diarization_amd.eend_eda.infer import chunk_groups, gen_chunk_indices, shard_chunks
from speaker_diarization_amd.eend_eda.models import _replay_construction_rng
from speaker_diarization_amd.weights import EDAConfig, eda_state_dict, to_torch
from tests.golden.make_golden import EDA_CASES, FEATURE_CASES, eda_inputs, feature_wav

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def _load(name):
    return dict(np.load(os.path.join(GOLD, name + ".npz")))


def _cfg(name):
    mtype, L = EDA_CASES[name][:2]
    return EDAConfig(model_type=mtype, n_layers=L)


@pytest.mark.parametrize("name", list(FEATURE_CASES))
def test_feature_pipeline_matches_reference_glue(name):
    n, sr, tr, fs, fsh, ctx, sub, seed = FEATURE_CASES[name]
    g = _load(name)
    got = eend_ref.features(feature_wav(n, seed), sr, fs, fsh, ctx, sub, tr)
    assert got.shape == g["feats"].shape
    np.testing.assert_array_equal(got, g["feats"])
    # frame count of feature.stft (drops the last frame when divisible)
    nf = feature.stft_num_frames(n, fsh)
    assert got.shape[0] == -(-nf // sub)


def test_slaney_mel_product_equals_oracle():
    for sr, n_fft in ((16000, 512), (8000, 256)):
        np.testing.assert_array_equal(feature.slaney_mel(sr, n_fft, 23), eend_ref.slaney_mel(sr, n_fft, 23))


def test_librosa_stft_restatement_is_a_centred_dft():
    rng = np.random.default_rng(0)
    y = rng.standard_normal(1000)
    Y = eend_ref.librosa_stft(y, 512, 160, 400)
    assert Y.shape == (257, 1 + 1000 // 160)
    t = 3
    win = np.zeros(512)
    win[56:456] = eend_ref.hann_periodic(400)
    yp = np.pad(y, 256)
    frame = yp[t * 160: t * 160 + 512] * win
    k = np.arange(257)[:, None]
    dft = (frame[None, :] * np.exp(-2j * np.pi * k * np.arange(512)[None, :] / 512)).sum(1)
    np.testing.assert_allclose(Y[:, t], dft, rtol=1e-10, atol=1e-9)


@pytest.mark.parametrize("name", list(EDA_CASES))
def test_eda_oracle_matches_reference(name):
    mtype, L, lens, nspk, iseed, wseed = EDA_CASES[name]
    g = _load(name)
    cfg = _cfg(name)
    sd = to_torch(eda_state_dict(cfg, seed=wseed))
    xs = eda_inputs(lens, seed=iseed)
    offs = np.cumsum([0] + lens)
    for i, x in enumerate(xs):
        perm = torch.from_numpy(g["perms"][offs[i]:offs[i + 1]])
        act, probs = eend_ref.infer_full(sd, cfg, [torch.from_numpy(x)], [perm])
        np.testing.assert_allclose(probs[0].numpy(), g["probs"][i], atol=1e-5)
        np.testing.assert_allclose(act[0].numpy(), g["act"][i, : lens[i]], atol=1e-5)
        if g["index_error"][i]:
            with pytest.raises(IndexError):
                eend_ref.select(act, probs, cfg.variant, None if nspk is None else nspk)
        else:
            ys = eend_ref.select(act, probs, cfg.variant, None if nspk is None else nspk)[0]
            assert ys.shape[1] == g["nsel"][i]


@pytest.mark.parametrize("name", ["eda_tfm_l2", "eda_eend_l4", "eda_conformer_l2"])
def test_construction_rng_replay_reproduces_reference_permutations(name):
    """Seed 777 -> construct -> randperm per chunk (infer_eda.py:39-112)."""
    mtype, L, lens = EDA_CASES[name][:3]
    g = _load(name)
    torch.manual_seed(777)
    _replay_construction_rng(_cfg(name), 0.5)
    perms = np.concatenate([torch.randperm(n).numpy() for n in lens])
    np.testing.assert_array_equal(perms, g["perms"])


def test_chunk_planning():
    chunks = list(gen_chunk_indices(4567, 2000))
    assert chunks == [(0, 2000), (2000, 4000), (4000, 4567)]
    assert chunk_groups(chunks, 8) == [(0, 2, 2000), (2, 3, 567)]
    assert chunk_groups(list(gen_chunk_indices(6000 * 6, 2000)), 8) == [(0, 8, 2000), (8, 16, 2000),
                                                                         (16, 18, 2000)]
    assert [shard_chunks(18, 4, r) for r in range(4)] == [(0, 5), (5, 10), (10, 14), (14, 18)]


def test_eda_oracle_batched_list_matches_reference():
    """B=2 list of different lengths in one infer(): pad_sequence(-1), no key mask."""
    g = _load("eda_tfm_batch")
    cfg = EDAConfig(model_type="TransformerEda", n_layers=2)
    torch.manual_seed(777)
    _replay_construction_rng(cfg, 0.5)
    lens = [int(v) for v in g["lens"]]
    perms = [torch.randperm(n) for n in lens]
    sd = to_torch(eda_state_dict(cfg, seed=785))
    xs = [torch.from_numpy(x) for x in eda_inputs(lens, seed=15)]
    act, probs = eend_ref.infer_full(sd, cfg, xs, perms)
    np.testing.assert_allclose(probs.numpy(), g["probs"], atol=1e-5)
    ys = eend_ref.select([act[i, : lens[i]] for i in range(2)], probs, 0, None, 0.5)
    assert [y.shape[1] for y in ys] == list(g["nsel"])
    np.testing.assert_allclose(np.concatenate([y.numpy().reshape(-1) for y in ys]), g["ys"], atol=1e-5)
