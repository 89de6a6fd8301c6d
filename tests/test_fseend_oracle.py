"""FS-EEND and plain-EEND oracles (oracle/fseend_ref.py) against the reference goldens."""
import os

import numpy as np
import pytest
import torch

from oracle import fseend_ref
from speaker_diarization_amd.weights import (EDAConfig, FSEENDConfig, eend_layout, fseend_state_dict,
                                             synthetic_state_dict, to_torch)
from tests.golden.make_golden import EEND_CASES, FSEEND_CASES, eda_inputs

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def _load(name):
    return dict(np.load(os.path.join(GOLD, name + ".npz")))


@pytest.mark.parametrize("name", list(FSEEND_CASES))
def test_fseend_oracle_matches_reference(name):
    lens, C, delay, iseed, wseed = FSEEND_CASES[name]
    g = _load(name)
    cfg = FSEENDConfig(mask_delay=delay)
    sd = to_torch(fseend_state_dict(cfg, seed=wseed))
    xs = [torch.from_numpy(x) for x in eda_inputs(lens, seed=iseed)]
    out, emb, att = fseend_ref.fseend_test(sd, cfg, xs, lens, C)
    np.testing.assert_allclose(torch.cat(out).numpy(), g["out"], atol=1e-5)
    np.testing.assert_allclose(torch.cat(emb).numpy(), g["emb"], atol=1e-5)
    np.testing.assert_allclose(torch.cat([a[:24] for a in att]).numpy(), g["att_head"], atol=1e-5)


def test_fseend_state_dict_shares_decoder_layers():
    sd = fseend_state_dict(FSEENDConfig(), seed=1)
    a = [k for k in sd if k.startswith("dec.attractor_decoder.0.")]
    assert len(a) == 20
    for k in a:
        assert np.array_equal(sd[k], sd[k.replace(".0.", ".1.", 1)])


@pytest.mark.parametrize("name", list(EEND_CASES))
def test_eend_oracle_matches_reference(name):
    nspk, L, lens, iseed, wseed = EEND_CASES[name]
    g = _load(name)
    sd = to_torch(synthetic_state_dict(eend_layout(EDAConfig(n_speakers=nspk, n_layers=L)), wseed))
    xs = [torch.from_numpy(x) for x in eda_inputs(lens, seed=iseed)]
    ys = fseend_ref.eend_forward(sd, L, 4, xs)
    np.testing.assert_allclose(torch.cat(ys).numpy(), g["ys"], atol=1e-5)
