"""SSND oracle (oracle/ssnd_ref.py) pinned to the reference module's outputs
(tests/golden/ssnd_*.npz from tests/golden/make_ssnd_golden.py, which imports
egs/alimeeting/ssnd/ssnd_model.py here)."""
import os

import numpy as np
import pytest
import torch

from make_ssnd_golden import SSND_CASES, ssnd_cfg, ssnd_inputs
from oracle import ssnd_ref
from speaker_diarization_amd.weights import ssnd_state_dict, to_torch

GOLD = os.path.join(os.path.dirname(__file__), "golden")


@pytest.mark.parametrize("name", list(SSND_CASES))
def test_ssnd_oracle_matches_reference(name):
    kind, B, T, N, iseed, wseed = SSND_CASES[name]
    cfg = ssnd_cfg(N)
    sd = to_torch(ssnd_state_dict(cfg, seed=wseed))
    g = np.load(os.path.join(GOLD, name + ".npz"))
    with torch.no_grad():
        if kind == "decode":
            enc, x, spk = (torch.from_numpy(a) for a in ssnd_inputs(kind, B, T, N, iseed, cfg))
            vad, emb = ssnd_ref.decode(sd, cfg, enc, x, spk)
        else:
            feats, spk = (torch.from_numpy(a) for a in ssnd_inputs(kind, B, T, N, iseed, cfg))
            vad, emb = ssnd_ref.infer(sd, cfg, feats, spk)
    np.testing.assert_allclose(vad.numpy(), g["vad_pred"], atol=2e-5, rtol=1e-5)
    np.testing.assert_allclose(emb.numpy(), g["emb_pred"], atol=2e-5, rtol=1e-5)


def test_ssnd_layout_keys():
    from speaker_diarization_amd.weights import SSNDConfig, ssnd_layout
    keys = [k for k, _, _ in ssnd_layout(SSNDConfig())]
    assert len(keys) == len(set(keys)) == 1272
