"""TS-VAD output stage pinned to a run of the reference itself: tests/golden/postprocess_*.npz
hold res_dicts and the res_rttm_<thr> files + der_result that ts_vad2/infer.py postprocess
(:72-163, imported from the reference and run here by make_postprocess_golden.py) wrote for
them.  Checked here (CPU): the oracle restatement (oracle/postprocess_ref.py) and the product's
host writer reproduce every RTTM byte for byte, and the md-eval restatement
(speaker_diarization_amd/der.py) reproduces the printed DER/MS/FA/SC.  The GPU writer is
checked against the same goldens in test_gpu_postprocess.py."""
import os
import re

import numpy as np
import pytest

from make_postprocess_golden import POSTPROCESS_CASES, THRESHOLDS, load_res_dict
from oracle.postprocess_ref import rttm_lines
from speaker_diarization_amd import der as der_mod
from speaker_diarization_amd.ts_vad.postprocess import posteriors_to_rttm

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def averaged(res):
    """infer.py:88-93: frames sorted, np.mean of each frame's float32 list."""
    return {k: np.array([np.mean(v) for v in lists], np.float32) for k, lists in res.items()}


@pytest.mark.parametrize("name", list(POSTPROCESS_CASES))
def test_oracle_rttm_matches_reference_run(name):
    g = np.load(os.path.join(GOLD, name + ".npz"))
    post = averaged(load_res_dict(os.path.join(GOLD, name + ".npz")))
    got = rttm_lines(post)
    for j, thr in enumerate(THRESHOLDS):
        assert "".join(got[thr]) == str(g["rttm"][j]), thr


@pytest.mark.parametrize("name", list(POSTPROCESS_CASES))
def test_host_writer_matches_reference_run(name):
    g = np.load(os.path.join(GOLD, name + ".npz"))
    post = averaged(load_res_dict(os.path.join(GOLD, name + ".npz")))
    got = posteriors_to_rttm(post)
    for j, thr in enumerate(THRESHOLDS):
        assert "".join(got[thr]) == str(g["rttm"][j]), thr


@pytest.mark.parametrize("name", list(POSTPROCESS_CASES))
def test_der_matches_reference_md_eval(name):
    """der_result lines 'Eval for threshold T: DER a%, MS b%, FA c%, SC d%' (md-eval.pl
    -c 0.25 against the reference RTTM) vs the restated scorer, to the printed 0.01."""
    g = np.load(os.path.join(GOLD, name + ".npz"))
    ref = der_mod.read_rttm(str(g["ref_rttm"]).splitlines(keepends=True))
    printed = re.findall(r"threshold ([\d.]+): DER ([\d.]+)%, MS ([\d.]+)%, FA ([\d.]+)%, SC ([\d.]+)%",
                         str(g["der_result"]))
    assert len(printed) == len(THRESHOLDS)
    for j, (thr, d, ms, fa, sc) in enumerate(printed):
        sys_ = der_mod.read_rttm(str(g["rttm"][j]).splitlines(keepends=True))
        if not sys_:
            continue          # md-eval scores an empty system file as all-miss; covered in test_der.py
        r = der_mod.md_eval(ref, sys_, collar=0.25)
        for got, want in ((r.der, d), (r.ms, ms), (r.fa, fa), (r.sc, sc)):
            assert abs(got - float(want)) <= 0.0051, (thr, got, want)
