"""DER scorer vs md-eval.pl's own output (tests/golden/make_der_golden.py).

md-eval prints percentages with two decimals, so each case must agree to
within rounding (0.005 + float slack); the north-star bar is +-0.1.
"""
import gzip
import io
import json
import os

import pytest

from speaker_diarization_amd import der

GOLD = os.path.join(os.path.dirname(__file__), "golden", "der")
CASES = json.load(open(os.path.join(GOLD, "expected.json")))


def _src(rel):
    p = os.path.join(GOLD, rel)
    if os.path.exists(p + ".gz"):
        return io.TextIOWrapper(gzip.open(p + ".gz"), encoding="utf-8")
    return p


@pytest.mark.parametrize("case", CASES, ids=lambda c: f"{c['ref']}|{c['sys']}|c{c['collar']}|1={c['ignore_overlap']}")
def test_md_eval_known_answers(case):
    kw = dict(collar=case["collar"], ignore_overlap=case["ignore_overlap"],
              uem=os.path.join(GOLD, case["uem"]) if case.get("uem") else None)
    if case["line"].startswith("error"):
        with pytest.raises(ZeroDivisionError):
            der.md_eval(_src(case["ref"]), _src(case["sys"]), **kw)
        return
    st = der.md_eval(_src(case["ref"]), _src(case["sys"]), **kw)
    want = [float(x) for x in case["line"].split("/")]
    got = [st.der, st.ms, st.fa, st.sc]
    assert all(abs(g - w) <= 0.005 + 1e-6 for g, w in zip(got, want)), (got, want)


def test_perfect_and_empty_system():
    ref = ["SPEAKER m 1 0.00 2.00 <NA> <NA> a <NA> <NA>\n", "SPEAKER m 1 1.00 3.00 <NA> <NA> b <NA> <NA>\n"]
    renamed = [l.replace(" a ", " x ").replace(" b ", " y ") for l in ref]
    assert der.md_eval(ref, renamed).der == 0.0
    st = der.md_eval(ref, [])
    assert st.ms == 100.0 and st.fa == 0.0 and st.sc == 0.0
    # scored speaker time: a 2 s + b 3 s
    assert abs(st.scored_speaker - 5.0) < 1e-9


def test_speaker_confusion_mapping():
    # sys swaps labels half-way; the optimal map keeps the longer agreement.
    ref = ["SPEAKER m 1 0 10 <NA> <NA> a <NA> <NA>\n", "SPEAKER m 1 10 4 <NA> <NA> b <NA> <NA>\n"]
    sys_ = ["SPEAKER m 1 0 6 <NA> <NA> 1 <NA> <NA>\n", "SPEAKER m 1 6 8 <NA> <NA> 2 <NA> <NA>\n"]
    st = der.md_eval(ref, sys_)
    # a->1 (6 s) and b->2 (4 s): error on [6,10) = 4 s of 14 s
    assert abs(st.sc - 100 * 4 / 14) < 1e-9 and st.ms == 0 and st.fa == 0


def test_rttm_roundtrip_format():
    line = der.format_rttm_line("R1_M1", 1.2, 0.84, 3)
    assert line == "SPEAKER R1_M1 1 1.200 0.840 <NA> <NA> 3 <NA> <NA>\n"
    rec = der.read_rttm([line])[("R1_M1", "1")]
    assert abs(rec.speakers["3"][0].tend - 2.04) < 1e-12


def test_collar_must_be_nonnegative():
    with pytest.raises(ValueError):
        der.md_eval(["SPEAKER m 1 0 1 <NA> <NA> a <NA> <NA>\n"], [], collar=-0.1)
