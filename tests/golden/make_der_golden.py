"""Known-answer DER fixtures from the reference's own scorer.

Runs the reference's md-eval.pl (SCTK 2.4.12, shipped as perl source in the
reference tree, run here in this container only) on
  * the reference's RTTM fixtures egs/magicdata-ramc/tests/alimeeting/{eval,test}
    (copied gzipped into tests/golden/der/ as data), and
  * seeded synthetic RTTM pairs covering the edge cases md-eval handles
    (overlapping turns of one speaker, zero-length turns, NOSCORE tokens, more
    system than reference speakers, recordings missing from the system output,
    sub-collar turns, a UEM file),
at several collars, with and without ``-1``, and stores md-eval's printed
``DER/MS/FA/SC`` line per case in tests/golden/der/expected.json.

    python tests/golden/make_der_golden.py      (needs /root/reference and perl)
"""
import gzip
import json
import os
import shutil
import subprocess
import sys

import numpy as np

REF = "/root/reference"
MDEVAL = f"{REF}/egs/alimeeting/SCTK-2.4.12/src/md-eval/md-eval.pl"
FIX = f"{REF}/egs/magicdata-ramc/tests/alimeeting"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "der")

FIXTURE_FILES = {
    "eval": ["alimeeting_eval.rttm", "tsvad_sys.rttm", "alimeeting_eval_oracle_sad_rttm_cam++_advanced.rttm",
             "alimeeting_eval_1.0dur.rttm", "tsvad_sys_1.0dur.rttm", "tsvad_sys_strict_2dur.rttm"],
    "test": ["alimeeting_test.rttm", "tsvad_sys.rttm"],
}
# (ref, sys) pairs scored on the fixtures.
FIXTURE_PAIRS = [
    ("eval/alimeeting_eval.rttm", "eval/tsvad_sys.rttm"),
    ("eval/alimeeting_eval.rttm", "eval/alimeeting_eval_oracle_sad_rttm_cam++_advanced.rttm"),
    ("eval/alimeeting_eval_1.0dur.rttm", "eval/tsvad_sys_1.0dur.rttm"),
    ("eval/alimeeting_eval.rttm", "eval/tsvad_sys_strict_2dur.rttm"),
    ("test/alimeeting_test.rttm", "test/tsvad_sys.rttm"),
]
COLLARS = [0.0, 0.25, 0.5]


def md_eval(ref, sys_, collar, one=False, uem=None):
    cmd = ["perl", MDEVAL] + (["-1"] if one else []) + ["-c", str(collar), "-r", ref, "-s", sys_]
    if uem:
        cmd += ["-u", uem]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        # md-eval dies when nothing is left to score (all time inside collars).
        assert "division by zero" in r.stderr, r.stderr
        return "error: division by zero"
    return r.stdout.strip().splitlines()[-1]


def synth_pair(seed):
    """A random meeting set: (ref_lines, sys_lines, uem_lines)."""
    rng = np.random.default_rng(seed)
    ref, sys_, uem = [], [], []
    n_files = int(rng.integers(1, 4))
    for fi in range(n_files):
        name = f"M{seed:03d}_{fi}"
        dur = float(rng.uniform(20, 120))
        n_ref = int(rng.integers(1, 5))
        for s in range(n_ref):
            t = float(rng.uniform(0, 3))
            while t < dur:
                d = float(rng.choice([rng.uniform(0.05, 0.6), rng.uniform(0.5, 8.0)]))
                ref.append((name, t, d, f"r{s}"))
                # Same-speaker overlapping turn now and then (md-eval accepts it).
                if rng.random() < 0.05:
                    ref.append((name, t + d * 0.5, d, f"r{s}"))
                t += d + float(rng.exponential(2.0))
        if rng.random() < 0.3:
            ref.append((name, float(rng.uniform(0, dur)), 0.0, "r0"))      # zero-length turn
        if seed % 5 == 4 and fi == n_files - 1:
            continue                                                     # no system output
        n_sys = n_ref + int(rng.integers(-1, 3))
        for s in range(max(n_sys, 1)):
            t = float(rng.uniform(0, 3))
            while t < dur:
                d = float(rng.uniform(0.1, 6.0))
                sys_.append((name, t, d, f"s{(s * 7 + seed) % 10}"))
                t += d + float(rng.exponential(1.5))
        if seed % 3 == 0:
            a = float(rng.uniform(0, 10))
            uem.append(f"{name} 1 {a:.2f} {a + dur * 0.6:.2f}\n")
    fmt = lambda r: "SPEAKER %s 1 %.3f %.3f <NA> <NA> %s <NA> <NA>\n" % r
    ref_lines = [fmt(r) for r in ref]
    if seed % 4 == 1:   # NOSCORE region in the reference
        name, t, d, _ = ref[len(ref) // 2]
        ref_lines.append(f"NOSCORE {name} 1 {t:.3f} {min(d, 3.0):.3f} <NA> <NA> <NA> <NA> <NA>\n")
    return ref_lines, [fmt(r) for r in sys_], uem


def main():
    if not os.path.exists(MDEVAL):
        sys.exit("needs the reference tree (md-eval.pl)")
    os.makedirs(OUT, exist_ok=True)
    for sub, files in FIXTURE_FILES.items():
        os.makedirs(os.path.join(OUT, sub), exist_ok=True)
        for f in files:
            with open(os.path.join(FIX, sub, f), "rb") as src, \
                    open(os.path.join(OUT, sub, f + ".gz"), "wb") as raw, \
                    gzip.GzipFile(fileobj=raw, mode="wb", compresslevel=9, mtime=0) as dst:
                shutil.copyfileobj(src, dst)
    cases = []
    for ref, sys_ in FIXTURE_PAIRS:
        for c in COLLARS:
            for one in (False, True):
                cases.append(dict(ref=ref, sys=sys_, collar=c, ignore_overlap=one,
                                  line=md_eval(f"{FIX}/{ref}", f"{FIX}/{sys_}", c, one)))
                print(cases[-1])
    synth = os.path.join(OUT, "synth")
    os.makedirs(synth, exist_ok=True)
    for seed in range(24):
        r, s, u = synth_pair(seed)
        rp, sp, up = (os.path.join(synth, f"{seed:02d}.{k}") for k in ("ref.rttm", "sys.rttm", "uem"))
        for p, lines in ((rp, r), (sp, s), (up, u)):
            with open(p, "w") as f:
                f.writelines(lines)
        if not u:
            os.remove(up)
        for c in (0.0, 0.25):
            for one in (False, True):
                cases.append(dict(ref=f"synth/{seed:02d}.ref.rttm", sys=f"synth/{seed:02d}.sys.rttm",
                                  uem=f"synth/{seed:02d}.uem" if u else None, collar=c, ignore_overlap=one,
                                  line=md_eval(rp, sp, c, one, up if u else None)))
    with open(os.path.join(OUT, "expected.json"), "w") as f:
        json.dump(cases, f, indent=1)
    print(len(cases), "cases")


if __name__ == "__main__":
    main()
