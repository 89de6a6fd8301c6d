"""Diarization error rate, scored the way the recipes score it.

Every recipe in the reference scores its RTTM with NIST md-eval (SCTK 2.4.12,
``egs/alimeeting/SCTK-2.4.12/src/md-eval/md-eval.pl``) invoked as
``perl md-eval.pl -c <collar> -s <sys> -r <ref>`` (ts_vad2/infer.py:136-151) or
with ``-1`` to drop overlapped speech (sond/.../cluster.py:174), and parses the
one line it prints: ``DER/MS/FA/SC`` in percent of scored speaker time.  This
module restates the speaker-diarization half of md-eval so a user of this
package needs neither perl nor the SCTK tree; it is pinned against md-eval's
own output on the reference's RTTM fixtures (tests/golden/der/, test_der.py).

What is restated (md-eval.pl line numbers):
  * RTTM parsing, get_rttm_file (500-611): whitespace fields, ``*`` stripped
    from times, ``<NA>`` duration -> 0, channel lower-cased.  The per-speaker
    overlap check there never fires (``$prev_token`` is never assigned), so
    overlapping turns of one speaker are accepted; they count once, as in
    create_speaker_segs.
  * The evaluation map: a UEM file (get_uem_data 435-480) or, without one,
    [min start, max end] of the reference tokens (uem_from_rttm 2245-2257);
    NOSCORE tokens cut no-eval / no-score zones (add_exclusion_zones_to_uem
    2132-2243).
  * Speaker mapping (score_speaker_diarization 1871-1925, map_speakers
    2461-2478): the one-to-one ref->sys map maximising total co-speaking time
    over the evaluation map (before collars), an assignment problem; md-eval
    solves it with its own Hungarian implementation (2675-2905), here
    scipy.optimize.linear_sum_assignment on the same cost matrix (including
    md-eval's "no edge costs slightly more than the worst edge" rule).
  * No-score collars of +-collar around every reference boundary
    (add_collars_to_uem 2034-2070) and optional exclusion of overlapped
    reference speech (exclude_overlapping_speech_from_uem 2072-2130, ``-1``).
  * Per scored segment (score_speaker_segments 1954-2018):
    missed = dur*max(nref-nsys,0), false alarm = dur*max(nsys-nref,0),
    speaker error = dur*(min(nref,nsys) - mapped matches); all summed over
    files and channels and divided by scored speaker time (print_sd_scores
    2367-2410).

Not restated: the word-mediated (``-w``/``-W``) and metadata (SU/EDIT/FILLER/IP)
scoring of md-eval, which no recipe of the reference uses for diarization.
"""
from __future__ import annotations

import dataclasses
import functools
import os
import re
from collections import defaultdict
from typing import Dict, Iterable, List, Optional, Tuple, Union

import numpy as np

EPSILON = 1e-8           # md-eval.pl:109
DEFAULT_EXTEND = 0.50    # md-eval.pl:188, max no-score zone extension
# Token types that define the default evaluation span (uem_from_rttm).
_UEM_TYPES = {"SEGMENT", "SPEAKER", "SU", "EDIT", "FILLER", "IP", "CB", "A/P", "LEXEME", "NON-LEX"}
# Default no-eval / no-score token sets for speaker diarization (md-eval.pl:170-181).
NOEVAL_SD = {"NOSCORE": {"<na>"}}
NOSCORE_SD = {"NOSCORE": {"<na>"}, "NON-LEX": {"laugh", "breath", "lipsmack", "cough", "sneeze", "other"}}

Uem = List[Tuple[float, float]]


@dataclasses.dataclass
class Token:
    type: str
    file: str
    chnl: str
    tbeg: float
    tdur: float
    subt: str
    spkr: str

    @property
    def tend(self) -> float:
        return self.tbeg + self.tdur


@dataclasses.dataclass
class Recording:
    tokens: List[Token] = dataclasses.field(default_factory=list)
    speakers: Dict[str, List[Token]] = dataclasses.field(default_factory=lambda: defaultdict(list))


RttmData = Dict[Tuple[str, str], Recording]


def _lines(src: Union[str, os.PathLike, Iterable[str]]) -> Iterable[str]:
    if isinstance(src, (str, os.PathLike)):
        with open(src) as f:
            yield from f
    else:
        yield from src


def _num(s: str) -> float:
    return float(s.replace("*", ""))


def read_rttm(src, data: Optional[RttmData] = None) -> RttmData:
    """Parse RTTM lines (a path or an iterable of lines) into per-(file, channel)
    recordings, md-eval.pl:500-611."""
    data = {} if data is None else data
    for rec in _lines(src):
        s = rec.strip()
        if not s or s[0] in "#;":
            continue
        f = s.split()
        if len(f) < 9:
            raise ValueError(f"insufficient number of fields in RTTM record: {rec!r}")
        dur = f[4].lower().replace("*", "")
        tok = Token(type=f[0].upper(), file=f[1], chnl=f[2].lower(), tbeg=_num(f[3]),
                    tdur=0.0 if dur == "<na>" else float(dur), subt=f[6].lower(),
                    spkr=f[7] if len(f) > 7 else "<na>")
        if tok.tdur < 0:
            raise ValueError(f"negative duration in RTTM record: {rec!r}")
        r = data.setdefault((tok.file, tok.chnl), Recording())
        if tok.type == "SPKR-INFO":
            continue
        r.tokens.append(tok)
        if tok.type == "SPEAKER":
            r.speakers[tok.spkr].append(tok)
    for r in data.values():
        for segs in r.speakers.values():
            segs.sort(key=lambda t: t.tbeg + t.tdur / 2)
    return data


def read_uem(src) -> Dict[Tuple[str, str], Uem]:
    """UEM ``<file> <chnl> <tbeg> <tend>`` records, md-eval.pl:435-480 (directory and
    extension stripped from the file field, as without ``-n``)."""
    out: Dict[Tuple[str, str], Uem] = defaultdict(list)
    for rec in _lines(src):
        s = rec.strip()
        if not s or s[0] in "#;":
            continue
        f = s.split()
        if len(f) < 4:
            raise ValueError(f"insufficient number of fields in UEM record: {rec!r}")
        name = re.sub(r"\.[^.]*", "", f[0].rsplit("/", 1)[-1], count=1)
        keep = lambda x: float(re.sub(r"[^0-9.]", "", x))
        out[(name, f[1].lower())].append((keep(f[2]), keep(f[3])))
    for key, segs in out.items():
        segs.sort()
        for (b0, e0), (b1, e1) in zip([(None, None)] + segs[:-1], segs):
            if e1 <= b1:
                raise ValueError(f"non-positive evaluation segment in UEM for {key}")
            if e0 is not None and b1 < e0:
                raise ValueError(f"overlapping evaluation segments in UEM for {key}")
    return dict(out)


def uem_from_rttm(tokens: List[Token]) -> Uem:
    """md-eval.pl:2245-2257."""
    tbeg, tend = 1e30, 0.0
    for t in tokens:
        if t.type in _UEM_TYPES:
            tbeg, tend = min(tbeg, t.tbeg), max(tend, t.tend)
    return [(tbeg, tend)]


def _sweep_uem(events, uem: Uem) -> Uem:
    """Intersect UEM segments with the complement of no-score zones.  `events` are
    (time, is_beg, 'NSZ'); shared by the two exclusion passes of md-eval
    (2223-2240, 2108-2127): ties sort END before BEG."""
    ev = list(events)
    for b, e in uem:
        if e - b > 0:
            ev += [(b, True, "UEM"), (e, False, "UEM")]
    ev.sort(key=_end_first)
    out, evl, nsz, evaluating, tbeg = [], 0, 0, False, 0.0
    for t, beg, kind in ev:
        if kind == "UEM":
            evl += 1 if beg else -1
        else:
            nsz += 1 if beg else -1
        if evaluating and (evl == 0 or nsz > 0) and t > tbeg:
            out.append((tbeg, t))
            evaluating = False
        elif evl > 0 and nsz == 0:
            tbeg, evaluating = t, True
    return out


def _end_first(ev):
    # Perl's tie rule ($a->{EVENT} eq "BEG") puts ENDs before BEGs at equal times.
    return (ev[0], bool(ev[1]))


def add_exclusion_zones(excluded, uem: Uem, tokens: List[Token], max_extend: Optional[float] = None) -> Uem:
    """Cut no-score zones around excluded tokens out of `uem`, md-eval.pl:2132-2243."""
    if not excluded:
        return uem
    ns = []
    for t in tokens:
        if t.tdur <= 0:
            continue
        if t.type == "LEXEME" and t.subt not in excluded.get("LEXEME", ()):
            kind = "LEX"
        elif t.type == "SPEAKER":
            kind = "SEG"
        elif t.subt in excluded.get(t.type, ()):
            kind = "NSZ"
        else:
            continue
        ns += [(t.tbeg, True, kind), (t.tend, False, kind)]
    ns.sort(key=_end_first)
    ext = EPSILON if not max_extend or max_extend < EPSILON else max_extend
    zones, evaluating = [], True
    tseg = tbeg_nsz = tbeg_lex = tend_nsz = tend_lex = 0.0
    lex = nsz = 0
    for t, beg, kind in ns:
        if kind == "LEX":
            if beg:
                if lex == 0:
                    tbeg_lex = t
                lex += 1
            else:
                if lex == 1:
                    tend_lex = t
                lex -= 1
        elif kind == "NSZ":
            if beg:
                if nsz == 0:
                    tbeg_nsz = t
                nsz += 1
            else:
                if nsz == 1:
                    tend_nsz = t
                nsz -= 1
        else:
            tseg = t
        if evaluating:
            if nsz == 0 or kind != "NSZ":
                continue
            tstop = t if lex > 0 else max(tend_lex, tseg, t - ext)
            zones.append((tstop, True, "NSZ"))
            evaluating = False
        elif nsz == 0 and (lex > 0 or kind == "SEG"):
            zones.append((min(tend_nsz + ext, t), False, "NSZ"))
            evaluating = True
        elif nsz == 1 and kind == "NSZ" and beg and t > tend_nsz + 2 * ext:
            zones += [(tend_nsz + ext, False, "NSZ"), (t - ext, True, "NSZ")]
            evaluating = False
    return _sweep_uem(zones, uem)


def add_collars(uem: Uem, ref_speakers: Dict[str, List[Token]], collar: float) -> Uem:
    """No-score collars around every reference boundary, md-eval.pl:2034-2070."""
    ev = []
    for b, e in uem:
        ev += [(b, True), (e, False)]
    for segs in ref_speakers.values():
        for s in segs:
            ev += [(s.tbeg - collar, False), (s.tbeg + collar, True),
                   (s.tend - collar, False), (s.tend + collar, True)]
    # Tie rule ($a->{EVENT} eq "END"): BEGs before ENDs at equal times.
    ev.sort(key=lambda x: (x[0], not x[1]))
    out, depth, tbeg = [], 0, 0.0
    for t, beg in ev:
        if beg:
            depth += 1
            if depth == 1:
                tbeg = t
        else:
            depth -= 1
            if depth == 0 and t > tbeg:
                out.append((tbeg, t))
    return out


def exclude_overlap(uem: Uem, tokens: List[Token]) -> Uem:
    """md-eval ``-1``: drop reference regions where >= 2 speakers talk (2072-2130)."""
    ev = []
    for t in tokens:
        if t.type == "SPEAKER" and t.tdur > 0:
            ev += [(t.tbeg, True), (t.tend, False)]
    ev.sort(key=_end_first)
    zones, cnt, t0 = [], 0, 0.0
    for t, beg in ev:
        if beg:
            cnt += 1
            if cnt == 2:
                t0 = t
        else:
            cnt -= 1
            if cnt == 1:
                zones += [(t0, True, "NSZ"), (t, False, "NSZ")]
    return _sweep_uem(zones, uem)


def speaker_segments(uem: Uem, ref: Dict[str, List[Token]], sys: Dict[str, List[Token]]):
    """Split the scored map at every ref/sys boundary, md-eval.pl:2261-2315.
    Yields (tbeg, tend, ref_speakers, sys_speakers) with frozenset speaker sets."""
    ev = []
    for b, e in uem:
        if e > b + EPSILON:
            ev += [(b, 1, "UEM", None), (e, 0, "UEM", None)]
    for side, spk in (("REF", ref), ("SYS", sys)):
        for name, segs in spk.items():
            for s in segs:
                if s.tdur > 0:
                    ev += [(s.tbeg, 1, side, name), (s.tend, 0, side, name)]

    def cmp(a, b):   # END before BEG within EPSILON, otherwise by time
        if a[0] < b[0] - EPSILON:
            return -1
        if a[0] > b[0] + EPSILON:
            return 1
        return -1 if a[1] == 0 else 1

    ev.sort(key=functools.cmp_to_key(cmp))
    counts = {"REF": defaultdict(int), "SYS": defaultdict(int)}
    out, evaluate, tbeg = [], False, 0.0
    for t, beg, side, name in ev:
        if evaluate and tbeg < t:
            out.append((tbeg, t, frozenset(k for k, v in counts["REF"].items() if v),
                        frozenset(k for k, v in counts["SYS"].items() if v)))
            tbeg = t
        if side == "UEM":
            evaluate = bool(beg)
            if evaluate:
                tbeg = t
        else:
            counts[side][name] += 1 if beg else -1
    return out


def map_speakers(overlap: Dict[str, Dict[str, float]]) -> Dict[str, str]:
    """Optimal one-to-one ref->sys mapping maximising co-speaking time
    (map_speakers + weighted_bipartite_graph_match, md-eval.pl:2461-2478, 2675-2905)."""
    from scipy.optimize import linear_sum_assignment
    if not overlap:
        return {}
    rows = sorted(overlap)
    cols = sorted({c for r in rows for c in overlap[r]})
    # md-eval: cost = -overlap shifted by its minimum; a missing edge costs
    # -min_score*(1+1e-12), i.e. a hair worse than the worst existing edge.
    min_score = min(-v for r in rows for v in overlap[r].values())
    n = max(len(rows), len(cols)) + 1
    no_edge = -min_score * (1 + 1e-12)
    cost = np.full((n, n), no_edge)
    for i, r in enumerate(rows):
        for c, v in overlap[r].items():
            cost[i, cols.index(c)] = -v - min_score
    ri, ci = linear_sum_assignment(cost)
    out = {}
    for i, j in zip(ri, ci):
        if i < len(rows) and j < len(cols) and cols[j] in overlap[rows[i]]:
            out[rows[i]] = cols[j]
    return out


@dataclasses.dataclass
class DerStats:
    eval_time: float = 0.0
    eval_speech: float = 0.0
    scored_time: float = 0.0
    scored_speech: float = 0.0
    missed_speech: float = 0.0
    falarm_speech: float = 0.0
    scored_speaker: float = 0.0
    missed_speaker: float = 0.0
    falarm_speaker: float = 0.0
    speaker_error: float = 0.0

    def __iadd__(self, o: "DerStats"):
        for f in dataclasses.fields(self):
            setattr(self, f.name, getattr(self, f.name) + getattr(o, f.name))
        return self

    def _pct(self, x):
        return 100.0 * x / self.scored_speaker if self.scored_speaker else float("nan")

    @property
    def der(self):
        return self._pct(self.missed_speaker + self.falarm_speaker + self.speaker_error)

    @property
    def ms(self):
        return self._pct(self.missed_speaker)

    @property
    def fa(self):
        return self._pct(self.falarm_speaker)

    @property
    def sc(self):
        return self._pct(self.speaker_error)

    def line(self) -> str:
        """md-eval's one output line, ``DER/MS/FA/SC`` (print_sd_scores)."""
        return "%.2f/%.2f/%.2f/%.2f" % (self.der, self.ms, self.fa, self.sc)


def score_recording(ref: Recording, sys: Optional[Recording], uem: Uem, collar: float = 0.0,
                    ignore_overlap: bool = False, mapping_out: Optional[dict] = None) -> DerStats:
    """score_speaker_diarization for one (file, channel), md-eval.pl:1871-1925."""
    st = DerStats()
    sys_spk = sys.speakers if sys is not None else {}
    uem_eval = add_exclusion_zones(NOEVAL_SD, uem, ref.tokens)
    for b, e in uem_eval:
        st.eval_time += e - b
    overlap: Dict[str, Dict[str, float]] = defaultdict(lambda: defaultdict(float))
    for b, e, rs, ss in speaker_segments(uem_eval, ref.speakers, sys_spk):
        if not rs:
            continue
        st.eval_speech += e - b
        for r in rs:
            for s in ss:
                overlap[r][s] += e - b
    mapping = map_speakers({r: dict(v) for r, v in overlap.items()}) if overlap else {}
    if mapping_out is not None:
        mapping_out.update(mapping)
    uem_score = add_collars(uem_eval, ref.speakers, collar) if collar > 0 else uem_eval
    uem_score = add_exclusion_zones(NOSCORE_SD, uem_score, ref.tokens)
    uem_score = add_exclusion_zones({"NON-LEX": NOSCORE_SD["NON-LEX"]}, uem_score, ref.tokens, DEFAULT_EXTEND)
    if ignore_overlap:
        uem_score = exclude_overlap(uem_score, ref.tokens)
    for b, e, rs, ss in speaker_segments(uem_score, ref.speakers, sys_spk):
        d, nref, nsys = e - b, len(rs), len(ss)
        st.scored_time += d
        st.scored_speech += d if nref else 0.0
        st.missed_speech += d if nref and not nsys else 0.0
        st.falarm_speech += d if nsys and not nref else 0.0
        st.scored_speaker += d * nref
        st.missed_speaker += d * max(nref - nsys, 0)
        st.falarm_speaker += d * max(nsys - nref, 0)
        nmap = sum(1 for r in rs if r in mapping and mapping[r] in ss)
        st.speaker_error += d * (min(nref, nsys) - nmap)
    return st


def md_eval(ref_rttm, sys_rttm, collar: float = 0.0, ignore_overlap: bool = False,
            uem=None, per_file: bool = False):
    """Score a system RTTM against a reference RTTM like
    ``md-eval.pl [-1] -c <collar> -r <ref> -s <sys> [-u <uem>]``.

    ref_rttm / sys_rttm: path, iterable of RTTM lines, or a parsed RttmData.
    Returns the pooled DerStats (``.der/.ms/.fa/.sc`` in percent, ``.line()`` is
    md-eval's printout) or, with per_file=True, (pooled, {(file, chnl): DerStats}).
    Only recordings present in the reference are scored (evaluate, 613-690).
    """
    if collar < 0:
        raise ValueError("Speaker Diarization scoring collar must be non-negative")
    ref = ref_rttm if isinstance(ref_rttm, dict) else read_rttm(ref_rttm)
    sys = sys_rttm if isinstance(sys_rttm, dict) else read_rttm(sys_rttm)
    uems = None if uem is None else (uem if isinstance(uem, dict) else read_uem(uem))
    total, files = DerStats(), {}
    for key in sorted(ref):
        r = ref[key]
        if not r.speakers:
            continue
        u = uems.get(key) if uems is not None else None
        if u is None:
            u = uem_from_rttm(r.tokens)
        st = score_recording(r, sys.get(key), u, collar, ignore_overlap)
        files[key] = st
        total += st
    if not total.scored_speaker > 0:
        # md-eval dies here ("Illegal division by zero", print_sd_scores).
        raise ZeroDivisionError("no scored speaker time (every reference turn lies inside the collars?)")
    return (total, files) if per_file else total


def format_rttm_line(name: str, tbeg: float, tdur: float, speaker) -> str:
    """The SPEAKER line the recipes write (ts_vad2/infer.py:104-112)."""
    return ("SPEAKER " + str(name) + " 1 %.3f" % tbeg + " %.3f " % tdur + "<NA> <NA> " + str(speaker)
            + " <NA> <NA>\n")
