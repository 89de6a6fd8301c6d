"""Two-stream critical-path account of one TS-VAD step from a rocprofv3 kernel trace (round-4 verdict item 3).

    python tools/stream_timeline.py <kernel_trace.csv> [--step K]

The trace is `rocprofv3 --kernel-trace --output-format csv` of `bench.py --workload c2` WITHOUT
SDIAR_CAM_ONE_STREAM, i.e. the shipped schedule: two window slices on two HIP streams (tsvad.cpp
`slice`), then the BiLSTM and the tail on the main stream.  A step is the span from one `fbank_kernel`
launch to the next.  For the chosen step (default: the last complete one) it prints, per stream, the
spans of the kernel families (CAM++ trunk, conformer stack, BiLSTM, tail), the time both streams have
kernels in flight, the idle gaps, and which stream's last kernel ends the slice phase - the stream that
bounds the step.  The family sums plus gaps add up to the step span by construction, so every later perf
claim can be checked against it."""
from __future__ import annotations

import argparse
import csv
import re
from collections import defaultdict

FAMILIES = [
    ("frontend", r"fbank_kernel|window_cmn|nonfinite_windows|zero_fill"),
    ("campp", r"fcm_conv3x3|cam_dense|cam_local|cam_context|gemm_ring_kernel<true|gemm_dma_kernel|stats_pool"),
    ("down+gsp", r"gemm_bf16_kernel|gsp_fc"),
    ("conformer", r"rowprog_kernel|mha_block|gemm_areg|dwconv_pk|dwconv_pp|glu_dwconv"),
    ("lstm", r"lstm_group|lstm_step|gemm_ring_kernel<false"),
    ("tail", r"poison_windows|overlap_average|overlap_mean|elementwise|FillFunctor|medfilt|run_segments"),
    ("copy", r"__amd_rocclr"),
]


def family(name: str) -> str:
    for f, pat in FAMILIES:
        if re.search(pat, name):
            return f
    return "other"


def load(path):
    rows = list(csv.DictReader(open(path)))
    if not rows:
        raise SystemExit("empty trace")
    keys = rows[0].keys()
    skey = "Stream_Id" if "Stream_Id" in keys else "Queue_Id"
    out = []
    for r in rows:
        out.append(dict(name=r["Kernel_Name"], s=int(r["Start_Timestamp"]), e=int(r["End_Timestamp"]),
                        stream=r[skey], fam=family(r["Kernel_Name"])))
    out.sort(key=lambda k: k["s"])
    return out, skey


def union(iv):
    iv = sorted(iv)
    tot, cur = 0, None
    for s, e in iv:
        if cur is None or s > cur[1]:
            if cur:
                tot += cur[1] - cur[0]
            cur = [s, e]
        else:
            cur[1] = max(cur[1], e)
    if cur:
        tot += cur[1] - cur[0]
    return tot


def overlap(a, b):
    """time both interval sets cover"""
    ev = [(s, 0, 1) for s, e in a] + [(e, 0, -1) for s, e in a] + [(s, 1, 1) for s, e in b] + [(e, 1, -1) for s, e in b]
    ev.sort()
    cnt, last, tot = [0, 0], None, 0
    for t, w, d in ev:
        if last is not None and cnt[0] > 0 and cnt[1] > 0:
            tot += t - last
        cnt[w] += d
        last = t
    return tot


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--step", type=int, default=-1)
    a = ap.parse_args()
    ks, skey = load(a.trace)
    starts = [i for i, k in enumerate(ks) if "fbank_kernel" in k["name"]]
    steps = [(starts[i], starts[i + 1]) for i in range(len(starts) - 1)] + [(starts[-1], len(ks))]
    # the last step may carry the bench's after-step work; prefer the last complete one
    i0, i1 = steps[a.step] if len(steps) == 1 else steps[a.step - 1 if a.step == -1 else a.step]
    st = ks[i0:i1]
    t0 = st[0]["s"]
    ms = lambda ns: ns / 1e6  # noqa: E731
    # the step ends at its last tail kernel (overlap average)
    tail_end = max(k["e"] for k in st if k["fam"] in ("tail", "lstm")) if any(k["fam"] == "tail" for k in st) else max(k["e"] for k in st)
    st = [k for k in st if k["s"] <= tail_end]
    span = tail_end - t0
    streams = defaultdict(list)
    for k in st:
        streams[k["stream"]].append(k)
    print(f"{len(steps)} steps in trace ({skey}); step {a.step}: {len(st)} kernels, span {ms(span):.3f} ms")
    print(f"busy (any stream) {ms(union([(k['s'], k['e']) for k in st])):.3f} ms; "
          f"kernel time summed {ms(sum(k['e'] - k['s'] for k in st)):.3f} ms")
    for sid, kk in streams.items():
        fam = defaultdict(list)
        for k in kk:
            fam[k["fam"]].append((k["s"], k["e"]))
        print(f"stream {sid}: {len(kk)} kernels, first {ms(kk[0]['s'] - t0):.3f} last end {ms(max(k['e'] for k in kk) - t0):.3f} ms,"
              f" busy {ms(union([(k['s'], k['e']) for k in kk])):.3f} ms")
        for f, iv in sorted(fam.items(), key=lambda x: min(s for s, _ in x[1])):
            print(f"   {f:10s} {ms(min(s for s, _ in iv) - t0):8.3f} -> {ms(max(e for _, e in iv) - t0):8.3f} ms"
                  f"  busy {ms(union(iv)):7.3f}  summed {ms(sum(e - s for s, e in iv)):7.3f}  n={len(iv)}")
    sids = list(streams)
    if len(sids) >= 2:
        # the two slice streams: the two with the most conformer kernels
        sl = sorted(sids, key=lambda s: -sum(1 for k in streams[s] if k["fam"] == "conformer"))[:2]
        a_iv = [(k["s"], k["e"]) for k in streams[sl[0]]]
        b_iv = [(k["s"], k["e"]) for k in streams[sl[1]]]
        print(f"both slice streams busy {ms(overlap(a_iv, b_iv)):.3f} ms")
        for s in sl:
            conf = [k for k in streams[s] if k["fam"] == "conformer"]
            cam = [k for k in streams[s] if k["fam"] == "campp"]
            print(f"  stream {s}: campp {ms(cam[0]['s'] - t0):.3f}-{ms(cam[-1]['e'] - t0):.3f}, "
                  f"conformer {ms(conf[0]['s'] - t0):.3f}-{ms(conf[-1]['e'] - t0):.3f} ms")
        ends = {s: max(k["e"] for k in streams[s] if k["fam"] in ("campp", "conformer", "down+gsp")) for s in sl}
        bound = max(ends, key=ends.get)
        print(f"slice phase ends {ms(ends[bound] - t0):.3f} ms on stream {bound} (other stream {ms(min(ends.values()) - t0):.3f})")
    # sequential phases on the whole step: frontend, slices, lstm, tail, with gaps between kernels
    gaps = []
    allk = sorted(st, key=lambda k: k["s"])
    cur_end = allk[0]["e"]
    for k in allk[1:]:
        if k["s"] > cur_end:
            gaps.append(k["s"] - cur_end)
        cur_end = max(cur_end, k["e"])
    print(f"idle gaps (no kernel on any stream): {len(gaps)} totalling {ms(sum(gaps)):.3f} ms, largest {ms(max(gaps) if gaps else 0):.3f}")
    cur_end, prev = allk[0]["e"], allk[0]
    big = []
    for k in allk[1:]:
        if k["s"] > cur_end:
            big.append((k["s"] - cur_end, cur_end - t0, prev["name"], k["name"]))
        if k["e"] >= cur_end:
            cur_end, prev = k["e"], k
    short = lambda n: re.sub(r"\(.*", "", n.replace("(anonymous namespace)::", ""))[:48]  # noqa: E731
    for gap, at, a_, b_ in sorted(big, reverse=True)[:6]:
        print(f"   gap {ms(gap):.3f} ms at {ms(at):.3f}: after {short(a_)} -> {short(b_)}")
    # per-kernel duration table for the step (name -> n, summed)
    agg = defaultdict(lambda: [0, 0])
    for k in st:
        n = re.sub(r"\(.*", "", k["name"].replace("(anonymous namespace)::", ""))[:70]
        agg[n][0] += 1
        agg[n][1] += k["e"] - k["s"]
    print("top kernels in the step (two-stream durations):")
    for n, (c, t) in sorted(agg.items(), key=lambda x: -x[1][1])[:20]:
        print(f"   {ms(t):7.3f} ms  n={c:4d}  {n}")


if __name__ == "__main__":
    main()
