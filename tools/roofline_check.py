"""Recompute every committed bench line's `roofline` from the rocprofv3 kernel-stats CSV committed beside it.

    python tools/roofline_check.py profiles/r04

For each bench_<wl>.json: the dominant kernel's rocprof launches and mean duration (kernel_stats_<wl>.csv,
symbols grouped by tools/pmc_traffic.py CATEGORIES), then
  - flop / byte roofs: achieved = flops (or algorithmic bytes) per launch / rocprof mean duration, frac = / peak;
  - the LSTM latency roof (C1 / C3): us per recurrence step = rocprof mean duration / steps per launch, frac =
    measured hand-off floor / that;
  - the C5 latency-mode line (c5s): the line's own model (pushes -> device ops x boundary + weight bytes) against
    its p50; rocprof gives the device time per push (sum of kernel time / pushes) beside it.
and prints them next to the line's live-timer values (HIP events on the launch stream)."""
import csv
import json
import os
import re
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_traffic import CATEGORIES  # noqa: E402


def line(path):
    return json.loads([x for x in open(path) if x.startswith("{")][-1])


def stats(path):
    with open(path) as fh:
        return list(csv.DictReader(fh))


def group(rows, cat):
    pat = re.compile(CATEGORIES[cat]) if cat in CATEGORIES else re.compile(re.escape(cat))
    calls, total = 0, 0.0
    for r in rows:
        if pat.search(r["Name"].replace("(anonymous namespace)::", "")):
            calls += int(r["Calls"])
            total += float(r["TotalDurationNs"])
    return calls, total


def main(d):
    out = []
    for f in sorted(os.listdir(d)):
        m = re.match(r"bench_(\w+)\.json$", f)
        if not m:
            continue
        wl = m.group(1)
        csvp = os.path.join(d, f"kernel_stats_{wl}.csv")
        if not os.path.exists(csvp):
            continue
        L = line(os.path.join(d, f))
        r = L.get("roofline")
        rows = stats(csvp)
        if not r:
            out.append(f"{wl}: NO roofline")
            continue
        if r.get("unit") == "us/push":
            tot = sum(float(x["TotalDurationNs"]) for x in rows)
            mdl = r.get("model", {})
            pushes = L["config"].get("pushes_per_step", 0) * (L["steps"] + L["warmup"])
            out.append(f"{wl}: latency model {r['peak']} us floor / p50 {r['achieved']} us = frac {r['frac']} "
                       f"(line); rocprof device time {tot / 1e3:.0f} us over the profiled run = "
                       f"{tot / 1e3 / max(pushes, 1):.1f} us of kernels per push ({pushes} pushes), "
                       f"device ops per push {mdl.get('device_ops_per_push')}, boundary {mdl.get('kernel_boundary_us')} us")
            continue
        calls, total = group(rows, r["kernel"])
        steps = L["steps"] + L["warmup"]
        per_launch_ns = total / calls if calls else float("nan")
        if r.get("unit") == "us/step":
            us = per_launch_ns / 1e3 / r["steps_per_launch"]
            # the floor probe (bench.py lstm_handoff_floor_us: one launch of 4000 exchange-only steps) is in the CSV too
            pc, pt = group(rows, "lstm_handoff_probe_kernel")
            floor = pt / pc / 1e3 / 4000 if pc else r["peak"]
            out.append(f"{wl}: {r['kernel']} rocprof {calls} launches, {per_launch_ns / 1e6:.4f} ms each -> "
                       f"{us:.4f} us/step vs floor {floor:.4f} (rocprof probe: {pc} launches of 4000 steps) -> frac "
                       f"{floor / us:.4f} (line: {r['achieved']} us/step vs {r['peak']}, frac {r['frac']})")
            continue
        if r["bound"] == "mfma":
            ach = r["flops_per_launch"] / (per_launch_ns * 1e-9) / 1e12
        else:
            ach = r["algorithmic_bytes_per_launch"] / (per_launch_ns * 1e-9) / 1e9
        # steps in the PROFILED run: its rocprof launches / the line's launches per step (the profiled command's
        # step count differs from the line's steps + warmup: the kernel-timer step, parity legs)
        per_step = r.get("launches") or 0
        prof_steps = f"{calls / per_step:.1f} steps of {per_step} launches" if per_step else f"line steps {steps}"
        out.append(f"{wl}: {r['kernel']} ({r['bound']}) rocprof {calls} launches over the profiled run "
                   f"({prof_steps}), {per_launch_ns / 1e6:.4f} ms each -> {ach:.1f} {r['unit']} "
                   f"= frac {ach / r['peak']:.4f} (line, live HIP-event timer: {r['avg_launch_ms']} ms, frac {r['frac']})")
    print("\n".join(out))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "profiles/r04")
