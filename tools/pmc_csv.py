"""Per-kernel summary of rocprofv3 CSV passes made by tools/profile_c2.sh.

    python tools/pmc_csv.py <dir with trace/ fetch/ write/ mfma/> [steps] [out.json]

For every kernel symbol (argument list dropped): dispatches per step, mean duration (kernel
trace), HBM bytes per dispatch = 2 x FETCH_SIZE + WRITE_SIZE (KiB units; gfx950 tallies a 128-B
streaming read request as 64 B, MI355X_MICROARCH.md "HBM"), MFMA utilisation =
SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE x 1024 SIMDs) and MFMA flops from
SQ_INSTS_VALU_MFMA_MOPS_BF16 x 512, SQ_WAIT_ANY / SQ_WAVE_CYCLES (share of wave cycles parked on
s_waitcnt / barrier).  Also groups them by the live-timer family bench.py reports
(tools/pmc_traffic.py CATEGORIES) and writes profiles/pmc_traffic.json-style traffic.
"""
import collections
import csv
import glob
import json
import os
import re
import sys

csv.field_size_limit(1 << 30)


def base(name):
    n = name.replace("(anonymous namespace)::", "").replace("void ", "")
    depth, out = 0, []
    for ch in n:
        if ch == "(" and depth == 0:
            break
        depth += ch == "<"
        depth -= ch == ">"
        out.append(ch)
    return "".join(out).strip()


def read_pmc(d):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    n = collections.Counter()
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = base(r["Kernel_Name"])
            agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
            n[(k, r["Counter_Name"])] += 1
    return agg, n


def read_trace(d):
    dur = collections.defaultdict(list)
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            dur[base(r["Kernel_Name"])].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    return dur


def main():
    root = sys.argv[1]
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 4     # warmup + steps + e2e runs of the traced bench
    dur = read_trace(os.path.join(root, "trace"))
    fetch, nf = read_pmc(os.path.join(root, "fetch"))
    write, nw = read_pmc(os.path.join(root, "write"))
    mfma, nm = read_pmc(os.path.join(root, "mfma"))
    rows = {}
    for k, ds in dur.items():
        calls = len(ds)
        r = {"dispatches": calls, "avg_us": round(sum(ds) / calls, 2), "total_ms": round(sum(ds) / 1e3, 3)}
        if k in fetch:
            c = nf[(k, "FETCH_SIZE")]
            r["hbm_bytes_per_dispatch"] = round((2 * fetch[k]["FETCH_SIZE"] / c +
                                                 write[k].get("WRITE_SIZE", 0.0) / max(nw[(k, "WRITE_SIZE")], 1)) * 1024)
            r["achieved_hbm_gbs"] = round(r["hbm_bytes_per_dispatch"] / (r["avg_us"] * 1e3), 1)
        if k in mfma:
            m = mfma[k]
            g = m.get("GRBM_GUI_ACTIVE", 0.0)
            r["mfma_util_pct"] = round(100 * m.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / (g * 1024), 2) if g else None
            c = nm[(k, "SQ_INSTS_VALU_MFMA_MOPS_BF16")] or 1
            r["mfma_bf16_flops_per_dispatch"] = m.get("SQ_INSTS_VALU_MFMA_MOPS_BF16", 0.0) * 512 / c
            if r["mfma_bf16_flops_per_dispatch"]:
                r["achieved_bf16_tflops"] = round(r["mfma_bf16_flops_per_dispatch"] / (r["avg_us"] * 1e-6) / 1e12, 1)
            wc = m.get("SQ_WAVE_CYCLES", 0.0)
            r["wait_any_share"] = round(m.get("SQ_WAIT_ANY", 0.0) / wc, 3) if wc else None
        rows[k] = r
    tot = sum(r["total_ms"] for r in rows.values())
    for r in rows.values():
        r["share"] = round(r["total_ms"] / tot, 4)
    out = dict(sorted(rows.items(), key=lambda kv: -kv[1]["total_ms"]))
    dst = sys.argv[3] if len(sys.argv) > 3 else os.path.join(root, "kernels.json")
    json.dump(out, open(dst, "w"), indent=1)
    for k, r in list(out.items())[:20]:
        print(f"{k[:58]:58s} {r['share']*100:5.1f}% {r['avg_us']:8.1f}us n={r['dispatches']:4d} "
              f"hbm={r.get('achieved_hbm_gbs', '-')} mfma%={r.get('mfma_util_pct', '-')} "
              f"tf={r.get('achieved_bf16_tflops', '-')} wait={r.get('wait_any_share', '-')}")


if __name__ == "__main__":
    main()
