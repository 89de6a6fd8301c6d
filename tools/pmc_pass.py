"""Sum rocprofv3 --pmc counters per kernel (argument list dropped) over a counter_collection run.

    python tools/pmc_pass.py <rocprofv3 -d dir> [kernel-substring ...]
"""
import collections
import csv
import glob
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_csv import base  # noqa: E402

csv.field_size_limit(1 << 30)
d = sys.argv[1]
filt = sys.argv[2:]
agg = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(set)
for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        k = base(r["Kernel_Name"])
        if filt and not any(s in k for s in filt):
            continue
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[k].add(r.get("Dispatch_Id", r.get("Correlation_Id", "")))
for k, c in sorted(agg.items()):
    n = max(1, len(disp[k]))
    print(k, f"dispatches={n}")
    wc = c.get("SQ_WAVE_CYCLES", 0.0)
    for name, v in sorted(c.items()):
        extra = f"  ({v / wc:.3f} of wave cycles)" if wc and name.startswith("SQ_WAIT") or name == "SQ_ACTIVE_INST_ANY" and wc else ""
        print(f"  {name:32s} {v / n:16.4g} per dispatch{extra}")
