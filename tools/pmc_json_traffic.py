"""Refresh profiles/pmc_traffic.json[workload] from a tools/pmc_csv.py summary (per-symbol HBM bytes per dispatch,
2 x FETCH_SIZE + WRITE_SIZE), grouped into bench.py's live-timer categories (tools/pmc_traffic.py CATEGORIES,
dispatch-weighted mean per category).

    python tools/pmc_json_traffic.py profiles/r05/pmc_c2.json c2 [profiles/pmc_traffic.json]
"""
import json
import os
import re
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_traffic import CATEGORIES  # noqa: E402


def main():
    src, wl = sys.argv[1], sys.argv[2]
    out = sys.argv[3] if len(sys.argv) > 3 else os.path.join(os.path.dirname(__file__), "..", "profiles", "pmc_traffic.json")
    per = json.load(open(src))
    cat = {}
    for name, rec in per.items():
        if not isinstance(rec, dict) or "hbm_bytes_per_dispatch" not in rec:
            continue
        for c, pat in CATEGORIES.items():
            if re.search(pat, name):
                s = cat.setdefault(c, [0.0, 0])
                s[0] += rec["hbm_bytes_per_dispatch"] * rec["dispatches"]
                s[1] += rec["dispatches"]
                break
    traffic = {c: int(round(v / n)) for c, (v, n) in cat.items() if n}
    data = json.load(open(out)) if os.path.exists(out) else {}
    data[wl] = traffic
    data.setdefault("_detail", {})[wl] = f"from {src} (round 5)"
    json.dump(data, open(out, "w"), indent=1, sort_keys=True)
    print(wl, traffic)


if __name__ == "__main__":
    main()
