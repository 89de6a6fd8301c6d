"""Per-kernel duration summary of a rocprofv3 (rocpd) .db: calls, total/avg/min/max us, share.
Usage: python tools/kstats_db.py run_results.db [name-filter] [--last N]  (last N dispatches only)"""
import collections
import sqlite3
import sys

db = sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 and not sys.argv[2].startswith("--") else ""
last = int(sys.argv[sys.argv.index("--last") + 1]) if "--last" in sys.argv else 0
c = sqlite3.connect(db)
tabs = [r[0] for r in c.execute("select name from sqlite_master where type='table'")]
sfx = [t for t in tabs if t.startswith("rocpd_kernel_dispatch")][0][len("rocpd_kernel_dispatch"):]
ks = dict(c.execute(f"select id, kernel_name from rocpd_info_kernel_symbol{sfx}"))
rows = list(c.execute(f"select kernel_id, start, end from rocpd_kernel_dispatch{sfx} order by start"))
if last:
    rows = rows[-last:]
agg = collections.defaultdict(list)
for kid, st, en in rows:
    kn = ks.get(kid, str(kid))
    if flt in kn:
        agg[kn].append((en - st) / 1e3)
tot = sum(sum(v) for v in agg.values())
print(f"{'kernel':80s} {'calls':>7s} {'total_us':>10s} {'avg_us':>8s} {'min':>7s} {'max':>8s} {'share':>6s}")
for kn, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
    print(f"{kn[:80]:80s} {len(v):7d} {sum(v):10.1f} {sum(v)/len(v):8.2f} {min(v):7.2f} {max(v):8.2f} {sum(v)/tot:6.3f}")
print(f"total kernel time {tot:.1f} us over {sum(len(v) for v in agg.values())} dispatches")
