"""Summarise a rocprofv3 .db (PMC run): per kernel name, mean of each counter and duration."""
import sqlite3, sys, collections
db = sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 else ""
c = sqlite3.connect(db)
tabs = [r[0] for r in c.execute("select name from sqlite_master where type='table'")]
sfx = [t for t in tabs if t.startswith("rocpd_pmc_event")][0][len("rocpd_pmc_event"):]
T = lambda n: f"rocpd_{n}{sfx}"
names = dict(c.execute(f"select id, name from {T('info_pmc')}"))
ks = dict(c.execute(f"select id, kernel_name from {T('info_kernel_symbol')}"))
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for kid, ev, st, en in c.execute(f"select kernel_id, event_id, start, end from {T('kernel_dispatch')}"):
    kn = ks.get(kid, str(kid))
    if flt not in kn: continue
    agg[kn]["dur_us"].append((en - st) / 1e3)
    for pid, val in c.execute(f"select pmc_id, value from {T('pmc_event')} where event_id=?", (ev,)):
        agg[kn][names[pid]].append(val)
for kn, d in agg.items():
    print(kn[:110])
    for k, v in d.items():
        print(f"   {k:28s} n={len(v):4d} mean={sum(v)/len(v):.4g}")
