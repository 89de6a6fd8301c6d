#!/bin/bash
# C4 (60-min meeting) step time per device batch (windows per launch), on one box: bash c4_batch_sweep.sh 640 1200 ...
set -euo pipefail
mkdir -p gpurun_out/c4b
for db in "$@"; do
  timeout -k 10 300 python3 bench.py --workload c4 --steps 3 --warmup 1 --no-cpu-baseline --no-c4-ref --device-batch "$db" \
    > "gpurun_out/c4b/db_$db.json" 2> "gpurun_out/c4b/db_$db.err"
  python3 - "$db" "gpurun_out/c4b/db_$db.json" <<'PY'
import json, sys
d = json.loads([x for x in open(sys.argv[2]) if x.startswith("{")][-1])
top = sorted(d.get("kernels", {}).items(), key=lambda kv: -kv[1]["ms"])[:5]
print("db", sys.argv[1], d["ms_per_step"], " ".join(f"{k}={v['ms']:.2f}" for k, v in top), flush=True)
PY
done
