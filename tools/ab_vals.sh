#!/bin/bash
# A/B of one env variable over several values on one box: bash ab_vals.sh VAR rounds workload v1 v2 ...
# (value "-" = unset).  Prints ms per step and the top kernels per run.
set -euo pipefail
V=$1; R=$2; WL=$3; shift 3
mkdir -p gpurun_out/ab
for i in $(seq 1 "$R"); do
  for val in "$@"; do
    if [ "$val" = "-" ]; then unset "$V"; else export "$V"="$val"; fi
    out="gpurun_out/ab/${V}_${val}_$i.json"
    timeout -k 10 300 python3 bench.py --workload "$WL" --steps 5 --warmup 2 --no-cpu-baseline --no-c4-ref > "$out" 2> "${out%.json}.err"
    python3 - "$V=$val" "$out" <<'PY'
import json, sys
d = json.loads([x for x in open(sys.argv[2]) if x.startswith("{")][-1])
top = sorted(d.get("kernels", {}).items(), key=lambda kv: -kv[1]["ms"])[:12]
print(sys.argv[1], d["ms_per_step"], " ".join(f"{k}={v['ms']:.3f}" for k, v in top), flush=True)
PY
  done
done
