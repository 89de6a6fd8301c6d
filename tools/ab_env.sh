#!/bin/bash
# A/B of one env switch on one box: bash ab_env.sh VAR rounds workload
set -euo pipefail
V=$1; R=${2:-2}; WL=${3:-c2}
mkdir -p gpurun_out/ab
for i in $(seq 1 "$R"); do
  for tag in A B; do
    if [ "$tag" = B ]; then export $V=1; else unset $V; fi
    timeout -k 10 300 python3 bench.py --workload "$WL" --steps 5 --warmup 2 --no-cpu-baseline --no-c4-ref > "gpurun_out/ab/${tag}_$i.json" 2> "gpurun_out/ab/${tag}_$i.err"
    python3 - "$tag" "gpurun_out/ab/${tag}_$i.json" <<'PY'
import json, sys
d = json.loads([x for x in open(sys.argv[2]) if x.startswith("{")][-1])
top = sorted(d.get("kernels", {}).items(), key=lambda kv: -kv[1]["ms"])[:10]
print(sys.argv[1], d["ms_per_step"], " ".join(f"{k}={v['ms']:.3f}" for k, v in top), flush=True)
PY
  done
done
