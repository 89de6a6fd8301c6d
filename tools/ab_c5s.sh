#!/bin/bash
# c5s p50 with the fused slot block on / off (one box): bash tools/ab_c5s.sh rounds
set -euo pipefail
R=${1:-1}
mkdir -p gpurun_out/ab
for i in $(seq 1 "$R"); do
  for tag in fused unfused; do
    if [ "$tag" = unfused ]; then export SDIAR_NO_SLOT_BLOCK=1; else unset SDIAR_NO_SLOT_BLOCK; fi
    out="gpurun_out/ab/c5s_${tag}_$i.json"
    timeout -k 10 300 python3 bench.py --workload c5s --steps 2 --warmup 1 --no-cpu-baseline > "$out" 2> "${out%.json}.err"
    python3 - "$tag" "$out" <<'PY'
import json, sys
d = json.loads([x for x in open(sys.argv[2]) if x.startswith("{")][-1])
lat = d.get("latency_ms", d.get("latency", {}))
print(sys.argv[1], d["ms_per_step"], json.dumps(lat)[:200], json.dumps(d.get("roofline"))[:300], flush=True)
PY
  done
done
