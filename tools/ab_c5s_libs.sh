#!/bin/bash
# c5s p50 A/B over builds and switches on ONE box, alternating:
#   bash tools/ab_c5s_libs.sh rounds label=lib[,ENV=1] ...
set -euo pipefail
R=$1; shift
mkdir -p gpurun_out/ab
for i in $(seq 1 "$R"); do
  for spec in "$@"; do
    tag=${spec%%=*}; rest=${spec#*=}; lib=${rest%%,*}; envs=""
    [ "$rest" != "$lib" ] && envs=${rest#*,}
    out="gpurun_out/ab/c5s_${tag}_$i.json"
    env SDIAR_LIB="$lib" $envs timeout -k 10 300 python3 bench.py --workload c5s --steps 2 --warmup 1 \
      --no-cpu-baseline > "$out" 2> "${out%.json}.err"
    python3 - "$tag" "$out" <<'PY'
import json, sys
d = json.loads([x for x in open(sys.argv[2]) if x.startswith("{")][-1])
lat = d["latency_ms"]
print(sys.argv[1], "p50", lat["p50"], "p90", lat["p90"], "mean", lat["mean"], "floor", d["roofline"]["peak"], flush=True)
PY
  done
done
