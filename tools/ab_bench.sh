#!/bin/bash
# A/B of two builds of libsdiar on ONE box (boxes differ by a few % in clock): alternating C2 bench runs
# with SDIAR_LIB pointing at each build; prints ms_per_step and the top kernels per run.
#   bash tools/ab_bench.sh <libA.so> <libB.so> [rounds] [workload]
set -euo pipefail
A=$1; B=$2; R=${3:-2}; WL=${4:-c2}
mkdir -p gpurun_out/ab
for i in $(seq 1 "$R"); do
  for tag in A B; do
    lib=$A; [ "$tag" = B ] && lib=$B
    SDIAR_LIB=$lib timeout -k 10 300 python3 bench.py --workload "$WL" --steps 5 --warmup 2 --no-cpu-baseline \
      --no-c4-ref > "gpurun_out/ab/${tag}_$i.json" 2> "gpurun_out/ab/${tag}_$i.err"
    python3 - "$tag" "gpurun_out/ab/${tag}_$i.json" <<'PY'
import json, sys
d = json.loads([x for x in open(sys.argv[2]) if x.startswith("{")][-1])
top = sorted(d.get("kernels", {}).items(), key=lambda kv: -kv[1]["ms"])[:8]
print(sys.argv[1], d["ms_per_step"], " ".join(f"{k}={v['ms']:.3f}" for k, v in top), flush=True)
PY
  done
done
