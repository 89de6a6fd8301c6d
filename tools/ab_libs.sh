#!/bin/bash
# A/B/C... of several builds of libsdiar on ONE box: rounds x libs alternating bench lines (SDIAR_LIB), printing
# ms_per_step and the top kernels of each run.
#   bash tools/ab_libs.sh <outdir> <rounds> <workload> <lib.so> [<lib.so> ...]
set -uo pipefail
O=$1; R=$2; WL=$3; shift 3
mkdir -p "$O"
for i in $(seq 1 "$R"); do
  for lib in "$@"; do
    tag=$(basename "$lib" .so)
    SDIAR_LIB=$lib timeout -k 10 300 python3 bench.py --workload "$WL" --steps 10 --warmup 2 --no-cpu-baseline \
      --no-c4-ref > "$O/${tag}_$i.json" 2> "$O/${tag}_$i.err" || { echo "$tag failed"; tail -3 "$O/${tag}_$i.err"; exit 1; }
    python3 - "$tag" "$O/${tag}_$i.json" <<'PY'
import json, sys
d = json.loads([x for x in open(sys.argv[2]) if x.startswith("{")][-1])
top = sorted(d.get("kernels", {}).items(), key=lambda kv: -kv[1]["ms"])[:6]
print(sys.argv[1], d["ms_per_step"], " ".join(f"{k}={v['ms']:.3f}" for k, v in top), flush=True)
PY
  done
done
