#!/bin/bash
# rocprofv3 kernel stats of a 1-minute c5s stream, fused slot block on and off: bash tools/prof_c5s.sh OUT
set -euo pipefail
OUT=${1:-gpurun_out/c5sprof}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for tag in fused unfused; do
  if [ "$tag" = unfused ]; then export SDIAR_NO_SLOT_BLOCK=1; else unset SDIAR_NO_SLOT_BLOCK; fi
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/$tag" -o run -- \
    python3 bench.py --workload c5s --steps 1 --warmup 0 --no-cpu-baseline --minutes 1 > "$OUT/$tag.json" 2> "$OUT/$tag.err"
  f=$(find "$OUT/$tag" -name '*kernel_stats.csv' | head -1)
  cp "$f" "$OUT/kernel_stats_$tag.csv"
done
