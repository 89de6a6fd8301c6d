#!/bin/bash
# Per-workload evidence for DESIGN.md §6 (run on the GPU box from the repo root):
#   bench JSON line (5 timed steps; with CPU baseline + parity block when FULL=1) + rocprofv3 kernel-trace
#   stats of the same command (no CPU baseline).
#   [FULL=1] bash tools/profile_round.sh <outdir> c1 c3 c5 ...
set -euo pipefail
OUT=$1; shift
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for WL in "$@"; do
  # --no-c4-ref: the C2 line would otherwise also run the 60-min C4 meeting (c4_60min_ms), whose kernels
  # would land in C2's kernel-trace table; C4 is profiled as its own workload
  BENCH="bench.py --workload $WL --steps 5 --warmup 2 --no-cpu-baseline --no-c4-ref"
  if [ "${FULL:-0}" = 1 ]; then
    timeout -k 10 400 python3 bench.py --workload $WL --steps 5 --warmup 2 --no-c4-ref > "$OUT/bench_$WL.json" 2> "$OUT/bench_$WL.err"
  else
    timeout -k 10 240 python3 $BENCH > "$OUT/bench_$WL.json" 2> "$OUT/bench_$WL.err"
  fi
  # kernel stats on one stream (see tools/profile_c2.sh)
  SDIAR_CAM_ONE_STREAM=1 timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace_$WL" -o run -- python3 $BENCH \
    > "$OUT/trace_$WL.log" 2>&1
  cp "$(find "$OUT/trace_$WL" -name '*kernel_stats.csv' | head -1)" "$OUT/kernel_stats_$WL.csv"
  rm -rf "$OUT/trace_$WL"   # the full traces exceed what gpurun copies back
  echo "$WL ok"
done
