#!/bin/bash
# rocprofv3 evidence for the bench line (run on the GPU box from the repo root):
#   1. kernel trace + stats of the C2 bench            -> $OUT/trace/*kernel_stats.csv
#   2. PMC pass FETCH_SIZE (own run)                    -> $OUT/fetch
#   3. PMC pass WRITE_SIZE (own run)                    -> $OUT/write
#   4. PMC pass MFMA / busy counters (own run)          -> $OUT/mfma   (counters from $MFMA_PMC)
# Every pass is a separate process with its own time limit; a failing pass ends the script.
set -euo pipefail
OUT=${1:-gpurun_out/prof}
WL=${WL:-c2}
MFMA_PMC=${MFMA_PMC:-"SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_VALU_MFMA_BF16 GRBM_GUI_ACTIVE"}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
BENCH="bench.py --workload $WL --steps 2 --warmup 1 --no-cpu-baseline --no-kernel-timing --no-c4-ref"
# per-kernel evidence on ONE stream (the TS-VAD forward otherwise runs the CAM++ trunk and the conformer stack
# as two concurrent window slices, whose kernels share the GPU): matches bench.py's single-stream profiled step
export SDIAR_CAM_ONE_STREAM=1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- python3 $BENCH > "$OUT/trace.log" 2>&1
echo "trace ok"
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run -- python3 $BENCH > "$OUT/fetch.log" 2>&1
echo "fetch ok"
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o run -- python3 $BENCH > "$OUT/write.log" 2>&1
echo "write ok"
timeout -s KILL 300 rocprofv3 --pmc $MFMA_PMC --output-format csv -d "$OUT/mfma" -o run -- python3 $BENCH > "$OUT/mfma.log" 2>&1
echo "mfma ok"
