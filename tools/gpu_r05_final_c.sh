#!/bin/bash
# Round-5 evidence, part C (after the late C2 / C5 changes): C5 line + kernel stats, the C2 and C5 PMC passes,
# the two-stream C2 trace
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
O=gpurun_out/r05
mkdir -p $O
FULL=1 bash tools/profile_round.sh $O c5 || { echo "profile_round failed"; exit 1; }
WL=c2 bash tools/profile_c2.sh $O/pmc_c2 || { echo "pmc failed"; exit 1; }
python3 tools/pmc_csv.py $O/pmc_c2 7 $O/pmc_c2.json > $O/pmc_c2.txt || true
cp $(find $O/pmc_c2/trace -name '*kernel_stats.csv' | head -1) $O/pmc_c2_kernel_stats.csv
rm -rf $O/pmc_c2/trace $O/pmc_c2/fetch $O/pmc_c2/write $O/pmc_c2/mfma
WL=c5 MFMA_PMC="SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_WAVE_CYCLES SQ_WAIT_ANY GRBM_GUI_ACTIVE" bash tools/profile_c2.sh $O/pmc_c5 || { echo "pmc c5 failed"; exit 1; }
python3 tools/pmc_csv.py $O/pmc_c5 3 $O/pmc_c5.json > $O/pmc_c5.txt || true
rm -rf $O/pmc_c5/trace $O/pmc_c5/fetch $O/pmc_c5/write $O/pmc_c5/mfma
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tl -o run -- python3 bench.py --workload c2 --steps 3 --warmup 1 --no-cpu-baseline --no-kernel-timing --no-c4-ref > $O/tl.log 2>&1 || { echo "trace failed"; exit 1; }
f=$(find $O/tl -name '*kernel_trace.csv' | head -1); python3 tools/stream_timeline.py "$f" --step 2 > $O/timeline_c2.txt; gzip -c "$f" > $O/kernel_trace_c2_2stream.csv.gz; rm -rf $O/tl
echo done
