#!/bin/bash
# round 5: the C2 BiLSTM input projection (90000 x 2048 x 1536, bf16 A, fp32 out): ring vs dma path vs hipBLASLt
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
O=gpurun_out/r05z; mkdir -p $O
GEMM_PROBE_TORCH=1 timeout -k 10 300 python3 tools/gemm_probe.py 90000x2048x1536 45056x2048x1536 > $O/probe.log 2>&1 || { echo probe failed; tail -5 $O/probe.log; exit 1; }
cat $O/probe.log
SDIAR_NO_RING_GEMM=1 timeout -k 10 300 python3 tools/gemm_probe.py 90000x2048x1536 > $O/probe_noring.log 2>&1 || { echo probe failed; tail -5 $O/probe_noring.log; exit 1; }
cat $O/probe_noring.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p -o run -- python3 tools/gemm_probe.py 90000x2048x1536 > $O/p.log 2>&1 || { echo "prof failed"; exit 1; }
f=$(find $O/p -name '*kernel_stats.csv' | head -1); cp "$f" $O/kernel_stats.csv; rm -rf $O/p
python3 - "$O/kernel_stats.csv" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    print(r['Name'][:90], r['Calls'], round(float(r['AverageNs']) / 1e3, 1), 'us')
PY
