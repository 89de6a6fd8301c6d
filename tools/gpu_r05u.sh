#!/bin/bash
# round 5: mha_block phase probe (C2 shape) under rocprofv3
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
O=gpurun_out/r05u; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p -o run -- python3 tools/mha_phase.py > $O/p.log 2>&1 || { echo "prof failed"; tail -5 $O/p.log; exit 1; }
f=$(find $O/p -name '*kernel_stats.csv' | head -1); cp "$f" $O/kernel_stats.csv; rm -rf $O/p
python3 - "$O/kernel_stats.csv" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if 'mha_block' in r['Name']:
        print(r['Name'].split('(')[0][-50:], r['Calls'], round(float(r['AverageNs']) / 1e3, 1), 'us')
PY
