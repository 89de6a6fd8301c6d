#!/bin/bash
# round 5: C2 BiLSTM recurrence time vs rows per group (SDIAR_LSTM_MT), one-stream rocprof
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
O=gpurun_out/r05x; mkdir -p $O
for m in 2 3 4 6; do
  SDIAR_LSTM_MT=$m SDIAR_CAM_ONE_STREAM=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p$m -o run -- python3 bench.py --workload c2 --steps 2 --warmup 1 --no-cpu-baseline --no-kernel-timing --no-c4-ref > $O/p$m.log 2>&1 || { echo "prof failed"; exit 1; }
  f=$(find $O/p$m -name '*kernel_stats.csv' | head -1); cp "$f" $O/kernel_stats_$m.csv; rm -rf $O/p$m
  python3 - "$O/kernel_stats_$m.csv" $m <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if 'lstm_group' in r['Name']:
        print('MT', sys.argv[2], r['Name'][:55], r['Calls'], round(float(r['AverageNs']) / 1e3, 1), 'us')
PY
done
