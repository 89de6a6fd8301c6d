#!/bin/bash
# round 5: BiLSTM on 8 waves per workgroup (two waves per unit tile): bit identity, lstm status, C2 A/B, rocprof
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
O=gpurun_out/r05y; mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_switches.py -k "lstm" > $O/t.log 2>&1; r=$?
echo "tests rc=$r"; tail -4 $O/t.log
[ $r -eq 0 ] || exit 1
SDIAR_LSTM_WV=8 SDIAR_LSTM_MT=2 timeout -k 10 300 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_lstm_status.py > $O/ts.log 2>&1; r=$?
echo "status tests rc=$r"; tail -3 $O/ts.log
[ $r -eq 0 ] || exit 1
for m in 4 8; do
  SDIAR_LSTM_WV=$m SDIAR_CAM_ONE_STREAM=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p$m -o run -- python3 bench.py --workload c2 --steps 2 --warmup 1 --no-cpu-baseline --no-kernel-timing --no-c4-ref > $O/p$m.log 2>&1 || { echo "prof failed"; exit 1; }
  f=$(find $O/p$m -name '*kernel_stats.csv' | head -1); cp "$f" $O/kernel_stats_wv$m.csv; rm -rf $O/p$m
  python3 - "$O/kernel_stats_wv$m.csv" $m <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if 'lstm_group' in r['Name']:
        print('WV', sys.argv[2], r['Name'][:60], r['Calls'], round(float(r['AverageNs']) / 1e3, 1), 'us')
PY
done
for i in 1 2 3; do
for m in 4 8; do
  SDIAR_LSTM_WV=$m timeout -k 10 300 python3 bench.py --workload c2 --steps 20 --warmup 3 --no-cpu-baseline --no-c4-ref > $O/c2_wv$m$i.json 2> $O/c2_wv$m$i.err || { echo "c2 wv$m failed"; tail -5 $O/c2_wv$m$i.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['ms_per_step'])" $O/c2_wv$m$i.json
done
done
