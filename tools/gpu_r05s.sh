#!/bin/bash
# round 5: window CMN load batching (bit-identical), granule LSTM exchange on C2's 152-workgroup BiLSTM (A/B)
set -uo pipefail
O=gpurun_out/r05s; mkdir -p $O
timeout -k 10 500 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_ops.py tests/test_gpu_tsvad.py tests/test_gpu_shard.py -k "cmn or fbank or tsvad or shard" > $O/t.log 2>&1; r=$?
echo "tests rc=$r"; tail -3 $O/t.log
[ $r -eq 0 ] || exit 1
for i in 1 2 3; do
for g in counter granule; do
  unset SDIAR_LSTM_GRANULE
  [ $g = granule ] && export SDIAR_LSTM_GRANULE=1
  timeout -k 10 300 python3 bench.py --workload c2 --steps 20 --warmup 3 --no-cpu-baseline --no-c4-ref > $O/c2_$g$i.json 2> $O/c2_$g$i.err || { echo "c2 $g failed"; tail -5 $O/c2_$g$i.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['ms_per_step'])" $O/c2_$g$i.json
done
done
unset SDIAR_LSTM_GRANULE
SDIAR_CAM_ONE_STREAM=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p -o run -- python3 bench.py --workload c2 --steps 2 --warmup 1 --no-cpu-baseline --no-kernel-timing --no-c4-ref > $O/p.log 2>&1 || { echo "prof failed"; exit 1; }
f=$(find $O/p -name '*kernel_stats.csv' | head -1); cp "$f" $O/kernel_stats.csv; rm -rf $O/p
python3 - "$O/kernel_stats.csv" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if 'window_cmn' in r['Name'] or 'lstm' in r['Name'] or 'fbank' in r['Name']:
        print(r['Name'][:60], r['Calls'], round(float(r['AverageNs']) / 1e3, 1), 'us')
PY
