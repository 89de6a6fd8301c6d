#!/bin/bash
# round 5: the whole-recording 512-point EEND STFT as three register FFT passes: hashes (8 kHz / 256-point
# must be unchanged), eda / feature / stream tests, rocprof C1 / C3, C1 / C3 lines
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
O=gpurun_out/r05af; mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_eda.py tests/test_gpu_fseend_stream.py tests/test_gpu_real_speech.py > $O/t.log 2>&1; r=$?
echo "tests rc=$r"; tail -3 $O/t.log
[ $r -eq 0 ] || exit 1
timeout -k 10 120 python3 tools/fbank_hash.py > $O/hash.log 2>&1 || { echo hash failed; tail -3 $O/hash.log; exit 1; }
grep eend $O/hash.log
for w in c1 c3; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p$w -o run -- python3 bench.py --workload $w --steps 2 --warmup 1 --no-cpu-baseline --no-kernel-timing --no-c4-ref > $O/p$w.log 2>&1 || { echo "prof failed"; exit 1; }
  f=$(find $O/p$w -name '*kernel_stats.csv' | head -1); cp "$f" $O/kernel_stats_$w.csv; rm -rf $O/p$w
  python3 - "$O/kernel_stats_$w.csv" $w <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if 'stft' in r['Name']:
        print(sys.argv[2], r['Name'][:60], r['Calls'], round(float(r['AverageNs']) / 1e3, 1), 'us')
PY
done
for i in 1 2; do
  for w in c1 c3; do
    timeout -k 10 300 python3 bench.py --workload $w --steps 10 --warmup 2 --no-cpu-baseline --no-c4-ref > $O/${w}_$i.json 2> $O/${w}_$i.err || { echo "$w failed"; tail -5 $O/${w}_$i.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['ms_per_step'])" $O/${w}_$i.json
  done
done
