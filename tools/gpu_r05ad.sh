#!/bin/bash
# round 5: EEND STFT log-mel (whole recording) with the mel runs in LDS and workgroups walking frame groups vs one
# workgroup per 8 frames (SDIAR_STFT_PER_GROUP=1): bit identity, eda / stream tests, rocprof, C1 / C5 A/B
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
O=gpurun_out/r05ad; mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_eda.py tests/test_gpu_fseend_stream.py tests/test_gpu_ops.py -k "feature or eda or stream or fbank" > $O/t.log 2>&1; r=$?
echo "tests rc=$r"; tail -3 $O/t.log
[ $r -eq 0 ] || exit 1
timeout -k 10 120 python3 tools/fbank_hash.py > $O/hash_walk.log 2>&1 || { echo hash failed; tail -3 $O/hash_walk.log; exit 1; }
SDIAR_STFT_PER_GROUP=1 SDIAR_FBANK_PER_GROUP=1 timeout -k 10 120 python3 tools/fbank_hash.py > $O/hash_group.log 2>&1 || { echo hash failed; exit 1; }
cat $O/hash_walk.log $O/hash_group.log | grep "fbank\|eend"
for w in c1 c5; do
for m in walk group; do
  unset SDIAR_STFT_PER_GROUP; [ $m = group ] && export SDIAR_STFT_PER_GROUP=1
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p$w$m -o run -- python3 bench.py --workload $w --steps 2 --warmup 1 --no-cpu-baseline --no-kernel-timing --no-c4-ref > $O/p$w$m.log 2>&1 || { echo "prof failed"; exit 1; }
  f=$(find $O/p$w$m -name '*kernel_stats.csv' | head -1); cp "$f" $O/kernel_stats_$w$m.csv; rm -rf $O/p$w$m
  python3 - "$O/kernel_stats_$w$m.csv" $w$m <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if 'stft' in r['Name']:
        print(sys.argv[2], r['Name'][:60], r['Calls'], round(float(r['AverageNs']) / 1e3, 1), 'us')
PY
done
done
unset SDIAR_STFT_PER_GROUP
for i in 1 2; do
for m in walk group; do
  unset SDIAR_STFT_PER_GROUP; [ $m = group ] && export SDIAR_STFT_PER_GROUP=1
  for w in c1 c5; do
    timeout -k 10 300 python3 bench.py --workload $w --steps 10 --warmup 2 --no-cpu-baseline --no-c4-ref > $O/${w}_$m$i.json 2> $O/${w}_$m$i.err || { echo "$w $m failed"; tail -5 $O/${w}_$m$i.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['ms_per_step'])" $O/${w}_$m$i.json
  done
done
done
