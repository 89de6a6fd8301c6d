#!/bin/bash
# round 5: Kaldi fbank with per-workgroup tables (mel runs in LDS) built once, workgroups walking frame groups, vs one workgroup per
# 8-frame group: bit identity, fbank / tsvad tests, rocprof, C2 A/B
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
O=gpurun_out/${OUT:-r05ab}; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_ops.py tests/test_gpu_tsvad.py -k "fbank or cmn or tsvad" > $O/t.log 2>&1; r=$?
echo "tests rc=$r"; tail -3 $O/t.log
[ $r -eq 0 ] || exit 1
timeout -k 10 120 python3 tools/fbank_hash.py > $O/hash_walk.log 2>&1 || { echo hash failed; tail -3 $O/hash_walk.log; exit 1; }
SDIAR_FBANK_PER_GROUP=1 timeout -k 10 120 python3 tools/fbank_hash.py > $O/hash_group.log 2>&1 || { echo hash failed; exit 1; }
grep fbank $O/hash_walk.log $O/hash_group.log
for m in walk group; do
  unset SDIAR_FBANK_PER_GROUP; [ $m = group ] && export SDIAR_FBANK_PER_GROUP=1
  SDIAR_CAM_ONE_STREAM=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p$m -o run -- python3 bench.py --workload c2 --steps 2 --warmup 1 --no-cpu-baseline --no-kernel-timing --no-c4-ref > $O/p$m.log 2>&1 || { echo "prof failed"; exit 1; }
  f=$(find $O/p$m -name '*kernel_stats.csv' | head -1); cp "$f" $O/kernel_stats_$m.csv; rm -rf $O/p$m
  python3 - "$O/kernel_stats_$m.csv" $m <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if 'fbank' in r['Name'] or 'window_cmn' in r['Name']:
        print(sys.argv[2], r['Name'][:60], r['Calls'], round(float(r['AverageNs']) / 1e3, 1), 'us')
PY
done
unset SDIAR_FBANK_PER_GROUP
for i in 1 2 3; do
for m in walk group; do
  unset SDIAR_FBANK_PER_GROUP; [ $m = group ] && export SDIAR_FBANK_PER_GROUP=1
  timeout -k 10 300 python3 bench.py --workload c2 --steps 20 --warmup 3 --no-cpu-baseline --no-c4-ref > $O/c2_$m$i.json 2> $O/c2_$m$i.err || { echo "c2 $m failed"; tail -5 $O/c2_$m$i.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['ms_per_step'])" $O/c2_$m$i.json
done
done
