#!/bin/bash
# round 5: persistent dwconv with LDS-only barriers (its next-sequence prefetch no longer drained): bit identity, C2
set -uo pipefail
O=gpurun_out/r05w; mkdir -p $O
timeout -k 10 500 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_switches.py tests/test_gpu_tsvad.py -k "dwconv_pp or group or tsvad" > $O/t.log 2>&1; r=$?
echo "tests rc=$r"; tail -3 $O/t.log
[ $r -eq 0 ] || exit 1
for i in 1 2 3; do
for g in pp pk; do
  unset SDIAR_NO_DWCONV_PP
  [ $g = pk ] && export SDIAR_NO_DWCONV_PP=1
  timeout -k 10 300 python3 bench.py --workload c2 --steps 20 --warmup 3 --no-cpu-baseline --no-c4-ref > $O/c2_$g$i.json 2> $O/c2_$g$i.err || { echo "c2 $g failed"; tail -5 $O/c2_$g$i.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['ms_per_step'])" $O/c2_$g$i.json
done
done
unset SDIAR_NO_DWCONV_PP
SDIAR_CAM_ONE_STREAM=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p -o run -- python3 bench.py --workload c2 --steps 2 --warmup 1 --no-cpu-baseline --no-kernel-timing --no-c4-ref > $O/p.log 2>&1 || { echo "prof failed"; exit 1; }
f=$(find $O/p -name '*kernel_stats.csv' | head -1); cp "$f" $O/kernel_stats.csv; rm -rf $O/p
python3 - "$O/kernel_stats.csv" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if 'dwconv' in r['Name'] or 'mha_block' in r['Name']:
        print(r['Name'][:60], r['Calls'], round(float(r['AverageNs']) / 1e3, 1), 'us')
PY
