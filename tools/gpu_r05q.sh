#!/bin/bash
# round 5: dwconv output tiled for the pw2 program: bit identity, C2 A/B
set -uo pipefail
O=gpurun_out/r05q; mkdir -p $O
timeout -k 10 500 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_switches.py tests/test_gpu_tsvad.py tests/test_gpu_mha_block.py tests/test_gpu_shard.py -k "rowmajor or two_stream or group or tsvad or mha or shard" > $O/t.log 2>&1; r=$?
echo "tests rc=$r"; tail -4 $O/t.log
[ $r -eq 0 ] || exit 1
for i in 1 2 3; do
for g in tiled rowdw; do
  unset SDIAR_RP_ROWMAJOR_DW
  [ $g = rowdw ] && export SDIAR_RP_ROWMAJOR_DW=1
  timeout -k 10 300 python3 bench.py --workload c2 --steps 20 --warmup 3 --no-cpu-baseline --no-c4-ref > $O/c2_$g$i.json 2> $O/c2_$g$i.err || { echo "c2 $g failed"; tail -5 $O/c2_$g$i.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['ms_per_step'])" $O/c2_$g$i.json
done
done
unset SDIAR_RP_ROWMAJOR_DW
for g in tiled rowdw; do
  [ $g = rowdw ] && export SDIAR_RP_ROWMAJOR_DW=1
  SDIAR_CAM_ONE_STREAM=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p$g -o run -- python3 bench.py --workload c2 --steps 2 --warmup 1 --no-cpu-baseline --no-kernel-timing --no-c4-ref > $O/p$g.log 2>&1 || { echo "prof failed"; exit 1; }
  f=$(find $O/p$g -name '*kernel_stats.csv' | head -1); cp "$f" $O/kernel_stats_$g.csv; rm -rf $O/p$g
  python3 - "$O/kernel_stats_$g.csv" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if 'rowprog' in r['Name'] or 'dwconv' in r['Name']:
        print(r['Name'][:50], r['Calls'], round(float(r['AverageNs']) / 1e3, 1), 'us')
PY
done
