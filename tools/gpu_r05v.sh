#!/bin/bash
# round 5: mha_block piece / head barriers without the release fence's vmcnt(0): tests, C2 A/B, phase probe
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
O=gpurun_out/r05v; mkdir -p $O
timeout -k 10 500 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_mha_block.py tests/test_gpu_tsvad.py tests/test_gpu_switches.py -k "mha or tsvad or group or schedule" > $O/t.log 2>&1; r=$?
echo "tests rc=$r"; tail -3 $O/t.log
[ $r -eq 0 ] || exit 1
for i in 1 2 3; do
for g in light full; do
  unset SDIAR_MHA_FULL_BARRIER
  [ $g = full ] && export SDIAR_MHA_FULL_BARRIER=1
  timeout -k 10 300 python3 bench.py --workload c2 --steps 20 --warmup 3 --no-cpu-baseline --no-c4-ref > $O/c2_$g$i.json 2> $O/c2_$g$i.err || { echo "c2 $g failed"; tail -5 $O/c2_$g$i.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['ms_per_step'])" $O/c2_$g$i.json
done
done
unset SDIAR_MHA_FULL_BARRIER
for g in light full; do
  [ $g = full ] && export SDIAR_MHA_FULL_BARRIER=1
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p$g -o run -- python3 tools/mha_phase.py > $O/p$g.log 2>&1 || { echo "prof failed"; tail -5 $O/p$g.log; exit 1; }
  f=$(find $O/p$g -name '*kernel_stats.csv' | head -1); cp "$f" $O/kernel_stats_$g.csv; rm -rf $O/p$g
  python3 - "$O/kernel_stats_$g.csv" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    n = r['Name']
    if 'mha_block' in n:
        i = n.find('mha_block_kernel'); print(sys.argv[1][-20:], n[i:i + 36], r['Calls'], round(float(r['AverageNs']) / 1e3, 1), 'us')
PY
done
