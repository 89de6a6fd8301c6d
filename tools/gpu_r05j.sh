#!/bin/bash
# round 5: mha_block layouts 0 / 3 / 7 (4-slot ring) on C2 + layout equality test
set -uo pipefail
O=gpurun_out/r05j; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_mha_block.py > $O/mha_tests.log 2>&1; r=$?
echo "mha tests rc=$r"; tail -4 $O/mha_tests.log
[ $r -eq 0 ] || exit 1
for i in 1 2 3; do
for v in 0 3 7; do
  SDIAR_MHA_VARIANT=$v timeout -k 10 300 python3 bench.py --workload c2 --steps 20 --warmup 3 --no-cpu-baseline --no-c4-ref > $O/c2_v$v$i.json 2> $O/c2_v$v$i.err || { echo "c2 v$v failed"; tail -5 $O/c2_v$v$i.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['ms_per_step'])" $O/c2_v$v$i.json
done
done
for v in 0 3 7; do
  SDIAR_MHA_VARIANT=$v SDIAR_CAM_ONE_STREAM=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p$v -o run -- python3 bench.py --workload c2 --steps 2 --warmup 1 --no-cpu-baseline --no-kernel-timing --no-c4-ref > $O/p$v.log 2>&1 || { echo "prof failed"; exit 1; }
  f=$(find $O/p$v -name '*kernel_stats.csv' | head -1); grep mha_block "$f" | cut -d, -f1-4; rm -rf $O/p$v
done
