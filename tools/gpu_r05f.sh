#!/bin/bash
# round 5: second-slice stream priority / start A/B on C2
set -uo pipefail
O=gpurun_out/r05f; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_switches.py -k "side_sched" > $O/switches.log 2>&1; r=$?
echo "switches rc=$r"; tail -4 $O/switches.log
[ $r -eq 0 ] || exit 1
for i in 1 2; do
for g in base tail prio after both; do
  unset SDIAR_SIDE_PRIO SDIAR_SIDE_AFTER_CAM SDIAR_LSTM_GATES_TAIL
  case $g in tail) export SDIAR_LSTM_GATES_TAIL=1;; prio) export SDIAR_SIDE_PRIO=1;; after) export SDIAR_SIDE_AFTER_CAM=1;; both) export SDIAR_SIDE_PRIO=1 SDIAR_SIDE_AFTER_CAM=1;; esac
  timeout -k 10 300 python3 bench.py --workload c2 --steps 20 --warmup 3 --no-cpu-baseline --no-c4-ref > $O/c2_$g$i.json 2> $O/c2_$g$i.err || { echo "c2 $g failed"; tail -5 $O/c2_$g$i.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['ms_per_step'], d['value'])" $O/c2_$g$i.json
done
done
unset SDIAR_SIDE_PRIO SDIAR_SIDE_AFTER_CAM
for g in prio both; do
  case $g in prio) export SDIAR_SIDE_PRIO=1;; both) export SDIAR_SIDE_PRIO=1 SDIAR_SIDE_AFTER_CAM=1;; esac
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tl -o run -- python3 bench.py --workload c2 --steps 3 --warmup 1 --no-cpu-baseline --no-kernel-timing --no-c4-ref > $O/tl.log 2>&1 || { echo "trace failed"; exit 1; }
  f=$(find $O/tl -name '*kernel_trace.csv' | head -1); python3 tools/stream_timeline.py "$f" --step 2 > $O/timeline_c2_$g.txt; rm -rf $O/tl
  head -24 $O/timeline_c2_$g.txt
done
