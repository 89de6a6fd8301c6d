#!/bin/bash
# round 5: schedule-switch bit identity (incl. the granule LSTM exchange), C1 granule A/B, host enqueue time
set -uo pipefail
O=gpurun_out/r05d; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_switches.py > $O/switches.log 2>&1; r=$?
echo "switches rc=$r"; tail -15 $O/switches.log
[ $r -eq 0 ] || [ $r -eq 1 ] || exit 1
for g in 0 1; do
  SDIAR_LSTM_GRANULE=$g timeout -k 10 300 python3 bench.py --workload c1 --steps 20 --warmup 3 --no-cpu-baseline --no-c4-ref > $O/c1_g$g.json 2> $O/c1_g$g.err || { echo "c1 g$g failed"; tail -5 $O/c1_g$g.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['ms_per_step'], d['value'])" $O/c1_g$g.json
done
timeout -k 10 300 python3 tools/enqueue_time.py c2 > $O/enqueue.log 2>&1; echo "enqueue rc=$?"; tail -3 $O/enqueue.log
