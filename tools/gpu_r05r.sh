#!/bin/bash
# round 5: LSTM output rows stored after the h hand-off: tests, C1 / C2 A/B
set -uo pipefail
O=gpurun_out/r05r; mkdir -p $O
timeout -k 10 500 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_eda.py tests/test_gpu_lstm_status.py tests/test_gpu_tsvad.py tests/test_gpu_switches.py -k "eda or lstm or tsvad or group or schedule" > $O/t.log 2>&1; r=$?
echo "tests rc=$r"; tail -3 $O/t.log
[ $r -eq 0 ] || exit 1
for i in 1 2 3; do
for g in late early; do
  unset SDIAR_LSTM_OUT_EARLY
  [ $g = early ] && export SDIAR_LSTM_OUT_EARLY=1
  for w in c1 c2; do
    timeout -k 10 300 python3 bench.py --workload $w --steps 10 --warmup 2 --no-cpu-baseline --no-c4-ref > $O/${w}_$g$i.json 2> $O/${w}_$g$i.err || { echo "$w $g failed"; tail -5 $O/${w}_$g$i.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(sys.argv[1], d['ms_per_step'], r.get('kernel'), r.get('achieved'))" $O/${w}_$g$i.json
  done
done
done
