#!/bin/bash
# round-5 check: changed GPU tests, the C2 line (with the spread-variant DER block), a two-stream timeline
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
O=gpurun_out/r05b; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_lstm_status.py::test_lstm_exchange_probes -s > $O/pytest.log 2>&1; echo "pytest rc=$?"
tail -3 $O/pytest.log
timeout -k 10 400 python3 bench.py --workload c2 --steps 10 --warmup 3 --no-c4-ref > $O/bench_c2.json 2> $O/bench_c2.err || { echo bench failed; tail -20 $O/bench_c2.err; exit 1; }
echo bench ok
for r in 1; do
  SDIAR_MHA_SEQ2=1 timeout -k 10 300 python3 bench.py --workload c2 --steps 10 --warmup 3 --no-cpu-baseline --no-c4-ref --no-kernel-timing > $O/bench_c2_seq2_$r.json 2>/dev/null || exit 1
  timeout -k 10 300 python3 bench.py --workload c2 --steps 10 --warmup 3 --no-cpu-baseline --no-c4-ref --no-kernel-timing > $O/bench_c2_seq1_$r.json 2>/dev/null || exit 1
done
echo ab ok
SDIAR_RP_PRIO=1 timeout -k 10 300 python3 bench.py --workload c2 --steps 10 --warmup 3 --no-cpu-baseline --no-c4-ref --no-kernel-timing > $O/bench_c2_prio1.json 2>/dev/null || exit 1
echo prio ok
for r in 1 2; do
  for k in 3 4; do
    SDIAR_SLICES=$k timeout -k 10 300 python3 bench.py --workload c2 --steps 10 --warmup 3 --no-cpu-baseline --no-c4-ref --no-kernel-timing > $O/bench_c2_slices${k}_$r.json 2>/dev/null || exit 1
  done
done
echo slices ok
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tl -o run -- python3 bench.py --workload c2 --steps 3 --warmup 1 --no-cpu-baseline --no-kernel-timing --no-c4-ref > $O/tl.log 2>&1 || { echo trace failed; exit 1; }
f=$(find $O/tl -name '*kernel_trace.csv' | head -1); cp "$f" $O/kernel_trace_c2_2stream.csv; rm -rf $O/tl
python3 tools/stream_timeline.py $O/kernel_trace_c2_2stream.csv --step 2 > $O/timeline.txt
echo done
