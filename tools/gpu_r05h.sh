#!/bin/bash
# round 5: attention + out-projection in one launch in the FS-EEND stream: tests, c5s A/B, kernel stats
set -uo pipefail
O=gpurun_out/r05h; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_fseend_stream.py > $O/fs_tests.log 2>&1; r=$?
echo "fs tests rc=$r"; tail -8 $O/fs_tests.log
[ $r -eq 0 ] || exit 1
for i in 1 2; do
for g in op noop; do
  unset SDIAR_NO_ATTN_OUTPROJ
  [ $g = noop ] && export SDIAR_NO_ATTN_OUTPROJ=1
  timeout -k 10 300 python3 bench.py --workload c5s --steps 3 --warmup 1 --no-cpu-baseline > $O/c5s_$g$i.json 2> $O/c5s_$g$i.err || { echo "c5s $g failed"; tail -5 $O/c5s_$g$i.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['latency_ms'], d['roofline']['model']['encoder_graph_nodes'], d['roofline']['model']['decoder_graph_nodes'])" $O/c5s_$g$i.json
done
done
unset SDIAR_NO_ATTN_OUTPROJ
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --workload c5s --steps 2 --warmup 1 --no-cpu-baseline > $O/prof.log 2>&1 || { echo "prof failed"; exit 1; }
f=$(find $O/prof -name '*kernel_stats.csv' | head -1); cp "$f" $O/kernel_stats_c5s.csv; rm -rf $O/prof
head -12 $O/kernel_stats_c5s.csv | cut -c1-160
