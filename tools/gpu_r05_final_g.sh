#!/bin/bash
# Round-5 evidence, part G: the two-stream C2 trace and its per-stream timeline on the final binary
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
O=gpurun_out/r05
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tl -o run -- python3 bench.py --workload c2 --steps 3 --warmup 1 --no-cpu-baseline --no-kernel-timing --no-c4-ref > $O/tl.log 2>&1 || { echo "trace failed"; exit 1; }
f=$(find $O/tl -name '*kernel_trace.csv' | head -1); python3 tools/stream_timeline.py "$f" --step 2 > $O/timeline_c2.txt; gzip -c "$f" > $O/kernel_trace_c2_2stream.csv.gz; rm -rf $O/tl
cat $O/timeline_c2.txt
echo done
