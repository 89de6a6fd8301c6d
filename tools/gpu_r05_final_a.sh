#!/bin/bash
# Round-5 evidence, part A: C2 / C4 / C1 / C3 bench lines (CPU baseline + parity, FULL=1) with rocprofv3 kernel
# stats, and the driver's default command's line.
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
O=gpurun_out/r05
mkdir -p $O
FULL=1 bash tools/profile_round.sh $O c2 c4 c1 c3 || { echo "profile_round failed"; exit 1; }
timeout -k 10 600 python3 bench.py > $O/bench_default.json 2> $O/bench_default.err || { echo "default bench failed"; exit 1; }
echo done
