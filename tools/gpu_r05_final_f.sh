#!/bin/bash
# Round-5 evidence, part F (after the register-pass fbank): the lines whose step runs the Kaldi fbank -- C2, C4,
# emb, tss (CPU baseline + parity) with kernel stats -- and the driver's default line
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
O=gpurun_out/r05
mkdir -p $O
FULL=1 bash tools/profile_round.sh $O c2 c4 emb tss || { echo "profile_round failed"; exit 1; }
timeout -k 10 600 python3 bench.py > $O/bench_default.json 2> $O/bench_default.err || { echo "default bench failed"; exit 1; }
echo done
