#!/bin/bash
# rocprofv3 kernel stats of a 1-minute c5s stream per environment setting: bash tools/prof_c5s_env.sh OUT tag=ENV=1 ...
set -euo pipefail
OUT=$1; shift
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for spec in "$@"; do
  tag=${spec%%=*}; envs=${spec#*=}; [ "$envs" = "-" ] && envs=""
  env $envs timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/$tag" -o run -- \
    python3 bench.py --workload c5s --steps 1 --warmup 0 --no-cpu-baseline --minutes 1 > "$OUT/$tag.json" 2> "$OUT/$tag.err"
  cp "$(find "$OUT/$tag" -name '*kernel_stats.csv' | head -1)" "$OUT/kernel_stats_$tag.csv"
  rm -rf "$OUT/$tag"
done
