#!/bin/bash
# GPU-box iteration step: selected -m gpu tests (one process, per-test timeout), then the C2 bench line.
#   bash tools/gpu_check.sh "<pytest -k expr or test files>" [bench args...]
set -euo pipefail
mkdir -p gpurun_out
T=${1:-tests}; shift || true
timeout -k 10 900 python3 -u -m pytest $T -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/tests.log 2>&1 \
  || { tail -30 gpurun_out/tests.log; exit 1; }
tail -3 gpurun_out/tests.log
if [ "${BENCH:-1}" = 1 ]; then
  timeout -k 10 300 python3 bench.py --no-c4-ref --no-cpu-baseline "$@" > gpurun_out/bench.json 2> gpurun_out/bench.err
  python3 - <<'PY'
import json
d = json.loads([x for x in open("gpurun_out/bench.json") if x.startswith("{")][-1])
print("ms_per_step", d["ms_per_step"], "value", d["value"])
for k, v in sorted(d.get("kernels", {}).items(), key=lambda kv: -kv[1]["ms"])[:12]:
    print(f"  {k:28s} {v['ms']:7.3f} ms  x{v['launches']:3d}  {v['bound']} {v['frac']}")
PY
fi
