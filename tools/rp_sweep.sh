#!/bin/bash
# rowprog A/B on the GPU box: C2 bench per variant (SDIAR_RP_TT token tiles per wave, SDIAR_RP_PROBE timing probes).
set -uo pipefail
OUT=${1:-gpurun_out/rp}
mkdir -p "$OUT"
B="python bench.py --steps 3 --warmup 1 --no-cpu-baseline"
run() {   # name env...
  local name=$1; shift
  env "$@" timeout -k 10 200 $B > "$OUT/$name.json" 2> "$OUT/$name.err" || { echo "$name failed"; exit 1; }
  python - "$OUT/$name.json" "$name" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
ks = {k: v for k, v in d["kernels"].items() if k.startswith("rowprog")}
print(sys.argv[2], d["ms_per_step"], {k: (v["ms"], v["launches"]) for k, v in ks.items()})
PY
}
for v in "$@"; do
  case $v in
    tt1) run tt1 SDIAR_RP_TT=1 ;;
    tt2) run tt2 SDIAR_RP_TT=2 ;;
    p1) run p1 SDIAR_RP_PROBE=1 ;;
    p2) run p2 SDIAR_RP_PROBE=2 ;;
    p3) run p3 SDIAR_RP_PROBE=3 ;;
    p4) run p4 SDIAR_RP_PROBE=4 ;;
    unfused) run unfused SDIAR_NO_ROWPROG=1 ;;
  esac
done
