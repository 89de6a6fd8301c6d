#!/bin/bash
# One parameterised GPU-box runner (replaces round 5's one-off tools/gpu_r05*.sh scripts).
#
#   bash tools/gpu_run.sh <outdir> <step> [<step> ...]
#
# Steps (each runs under its own time limit; the first failure ends the call, nothing is retried):
#   tests[:<pytest -k expr>]           the -m gpu suite (or the selected tests) -> <outdir>/tests*.log
#   file:<test file>[:<-k expr>]       one test file -> <outdir>/<file stem>.log
#   smoke                              __graft_entry__.smoke()
#   bench:<name>:<bench.py args>       one bench line -> <outdir>/<name>.json (+ .err)
#   prof:<name>:<bench.py args>        rocprofv3 --kernel-trace --stats of a bench command (one stream)
#                                      -> <outdir>/kernel_stats_<name>.csv
#   pmc:<name>:<counters>:<bench args> one rocprofv3 --pmc pass -> <outdir>/pmc_<name>.csv
#   py:<name>:<script> [args]          python3 <script> [args] -> <outdir>/<name>.log
# Environment variables given before the command apply to every step (e.g. SDIAR_CAM_ONE_STREAM=1).
set -uo pipefail
OUT=$1; shift
mkdir -p "$OUT"
export TMPDIR=/tmp
ROOT=$(pwd)
T_TEST=${T_TEST:-900}
T_BENCH=${T_BENCH:-400}

line_ms() {  # print the ms_per_step / value of a bench line
  python3 - "$1" <<'PY'
import json, sys
try:
    d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
    print(sys.argv[1], "ms_per_step", d.get("ms_per_step"), "value", d.get("value"), d.get("unit"),
          "frac", (d.get("roofline") or {}).get("frac"), "parity", (d.get("parity") or {}).get("max_abs_diff"))
except Exception as e:  # noqa: BLE001
    print(sys.argv[1], "unreadable:", e)
PY
}

for STEP in "$@"; do
  KIND=${STEP%%:*}
  REST=${STEP#*:}
  [ "$REST" = "$STEP" ] && REST=""
  case "$KIND" in
    tests)
      K=()
      [ -n "$REST" ] && K=(-k "$REST")
      timeout -k 10 "$T_TEST" python3 -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread "${K[@]}" \
        > "$OUT/tests.log" 2>&1; r=$?
      echo "tests rc=$r"; tail -4 "$OUT/tests.log"
      [ $r -eq 0 ] || exit 1 ;;
    file)
      F=${REST%%:*}; KX=${REST#*:}; [ "$KX" = "$REST" ] && KX=""
      K=(); [ -n "$KX" ] && K=(-k "$KX")
      N=$(basename "$F" .py)
      timeout -k 10 "$T_TEST" python3 -u -m pytest "$F" -x -v -s --timeout 240 --timeout-method thread "${K[@]}" \
        > "$OUT/$N.log" 2>&1; r=$?
      echo "$F rc=$r"; tail -4 "$OUT/$N.log"
      [ $r -eq 0 ] || exit 1 ;;
    smoke)
      timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1; r=$?
      echo "smoke rc=$r"; tail -2 "$OUT/smoke.log"
      [ $r -eq 0 ] || exit 1 ;;
    bench)
      N=${REST%%:*}; A=${REST#*:}; [ "$A" = "$REST" ] && A=""
      # shellcheck disable=SC2086
      timeout -k 10 "$T_BENCH" python3 bench.py $A > "$OUT/$N.json" 2> "$OUT/$N.err"; r=$?
      [ $r -eq 0 ] || { echo "bench $N rc=$r"; tail -5 "$OUT/$N.err"; exit 1; }
      line_ms "$OUT/$N.json" ;;
    prof)
      N=${REST%%:*}; A=${REST#*:}; [ "$A" = "$REST" ] && A=""
      D="$OUT/trace_$N"
      # shellcheck disable=SC2086
      SDIAR_CAM_ONE_STREAM=1 timeout -k 10 "$T_BENCH" rocprofv3 --kernel-trace --stats --output-format csv -d "$D" -o run \
        -- python3 bench.py $A > "$OUT/prof_$N.log" 2>&1; r=$?
      [ $r -eq 0 ] || { echo "prof $N rc=$r"; tail -5 "$OUT/prof_$N.log"; exit 1; }
      cp "$(find "$D" -name '*kernel_stats.csv' | head -1)" "$OUT/kernel_stats_$N.csv"
      rm -rf "$D"
      echo "prof $N ok" ;;
    pmc)
      N=${REST%%:*}; R2=${REST#*:}; C=${R2%%:*}; A=${R2#*:}; [ "$A" = "$R2" ] && A=""
      D="$OUT/pmc_$N"
      # shellcheck disable=SC2086
      SDIAR_CAM_ONE_STREAM=1 timeout -s KILL 300 rocprofv3 --pmc ${C//,/ } --output-format csv -d "$D" -o run \
        -- python3 bench.py $A > "$OUT/pmc_$N.log" 2>&1; r=$?
      [ $r -eq 0 ] || { echo "pmc $N rc=$r"; tail -5 "$OUT/pmc_$N.log"; exit 1; }
      cp "$(find "$D" -name '*counter_collection.csv' | head -1)" "$OUT/pmc_$N.csv"
      rm -rf "$D"
      echo "pmc $N ok" ;;
    py)
      N=${REST%%:*}; A=${REST#*:}
      # shellcheck disable=SC2086
      timeout -k 10 "$T_BENCH" python3 $A > "$OUT/$N.log" 2>&1; r=$?
      echo "py $N rc=$r"; tail -6 "$OUT/$N.log"
      [ $r -eq 0 ] || exit 1 ;;
    *)
      echo "unknown step $STEP"; exit 2 ;;
  esac
done
echo "all steps done"
cd "$ROOT" || true
