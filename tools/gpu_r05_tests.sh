#!/bin/bash
# Round-5: the whole -m gpu suite and smoke() on the final tree
set -uo pipefail
O=gpurun_out/r05t; mkdir -p $O
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $O/gpu_tests.log 2>&1; r=$?
echo "gpu tests rc=$r"; tail -5 $O/gpu_tests.log
[ $r -eq 0 ] || exit 1
timeout -k 10 150 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; echo "smoke rc=$?"; tail -3 $O/smoke.log
