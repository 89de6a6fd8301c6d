#!/bin/bash
set -uo pipefail
O=gpurun_out/r05c; mkdir -p $O
timeout -k 10 200 python3 tools/mha_diag.py > $O/mha_diag.log 2>&1; echo "rc=$?"; cat $O/mha_diag.log | tail -60
