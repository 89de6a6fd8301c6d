#!/bin/bash
set -uo pipefail
O=gpurun_out/r05c; mkdir -p $O
timeout -k 10 300 python3 tools/shard_diag.py > $O/shard_diag.log 2>&1; echo "rc=$?"; tail -12 $O/shard_diag.log
