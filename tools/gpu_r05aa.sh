#!/bin/bash
# round 5: the LSTM input projection GEMM (gemm_ring, 16 N tiles): row-major tile order vs 4 x 8 XCD blocks vs the
# persistent wide ring; output hashes must agree
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
O=gpurun_out/r05aa; mkdir -p $O
for i in 1 2 3; do
  timeout -k 10 200 python3 tools/gemm_probe.py 90000x2048x1536 >> $O/probe_row.log 2>&1 || { echo probe failed; tail -5 $O/probe_row.log; exit 1; }
  SDIAR_RING_BLOCK=1 timeout -k 10 200 python3 tools/gemm_probe.py 90000x2048x1536 >> $O/probe_block.log 2>&1 || { echo probe failed; tail -5 $O/probe_block.log; exit 1; }
  SDIAR_RING_WIDE=1 timeout -k 10 200 python3 tools/gemm_probe.py 90000x2048x1536 45000x2048x1536 >> $O/probe_wide.log 2>&1 || { echo probe failed; tail -5 $O/probe_wide.log; exit 1; }
done
timeout -k 10 200 python3 tools/gemm_probe.py 45000x2048x1536 >> $O/probe_row.log 2>&1 || { echo probe failed; exit 1; }
grep -h "gemm_\|sha" $O/probe_row.log $O/probe_block.log $O/probe_wide.log
