#!/bin/bash
# Two SQ counter passes (one process each) over a short run, summarised for kernels matching a substring.
#   bash tools/pmc_attn.sh <outdir> <kernel-substring> <python script and args...>
set -euo pipefail
OUT=$1; KS=$2; shift 2
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
A="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES"
B="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES"
timeout -s KILL 120 rocprofv3 --pmc $A --output-format csv -d "$OUT/a" -o run -- python3 "$@" > "$OUT/a.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc $B --output-format csv -d "$OUT/b" -o run -- python3 "$@" > "$OUT/b.log" 2>&1
python3 tools/pmc_pass.py "$OUT/a" $KS
python3 tools/pmc_pass.py "$OUT/b" $KS
