#!/bin/bash
# round 5: mha_block layout variants on C2 (ring depth vs workgroups per CU), one box
set -uo pipefail
O=gpurun_out/r05i; mkdir -p $O
for i in 1 2; do
for v in 0 1 2 3 4 5 6; do
  SDIAR_MHA_VARIANT=$v timeout -k 10 300 python3 bench.py --workload c2 --steps 20 --warmup 3 --no-cpu-baseline --no-c4-ref > $O/c2_v$v$i.json 2> $O/c2_v$v$i.err || { echo "c2 v$v failed"; tail -5 $O/c2_v$v$i.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['ms_per_step'])" $O/c2_v$v$i.json
done
done
