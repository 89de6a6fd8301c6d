#!/bin/bash
# round 5: small-grid XCD grouping of the long attention (FS-EEND encoder): tests, C5 A/B, FETCH_SIZE per launch
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
O=gpurun_out/r05n; mkdir -p $O
timeout -k 10 500 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_fseend.py tests/test_gpu_attention_mask.py tests/test_gpu_eda.py tests/test_gpu_ops.py -k "attention or attn or fseend or eda" > $O/t.log 2>&1; r=$?
echo "tests rc=$r"; tail -3 $O/t.log
[ $r -eq 0 ] || exit 1
for i in 1 2; do
for g in group flat; do
  unset SDIAR_ATTN_NO_GROUP_REMAP
  [ $g = flat ] && export SDIAR_ATTN_NO_GROUP_REMAP=1
  timeout -k 10 300 python3 bench.py --workload c5 --steps 5 --warmup 2 --no-cpu-baseline > $O/c5_$g$i.json 2> $O/c5_$g$i.err || { echo "c5 $g failed"; tail -5 $O/c5_$g$i.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['ms_per_step'], d['roofline']['frac'], d['roofline'].get('avg_launch_ms'))" $O/c5_$g$i.json
done
done
unset SDIAR_ATTN_NO_GROUP_REMAP
for g in group flat; do
  [ $g = flat ] && export SDIAR_ATTN_NO_GROUP_REMAP=1
  timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/f$g -o run -- python3 bench.py --workload c5 --steps 2 --warmup 1 --no-cpu-baseline --no-kernel-timing > $O/f$g.log 2>&1 || { echo "fetch failed"; exit 1; }
  f=$(find $O/f$g -name '*counter_collection.csv' | head -1)
  python3 - "$f" <<'PY'
import csv, sys, collections
tot = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    n = r.get('Kernel_Name', r.get('Kernel-Name', ''))
    if 'attn_long' in n:
        tot[n.split('(')[0][-40:]].append(float(r['Counter_Value']))
for k, v in tot.items():
    print(k, len(v), 'FETCH_SIZE KiB per launch (x2 for gfx950 bytes):', round(sum(v) / len(v)))
PY
  rm -rf $O/f$g
done
