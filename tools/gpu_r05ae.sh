#!/bin/bash
# round 5: Kaldi fbank FFT in three register passes vs the nine-stage LDS form (SDIAR_FBANK_LDS_FFT=1): hashes,
# fbank / tsvad / embedding tests, rocprof, C2 A/B
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
O=gpurun_out/r05ae; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_ops.py tests/test_gpu_tsvad.py tests/test_gpu_campp.py -k "fbank or cmn or tsvad or campp or embed" > $O/t.log 2>&1; r=$?
echo "tests rc=$r"; tail -3 $O/t.log
[ $r -eq 0 ] || exit 1
timeout -k 10 120 python3 tools/fbank_hash.py > $O/hash_reg.log 2>&1 || { echo hash failed; tail -3 $O/hash_reg.log; exit 1; }
SDIAR_FBANK_LDS_FFT=1 timeout -k 10 120 python3 tools/fbank_hash.py > $O/hash_lds.log 2>&1 || { echo hash failed; exit 1; }
grep -h fbank $O/hash_reg.log $O/hash_lds.log
for m in reg lds; do
  unset SDIAR_FBANK_LDS_FFT; [ $m = lds ] && export SDIAR_FBANK_LDS_FFT=1
  SDIAR_CAM_ONE_STREAM=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p$m -o run -- python3 bench.py --workload c2 --steps 2 --warmup 1 --no-cpu-baseline --no-kernel-timing --no-c4-ref > $O/p$m.log 2>&1 || { echo "prof failed"; exit 1; }
  f=$(find $O/p$m -name '*kernel_stats.csv' | head -1); cp "$f" $O/kernel_stats_$m.csv; rm -rf $O/p$m
  python3 - "$O/kernel_stats_$m.csv" $m <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if 'fbank' in r['Name']:
        print(sys.argv[2], r['Name'][:60], r['Calls'], round(float(r['AverageNs']) / 1e3, 1), 'us')
PY
done
unset SDIAR_FBANK_LDS_FFT
for i in 1 2; do
for m in reg lds; do
  unset SDIAR_FBANK_LDS_FFT; [ $m = lds ] && export SDIAR_FBANK_LDS_FFT=1
  timeout -k 10 300 python3 bench.py --workload c2 --steps 20 --warmup 3 --no-cpu-baseline --no-c4-ref > $O/c2_$m$i.json 2> $O/c2_$m$i.err || { echo "c2 $m failed"; tail -5 $O/c2_$m$i.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['ms_per_step'])" $O/c2_$m$i.json
done
done
