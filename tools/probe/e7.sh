set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${RUN:-e7}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_tsvad.py tests/test_gpu_campp.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 1; }
timeout -k 10 200 python -u bench.py --no-cpu-baseline > $O/c2.json 2> $O/c2.err || exit 2
timeout -k 10 200 python -u bench.py --workload emb --steps 3 --warmup 1 > $O/emb.json 2> $O/emb.err || exit 3
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/f -o f -- python bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-kernel-timing > $O/f.log 2>&1 || exit 4
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/w -o w -- python bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-kernel-timing > $O/w.log 2>&1 || exit 5
python tools/pmc_traffic.py $O/f $O/w c2 $O/pmc_traffic.json > $O/pmc.txt 2>&1
tail -2 $O/tests.log; cat $O/c2.json $O/emb.json; cat $O/pmc.txt | tail -10
