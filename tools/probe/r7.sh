# Round-end refresh: default bench (with CPU baseline), kernel-trace stats, PMC traffic.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${RUN:-r01_v7}
mkdir -p $O
timeout -k 10 400 python -u bench.py > $O/bench_c2.json 2> $O/bench_c2.err || exit 1
timeout -s KILL 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o kt -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline > $O/bench_c2_under_rocprof.json 2> $O/kt.err || exit 2
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/f -o f -- python bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-kernel-timing > $O/f.log 2>&1 || exit 3
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/w -o w -- python bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-kernel-timing > $O/w.log 2>&1 || exit 4
python tools/pmc_traffic.py $O/f $O/w c2 $O/pmc_traffic.json > $O/pmc.txt 2>&1
find $O/kt -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats_c2.csv \;
cat $O/bench_c2.json; tail -5 $O/pmc.txt
