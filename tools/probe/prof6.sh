set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/p6
mkdir -p $O
timeout -s KILL 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o kt -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/kt.log 2>&1 || exit 2
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/f -o f -- python bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-kernel-timing > $O/f.log 2>&1 || exit 3
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/w -o w -- python bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-kernel-timing > $O/w.log 2>&1 || exit 4
python tools/pmc_traffic.py $O/f $O/w c2 $O/pmc_traffic.json > $O/pmc.txt 2>&1 || echo pmcfail
find $O/kt -name '*kernel_stats.csv' | head -1 | xargs -I{} cp {} $O/kernel_stats.csv
head -12 $O/kernel_stats.csv; cat $O/pmc.txt | tail -12; grep '"metric"' $O/kt.log | head -1
