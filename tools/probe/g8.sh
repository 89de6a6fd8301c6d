set -o pipefail
mkdir -p gpurun_out/g8
export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE TCC_HIT_sum -d gpurun_out/g8/p1 -o p1 -- python tools/gemm_micro.py --reps 2 --shapes 1152x384,384x384 > gpurun_out/g8/p1.log 2>&1 || exit 2
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE TCC_MISS_sum -d gpurun_out/g8/p2 -o p2 -- python tools/gemm_micro.py --reps 2 --shapes 1152x384,384x384 > gpurun_out/g8/p2.log 2>&1 || exit 3
timeout -s KILL 90 rocprofv3 --pmc TA_BUSY_avr TA_FLAT_READ_WAVEFRONTS_sum TD_BUSY_avr TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum -d gpurun_out/g8/p3 -o p3 -- python tools/gemm_micro.py --reps 2 --shapes 1152x384,384x384 > gpurun_out/g8/p3.log 2>&1 || echo p3fail
for p in p1 p2 p3; do f=$(find gpurun_out/g8/$p -name '*.db' | head -1); [ -n "$f" ] && python tools/pmc_db.py "$f" gemm > gpurun_out/g8/$p.txt; done
cat gpurun_out/g8/p1.txt gpurun_out/g8/p2.txt gpurun_out/g8/p3.txt; grep -i error gpurun_out/g8/p3.log | head -3
