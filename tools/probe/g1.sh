set -o pipefail
mkdir -p gpurun_out/g1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 120 python -u tools/gemm_micro.py > gpurun_out/g1/micro.txt 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT -d gpurun_out/g1/p1 -o p1 -- python tools/gemm_micro.py --reps 2 --shapes 384x512,384x384 > gpurun_out/g1/p1.log 2>&1 || exit 2
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE TCC_HIT_sum -d gpurun_out/g1/p2 -o p2 -- python tools/gemm_micro.py --reps 2 --shapes 384x512,384x384 > gpurun_out/g1/p2.log 2>&1 || exit 3
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE TCC_MISS_sum -d gpurun_out/g1/p3 -o p3 -- python tools/gemm_micro.py --reps 2 --shapes 384x512,384x384 > gpurun_out/g1/p3.log 2>&1 || exit 4
for p in p1 p2 p3; do f=$(find gpurun_out/g1/$p -name '*.db' | head -1); python tools/pmc_db.py "$f" gemm > gpurun_out/g1/$p.txt; done
cat gpurun_out/g1/micro.txt gpurun_out/g1/p1.txt gpurun_out/g1/p2.txt gpurun_out/g1/p3.txt
