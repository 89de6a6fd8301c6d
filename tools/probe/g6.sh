set -o pipefail
mkdir -p gpurun_out/g6
export TMPDIR=/tmp
C="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT"
timeout -s KILL 90 rocprofv3 --pmc $C -d gpurun_out/g6/p1 -o p1 -- python tools/gemm_micro.py --reps 2 --shapes 1152x384 > gpurun_out/g6/p1.log 2>&1 || exit 2
SDIAR_NO_AREG_GEMM=1 timeout -s KILL 90 rocprofv3 --pmc $C -d gpurun_out/g6/p2 -o p2 -- python tools/gemm_micro.py --reps 2 --shapes 1152x384 > gpurun_out/g6/p2.log 2>&1 || exit 3
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_MFMA SQ_WAVES SQ_INSTS_VMEM_WR SQ_INST_CYCLES_VMEM_RD -d gpurun_out/g6/p3 -o p3 -- python tools/gemm_micro.py --reps 2 --shapes 1152x384 > gpurun_out/g6/p3.log 2>&1 || echo p3fail
for p in p1 p2 p3; do f=$(find gpurun_out/g6/$p -name '*.db' | head -1); [ -n "$f" ] && python tools/pmc_db.py "$f" gemm > gpurun_out/g6/$p.txt; done
cat gpurun_out/g6/p1.txt gpurun_out/g6/p2.txt gpurun_out/g6/p3.txt; tail -3 gpurun_out/g6/p3.log
