# PMC counter passes over the probe GEMM (gemm_bench.py at 8192^3): MFMA busy, LDS bank conflicts, L2 hit rate.
# One rocprofv3 run per pass, each within the per-block counter limits (<=8 SQ, <=4 TCC, <=2 GRBM).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
timeout -s KILL 90 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE \
  --kernel-trace --output-format csv -d gpurun_out/pmc/p1 -o p1 -- python3 scripts/gemm_bench.py --sizes 8192 --rounds 1 --reps 3 > gpurun_out/pmc/p1.txt 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum SQ_WAIT_INST_LDS SQ_WAIT_INST_ANY \
  --kernel-trace --output-format csv -d gpurun_out/pmc/p2 -o p2 -- python3 scripts/gemm_bench.py --sizes 8192 --rounds 1 --reps 3 > gpurun_out/pmc/p2.txt 2>&1
rc=$?
find gpurun_out/pmc -name "*.csv" > gpurun_out/pmc/files.txt
exit $rc
