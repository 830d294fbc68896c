# One PMC pass over the fused readiness probe (20 calls): LDS bank conflicts and LDS waits per
# kernel. Counters stay within one pass's limits (6 SQ + 1 GRBM); kernel trace only, no API tracing.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc_ready
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE \
  --kernel-trace --output-format csv -d gpurun_out/pmc_ready/p1 -o p1 -- python3 scripts/dev/readiness_loop.py 20 > gpurun_out/pmc_ready/p1.txt 2>&1
rc=$?
find gpurun_out/pmc_ready -name "*.csv" > gpurun_out/pmc_ready/files.txt
exit $rc
