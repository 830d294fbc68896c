# GEMM kernel validation + benchmark + kernel trace on one MI355X
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out

timeout -k 10 300 python -m pytest tests/test_gpu_ops.py -q -m gpu -k gemm > gpurun_out/gemm_tests.txt 2>&1 && \
timeout -k 10 300 python scripts/gemm_bench.py --sizes 4096,8192 --rounds 7 > gpurun_out/gemm_bench.json 2> gpurun_out/gemm_bench.err && \
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_gemm -o gemm -- python3 $GRAFT_REPO_ROOT/scripts/gemm_bench.py --sizes 8192 --rounds 2 --reps 3 > $GRAFT_REPO_ROOT/gpurun_out/prof_gemm.log 2>&1
