# rocprofv3 kernel trace + stats of the full GPU health probe and of one bench step
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/health -o health -- python3 -m dcos_commons_amd.ops.gpu_health --full --json > gpurun_out/prof/health_stdout.txt 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/bench -o bench -- python3 bench.py --steps 1 --warmup 0 > gpurun_out/prof/bench_stdout.txt 2>&1
find gpurun_out/prof -name "*stats*" > gpurun_out/prof/files.txt
