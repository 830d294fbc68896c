# Round validation on one MI355X: GPU tests, smoke, bench N=1 (both profiles), rocprofv3 kernel stats of a bench step.
# Natives are built on the CPU host beforehand (python -c "import __graft_entry__ as g; g.build()").
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.txt 2>&1 && \
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.txt 2>&1 && \
timeout -k 10 600 python -u bench.py --steps 5 --warmup 1 > gpurun_out/bench1.txt 2>&1 && \
timeout -k 10 600 python -u bench.py --steps 2 --warmup 0 --profile reference > gpurun_out/bench1_ref.txt 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/bench -o bench -- python3 bench.py --steps 1 --warmup 0 > gpurun_out/prof/bench_stdout.txt 2>&1
rc=$?
find gpurun_out/prof -name "*stats*" > gpurun_out/prof/files.txt
exit $rc
