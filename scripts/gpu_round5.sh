# Round-5 validation on one MI355X (one gpurun call): node discovery dump, GPU tests, smoke, bench N=1
# (headline + the reference gpu_resource.yml serial row), framework benches on the reference's
# unchanged packages and the repo's (needs scripts/stage_reference_inputs.sh beforehand), the one-GPU
# scaling rehearsal, and a rocprofv3 kernel trace of one bench step.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
bash scripts/dev/dump_gpu_discovery.sh > gpurun_out/discovery_stdout.txt 2>&1 && \
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.txt 2>&1 && \
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.txt 2>&1 && \
timeout -k 10 600 python -u bench.py --steps 5 --warmup 1 > gpurun_out/bench1.txt 2>&1 && \
timeout -k 10 600 python -u -m dcos_commons_amd.benchmarks.framework_bench --cycles 5 > gpurun_out/framework_bench.txt 2>&1 && \
bash scripts/gpu_scale_rehearsal.sh && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/bench -o bench -- python3 bench.py --steps 1 --warmup 0 --reference-steps 0 > gpurun_out/prof/bench_stdout.txt 2>&1
rc=$?
find gpurun_out/prof -name "*stats*" > gpurun_out/prof/files.txt
exit $rc
