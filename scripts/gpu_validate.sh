# GPU validation: build natives for gfx950, GPU tests, smoke, health probes, bench N=1
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.txt 2>&1 && \
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.txt 2>&1 && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.txt 2>&1 && \
timeout -k 10 120 ./native/build/amd-gpu-probe --full --json > gpurun_out/probe_full.json 2>&1 && \
timeout -k 10 120 ./native/build/amd-gpu-probe --readiness --json > gpurun_out/probe_readiness.json 2>&1 && \
timeout -k 10 600 python bench.py --steps 5 --warmup 1 > gpurun_out/bench1.txt 2>&1 && \
timeout -k 10 600 python bench.py --steps 2 --warmup 0 --profile reference > gpurun_out/bench1_ref.txt 2>&1
