set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
python -c "import torch;print(torch.cuda.get_device_name(0), torch.cuda.device_count())" > gpurun_out/dev.txt 2>&1
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.txt 2>&1 && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.txt 2>&1 && \
timeout -k 10 300 python -m dcos_commons_amd.ops.gpu_health --json > gpurun_out/health.json 2>&1 && \
timeout -k 10 600 python bench.py --steps 3 --warmup 1 > gpurun_out/bench1.txt 2>&1
