# One GPU call for a full validation: round script (GPU tests, smoke, bench N=1 in both profiles,
# kernel trace), framework benches, one-GPU scaling rehearsal, cluster-mode bench.
set -o pipefail
bash scripts/gpu_round.sh && \
timeout -k 10 300 python -u -m dcos_commons_amd.benchmarks.framework_bench --cycles 5 > gpurun_out/framework_bench.txt 2>&1 && \
bash scripts/gpu_scale_rehearsal.sh && \
bash scripts/gpu_cluster_bench.sh && \
mkdir -p gpurun_out/timeline && \
SDK_TRACE=1 timeout -k 10 120 python -u scripts/dev/deploy_timeline.py 1 --gpu > gpurun_out/timeline/n1.txt 2>&1 && \
SDK_TRACE=1 timeout -k 10 120 python -u scripts/dev/deploy_timeline.py 8 --gpu > gpurun_out/timeline/n8.txt 2>&1
