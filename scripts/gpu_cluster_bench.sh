# Cluster-mode bench on one MI355X box: the scheduler as its own process over the Mesos v1 HTTP API
# with ZooKeeper persistence and real task processes; the readiness check is first a device-export
# check, then the native HIP probe binary run by the agent on the pod's GPU (a HIP runtime per check),
# then the node's readiness service (amd-gpu-probed, runtime resident) with amd-gpu-ready as the check.
set -o pipefail
mkdir -p gpurun_out/cluster
timeout -k 10 300 python -u -m dcos_commons_amd.benchmarks.cluster_bench --agents 1 --cycles 5 \
  > gpurun_out/cluster/n1.json 2> gpurun_out/cluster/n1.err && \
timeout -k 10 300 python -u -m dcos_commons_amd.benchmarks.cluster_bench --agents 8 --cycles 3 \
  > gpurun_out/cluster/n8.json 2> gpurun_out/cluster/n8.err && \
timeout -k 10 300 python -u -m dcos_commons_amd.benchmarks.cluster_bench --agents 1 --cycles 5 \
  --probe-cmd "$GRAFT_REPO_ROOT/native/build/amd-gpu-probe --readiness" \
  > gpurun_out/cluster/n1_probe.json 2> gpurun_out/cluster/n1_probe.err && \
timeout -k 10 300 python -u -m dcos_commons_amd.benchmarks.cluster_bench --agents 1 --cycles 5 --probe-service \
  > gpurun_out/cluster/n1_service.json 2> gpurun_out/cluster/n1_service.err && \
timeout -k 10 300 python -u -m dcos_commons_amd.benchmarks.cluster_bench --agents 1 --cycles 1 --warmup 0 \
  --profile reference > gpurun_out/cluster/n1_ref.json 2> gpurun_out/cluster/n1_ref.err
