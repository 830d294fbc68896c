# Cluster mode (scheduler process, v1 HTTP API, ZooKeeper, real task processes) on one MI355X box,
# 1 and 8 pods, each with two readiness checks: the shell test of HIP_VISIBLE_DEVICES ("no GPU
# readiness") and the node's GPU readiness service (amd-gpu-ready -> amd-gpu-probed: the HIP probe on
# the pod's GPU; all 8 agents map their pod onto the box's one GPU). Interleaved, back to back.
set -o pipefail
out=gpurun_out/cluster_probe_r06
mkdir -p $out
run() {  # name, args...
  local name=$1; shift
  timeout -k 10 240 python -u -m dcos_commons_amd.benchmarks.cluster_bench "$@" > $out/$name.json 2> $out/$name.err
}
run n1_test --agents 1 --cycles 5 && \
run n1_service --agents 1 --cycles 5 --probe-service && \
run n8_test --agents 8 --cycles 5 && \
run n8_service --agents 8 --cycles 5 --probe-service && \
cat $out/*.json
