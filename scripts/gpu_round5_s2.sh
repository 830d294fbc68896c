# Round-5 second validation on one MI355X: the full round-5 run (scripts/gpu_round5.sh: discovery,
# GPU tests, smoke, bench N=1 + reference row, framework benches, scaling rehearsal, kernel trace),
# then the cluster-mode bench set (scripts/gpu_cluster_bench.sh).
set -o pipefail
bash scripts/gpu_round5.sh && bash scripts/gpu_cluster_bench.sh
