# Interleaved same-box A/B of cluster mode (scheduler process over the v1 HTTP API + ZooKeeper,
# real task processes): the round-4 final tree (ab_trees/old) against this tree, 8 and 1 pods,
# then the in-process A/B and deploy timelines of scripts/gpu_ab_check_thread.sh.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/cluster_ab
root=$(pwd)
for i in 1 2 3; do
  if [ $((i % 2)) -eq 1 ]; then order="ab_trees/old ."; else order=". ab_trees/old"; fi
  for tree in $order; do
    (cd "$tree" && timeout -k 10 240 python -u -m dcos_commons_amd.benchmarks.cluster_bench --agents 8 --cycles 5 \
      | sed "s|^|$tree n8 |" >> "$root/gpurun_out/cluster_ab/res.txt" 2>> "$root/gpurun_out/cluster_ab/err.txt") || exit $?
  done
done
for tree in ab_trees/old .; do
  (cd "$tree" && timeout -k 10 240 python -u -m dcos_commons_amd.benchmarks.cluster_bench --agents 1 --cycles 5 \
    | sed "s|^|$tree n1 |" >> "$root/gpurun_out/cluster_ab/res.txt" 2>> "$root/gpurun_out/cluster_ab/err.txt") || exit $?
done
PYTHONPATH=. timeout -k 10 240 python -u scripts/dev/cluster_timeline.py 8 3 > gpurun_out/cluster_ab/timeline_n8.txt 2>&1 && \
bash scripts/gpu_ab_check_thread.sh
