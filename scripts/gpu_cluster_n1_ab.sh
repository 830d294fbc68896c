# Same-box interleaved cluster-mode A/B at 1 pod (10 cycles per run, 3 rounds): the round-4 tree
# (ab_trees/old) against this tree.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/cn1
root=$(pwd)
for i in 1 2 3; do
  if [ $((i % 2)) -eq 1 ]; then order="ab_trees/old ."; else order=". ab_trees/old"; fi
  for tree in $order; do
    (cd "$tree" && timeout -k 10 240 python -u -m dcos_commons_amd.benchmarks.cluster_bench --agents 1 --cycles 10 \
      | sed "s|^|$tree n1 |" >> "$root/gpurun_out/cn1/res.txt" 2>> "$root/gpurun_out/cn1/err.txt") || exit $?
  done
done
