# Same-box interleaved cluster-mode A/B (round 5, helper-side sandbox set-up), 8 and 1 pods (5 cycles per run, 3 rounds): ab_trees/head
# (the previous commit) against this tree.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/cab4
root=$(pwd)
for i in 1 2 3; do
  if [ $((i % 2)) -eq 1 ]; then order="ab_trees/head ."; else order=". ab_trees/head"; fi
  for n in 8 1; do
    for tree in $order; do
      (cd "$tree" && timeout -k 10 240 python -u -m dcos_commons_amd.benchmarks.cluster_bench --agents $n --cycles 5 \
        | sed "s|^|$tree n$n |" >> "$root/gpurun_out/cab4/res.txt" 2>> "$root/gpurun_out/cab4/err.txt") || exit $?
    done
  done
done
PYTHONPATH=. timeout -k 10 240 python -u scripts/dev/cluster_timeline.py 8 3 > gpurun_out/cab4/timeline_n8.txt 2>&1
