# Same-box interleaved A/B in cluster mode (8 pods): ab_trees/head (a git archive of the previous
# commit) against this tree, three rounds; then an 8-pod timeline of this tree.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/cab2
root=$(pwd)
for i in 1 2 3; do
  if [ $((i % 2)) -eq 1 ]; then order="ab_trees/head ."; else order=". ab_trees/head"; fi
  for tree in $order; do
    (cd "$tree" && timeout -k 10 240 python -u -m dcos_commons_amd.benchmarks.cluster_bench --agents 8 --cycles 5 \
      | sed "s|^|$tree n8 |" >> "$root/gpurun_out/cab2/res.txt" 2>> "$root/gpurun_out/cab2/err.txt") || exit $?
  done
done
PYTHONPATH=. timeout -k 10 240 python -u scripts/dev/cluster_timeline.py 8 3 > gpurun_out/cab2/timeline_n8.txt 2>&1
