# Same-box interleaved framework-bench A/B (BASELINE configs 3 and 4 on the reference's unchanged
# packages): ab_trees/head (the previous commit) against this tree, 3 rounds, order alternating.
# Needs ref_inputs/ (scripts/stage_reference_inputs.sh) and ab_trees/head (git archive + built .so).
set -o pipefail
export TMPDIR=/tmp
export SDK_REFERENCE_ROOT="$(pwd)/ref_inputs"
mkdir -p gpurun_out/fab
root=$(pwd)
for i in 1 2 3; do
  if [ $((i % 2)) -eq 1 ]; then order="ab_trees/head ."; else order=". ab_trees/head"; fi
  for tree in $order; do
    (cd "$tree" && timeout -k 10 300 python -u -m dcos_commons_amd.benchmarks.framework_bench --framework all \
      --specs reference --cycles 7 2>> "$root/gpurun_out/fab/err.txt" | grep '^{' \
      | sed "s|^|$tree |" >> "$root/gpurun_out/fab/res.txt") || exit $?
  done
done
