# Interleaved A/B of two source trees on the box: ab_trees/old vs this tree, helloworld DeployBench
# (synthetic readiness) pinned to CPUs 4-7. AB_NS (default "1 8"), AB_REPS (30) and AB_ITERS (3)
# size the run; the order of the two trees alternates between iterations.
set -o pipefail
mkdir -p gpurun_out/abt
NS=${AB_NS:-"1 8"}; REPS=${AB_REPS:-30}; ITERS=${AB_ITERS:-3}; AB_EXTRA=${AB_EXTRA:-}
for i in $(seq 1 $ITERS); do
  if [ $((i % 2)) -eq 1 ]; then order="ab_trees/old ."; else order=". ab_trees/old"; fi
  for n in $NS; do
    for tree in $order; do
      timeout -k 10 200 python scripts/dev/ab_deploy.py $tree $n $REPS $AB_EXTRA >> gpurun_out/abt/res.jsonl 2>> gpurun_out/abt/err.txt || exit $?
    done
  done
done
