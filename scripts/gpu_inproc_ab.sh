# Same-box interleaved in-process A/B (scripts/dev/ab_deploy.py --gpu: the HIP readiness probe,
# 30 cycles per run): ab_trees/head (the previous commit) against this tree, N=1 and N=8, 3 rounds.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/iab
for i in 1 2 3; do
  if [ $((i % 2)) -eq 1 ]; then order="ab_trees/head ."; else order=". ab_trees/head"; fi
  for n in 1 8; do
    for tree in $order; do
      timeout -k 10 200 python scripts/dev/ab_deploy.py $tree $n 30 --gpu >> gpurun_out/iab/res.jsonl 2>> gpurun_out/iab/err.txt || exit $?
    done
  done
done
