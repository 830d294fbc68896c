# Interleaved same-box A/B of the round-4 final tree (ab_trees/old) against this tree, with the real
# HIP readiness probe (ab_deploy.py --gpu), N=1 and N=8 pods, plus an 8-pod deploy timeline of this tree.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/abt gpurun_out/timeline
for i in 1 2 3; do
  if [ $((i % 2)) -eq 1 ]; then order="ab_trees/old ."; else order=". ab_trees/old"; fi
  for n in 1 8; do
    for tree in $order; do
      timeout -k 10 200 python scripts/dev/ab_deploy.py $tree $n 30 --gpu >> gpurun_out/abt/res.jsonl 2>> gpurun_out/abt/err.txt || exit $?
    done
  done
done
SDK_TRACE=1 timeout -k 10 120 python -u scripts/dev/deploy_timeline.py 8 --gpu > gpurun_out/timeline/n8.txt 2>&1 && \
SDK_TRACE=1 timeout -k 10 120 python -u scripts/dev/deploy_timeline.py 1 --gpu > gpurun_out/timeline/n1.txt 2>&1
