# Interleaved A/B of two source trees on the box: ab_trees/old vs this tree, helloworld DeployBench
# (synthetic readiness) pinned to CPUs 4-7, N = 1 and 8.
set -o pipefail
mkdir -p gpurun_out/abt
for i in 1 2 3; do
  for n in 1 8; do
    timeout -k 10 200 python scripts/dev/ab_deploy.py ab_trees/old $n 30 >> gpurun_out/abt/res.jsonl 2>> gpurun_out/abt/err.txt || exit $?
    timeout -k 10 200 python scripts/dev/ab_deploy.py . $n 30 >> gpurun_out/abt/res.jsonl 2>> gpurun_out/abt/err.txt || exit $?
  done
done
