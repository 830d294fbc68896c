# Interleaved A/B of two source trees on the box (synthetic readiness): ab_trees/old vs this tree.
set -o pipefail
mkdir -p gpurun_out/abt
for i in 1 2 3; do
  (cd ab_trees/old && timeout -k 10 200 python scripts/ab_profiles.py --agents 1 8 --reps 10 --profile old=) >> gpurun_out/abt/res.jsonl 2>> gpurun_out/abt/err.txt || exit $?
  timeout -k 10 200 python scripts/ab_profiles.py --agents 1 8 --reps 10 --profile new= >> gpurun_out/abt/res.jsonl 2>> gpurun_out/abt/err.txt || exit $?
done
