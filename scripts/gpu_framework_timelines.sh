# Framework deploy timelines on one MI355X box (needs scripts/stage_reference_inputs.sh): one traced
# cycle of each framework on the reference's unchanged package and the repo's, plus two more
# framework bench runs for the spread.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/fwtl
for fw in cassandra hdfs; do
  for specs in reference repo; do
    SDK_TRACE=1 timeout -k 10 120 python -u scripts/dev/framework_timeline.py $fw $specs -v \
      > gpurun_out/fwtl/${fw}_${specs}.txt 2>&1 || exit $?
  done
done
for i in 1 2; do
  timeout -k 10 300 python -u -m dcos_commons_amd.benchmarks.framework_bench --cycles 5 2>/dev/null \
    | grep '^{' >> gpurun_out/fwtl/bench.jsonl || exit $?
done
