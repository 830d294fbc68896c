# Framework benches on one MI355X box (needs scripts/stage_reference_inputs.sh): three runs of
# 1 warm-up + 5 timed cycles each, on the reference's unchanged packages and the repo's.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/fw
for i in 1 2 3; do
  timeout -k 10 300 python -u -m dcos_commons_amd.benchmarks.framework_bench --cycles 5 --warmup 1 2>/dev/null \
    | grep '^{' >> gpurun_out/fw/bench.jsonl || exit $?
done
