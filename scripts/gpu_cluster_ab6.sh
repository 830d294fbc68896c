# Same-box interleaved cluster-mode A/B (round 5): the scheduler process's interpreter switch
# interval (SDK_GIL_SWITCH_INTERVAL_MS) at Python's 5 ms vs 0.5 ms, with the cluster process at its
# 0.5 ms default. 8 and 1 pods, 6 cycles per run, 4 rounds, order alternating.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/cab6
run() {  # label n extra...
  local label=$1 n=$2; shift 2
  timeout -k 10 240 python -u -m dcos_commons_amd.benchmarks.cluster_bench --agents $n --cycles 6 "$@" \
    2>> gpurun_out/cab6/err.txt | sed "s|^|$label n$n |" >> gpurun_out/cab6/res.txt
}
for i in 1 2 3 4; do
  for n in 8 1; do
    if [ $((i % 2)) -eq 1 ]; then
      run base $n && run s05 $n --scheduler-env SDK_GIL_SWITCH_INTERVAL_MS=0.5 || exit $?
    else
      run s05 $n --scheduler-env SDK_GIL_SWITCH_INTERVAL_MS=0.5 && run base $n || exit $?
    fi
  done
done
