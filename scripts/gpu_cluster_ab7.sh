# (Experiment record: SDK_MESOS_CALL_LANES was removed after this A/B, profiles/call_lanes_ab_r05_box.txt.)
# Same-box interleaved cluster-mode A/B (round 5): the v1 driver's call lanes
# (SDK_MESOS_CALL_LANES) 1 (one sender, one connection) vs 4 (per-agent lanes). 8 and 1 pods,
# 6 cycles per run, 4 rounds, order alternating.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/cab7
run() {  # label n extra...
  local label=$1 n=$2; shift 2
  timeout -k 10 240 python -u -m dcos_commons_amd.benchmarks.cluster_bench --agents $n --cycles 6 "$@" \
    2>> gpurun_out/cab7/err.txt | sed "s|^|$label n$n |" >> gpurun_out/cab7/res.txt
}
for i in 1 2 3 4; do
  for n in 8 1; do
    if [ $((i % 2)) -eq 1 ]; then
      run base $n && run lanes4 $n --scheduler-env SDK_MESOS_CALL_LANES=4 || exit $?
    else
      run lanes4 $n --scheduler-env SDK_MESOS_CALL_LANES=4 && run base $n || exit $?
    fi
  done
done
