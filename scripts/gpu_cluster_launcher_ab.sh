# Same-box interleaved A/Bs in cluster mode (8 pods, this tree): the local agents' launcher thread
# (SDK_AGENT_LAUNCHER_THREAD, the bench process) and a 1 ms interpreter switch interval in the
# scheduler process (SDK_GIL_SWITCH_INTERVAL_MS); then 1 pod for each launcher setting and an
# 8-pod timeline.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/launcher_ab
run() {  # label, launcher, extra args...
  local label=$1 l=$2; shift 2
  SDK_AGENT_LAUNCHER_THREAD=$l timeout -k 10 240 python -u -m dcos_commons_amd.benchmarks.cluster_bench --cycles 5 "$@" \
    | sed "s|^|$label |" >> gpurun_out/launcher_ab/res.txt 2>> gpurun_out/launcher_ab/err.txt
}
for i in 1 2 3; do
  if [ $((i % 2)) -eq 1 ]; then order="0 1"; else order="1 0"; fi
  for l in $order; do run "launcher=$l n8" $l --agents 8 || exit $?; done
  run "launcher=1 switch=1ms n8" 1 --agents 8 --scheduler-env SDK_GIL_SWITCH_INTERVAL_MS=1 || exit $?
done
for l in 0 1; do run "launcher=$l n1" $l --agents 1 || exit $?; done
SDK_AGENT_LAUNCHER_THREAD=1 PYTHONPATH=. timeout -k 10 240 python -u scripts/dev/cluster_timeline.py 8 3 > gpurun_out/launcher_ab/timeline_n8.txt 2>&1
