# (Experiment record: SDK_STATUS_UPDATE_WINDOW_US was removed after this A/B, profiles/status_window_ab_r05_box.txt.)
# Same-box interleaved cluster-mode A/B (round 5): the v1 driver's status update window
# (SDK_STATUS_UPDATE_WINDOW_US) 0 vs 300 us. 8 and 1 pods, 6 cycles per run, 4 rounds, order alternating.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/cab8
run() {  # label n extra...
  local label=$1 n=$2; shift 2
  timeout -k 10 240 python -u -m dcos_commons_amd.benchmarks.cluster_bench --agents $n --cycles 6 "$@" \
    2>> gpurun_out/cab8/err.txt | sed "s|^|$label n$n |" >> gpurun_out/cab8/res.txt
}
for i in 1 2 3 4; do
  for n in 8 1; do
    if [ $((i % 2)) -eq 1 ]; then
      run base $n && run w300 $n --scheduler-env SDK_STATUS_UPDATE_WINDOW_US=300 || exit $?
    else
      run w300 $n --scheduler-env SDK_STATUS_UPDATE_WINDOW_US=300 && run base $n || exit $?
    fi
  done
done
