# (Experiment record: the SDK_LAUNCH_YIELD_US flag was removed after this A/B, profiles/launch_yield_ab_r05_box.txt.)
# Same-box interleaved A/B of the offer loop's yield after each streamed launch
# (SDK_LAUNCH_YIELD_US) and of a 1 ms interpreter switch interval, on the one-GPU scaling rehearsal
# (N ranks share the card over gloo; remote ranks run the HIP readiness probe). 2 rounds.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/ly
run() {  # label n extra-args...
  local label=$1 n=$2; shift 2
  if [ "$n" = 1 ]; then
    timeout -k 10 240 python -u bench.py --steps 8 --warmup 1 --reference-steps 0 "$@" \
      2>> gpurun_out/ly/err.txt | sed "s|^|$label n$n |" >> gpurun_out/ly/res.txt
  else
    timeout -k 10 240 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
      --master-port $((29700 + n)) bench.py --gpus $n --steps 8 --warmup 1 --reference-steps 0 --dist-backend gloo "$@" \
      2>> gpurun_out/ly/err.txt | grep '^{' | sed "s|^|$label n$n |" >> gpurun_out/ly/res.txt
  fi
}
for i in 1 2; do
  for n in 8 1; do
    run base $n || exit $?
    run y0 $n --sched-env SDK_LAUNCH_YIELD_US=0 || exit $?
    run y50 $n --sched-env SDK_LAUNCH_YIELD_US=50 || exit $?
    run gil1 $n --sched-env SDK_GIL_SWITCH_INTERVAL_MS=1 || exit $?
  done
done
