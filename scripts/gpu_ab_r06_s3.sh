# Same-box interleaved A/B of this tree's bench (split topology): default vs SDK_OFFER_PREWARM=false,
# and vs SDK_AGENT_REPORT_WINDOW_MS=0; N=1 single process, N=8 torchrun over gloo (all ranks on the
# card); then the default's split timelines.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/ab_r06_s3
mkdir -p $out
run() {  # name n window_ms [bench args]
  local name=$1 n=$2 w=$3; shift 3
  if [ "$n" = 1 ]; then
    SDK_AGENT_REPORT_WINDOW_MS=$w timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --reference-steps 0 "$@" \
      > $out/${name}_n$n.json 2> $out/${name}_n$n.err
  else
    SDK_AGENT_REPORT_WINDOW_MS=$w timeout -k 10 240 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
      --master-addr 127.0.0.1 --master-port $((29600 + n + RANDOM % 200)) bench.py --gpus $n --steps 20 --warmup 3 \
      --dist-backend gloo --reference-steps 0 "$@" > $out/${name}_n$n.json 2> $out/${name}_n$n.err
  fi
}
for r in 1 2 3; do
  for n in 1 8; do
    run default_r$r $n 2 || exit $?
    run noprewarm_r$r $n 2 --sched-env SDK_OFFER_PREWARM=false || exit $?
    run nowindow_r$r $n 0 || exit $?
  done
done
for n in 1 8; do
  timeout -k 10 120 python -u scripts/dev/split_timeline.py $n --probe > $out/timeline_n$n.txt 2>&1 || exit $?
done
python - <<'PY' > $out/ab.txt
import glob, json, os
for f in sorted(glob.glob("gpurun_out/ab_r06_s3/*_r*_n*.json")):
    for line in open(f):
        if line.startswith("{"):
            d = json.loads(line)
            print("%-18s deploy %6.2f ms  from-subscribed %6.2f  restart %5.2f  replace %5.2f  step %6.2f" % (
                os.path.basename(f)[:-5], d["deploy_s"]["mean"] * 1e3, d["deploy_from_subscribed_s"]["mean"] * 1e3,
                d["mttr_restart_s"]["mean"] * 1e3, d["mttr_replace_s"]["mean"] * 1e3, d["ms_per_step"]))
PY
cat $out/ab.txt
