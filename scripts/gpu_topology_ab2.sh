# Same-box A/B: in-process vs split topology (after the agent runtime runs launches inline), and the
# split topology with a 0.5 ms interpreter switch interval in the master / agent processes.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/topology_ab2
mkdir -p $out
run() {  # name n extra-args...
  local name=$1 n=$2; shift 2
  if [ "$n" = 1 ]; then
    timeout -k 10 200 python -u bench.py --steps 10 --warmup 2 --reference-steps 0 "$@" > $out/${name}_n$n.json 2> $out/${name}_n$n.err
  else
    timeout -k 10 240 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
      --master-port $((29600 + n + RANDOM % 200)) bench.py --gpus $n --steps 10 --warmup 2 --dist-backend gloo \
      --reference-steps 0 "$@" > $out/${name}_n$n.json 2> $out/${name}_n$n.err
  fi
}
for r in 1 2; do
  for n in 1 8; do
    run inprocess_r$r $n --topology inprocess || exit $?
    run split_r$r $n --topology split || exit $?
    run split_si05_r$r $n --topology split --cluster-switch-interval-ms 0.5 || exit $?
    run split_si05_s05_r$r $n --topology split --cluster-switch-interval-ms 0.5 --sched-env SDK_GIL_SWITCH_INTERVAL_MS=0.5 || exit $?
  done
done
python - <<'PY'
import glob, json, os
for f in sorted(glob.glob("gpurun_out/topology_ab2/*.json")):
    for line in open(f):
        if line.startswith("{"):
            d = json.loads(line)
            print("%-26s deploy %6.2f ms  restart %5.2f  replace %5.2f  step %6.2f" % (
                os.path.basename(f)[:-5], d["deploy_s"]["mean"] * 1e3, d["mttr_restart_s"]["mean"] * 1e3,
                d["mttr_replace_s"]["mean"] * 1e3, d["ms_per_step"]))
PY
