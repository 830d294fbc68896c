# Box: where does agent 0 belong? Split-topology timelines with agent 0 in its own process vs on a
# thread of the scheduler's process (1 and 8 pods, HIP probe), then bench.py interleaved with
# --agent0 thread (default) vs process: N=1 single process, N=8 torchrun over gloo (all ranks on the card).
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/agent0_r06
mkdir -p $out
for a in process thread; do
  for n in 1 8; do
    timeout -k 10 120 python -u scripts/dev/split_timeline.py $n --probe --agent0 $a > $out/timeline_${a}_n$n.txt 2>&1 || exit $?
  done
done
run() {  # name n [bench args]
  local name=$1 n=$2; shift 2
  if [ "$n" = 1 ]; then
    timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --reference-steps 0 "$@" > $out/${name}_n$n.json 2> $out/${name}_n$n.err
  else
    timeout -k 10 240 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
      --master-port $((29600 + n + RANDOM % 200)) bench.py --gpus $n --steps 20 --warmup 3 --dist-backend gloo \
      --reference-steps 0 "$@" > $out/${name}_n$n.json 2> $out/${name}_n$n.err
  fi
}
for r in 1 2 3; do
  for n in 1 8; do
    run thread_r$r $n --agent0 thread || exit $?
    run process_r$r $n --agent0 process || exit $?
  done
done
python - <<'PY' > gpurun_out/agent0_r06/ab.txt
import glob, json, os
for f in sorted(glob.glob("gpurun_out/agent0_r06/*_r*_n*.json")):
    for line in open(f):
        if line.startswith("{"):
            d = json.loads(line)
            print("%-16s deploy %6.2f ms  from-subscribed %6.2f  restart %5.2f  replace %5.2f  step %6.2f" % (
                os.path.basename(f)[:-5], d["deploy_s"]["mean"] * 1e3, d["deploy_from_subscribed_s"]["mean"] * 1e3,
                d["mttr_restart_s"]["mean"] * 1e3, d["mttr_replace_s"]["mean"] * 1e3, d["ms_per_step"]))
PY
cat gpurun_out/agent0_r06/ab.txt
