# Box: split-topology timelines (1 and 8 pods, HIP probe in the agent processes), a cProfile of the
# scheduler side of an 8-pod deploy, and an interleaved A/B of the tree in ./ab_base_r06 (A) against
# this tree (B) through bench.py (N=1 single process; N=8 torchrun over gloo, all ranks on the card).
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/split_prof_r06
mkdir -p $out
timeout -k 10 120 python -u scripts/dev/split_timeline.py 1 --probe > $out/timeline_n1.txt 2>&1 || exit $?
timeout -k 10 120 python -u scripts/dev/split_timeline.py 8 --probe > $out/timeline_n8.txt 2>&1 || exit $?
timeout -k 10 180 python -u scripts/dev/prof_split_cycle.py 8 --cycles 30 --sort cumtime --limit 80 > $out/prof_n8_cum.txt 2>&1 || exit $?
timeout -k 10 180 python -u scripts/dev/prof_split_cycle.py 8 --cycles 30 --sort tottime --limit 50 > $out/prof_n8_tot.txt 2>&1 || exit $?
run() {  # tree name n [bench args]
  local dir=$1 name=$2 n=$3; shift 3
  if [ "$n" = 1 ]; then
    (cd $dir && timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --reference-steps 0 "$@") > $out/${name}_n$n.json 2> $out/${name}_n$n.err
  else
    (cd $dir && timeout -k 10 240 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
      --master-port $((29600 + n + RANDOM % 200)) bench.py --gpus $n --steps 20 --warmup 3 --dist-backend gloo \
      --reference-steps 0 "$@") > $out/${name}_n$n.json 2> $out/${name}_n$n.err
  fi
}
for r in 1 2 3; do
  for n in 1 8; do
    run ab_base_r06 A_r$r $n || exit $?
    run . B_r$r $n || exit $?
    run . C_nogate_r$r $n --sched-env SDK_STATUS_CYCLE_WAIT_MS=0 || exit $?
  done
done
python - <<'PY' > gpurun_out/split_prof_r06/ab.txt
import glob, json, os
for f in sorted(glob.glob("gpurun_out/split_prof_r06/[ABC]_*.json")):
    for line in open(f):
        if line.startswith("{"):
            d = json.loads(line)
            print("%-10s deploy %6.2f ms  restart %5.2f  replace %5.2f  step %6.2f" % (
                os.path.basename(f)[:-5], d["deploy_s"]["mean"] * 1e3, d["mttr_restart_s"]["mean"] * 1e3,
                d["mttr_replace_s"]["mean"] * 1e3, d["ms_per_step"]))
PY
cat gpurun_out/split_prof_r06/ab.txt
