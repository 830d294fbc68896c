# Same-box A/B of bench.py's two topologies on ONE MI355X: in-process (one interpreter holds the
# scheduler, the master and every agent's task lifecycle) vs split (master process; every agent,
# i.e. every rank, runs its own tasks and HIP readiness probe; scheduler over the framed v1
# stream). N ranks share the GPU over gloo (a rehearsal of the driver's N=1,2,4,8 run).
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/topology_ab
mkdir -p $out
run() {  # topology n round
  local t=$1 n=$2 r=$3
  if [ "$n" = 1 ]; then
    timeout -k 10 200 python -u bench.py --steps ${STEPS:-10} --warmup 2 --topology $t --reference-steps 2 \
      > $out/${t}_n${n}_r${r}.json 2> $out/${t}_n${n}_r${r}.err
  else
    timeout -k 10 240 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
      --master-port $((29600 + n + 10 * r)) bench.py --gpus $n --steps ${STEPS:-10} --warmup 2 --dist-backend gloo \
      --topology $t --reference-steps 2 > $out/${t}_n${n}_r${r}.json 2> $out/${t}_n${n}_r${r}.err
  fi
}
for r in 1 2; do
  for n in 1 8 2 4; do
    for t in inprocess split; do
      run $t $n $r || exit $?
    done
  done
done
python - <<'EOF'
import glob, json, os
rows = []
for f in sorted(glob.glob("gpurun_out/topology_ab/*.json")):
    for line in open(f):
        if line.startswith("{"):
            d = json.loads(line)
            rows.append((os.path.basename(f)[:-5], d["deploy_s"]["mean"] * 1e3, d["mttr_restart_s"]["mean"] * 1e3,
                         d["mttr_replace_s"]["mean"] * 1e3, d["ms_per_step"],
                         (d.get("reference_spec") or {}).get("deploy_s", {}).get("mean", 0) * 1e3))
for r in rows:
    print("%-22s deploy %7.2f ms  restart %6.2f  replace %6.2f  step %7.2f  ref-serial %6.2f" % r)
EOF
