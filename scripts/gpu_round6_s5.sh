# Round-6 validation s5 (final: hdfs parallel deploy default, startup-order flags off): GPU tests, smoke, bench N=1 and the one-GPU rehearsal N=2/4/8, cluster mode
# 1 / 8 pods with and without GPU readiness, and the cluster-mode framework benches on both package
# sets (the reference's are staged in ref_inputs/ by scripts/stage_reference_inputs.sh).
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r6s5
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $out/pytest_gpu.txt 2>&1 && \
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.txt 2>&1 || exit $?
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 > $out/bench_n1_r$r.json 2> $out/bench_n1_r$r.err || exit $?
  for n in 2 4 8; do
    timeout -k 10 240 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
      --master-port $((29600 + n + RANDOM % 200)) bench.py --gpus $n --steps 20 --warmup 3 --dist-backend gloo \
      > $out/scale_n${n}_r$r.json 2> $out/scale_n${n}_r$r.err || exit $?
  done
done
run() {  # name, args...
  local name=$1; shift
  timeout -k 10 240 python -u -m dcos_commons_amd.benchmarks.cluster_bench "$@" > $out/cluster_$name.json 2> $out/cluster_$name.err
}
run n1_test --agents 1 --cycles 5 && \
run n1_service --agents 1 --cycles 5 --probe-service && \
run n8_test --agents 8 --cycles 5 && \
run n8_service --agents 8 --cycles 5 --probe-service || exit $?
for fw in cassandra hdfs; do
  for s in reference repo; do
    timeout -k 10 400 python -u -m dcos_commons_amd.benchmarks.framework_cluster_bench --framework $fw --specs $s \
      --cycles 5 --warmup 1 > $out/fwcluster_${fw}_${s}.json 2> $out/fwcluster_${fw}_${s}.err || exit $?
  done
done
python - <<'PY' > $out/summary.txt
import glob, json, os
for f in sorted(glob.glob("gpurun_out/r6s5/*.json")):
    for line in open(f):
        if not line.startswith("{"):
            continue
        d = json.loads(line)
        name = os.path.basename(f)[:-5]
        if "deploy_s" in d and "mttr_restart_s" in d:
            print("%-22s deploy %7.2f ms  restart %6.2f  replace %6.2f" % (
                name, d["deploy_s"]["mean"] * 1e3, d["mttr_restart_s"]["mean"] * 1e3, d["mttr_replace_s"]["mean"] * 1e3))
        else:
            print("%-22s %s" % (name, {k: round(v["median"] * 1e3, 1) for k, v in d.items()
                                       if isinstance(v, dict) and "median" in v}))
PY
cat $out/summary.txt
