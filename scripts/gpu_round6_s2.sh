# Round-6 validation s2 (after the status gate, template moves, agent-0 process, prewarm): GPU tests,
# smoke, bench N=1 twice, the one-GPU scaling rehearsal N=2/4/8 (torchrun over gloo, every rank on
# the card) twice, split timelines for 1 and 8 pods, and a rocprofv3 kernel trace of one bench step.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r6s2
mkdir -p $out/prof
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
for n in 1 8; do
  timeout -k 10 120 python -u scripts/dev/split_timeline.py $n --probe > $out/timeline_n$n.txt 2>&1 || exit $?
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof/bench -o bench -- python3 bench.py --steps 1 --warmup 0 \
  --topology inprocess --reference-steps 0 > $out/prof/bench_stdout.txt 2>&1 || exit $?
python - <<'PY' > $out/summary.txt
import glob, json, os
for f in sorted(glob.glob("gpurun_out/r6s2/*_r[12].json")):
    for line in open(f):
        if line.startswith("{"):
            d = json.loads(line)
            print("%-16s deploy %6.2f ms  from-subscribed %6.2f  restart %5.2f  replace %5.2f  step %6.2f  ref-serial %s" % (
                os.path.basename(f)[:-5], d["deploy_s"]["mean"] * 1e3, d["deploy_from_subscribed_s"]["mean"] * 1e3,
                d["mttr_restart_s"]["mean"] * 1e3, d["mttr_replace_s"]["mean"] * 1e3, d["ms_per_step"],
                d.get("reference_spec", {}).get("deploy_s", {}).get("mean")))
PY
cat $out/summary.txt
