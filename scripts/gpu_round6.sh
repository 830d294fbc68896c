# Round-6 validation on one MI355X: GPU tests, smoke, bench N=1 (split topology, the default; the
# in-process topology and the reference cadence for comparison), the one-GPU scaling rehearsal in
# both topologies, a rocprofv3 kernel trace of one bench step (in-process topology: nothing is
# spawned under the profiler), and the cluster-mode framework benches (BASELINE configs 3/4) on the
# reference's unchanged packages (staged in ref_inputs/) and on this repository's.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r6
mkdir -p $out/prof
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $out/pytest_gpu.txt 2>&1 && \
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.txt 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 > $out/bench_n1_split.json 2> $out/bench_n1_split.err && \
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --topology inprocess > $out/bench_n1_inprocess.json 2> $out/bench_n1_inprocess.err && \
timeout -k 10 300 python -u bench.py --steps 2 --warmup 0 --profile reference --reference-steps 0 > $out/bench_n1_refcadence.json 2> $out/bench_n1_refcadence.err || exit $?
for n in 2 4 8; do
  for t in split inprocess; do
    timeout -k 10 240 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
      --master-port $((29600 + n)) bench.py --gpus $n --steps 10 --warmup 2 --dist-backend gloo --topology $t \
      > $out/scale_${t}_n$n.json 2> $out/scale_${t}_n$n.err || exit $?
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof/bench -o bench -- python3 bench.py --steps 1 --warmup 0 \
  --topology inprocess --reference-steps 0 > $out/prof/bench_stdout.txt 2>&1 || exit $?
find $out/prof -name "*stats*" > $out/prof/files.txt
for fw in cassandra hdfs; do
  for s in reference repo; do
    timeout -k 10 400 python -u -m dcos_commons_amd.benchmarks.framework_cluster_bench --framework $fw --specs $s \
      --cycles 5 --warmup 1 > $out/fwcluster_${fw}_${s}.json 2> $out/fwcluster_${fw}_${s}.err || exit $?
  done
done
echo done
