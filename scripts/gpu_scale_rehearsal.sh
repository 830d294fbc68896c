# Rehearsal of the driver's N=1,2,4,8 scaling run on ONE MI355X: N ranks share the GPU
# (gloo collectives, since RCCL refuses two ranks on one device). Every rank runs the real HIP
# readiness probe on the shared card. Not the official scaling measurement.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/scale
timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 > gpurun_out/scale/n1.json 2> gpurun_out/scale/n1.err || exit $?
for n in 2 4 8; do
  timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
    --master-port $((29600 + n)) bench.py --gpus $n --steps 5 --warmup 1 --dist-backend gloo \
    > gpurun_out/scale/n$n.json 2> gpurun_out/scale/n$n.err || exit $?
done
