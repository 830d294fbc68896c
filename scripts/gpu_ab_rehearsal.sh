# A/B of one scheduler flag in the 8-rank one-GPU rehearsal (real HIP probe per rank).
# usage: bash scripts/gpu_ab_rehearsal.sh KEY=VALUE
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
for i in 1 2; do
  for arm in base alt; do
    extra=""; [ "$arm" = alt ] && extra="--sched-env $1"
    timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
      --master-port $((29700 + i)) bench.py --gpus 8 --steps 8 --warmup 1 --dist-backend gloo $extra \
      >> gpurun_out/ab/$arm.jsonl 2>> gpurun_out/ab/$arm.err || exit $?
  done
done
