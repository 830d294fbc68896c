# Interleaved A/B of two source trees on the one-GPU box in the multi-rank bench: ab_trees/old vs
# this tree, N ranks sharing the card over gloo (AB_N, default 8), AB_ITERS alternating rounds.
set -o pipefail
mkdir -p gpurun_out/abr
N=${AB_N:-8}; ITERS=${AB_ITERS:-2}; PORT=29700
for i in $(seq 1 $ITERS); do
  if [ $((i % 2)) -eq 1 ]; then order="ab_trees/old ."; else order=". ab_trees/old"; fi
  for tree in $order; do
    PORT=$((PORT + 1))
    (cd $tree && timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node $N \
      --master-addr 127.0.0.1 --master-port $PORT bench.py --gpus $N --steps 10 --warmup 2 --dist-backend gloo) \
      2>> gpurun_out/abr/err.txt | grep metric | sed "s#^#$tree #" >> gpurun_out/abr/res.txt || exit $?
  done
done
