# Round-6 end: bench.py N=1 and the one-GPU rehearsal N=2/4/8 at HEAD, three rounds (auto backend:
# gloo, since the ranks share the card).
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r6final_scale
mkdir -p $out
for r in 1 2 3; do
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 > $out/n1_r$r.json 2> $out/n1_r$r.err || exit $?
  for n in 2 4 8; do
    timeout -k 10 240 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
      --master-port $((29600 + n + RANDOM % 200)) bench.py --gpus $n --steps 20 --warmup 3 \
      > $out/n${n}_r$r.json 2> $out/n${n}_r$r.err || exit $?
  done
done
cat $out/n*_r*.json | grep '^{"metric' > $out/all.jsonl
