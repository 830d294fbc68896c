# A/B of SDK_EARLY_SUBSCRIBE (SUBSCRIBE before the API server starts): bench.py N=1 and the one-GPU
# N=8 rehearsal, interleaved, 4 rounds.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/early_ab
mkdir -p $out
for r in 1 2 3 4; do
  for v in false true; do
    SDK_EARLY_SUBSCRIBE=$v timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 > $out/n1_${v}_r$r.json 2> $out/n1_${v}_r$r.err || exit $?
    SDK_EARLY_SUBSCRIBE=$v timeout -k 10 240 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
      --master-port $((29600 + RANDOM % 400)) bench.py --gpus 8 --steps 20 --warmup 3 --dist-backend gloo \
      > $out/n8_${v}_r$r.json 2> $out/n8_${v}_r$r.err || exit $?
  done
done
python - <<'PY' > $out/summary.txt
import glob, json, os
for f in sorted(glob.glob("gpurun_out/early_ab/*.json")):
    for line in open(f):
        if line.startswith('{"metric'):
            d = json.loads(line)
            print("%-16s %.3f ms/step  %s" % (os.path.basename(f)[:-5], d["ms_per_step"], d.get("value")))
PY
cat $out/summary.txt
