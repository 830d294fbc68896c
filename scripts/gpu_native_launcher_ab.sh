# Same-box interleaved cluster-mode A/B of the native agent launcher (SDK_NATIVE_AGENT_LAUNCHER:
# task processes and checks started by native/build/sdk-agent-launcher, or by the master's
# interpreter), 8 and 1 pods, 3 rounds; then an 8-pod timeline with it on.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/nl
for i in 1 2 3; do
  if [ $((i % 2)) -eq 1 ]; then order="0 1"; else order="1 0"; fi
  for n in 8 1; do
    for v in $order; do
      SDK_NATIVE_AGENT_LAUNCHER=$v timeout -k 10 240 python -u -m dcos_commons_amd.benchmarks.cluster_bench --agents $n --cycles 5 \
        | sed "s|^|native=$v n$n |" >> gpurun_out/nl/res.txt 2>> gpurun_out/nl/err.txt || exit $?
    done
  done
done
SDK_NATIVE_AGENT_LAUNCHER=1 PYTHONPATH=. timeout -k 10 240 python -u scripts/dev/cluster_timeline.py 8 3 > gpurun_out/nl/timeline_n8.txt 2>&1
