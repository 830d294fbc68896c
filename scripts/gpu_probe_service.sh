# GPU readiness service on one MI355X box: its GPU tests, then the cluster-mode bench with the
# per-check HIP probe binary vs the resident service (same box, back to back).
set -o pipefail
mkdir -p gpurun_out/svc
timeout -k 10 400 python -u -m pytest tests/test_probe_service.py -m gpu -x -v --timeout 200 --timeout-method thread \
  > gpurun_out/svc/pytest.txt 2>&1 && \
timeout -k 10 300 python -u -m dcos_commons_amd.benchmarks.cluster_bench --agents 1 --cycles 5 --probe-service \
  > gpurun_out/svc/n1_service.json 2> gpurun_out/svc/n1_service.err && \
timeout -k 10 300 python -u -m dcos_commons_amd.benchmarks.cluster_bench --agents 1 --cycles 5 \
  --probe-cmd "$GRAFT_REPO_ROOT/native/build/amd-gpu-probe --readiness" \
  > gpurun_out/svc/n1_probe.json 2> gpurun_out/svc/n1_probe.err
