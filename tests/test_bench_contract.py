"""bench.py contract: one JSON line from rank 0, whole-job value, multi-rank path over gloo.

The driver launches ``bench.py`` under ``torch.distributed.run`` with one rank per GPU; here the
same path runs on CPU (gloo, world size 2, synthetic readiness) so the distributed agent links are
covered without a GPU. The N=1 case runs in-process.
"""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REQUIRED = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
            "vs_baseline", "dtype", "data", "config"}


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _json_lines(out: str):
    return [json.loads(l) for l in out.splitlines() if l.startswith("{")]


def _check(rec, n, steps, warmup):
    assert REQUIRED <= set(rec)
    baseline = json.load(open(os.path.join(ROOT, "BASELINE.json")))
    assert rec["metric"] == baseline["metric"]
    assert rec["n_gpus"] == n and rec["steps"] == steps and rec["warmup"] == warmup
    assert rec["higher_is_better"] is False and rec["scaling"] == "weak"
    assert rec["config"]["pods"] == n and rec["config"]["agents"] == n
    assert rec["value"] > 0 and rec["ms_per_step"] > 0
    assert rec["mttr_restart_s"]["mean"] > 0 and rec["mttr_replace_s"]["mean"] > 0
    assert 0 < rec["deploy_from_subscribed_s"]["mean"] < rec["value"]


def test_bench_single_process():
    env = dict(os.environ, PYTHONPATH=ROOT)
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "1", "--warmup", "0",
                        "--no-gpu-probe", "--allocation-interval", "0.05"],
                       capture_output=True, text=True, timeout=240, env=env, cwd=ROOT)
    assert p.returncode == 0, p.stderr[-2000:]
    recs = _json_lines(p.stdout)
    assert len(recs) == 1
    _check(recs[0], 1, 1, 0)


@pytest.mark.timeout(300)
def test_bench_two_ranks_over_gloo():
    env = dict(os.environ, PYTHONPATH=ROOT, MASTER_ADDR="127.0.0.1", OMP_NUM_THREADS="1")
    env.pop("CUDA_VISIBLE_DEVICES", None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1", "--warmup", "1", "--no-gpu-probe",
           "--allocation-interval", "0.05"]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=280, env=env, cwd=ROOT)
    assert p.returncode == 0, p.stderr[-3000:]
    recs = _json_lines(p.stdout)
    assert len(recs) == 1, p.stdout            # only rank 0 prints
    _check(recs[0], 2, 1, 1)
    assert recs[0]["config"]["parallelism"] == "agents2-ranks2"


def test_deploy_bench_waits_on_status_events():
    """The timed waits re-check the plan when a status was processed (no 1 ms polling)."""
    import threading
    import time

    from dcos_commons_amd.benchmarks.deploy_bench import DeployBench

    b = DeployBench(1, timeout_s=5)
    ev, state = threading.Event(), {"done": False, "checks": 0}

    def pred():
        state["checks"] += 1
        return state["done"]

    def finish():
        time.sleep(0.05)
        state["done"] = True
        ev.set()

    threading.Thread(target=finish).start()
    waited = b._wait(pred, "test", ev)
    assert state["done"] and 0.04 < waited < 1.0
    assert state["checks"] < 30          # woken by the event / 5 ms ticks, not a 1 ms poll loop
