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


@pytest.mark.timeout(400)
def test_bench_four_ranks_build_agents_from_what_each_rank_registers(tmp_path):
    """The driver's N-GPU run, rehearsed on CPU: 4 ranks over gloo, each discovering "its" GPU
    from a recorded-format KFD tree of a 4-GPU node in two xGMI hives (``ops.gpu``). Checks that
    the offers came from each rank's registration (hostname, device, model, hive), every
    readiness check ran on the registering rank's own device, and the JSON reports n_gpus=4 with
    the time MAX-reduced over the ranks."""
    from dcos_commons_amd.ops import gpu as G

    fixture = tmp_path / "node"
    G.synthetic_kfd_tree(str(fixture / "kfd"), [0xA1, 0xA1, 0xB2, 0xB2])
    record = tmp_path / "record"
    env = dict(os.environ, PYTHONPATH=ROOT, MASTER_ADDR="127.0.0.1", OMP_NUM_THREADS="1",
               SDK_GPU_DISCOVERY_FIXTURE=str(fixture), SDK_BENCH_RECORD=str(record))
    env.pop("CUDA_VISIBLE_DEVICES", None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "4",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(ROOT, "bench.py"), "--gpus", "4", "--steps", "2", "--warmup", "1", "--no-gpu-probe",
           "--allocation-interval", "0.05", "--reference-steps", "1"]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=380, env=env, cwd=ROOT)
    assert p.returncode == 0, p.stderr[-3000:]
    recs = _json_lines(p.stdout)
    assert len(recs) == 1, p.stdout
    rec = recs[0]
    _check(rec, 4, 2, 1)
    assert rec["config"]["parallelism"] == "agents4-ranks4"
    assert rec["reference_spec"]["pods"] == 4 and rec["reference_spec"]["plan"] == "default serial deploy"
    ranks = {r: json.load(open(record / f"rank{r}.json")) for r in range(4)}
    hive = {0: "a1", 1: "a1", 2: "b2", 3: "b2"}
    for r, data in ranks.items():
        assert data["device"] == r and data["registered"]["devices"] == [r]
        assert data["registered"]["attributes"]["xgmi_hive"] == hive[r]
        # every check this rank served was for its own device, and ran there (rank 0's agent is a
        # process of its own by default: its checks are in its own record)
        checks = data["checks"] or json.load(open(record / f"agent{r}.json"))["checks"]
        assert checks and all(tuple(a) == (r,) and d == r and ok for a, d, ok in checks)
    # the agents rank 0 offered are exactly what the ranks registered
    agents = {a["hostname"]: a for a in ranks[0]["agents"]}
    for r, data in ranks.items():
        a = agents[data["registered"]["hostname"]]
        assert a["gpu_devices"] == [r] and a["attributes"]["xgmi_hive"] == hive[r]
        assert a["attributes"]["gpu_model"] == "MI355X" and a["attributes"]["gpu_arch"] == "gfx950"
    # one hello pod per agent (hostname:UNIQUE), each on that agent's device
    placed = {x["hostname"]: x for x in ranks[0]["placement"] if x["task"].startswith("hello-")}
    assert len(placed) == 4
    for host, x in placed.items():
        assert x["gpu_devices"] == agents[host]["gpu_devices"]
    # the reported time is the MAX over the ranks' own views of the timed window
    elapsed = [d["elapsed_local_s"] for d in ranks.values()]
    assert all(d["elapsed_max_s"] == max(elapsed) for d in ranks.values())
    assert abs(rec["ms_per_step"] - max(elapsed) * 1000 / 2) < 0.01


@pytest.mark.timeout(300)
@pytest.mark.parametrize("agent0", ["thread", "process"])
def test_bench_two_ranks_over_gloo(agent0):
    """Two ranks; rank 0's agent on a thread of the scheduler's process or in a process of its own."""
    env = dict(os.environ, PYTHONPATH=ROOT, MASTER_ADDR="127.0.0.1", OMP_NUM_THREADS="1")
    env.pop("CUDA_VISIBLE_DEVICES", None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1", "--warmup", "1", "--no-gpu-probe",
           "--allocation-interval", "0.05", "--agent0", agent0]
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


@pytest.mark.timeout(300)
def test_bench_single_process_with_agent_processes(tmp_path):
    """``--gpus 3 --agent0 thread`` without torchrun: the master process plus two helper agent
    processes (``parallel.agent_process``); the bench process is agent 0. One pod per agent."""
    record = tmp_path / "record"
    env = dict(os.environ, PYTHONPATH=ROOT, SDK_BENCH_RECORD=str(record))
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "3", "--steps", "1", "--warmup", "1",
                        "--no-gpu-probe", "--allocation-interval", "0.05", "--reference-steps", "1",
                        "--agent0", "thread"],
                       capture_output=True, text=True, timeout=280, env=env, cwd=ROOT)
    assert p.returncode == 0, p.stderr[-3000:]
    recs = _json_lines(p.stdout)
    assert len(recs) == 1
    rec = recs[0]
    _check(rec, 3, 1, 1)
    assert rec["config"]["topology"].startswith("split") and rec["config"]["agent_processes"] == 3
    data = json.load(open(record / "rank0.json"))
    assert sorted(a["rank"] for a in data["agents"]) == [0, 1, 2]
    hosts = {a["hostname"] for a in data["agents"]}
    placed = [x for x in data["placement"] if x["task"].startswith("hello-")]
    assert len(placed) == 3 and {x["hostname"] for x in placed} == hosts     # hostname:UNIQUE, one per agent
    assert data["checks"] and all(ok for _, _, ok in data["checks"])       # agent 0's checks ran here


def test_bench_inprocess_topology():
    env = dict(os.environ, PYTHONPATH=ROOT)
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1", "--warmup", "0",
                        "--no-gpu-probe", "--allocation-interval", "0.05", "--topology", "inprocess",
                        "--reference-steps", "0"],
                       capture_output=True, text=True, timeout=240, env=env, cwd=ROOT)
    assert p.returncode == 0, p.stderr[-2000:]
    rec = _json_lines(p.stdout)[0]
    _check(rec, 2, 1, 0)
    assert "topology" not in rec["config"]


@pytest.mark.parametrize("env", [{"SDK_EARLY_SUBSCRIBE": "true"}, {"SDK_THREAD_PRESTART": "before"},
                                 {"SDK_THREAD_PRESTART": "after", "SDK_EARLY_SUBSCRIBE": "true"}])
def test_startup_order_flags_deploy_and_recover(monkeypatch, env):
    """SUBSCRIBE before the API server (early offers wait for it) and the offer-loop threads created
    ahead of registration: a deploy, a restart and a replace still complete, and no offer was
    declined for want of the API server."""
    from dcos_commons_amd.benchmarks.deploy_bench import DeployBench
    from dcos_commons_amd.framework import framework_scheduler as FS

    for k, v in env.items():
        monkeypatch.setenv(k, v)
    declined = []
    orig = FS.decline_short
    monkeypatch.setattr(FS, "decline_short", lambda offers, *a, **k: (declined.extend(offers), orig(offers, *a, **k)))
    r = DeployBench(1, timeout_s=20, allocation_interval_s=0.05).run_cycle()
    assert r.deploy_s > 0 and r.mttr_restart_s > 0 and r.mttr_replace_s > 0
    assert declined == []
