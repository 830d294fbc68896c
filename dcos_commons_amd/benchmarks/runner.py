"""Drives ``DeployBench`` for ``bench.py`` on one process or across ``torchrun`` ranks.

Rank 0 owns the master + scheduler; with WORLD_SIZE > 1 every rank (rank 0 included, in
process) serves the agent for its own GPU, remote ranks over ``parallel.agent_link``. Timing
follows the bench contract: W untimed warmup steps, then exactly K steps bracketed by a barrier
and ``torch.cuda.synchronize()`` on both sides; the elapsed time is MAX-reduced over ranks.
"""
from __future__ import annotations

import os
import socket
import statistics
import time

from dcos_commons_amd.benchmarks.deploy_bench import (DeployBench, agent_spec_from_registration,
                                                      agent_specs_from_inventory, reference_spec)

METRIC = "deploy-plan COMPLETE wall-clock (s) + pod recovery MTTR, helloworld 1/2/4/8 pods"


def gpu_check_runner(device_map=None):
    """Readiness check that runs the HIP device probe on the task's (local) GPU."""
    from dcos_commons_amd.ops import gpu_health

    def run(task_info, devices):
        dev = devices[0] if devices else 0
        if device_map is not None:
            dev = device_map(dev)
        return gpu_health.readiness_probe(dev)["healthy"]
    run.inline = True   # one native call (~0.07 ms, interpreter released): the agent runs it itself
    return run


def _sync():
    import torch

    if torch.cuda.is_available():
        torch.cuda.synchronize()


def _sched_env(args) -> dict:
    return dict(kv.split("=", 1) for kv in getattr(args, "sched_env", None) or [])


def run_bench(args, rank: int, world: int, local_rank: int, use_gpu: bool, dist=None, cluster=None) -> dict:
    """``cluster``: the processes of the split topology (``split_cluster.SplitCluster``, started by
    ``bench.py`` before any GPU was initialised); None runs the in-process topology."""
    n = args.gpus if world == 1 else world
    if world > 1 and args.gpus != world:
        raise SystemExit(f"--gpus {args.gpus} does not match WORLD_SIZE {world}")
    if cluster is not None:
        if world == 1:
            return _run_single_split(args, n, use_gpu, cluster)
        return _run_distributed_split(args, rank, world, local_rank, use_gpu, dist, cluster)
    if world == 1:
        return _run_single(args, n, use_gpu)
    return _run_distributed(args, rank, world, local_rank, use_gpu, dist)


def _summary(args, n, cycles, elapsed, use_gpu, parallelism):
    deploy = [c.deploy_s for c in cycles]
    restart = [c.mttr_restart_s for c in cycles]
    replace = [c.mttr_replace_s for c in cycles]
    sub = [c.deploy_from_subscribed_s for c in cycles]
    value = statistics.mean(deploy)
    return {
        "metric": METRIC,
        "value": round(value, 6),
        "unit": "s",
        "n_gpus": n,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed * 1000.0 / max(1, args.steps), 3),
        "higher_is_better": False,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "bf16",
        "data": "synthetic task payloads; readiness = HIP MFMA/HBM device probe on each pod's GPU"
                if use_gpu else "synthetic task payloads; synthetic readiness",
        "config": {"model": "helloworld gpu.yml (gpus:1 per pod, hostname:UNIQUE, parallel deploy)",
                   "global_batch": n, "seq_len": 0, "parallelism": parallelism,
                   "pods": n, "agents": n, "profile": args.profile,
                   "allocation_interval_s": args.allocation_interval,
                   **({"scheduler_overrides": _sched_env(args)} if _sched_env(args) else {})},
        "deploy_s": {"mean": round(value, 6), "min": round(min(deploy), 6), "max": round(max(deploy), 6)},
        # BASELINE.md's protocol window (SUBSCRIBED -> deploy COMPLETE); `value` also counts the
        # scheduler's construction and API server start before SUBSCRIBE, as in rounds 1-3
        "deploy_from_subscribed_s": {"mean": round(statistics.mean(sub), 6), "min": round(min(sub), 6),
                                     "max": round(max(sub), 6)},
        "mttr_restart_s": {"mean": round(statistics.mean(restart), 6), "max": round(max(restart), 6)},
        "mttr_replace_s": {"mean": round(statistics.mean(replace), 6), "max": round(max(replace), 6)},
    }


def _reference_row(args, n, make_bench) -> dict:
    """BASELINE config #5 as the reference itself would run it: its unchanged helloworld
    ``gpu_resource.yml`` (``gpus: 1`` hello pods, ``hostname:UNIQUE``, no ``plans:`` so the default
    *serial* deploy of DeployPlanFactory.java:22 / DefaultPhaseFactory.java:35, no readiness
    check), on the same agents, after the timed region (it does not enter ``value``/``ms_per_step``)."""
    steps = getattr(args, "reference_steps", 0)
    path = reference_spec("gpu_resource.yml")
    if steps <= 0:
        return {}
    if path is None:
        # the repository's rewrite of the same scenario (also no plans: -> serial)
        path = os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))),
                            "frameworks", "helloworld", "specs", "gpu_resource.yml")
        which = ("repo frameworks/helloworld/specs/gpu_resource.yml: the reference scenario rewritten for this "
                 "repository (no reference tree on this machine); it builds the same ServiceSpec as the reference's "
                 "dist/gpu_resource.yml (tests/test_reference_conformance.py::"
                 "test_repo_gpu_resource_builds_the_reference_scenario)")
    else:
        which = "reference frameworks/helloworld/src/main/dist/gpu_resource.yml, unchanged"
    bench = make_bench(path)
    cycles = [bench.run_cycle() for _ in range(steps)]
    dep = [c.deploy_s for c in cycles]
    return {"reference_spec": {
        "spec": which, "plan": "default serial deploy", "steps": steps, "pods": n,
        "deploy_s": {"mean": round(statistics.mean(dep), 6), "min": round(min(dep), 6), "max": round(max(dep), 6)},
        "deploy_from_subscribed_s": {"mean": round(statistics.mean(c.deploy_from_subscribed_s for c in cycles), 6)},
        "mttr_restart_s": {"mean": round(statistics.mean(c.mttr_restart_s for c in cycles), 6)},
        "mttr_replace_s": {"mean": round(statistics.mean(c.mttr_replace_s for c in cycles), 6)}}}


# the reference example's world pods are not part of BASELINE config #5 (hello pods, one per GPU)
REFERENCE_ROW_ENV = {"WORLD_COUNT": "0"}


def _record(path, payload) -> None:
    """``SDK_BENCH_RECORD=<dir>``: each rank writes what it saw (tests of the multi-rank path)."""
    if not path:
        return
    import json

    os.makedirs(path, exist_ok=True)
    with open(os.path.join(path, f"rank{payload.get('rank', 0)}.json"), "w") as f:
        json.dump(payload, f, indent=1, sort_keys=True)


def _run_single(args, n, use_gpu):
    import torch

    runner = gpu_check_runner() if use_gpu else None
    ndev = torch.cuda.device_count() if use_gpu else 1
    devices = [i % max(1, ndev) for i in range(n)]
    # the agents advertise what node discovery finds for their device (ops.gpu)
    specs = agent_specs_from_inventory(devices)

    def make(spec_file="gpu.yml", spec_env=None):
        return DeployBench(n, profile=args.profile, check_runner=runner, gpu_devices=devices,
                           allocation_interval_s=args.allocation_interval, extra_env=_sched_env(args),
                           agent_specs=specs, spec_file=spec_file, spec_env=spec_env)
    bench = make()
    for _ in range(args.warmup):
        bench.run_cycle()
    _sync()
    t0 = time.perf_counter()
    cycles = [bench.run_cycle() for _ in range(args.steps)]
    _sync()
    elapsed = time.perf_counter() - t0
    out = _summary(args, n, cycles, elapsed, use_gpu, f"agents{n}")
    out["config"]["agent_attributes"] = specs[0].attributes
    out.update(_reference_row(args, n, lambda path: make(path, REFERENCE_ROW_ENV)))
    _record(os.environ.get("SDK_BENCH_RECORD"), {"rank": 0, "placement": bench.last_placement,
                                                 "agents": [_spec_view(s) for s in specs]})
    return out


def _spec_view(spec) -> dict:
    return {"hostname": spec.hostname, "gpus": spec.gpus, "gpu_devices": list(spec.gpu_devices or []),
            "attributes": dict(spec.attributes)}


def _local_agent_info(rank: int, local_rank: int, device: int) -> dict:
    """What this rank registers as its agent: a hostname of its own (one agent per GPU, so
    ``hostname:UNIQUE`` pins pods 1:1), the device it serves, and that device's discovered
    inventory entry (model, arch, xGMI hive and peers) for the agent's attributes."""
    from dcos_commons_amd.ops import gpu as G

    inv = G.node_inventory(device + 1)
    return {"rank": rank, "hostname": f"{socket.gethostname()}-gpu{local_rank}", "devices": [device],
            "gpus": 1, "inventory": inv.subset([device]).to_dict(),
            "attributes": inv.subset([device]).attributes()}


def _run_distributed(args, rank, world, local_rank, use_gpu, dist):
    import torch

    from dcos_commons_amd.parallel import agent_link

    master_addr = os.environ.get("MASTER_ADDR", "127.0.0.1")
    port_box = [0]
    server = None
    if rank == 0:
        server = agent_link.AgentLinkServer(host="127.0.0.1" if master_addr in ("127.0.0.1", "localhost") else
                                            master_addr)
        port_box[0] = server.port
    dist.broadcast_object_list(port_box, src=0)
    if torch.cuda.is_available():
        n_dev = torch.cuda.device_count()
    else:
        # no GPU (gloo rehearsal / CPU test): the node's discovered (or fixture) devices
        from dcos_commons_amd.ops import gpu as G

        n_dev = G.node_inventory(1).count
    device = local_rank % max(n_dev, 1)
    local_check = gpu_check_runner() if use_gpu else None
    # collectives run on the GPU under RCCL, on the host under gloo
    coll_dev = "cuda" if torch.cuda.is_available() and getattr(args, "dist_backend", "nccl") == "nccl" else "cpu"
    record = os.environ.get("SDK_BENCH_RECORD")
    checks = []  # (devices the master assigned, device the probe ran on, ok)

    def check(msg):
        assigned = list(msg.get("devices") or [device])
        if assigned != [device]:
            # the master assigns from the devices this agent registered: anything else is a bug
            checks.append((assigned, device, False))
            return False, f"check for devices {assigned} sent to the agent of device {device}"
        ok = True if local_check is None else local_check(None, [device])
        checks.append((assigned, device, bool(ok)))
        return ok, f"{'probe' if local_check is not None else 'synthetic'} on device {device}"

    info = _local_agent_info(rank, local_rank, device)
    if rank != 0:
        marks = []

        def on_barrier():
            _sync()
            dist.barrier()
            marks.append(time.perf_counter())
        agent_link.run_agent(master_addr, port_box[0], info, check, on_barrier=on_barrier)
        # this rank's view of the timed region (between rank 0's two barriers), MAX-reduced with
        # every other rank's
        elapsed = marks[-1] - marks[0] if len(marks) >= 2 else 0.0
        t = torch.tensor([elapsed], dtype=torch.float64, device=coll_dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        _record(record, {"rank": rank, "device": device, "registered": info, "checks": checks,
                         "elapsed_local_s": elapsed, "elapsed_max_s": float(t.item())})
        return {}

    remotes = server.wait_for(world - 1)

    def local_runner(task_info, devices):
        return check({"devices": devices})[0]
    local_runner.inline = True   # the local probe (or the synthetic pass) is one short call

    runners = [local_runner] + [agent_link.RemoteCheckRunner(r) for r in remotes]
    # every agent is what its rank registered: hostname, device, discovered attributes
    specs = [agent_spec_from_registration(info, 0)] + [agent_spec_from_registration(r.info, i + 1)
                                                       for i, r in enumerate(remotes)]

    def make(spec_file="gpu.yml", spec_env=None):
        return DeployBench(world, profile=args.profile, agent_runners=runners, agent_specs=specs,
                           allocation_interval_s=args.allocation_interval, extra_env=_sched_env(args),
                           spec_file=spec_file, spec_env=spec_env)
    bench = make()
    for _ in range(args.warmup):
        bench.run_cycle()

    def barrier():
        server.broadcast("barrier")
        _sync()
        dist.barrier()

    barrier()
    t0 = time.perf_counter()
    cycles = [bench.run_cycle() for _ in range(args.steps)]
    _sync()
    barrier()
    elapsed = time.perf_counter() - t0
    placement = bench.last_placement
    extra = _reference_row(args, world, lambda path: make(path, REFERENCE_ROW_ENV))
    server.close()
    t = torch.tensor([elapsed], dtype=torch.float64, device=coll_dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    _record(record, {"rank": 0, "device": device, "registered": info, "checks": checks, "placement": placement,
                     "agents": [_spec_view(s) for s in specs], "elapsed_local_s": elapsed,
                     "elapsed_max_s": float(t.item())})
    out = _summary(args, world, cycles, float(t.item()), use_gpu, f"agents{world}-ranks{world}")
    out["config"]["agent_attributes"] = specs[0].attributes
    out.update(extra)
    return out


# -- split topology: master process, agents that run their own tasks --------------------------
def _agent_check(device: int, use_gpu: bool, checks: list):
    """``check(msg)`` of this process's agent (its device): the HIP probe or a synthetic pass;
    every check is recorded as (assigned devices, device, ok)."""
    local = gpu_check_runner() if use_gpu else None

    def check(msg):
        assigned = list(msg.get("devices") or [device])
        if assigned != [device]:
            # the master assigns from the devices this agent registered: anything else is a bug
            checks.append((assigned, device, False))
            return False, f"check for devices {assigned} sent to the agent of device {device}"
        ok = True if local is None else local(None, [device])
        checks.append((assigned, device, bool(ok)))
        return ok, f"{'probe' if local is not None else 'synthetic'} on device {device}"
    return check


def _start_agent_thread(host: str, port: int, info: dict, check):
    import threading

    from dcos_commons_amd.parallel import agent_link

    registered = threading.Event()
    t = threading.Thread(target=agent_link.run_agent, args=(host, port, info, check),
                         kwargs={"on_registered": registered.set}, name="agent-link", daemon=True)
    t.start()
    if not registered.wait(120):
        raise TimeoutError("this process's agent did not register with the master process")
    return t


def _split_summary(args, n, cycles, elapsed, use_gpu, parallelism, infos):
    out = _summary(args, n, cycles, elapsed, use_gpu, parallelism)
    out["config"]["topology"] = ("split: master process; each agent (rank or helper process) runs its tasks' "
                                 "lifecycle and readiness checks; scheduler over the framed v1 stream")
    out["config"]["agent0"] = getattr(args, "agent0", "process")
    out["config"]["agent_attributes"] = agent_spec_from_registration(infos[0], 0).attributes
    return out


def _run_single_split(args, n, use_gpu, cluster):
    import torch

    from dcos_commons_amd.mesos.master_process import MasterClient

    ndev = torch.cuda.device_count() if use_gpu else 1
    checks: list = []
    info = _local_agent_info(0, 0, 0)
    agent = None
    if getattr(args, "agent0", "process") == "thread":
        agent = _start_agent_thread(cluster.host, cluster.ports["agents"], info, _agent_check(0, use_gpu, checks))
    client = MasterClient(cluster.host, cluster.ports["control"])
    infos = client.call("agents", n=n)

    def make(spec_file="gpu.yml", spec_env=None):
        return DeployBench(n, profile=args.profile, allocation_interval_s=args.allocation_interval,
                           extra_env=_sched_env(args), spec_file=spec_file, spec_env=spec_env, master_client=client)
    bench = make()
    for _ in range(args.warmup):
        bench.run_cycle()
    _sync()
    t0 = time.perf_counter()
    cycles = [bench.run_cycle() for _ in range(args.steps)]
    _sync()
    elapsed = time.perf_counter() - t0
    out = _split_summary(args, n, cycles, elapsed, use_gpu, f"agents{n}", infos)
    out["config"]["agent_processes"] = n
    out["config"]["devices"] = [i % max(1, ndev) for i in range(n)]
    placement = bench.last_placement
    out.update(_reference_row(args, n, lambda path: make(path, REFERENCE_ROW_ENV)))
    client.call("shutdown")
    if agent is not None:
        agent.join(10)
    _record(os.environ.get("SDK_BENCH_RECORD"), {"rank": 0, "placement": placement, "registered": info,
                                                 "checks": checks, "agents": infos})
    return out


def _run_distributed_split(args, rank, world, local_rank, use_gpu, dist, cluster):
    import torch

    from dcos_commons_amd.mesos.master_process import MasterClient

    box = [cluster.ports if cluster is not None and rank == 0 else None]
    dist.broadcast_object_list(box, src=0)
    ports = box[0]
    host = os.environ.get("MASTER_ADDR", "127.0.0.1")
    if torch.cuda.is_available():
        n_dev = torch.cuda.device_count()
    else:
        from dcos_commons_amd.ops import gpu as G

        n_dev = G.node_inventory(1).count
    device = local_rank % max(n_dev, 1)
    coll_dev = "cuda" if torch.cuda.is_available() and getattr(args, "dist_backend", "nccl") == "nccl" else "cpu"
    record = os.environ.get("SDK_BENCH_RECORD")
    checks: list = []
    info = _local_agent_info(rank, local_rank, device)
    agent = None
    if rank != 0 or getattr(args, "agent0", "process") != "process":
        agent = _start_agent_thread(host, ports["agents"], info, _agent_check(device, use_gpu, checks))
    # else: rank 0's agent is the process SplitCluster started for it (--agent0 process)

    def barrier():
        _sync()
        dist.barrier()

    if rank != 0:
        # this rank is an agent: its runtime serves launches and checks on its own threads while
        # the main thread marks the timed window between rank 0's barriers
        barrier()
        t0 = time.perf_counter()
        barrier()
        elapsed = time.perf_counter() - t0
        t = torch.tensor([elapsed], dtype=torch.float64, device=coll_dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        agent.join()    # until the master process shuts the agents down
        _record(record, {"rank": rank, "device": device, "registered": info, "checks": checks,
                         "elapsed_local_s": elapsed, "elapsed_max_s": float(t.item())})
        return {}

    client = MasterClient(cluster.host, ports["control"])
    infos = client.call("agents", n=world)

    def make(spec_file="gpu.yml", spec_env=None):
        return DeployBench(world, profile=args.profile, allocation_interval_s=args.allocation_interval,
                           extra_env=_sched_env(args), spec_file=spec_file, spec_env=spec_env, master_client=client)
    bench = make()
    for _ in range(args.warmup):
        bench.run_cycle()
    barrier()
    t0 = time.perf_counter()
    cycles = [bench.run_cycle() for _ in range(args.steps)]
    barrier()
    elapsed = time.perf_counter() - t0
    placement = bench.last_placement
    extra = _reference_row(args, world, lambda path: make(path, REFERENCE_ROW_ENV))
    t = torch.tensor([elapsed], dtype=torch.float64, device=coll_dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    client.call("shutdown")
    if agent is not None:
        agent.join(30)
    specs = [agent_spec_from_registration(x, i) for i, x in enumerate(infos)]
    _record(record, {"rank": 0, "device": device, "registered": info, "checks": checks, "placement": placement,
                     "agents": [_spec_view(s) for s in specs], "elapsed_local_s": elapsed,
                     "elapsed_max_s": float(t.item())})
    out = _split_summary(args, world, cycles, float(t.item()), use_gpu, f"agents{world}-ranks{world}", infos)
    out.update(extra)
    return out
