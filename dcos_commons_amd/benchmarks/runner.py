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

from dcos_commons_amd.benchmarks.deploy_bench import DeployBench

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


def run_bench(args, rank: int, world: int, local_rank: int, use_gpu: bool, dist=None) -> dict:
    n = args.gpus if world == 1 else world
    if world > 1 and args.gpus != world:
        raise SystemExit(f"--gpus {args.gpus} does not match WORLD_SIZE {world}")
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


def _run_single(args, n, use_gpu):
    import torch

    runner = gpu_check_runner() if use_gpu else None
    ndev = torch.cuda.device_count() if use_gpu else 1
    bench = DeployBench(n, profile=args.profile, check_runner=runner,
                        gpu_devices=[i % max(1, ndev) for i in range(n)],
                        allocation_interval_s=args.allocation_interval, extra_env=_sched_env(args))
    for _ in range(args.warmup):
        bench.run_cycle()
    _sync()
    t0 = time.perf_counter()
    cycles = [bench.run_cycle() for _ in range(args.steps)]
    _sync()
    elapsed = time.perf_counter() - t0
    return _summary(args, n, cycles, elapsed, use_gpu, f"agents{n}")


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
    n_dev = torch.cuda.device_count() if torch.cuda.is_available() else 1
    device = local_rank % max(n_dev, 1)
    local_check = gpu_check_runner() if use_gpu else None
    # collectives run on the GPU under RCCL, on the host under gloo
    coll_dev = "cuda" if torch.cuda.is_available() and getattr(args, "dist_backend", "nccl") == "nccl" else "cpu"

    def check(msg):
        if local_check is None:
            return True, "synthetic"
        ok = local_check(None, [device])
        return ok, "probe"

    if rank != 0:
        info = {"rank": rank, "hostname": f"{socket.gethostname()}-gpu{local_rank}", "devices": [device]}
        agent_link.run_agent(master_addr, port_box[0], info, check, on_barrier=lambda: (_sync(), dist.barrier()))
        # final MAX reduction of the timed region (rank 0 drives it)
        t = torch.zeros(1, dtype=torch.float64, device=coll_dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return {}

    remotes = server.wait_for(world - 1)

    def local_runner(task_info, devices):
        return check({})[0]
    local_runner.inline = True   # the local probe (or the synthetic pass) is one short call

    runners = [local_runner] + [agent_link.RemoteCheckRunner(r) for r in remotes]
    bench = DeployBench(world, profile=args.profile, agent_runners=runners, gpu_devices=list(range(world)),
                        allocation_interval_s=args.allocation_interval, extra_env=_sched_env(args))
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
    server.close()
    t = torch.tensor([elapsed], dtype=torch.float64, device=coll_dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return _summary(args, world, cycles, float(t.item()), use_gpu, f"agents{world}-ranks{world}")
