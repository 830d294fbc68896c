#!/usr/bin/env python3
"""Headline benchmark: helloworld deploy-plan COMPLETE wall-clock + pod recovery MTTR.

    python bench.py --gpus N --steps K --warmup W

N GPUs = N MI355X agents (one per GPU, ``gpus: 1`` pods pinned 1:1, readiness = HIP device
probe on the pod's GPU). A *step* is one full cycle on a fresh cluster and fresh state:
deploy -> inject TASK_FAILED (restart MTTR) -> ``pod replace`` (replace MTTR) -> teardown.
``value`` is the mean deploy-plan COMPLETE wall-clock over the K timed steps (seconds, lower is
better); the MTTRs are reported alongside. Weak scaling: one pod per GPU.

Under ``torchrun`` every rank owns the agent for its GPU (LOCAL_RANK) and rank 0 runs the
master + scheduler; agents talk to the master over TCP (``parallel.agent_link``).
"""
from __future__ import annotations

import argparse
import json
import logging
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def parse_args(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--profile", default="mi355x", choices=["mi355x", "reference"])
    ap.add_argument("--allocation-interval", type=float, default=1.0,
                    help="fake Mesos master allocation interval (Mesos default 1 s)")
    ap.add_argument("--no-gpu-probe", action="store_true", help="synthetic readiness (no HIP probe)")
    ap.add_argument("--dist-backend", default="auto", choices=["auto", "nccl", "gloo"],
                    help="torch.distributed backend (auto: nccl=RCCL on GPUs, gloo on CPU; gloo lets several "
                         "ranks share one GPU for a rehearsal)")
    ap.add_argument("--sched-env", action="append", default=[], metavar="KEY=VALUE",
                    help="scheduler flag override on top of --profile (A/B experiments)")
    ap.add_argument("--no-pin", action="store_true",
                    help="do not pin each rank to its own slice of the allowed CPUs")
    ap.add_argument("--reference-steps", type=int, default=None,
                    help="cycles of the reference's unchanged gpu_resource.yml (default serial deploy) run after "
                         "the timed region and reported as `reference_spec` (default: --steps; 0 = skip)")
    ap.add_argument("--topology", default="split", choices=["split", "inprocess"],
                    help="split: the master and every agent's task lifecycle run in processes of their own (a "
                         "master process; each rank, or a helper process per agent, runs its tasks), the "
                         "scheduler here over the framed v1 stream; inprocess: one interpreter holds all of it")
    ap.add_argument("--agent0", default="process", choices=["thread", "process"],
                    help="split topology: agent 0 (rank 0's agent under torchrun) runs on a thread of this "
                         "process (thread) or in a process of its own like the others (process)")
    ap.add_argument("--cluster-switch-interval-ms", type=float, default=0.0,
                    help="split topology: interpreter switch interval of the master and agent processes "
                         "(0: Python's 5 ms)")
    ap.add_argument("--verbose", action="store_true")
    args = ap.parse_args(argv)
    if args.reference_steps is None:
        args.reference_steps = args.steps
    return args


def pin_cpus(local_rank: int, local_world: int, per: int = 4, skip: int = 4) -> list:
    """Pin this rank (and every thread it starts afterwards) to its own ``per`` CPUs of the set it
    may run on, past the first ``skip`` (interrupt handling), like pinning a scheduler with
    taskset/cpusets in production. The scheduler is one interpreter whose offer loop, status path
    and agents hand work to each other: kept on a few warm cores those hand-offs do not wait for
    an idle core to wake (measured on the box: deploy 4.2-5.1 -> 2.8 ms, restart MTTR 2.7-3.0 ->
    1.9 ms). Too few CPUs for a slice each: no pinning."""
    try:
        allowed = sorted(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        return []
    if len(allowed) < skip + per * local_world:
        skip = 0
        per = len(allowed) // max(1, local_world)
    if per < 2:
        return []
    cpus = allowed[skip + local_rank * per: skip + (local_rank + 1) * per]
    try:
        os.sched_setaffinity(0, cpus)
    except OSError:
        return []
    return cpus


def main(argv=None) -> int:
    args = parse_args(argv)
    logging.basicConfig(level=logging.INFO if args.verbose else logging.ERROR,
                        format="%(asctime)s %(name)s %(levelname)s %(message)s")
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    local_world = int(os.environ.get("LOCAL_WORLD_SIZE", str(world)))
    cpus = [] if args.no_pin else pin_cpus(local_rank, local_world)

    cluster = None
    if args.topology == "split":
        # before anything initialises a GPU: such a process may not start programs
        from dcos_commons_amd.benchmarks.split_cluster import SplitCluster

        cluster = SplitCluster.start(args, rank, world)

    import torch

    use_gpu = torch.cuda.is_available() and not args.no_gpu_probe
    dist = None
    if world > 1:
        import torch.distributed as dist

        # auto: RCCL with one rank per GPU; more ranks than GPUs (a one-GPU rehearsal) cannot share a
        # device under RCCL ("Duplicate GPU detected"), so they use gloo
        backend = args.dist_backend if args.dist_backend != "auto" else (
            "nccl" if torch.cuda.is_available() and world <= torch.cuda.device_count() else "gloo")
        args.dist_backend = backend
        if torch.cuda.is_available():
            # one rank per GPU; more ranks than GPUs share them round-robin (gloo rehearsals)
            torch.cuda.set_device(local_rank % torch.cuda.device_count())
        dist.init_process_group(backend=backend)

    from dcos_commons_amd.benchmarks.runner import run_bench

    try:
        result = run_bench(args, rank=rank, world=world, local_rank=local_rank, use_gpu=use_gpu, dist=dist,
                           cluster=cluster)
    finally:
        if cluster is not None:
            cluster.close()
    if rank == 0 and result:
        result["config"]["cpus_per_rank"] = len(cpus) if cpus else None
    if rank == 0:
        print(json.dumps(result), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
