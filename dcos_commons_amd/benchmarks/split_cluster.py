"""The processes of ``bench.py``'s split topology, started before the bench initialises a GPU.

* rank 0 (or the only process) starts the master process (``mesos.master_process``): offers,
  reservations, ACCEPTs and status forwarding, as a Mesos master;
* it starts the agent processes (``parallel.agent_process``) that are not ranks: without
  ``torchrun``, all N agents; under ``torchrun``, rank 0's own agent (the other ranks are agents
  themselves). So every agent is a process of its own that runs its tasks' lifecycle and readiness
  checks, and the scheduler's interpreter runs only the scheduler, as on a cluster. ``--agent0
  thread`` keeps agent 0 on a thread of the bench process instead (same-box A/B: 1 pod 2.04 ->
  1.90 ms, 8 pods 5.81 -> 5.57 ms with the process, ``profiles/agent0_ab_r06_box.txt``);
* the scheduler stays in the bench process and subscribes over ``mesos.stream_api``.

A process that has initialised a GPU must not start programs (the box forbids the exec), which is
why ``bench.py`` calls ``SplitCluster.start`` before anything touches the GPU.
"""
from __future__ import annotations

import os
import subprocess
import sys
from typing import Dict, List, Optional


class SplitCluster:
    def __init__(self, host: str, ports: Optional[Dict[str, int]], procs: List[subprocess.Popen]):
        self.host = host
        self.ports = ports
        self.procs = procs

    @staticmethod
    def start(args, rank: int, world: int) -> "SplitCluster":
        from dcos_commons_amd.mesos import master_process

        addr = os.environ.get("MASTER_ADDR", "127.0.0.1")
        host = "127.0.0.1" if addr in ("127.0.0.1", "localhost") else addr
        if rank != 0:
            return SplitCluster(host, None, [])
        si = getattr(args, "cluster_switch_interval_ms", 0.0) or 0.0
        master, ports = master_process.spawn(args.allocation_interval, host=host, switch_interval_ms=si)
        procs = [master]
        agent0_process = getattr(args, "agent0", "process") == "process"
        first = 0 if agent0_process else 1
        # agent processes: without torchrun, agents first..N-1 (agent 0 is this process's thread
        # unless --agent0 process); under torchrun every other rank is an agent, and --agent0
        # process moves rank 0's own agent out of the scheduler's interpreter
        if world == 1:
            ranks = list(range(first, args.gpus))
        else:
            ranks = [0] if agent0_process else []
        if ranks:
            probe = "off"
            if not args.no_gpu_probe:
                import torch

                ndev = torch.cuda.device_count()   # counts devices without initialising them
                probe = "on" if ndev > 0 else "off"
            else:
                ndev = 0
            root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
            env = dict(os.environ)
            env["PYTHONPATH"] = root + (os.pathsep + env["PYTHONPATH"] if env.get("PYTHONPATH") else "")
            local = int(os.environ.get("LOCAL_RANK", "0")) if world > 1 else None
            for i in ranks:
                dev = (local if local is not None else i)
                dev = dev % ndev if ndev else dev
                procs.append(subprocess.Popen(
                    [sys.executable, "-m", "dcos_commons_amd.parallel.agent_process", "--host", host,
                     "--port", str(ports["agents"]), "--rank", str(i), "--device", str(dev), "--probe", probe,
                     "--switch-interval-ms", str(si)],
                    stdin=subprocess.DEVNULL, env=env, cwd=root))
        return SplitCluster(host, ports, procs)

    def close(self, timeout_s: float = 10.0) -> None:
        """Waits for the processes (the master process ends on ``shutdown`` or when the bench's
        control connection closes; agents when the master goes), killing any that linger."""
        for p in self.procs:
            try:
                p.wait(timeout_s)
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait(5)
