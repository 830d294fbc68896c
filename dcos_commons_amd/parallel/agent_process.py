"""One agent as a process of its own: registers with the master process over ``agent_link`` and
runs its tasks' lifecycle and readiness checks (``mesos.agent_runtime``) on its device.

``bench.py`` without ``torchrun`` but with ``--gpus N > 1`` starts N-1 of these (the bench
process itself is agent 0), so every agent is a separate process, as on a cluster and as under
``torchrun`` where every rank is one.

    python -m dcos_commons_amd.parallel.agent_process --port P --rank R --device D [--probe on|off]
"""
from __future__ import annotations

import argparse
import json
import logging
import os
import sys
from typing import Optional


def check_for(device: int, probe: bool, checks: Optional[list] = None):
    """``check(msg) -> (ok, detail)`` for the agent link: the fused HIP readiness probe on
    ``device`` (``probe``; a missing extension then fails loudly), else a synthetic pass. Each
    check is appended to ``checks`` as (assigned devices, device, ok)."""
    runner = None
    if probe:
        from dcos_commons_amd.benchmarks.runner import gpu_check_runner

        runner = gpu_check_runner()

    def check(msg):
        assigned = list(msg.get("devices") or [device])
        if assigned != [device]:
            if checks is not None:
                checks.append((assigned, device, False))
            return False, f"check for devices {assigned} sent to the agent of device {device}"
        ok = True if runner is None else bool(runner(None, [device]))
        if checks is not None:
            checks.append((assigned, device, ok))
        return ok, f"{'probe' if runner is not None else 'synthetic'} on device {device}"
    check.probing = runner is not None
    return check


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--host", default="127.0.0.1")
    ap.add_argument("--port", type=int, required=True)
    ap.add_argument("--rank", type=int, required=True)
    ap.add_argument("--device", type=int, default=0)
    ap.add_argument("--probe", choices=["on", "off"], default="off",
                    help="readiness = the HIP probe on --device (on), or a synthetic pass (off)")
    ap.add_argument("--switch-interval-ms", type=float, default=0.0,
                    help="interpreter thread switch interval of this process (0: Python's 5 ms)")
    args = ap.parse_args(argv)
    if args.switch_interval_ms > 0:
        sys.setswitchinterval(args.switch_interval_ms / 1000.0)
    logging.basicConfig(level=logging.ERROR)
    from dcos_commons_amd.benchmarks.runner import _local_agent_info
    from dcos_commons_amd.parallel import agent_link

    info = _local_agent_info(args.rank, args.rank, args.device)
    checks: list = []
    agent_link.run_agent(args.host, args.port, info, check_for(args.device, args.probe == "on", checks))
    record = os.environ.get("SDK_BENCH_RECORD")
    if record:
        # the bench's per-rank records (runner._record) get this agent's checks next to them
        os.makedirs(record, exist_ok=True)
        with open(os.path.join(record, f"agent{args.rank}.json"), "w") as f:
            json.dump({"rank": args.rank, "device": args.device, "registered": info, "checks": checks}, f)
    return 0


if __name__ == "__main__":
    sys.exit(main())
