"""The stand-in Mesos master as a process of its own, with agents that run their own tasks.

``bench.py`` used to keep the master, every agent's task lifecycle and the scheduler in one
interpreter (rank 0's), so each added pod cost the scheduler's process its launch, its status
updates and its checks as well as its evaluation. On a cluster these are separate processes, and
this module makes them so:

* the **master** (a ``LocalMaster``) runs here and keeps what a Mesos master keeps: offers,
  reservations, ACCEPT bookkeeping, and the forwarding of status updates;
* **agents** register over ``parallel.agent_link`` (one per ``torchrun`` rank, owning its GPU, or
  a helper process) and run their tasks' lifecycle and readiness checks themselves
  (``mesos.agent_runtime``); the master sends them ``launch`` / ``kill`` and turns their reports
  into status updates;
* the **scheduler** subscribes over ``mesos.stream_api`` (the v1 ``Call``/``Event`` messages on
  one framed socket).

A small JSON-lines control socket (loopback) lets the bench drive it: ``agents`` (wait for N
registrations), ``reset`` (a fresh master, same agents: the start of a bench cycle), ``placement``,
``fail_task`` (the task dies on its agent), ``shutdown``.

    python -m dcos_commons_amd.mesos.master_process [--allocation-interval 1.0]

prints one JSON line with its ports (``stream``, ``agents``, ``control``) and serves until
``shutdown`` or until its parent closes the control connection.
"""
from __future__ import annotations

import argparse
import json
import logging
import os
import socket
import subprocess
import sys
import threading
import time
from typing import Dict, List, Optional

LOGGER = logging.getLogger(__name__)


class _Runtime:
    """Master-side handle of a remote agent's runtime: ``send`` goes over its link."""

    def __init__(self, agent):
        self.agent = agent

    def send(self, msg: dict) -> None:
        self.agent.send(msg)


class MasterProcess:
    def __init__(self, host: str = "127.0.0.1", allocation_interval_s: float = 1.0):
        from dcos_commons_amd.mesos.local_master import LocalMaster
        from dcos_commons_amd.mesos.stream_api import StreamMaster
        from dcos_commons_amd.parallel.agent_link import AgentLinkServer

        self.host = host
        self.allocation_interval_s = allocation_interval_s
        self.links = AgentLinkServer(host=host)
        self.master: Optional[LocalMaster] = None
        self.stream = StreamMaster(LocalMaster(allocation_interval_s=allocation_interval_s), host=host).start()
        self.master = self.stream.master
        self.control = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
        self.control.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
        self.control.bind((host, 0))
        self.control.listen(4)
        self._done = threading.Event()

    def ports(self) -> Dict[str, int]:
        return {"stream": self.stream.port, "agents": self.links.port, "control": self.control.getsockname()[1],
                "pid": os.getpid()}

    # -- control ops ---------------------------------------------------------------------
    def op_agents(self, n: int, timeout: float = 120.0) -> List[dict]:
        return [a.info for a in self.links.wait_for(int(n), timeout)]

    def op_reset(self, allocation_interval_s: Optional[float] = None) -> dict:
        """A fresh master with every registered agent (in rank order), each told to forget its
        tasks: the start of a bench cycle, like a new cluster."""
        from dcos_commons_amd.benchmarks.deploy_bench import agent_spec_from_registration
        from dcos_commons_amd.mesos.local_master import LocalMaster

        if allocation_interval_s is not None:
            self.allocation_interval_s = float(allocation_interval_s)
        old = self.master
        lm = LocalMaster(allocation_interval_s=self.allocation_interval_s)
        agents = sorted(self.links.agents, key=lambda a: a.rank)
        for a in agents:
            a.send({"op": "reset"})
        for i, a in enumerate(agents):
            aid = lm.add_agent(agent_spec_from_registration(a.info, i), runtime=_Runtime(a))
            a.on_status = (lambda reports, aid=aid, lm=lm: lm.runtime_reports(aid, reports))
        self.stream.set_master(lm)
        self.master = lm
        if old is not None:
            old.shutdown()
        return {"stream": self.stream.address, "agents": len(agents)}

    def op_placement(self) -> list:
        return self.master.placement()

    def op_fail_task(self, task_id: str, message: str = "injected failure") -> None:
        self.master.fail_task(task_id, message=message)

    def op_task_states(self) -> dict:
        return self.master.task_states()

    def op_shutdown(self) -> None:
        self._done.set()

    # -- serving -------------------------------------------------------------------------
    def serve(self) -> None:
        threading.Thread(target=self._accept, name="master-control", daemon=True).start()
        self._done.wait()
        self.links.close()
        self.stream.stop()
        if self.master is not None:
            self.master.shutdown()

    def _accept(self) -> None:
        while not self._done.is_set():
            try:
                conn, _ = self.control.accept()
            except OSError:
                return
            conn.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
            threading.Thread(target=self._client, args=(conn,), daemon=True).start()

    def _client(self, conn: socket.socket) -> None:
        rfile = conn.makefile("r", encoding="utf-8", newline="\n")
        try:
            for line in rfile:
                req = json.loads(line)
                op = req.pop("op", "")
                fn = getattr(self, "op_" + op, None)
                try:
                    if fn is None:
                        raise ValueError(f"unknown op {op!r}")
                    out = {"ok": True, "result": fn(**req)}
                except Exception as e:  # noqa: BLE001
                    LOGGER.exception("control op %s failed", op)
                    out = {"ok": False, "error": f"{type(e).__name__}: {e}"}
                conn.sendall((json.dumps(out) + "\n").encode("utf-8"))
                if op == "shutdown":
                    return
        except (OSError, ValueError):
            pass
        finally:
            conn.close()
            # the bench (our parent) went away: nothing is left to serve
            self._done.set()


class MasterClient:
    """The bench's side of the control socket (blocking request/response)."""

    def __init__(self, host: str, port: int, timeout_s: float = 120.0):
        self.sock = socket.create_connection((host, port), timeout=timeout_s)
        self.sock.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
        self.rfile = self.sock.makefile("r", encoding="utf-8", newline="\n")
        self._lock = threading.Lock()

    def call(self, op: str, **fields):
        with self._lock:
            self.sock.sendall((json.dumps(dict(fields, op=op)) + "\n").encode("utf-8"))
            line = self.rfile.readline()
        if not line:
            raise ConnectionError("master process closed the control connection")
        out = json.loads(line)
        if not out.get("ok"):
            raise RuntimeError(f"master process: {op} failed: {out.get('error')}")
        return out.get("result")

    def close(self) -> None:
        try:
            self.sock.close()
        except OSError:
            pass


def spawn(allocation_interval_s: float = 1.0, host: str = "127.0.0.1", env: Optional[dict] = None,
          timeout_s: float = 120.0, switch_interval_ms: float = 0.0):
    """Starts a master process (a child: start it before this process initialises a GPU) and
    returns ``(Popen, ports)``."""
    root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    e = dict(os.environ)
    e.update(env or {})
    e["PYTHONPATH"] = root + (os.pathsep + e["PYTHONPATH"] if e.get("PYTHONPATH") else "")
    proc = subprocess.Popen([sys.executable, "-m", "dcos_commons_amd.mesos.master_process",
                             "--host", host, "--allocation-interval", str(allocation_interval_s),
                             "--switch-interval-ms", str(switch_interval_ms)],
                            stdout=subprocess.PIPE, stdin=subprocess.DEVNULL, env=e, cwd=root, text=True)
    deadline = time.monotonic() + timeout_s
    line = proc.stdout.readline()
    if not line or time.monotonic() > deadline:
        proc.kill()
        raise RuntimeError("master process did not start")
    return proc, json.loads(line)


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--host", default="127.0.0.1")
    ap.add_argument("--allocation-interval", type=float, default=1.0)
    ap.add_argument("--verbose", action="store_true")
    ap.add_argument("--switch-interval-ms", type=float, default=0.0,
                    help="interpreter thread switch interval of this process (0: Python's 5 ms)")
    args = ap.parse_args(argv)
    if args.switch_interval_ms > 0:
        sys.setswitchinterval(args.switch_interval_ms / 1000.0)
    logging.basicConfig(level=logging.INFO if args.verbose else logging.ERROR,
                        format="%(asctime)s master %(name)s %(levelname)s %(message)s")
    mp = MasterProcess(args.host, args.allocation_interval)
    print(json.dumps(mp.ports()), flush=True)
    mp.serve()
    return 0


if __name__ == "__main__":
    sys.exit(main())
