"""Master <-> remote-agent link: one agent process per GPU.

The reference's agents are Mesos slaves talking to the master over libprocess; here every
``torchrun`` rank owns the MI355X at ``LOCAL_RANK`` and runs an agent that connects to the
master (rank 0) over TCP. The master keeps the offer/reservation bookkeeping (``LocalMaster``);
the agent executes what must run *on its GPU*: task checks (the HIP device probe that gates GPU
pod readiness). Wire format: newline-delimited JSON, request ids for request/response pairs.

The listener binds to loopback (127.0.0.1) by default: the single-node benchmark and tests never
need more, and the link carries no authentication.

Ops (master -> agent): ``check`` {id, task, name, devices}, ``barrier`` {id}, ``shutdown``, and
for an agent that runs its tasks' lifecycle itself (``mesos.agent_runtime``) ``launch``, ``kill``,
``fail``, ``drop``, ``reset`` (no reply). Ops (agent -> master): ``register`` {hostname, gpus,
devices, attributes, rank}, ``result`` {id, ok, detail}, and unsolicited ``status`` {reports}.
"""
from __future__ import annotations

import json
import logging
import socket
import threading
from concurrent.futures import Future
from typing import Callable, Dict, List, Optional

LOGGER = logging.getLogger(__name__)
DEFAULT_HOST = "127.0.0.1"


class _Conn:
    def __init__(self, sock: socket.socket):
        self.sock = sock
        self.rfile = sock.makefile("r", encoding="utf-8", newline="\n")
        self._wlock = threading.Lock()

    def send(self, msg: dict) -> None:
        data = (json.dumps(msg) + "\n").encode("utf-8")
        with self._wlock:
            self.sock.sendall(data)

    def recv(self) -> Optional[dict]:
        line = self.rfile.readline()
        if not line:
            return None
        return json.loads(line)

    def close(self) -> None:
        try:
            self.sock.shutdown(socket.SHUT_RDWR)
        except OSError:
            pass
        self.sock.close()


class RemoteAgent:
    """Master-side handle of one connected agent."""

    def __init__(self, conn: _Conn, info: dict):
        self.conn = conn
        self.info = info
        self._next = 0
        self._pending: Dict[int, Future] = {}
        self._lock = threading.Lock()
        self.alive = True
        # unsolicited ``status`` messages of an agent running its own tasks (agent_runtime reports)
        self.on_status: Callable[[List[dict]], None] = lambda reports: None
        self._reader = threading.Thread(target=self._read_loop, daemon=True, name=f"agent-link-{info.get('rank')}")
        self._reader.start()

    @property
    def rank(self) -> int:
        return int(self.info.get("rank", -1))

    def _read_loop(self) -> None:
        while True:
            try:
                msg = self.conn.recv()
            except (OSError, ValueError):
                msg = None
            if msg is None:
                break
            if msg.get("op") == "status":
                try:
                    self.on_status(msg.get("reports") or [])
                except Exception:  # noqa: BLE001
                    LOGGER.exception("agent status reports failed")
                continue
            with self._lock:
                fut = self._pending.pop(msg.get("id"), None)
            if isinstance(fut, Future):
                fut.set_result(msg)
            elif fut is not None:
                fut(msg)  # an asynchronous request's callback, run on this reader thread
        with self._lock:
            self.alive = False   # under the lock: a request registered after this fails at once
            pending, self._pending = self._pending, {}
        for f in pending.values():
            if isinstance(f, Future):
                f.set_exception(ConnectionError("agent disconnected"))
            else:
                f({"ok": False, "detail": "agent disconnected"})

    def request(self, op: str, timeout: Optional[float] = None, **fields) -> dict:
        with self._lock:
            if not self.alive:
                raise ConnectionError("agent disconnected")
            self._next += 1
            rid = self._next
            fut: Future = Future()
            self._pending[rid] = fut
        self.conn.send(dict(fields, op=op, id=rid))
        return fut.result(timeout)

    def request_async(self, op: str, callback: Callable[[dict], None], **fields) -> None:
        """Sends ``op`` and returns at once; ``callback(reply)`` runs on the link's reader thread
        (with ``{"ok": False}`` if the agent disconnects first)."""
        with self._lock:
            alive = self.alive
            if alive:
                self._next += 1
                rid = self._next
                self._pending[rid] = callback
        if not alive:
            callback({"ok": False, "detail": "agent disconnected"})
            return
        try:
            self.conn.send(dict(fields, op=op, id=rid))
        except OSError:
            with self._lock:
                self._pending.pop(rid, None)
            callback({"ok": False, "detail": "agent link send failed"})

    def run_check(self, task_info, devices: List[int]) -> bool:
        """Check runner for ``LocalMaster``: executes the task's check on this agent's GPU."""
        r = self.request("check", timeout=300, task=task_info.task_id.value, name=task_info.name, devices=devices)
        return bool(r.get("ok"))

    def run_check_async(self, task_info, devices: List[int], done: Callable[[bool], None]) -> None:
        """``LocalMaster``'s asynchronous check protocol: the request goes out from the master's
        thread and the reply's callback reports the result from the reader thread, so no worker
        thread sits blocked on the round trip and the result reaches the master one thread hop
        sooner."""
        self.request_async("check", lambda r: done(bool(r.get("ok"))), task=task_info.task_id.value,
                           name=task_info.name, devices=devices)


    def send(self, msg: dict) -> None:
        """A runtime message (``launch``, ``kill``, ...): no reply; a dead link is logged."""
        try:
            self.conn.send(msg)
        except OSError as e:
            LOGGER.warning("agent link to rank %s: %s dropped (%s)", self.rank, msg.get("op"), e)

    def shutdown(self) -> None:
        try:
            self.conn.send({"op": "shutdown", "id": 0})
        except OSError:
            pass


class RemoteCheckRunner:
    """A check runner bound to a remote agent: callable (blocking) and with ``run_async``."""

    def __init__(self, agent: "RemoteAgent"):
        self.agent = agent

    def __call__(self, task_info, devices: List[int]) -> bool:
        return self.agent.run_check(task_info, devices)

    def run_async(self, task_info, devices: List[int], done: Callable[[bool], None]) -> None:
        self.agent.run_check_async(task_info, devices, done)


class AgentLinkServer:
    """Accepts agent registrations (rank 0)."""

    def __init__(self, host: str = DEFAULT_HOST, port: int = 0):
        self.sock = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
        self.sock.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
        self.sock.bind((host, port))
        self.sock.listen(64)
        self.port = self.sock.getsockname()[1]
        self.agents: List[RemoteAgent] = []
        self._cond = threading.Condition()
        self._thread = threading.Thread(target=self._accept_loop, daemon=True, name="agent-link-accept")
        self._thread.start()

    def _accept_loop(self) -> None:
        while True:
            try:
                s, _ = self.sock.accept()
            except OSError:
                return
            s.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
            conn = _Conn(s)
            try:
                reg = conn.recv()
            except (OSError, ValueError):
                conn.close()
                continue
            if not reg or reg.get("op") != "register":
                conn.close()
                continue
            agent = RemoteAgent(conn, reg)
            conn.send({"op": "registered", "id": reg.get("id", 0)})
            with self._cond:
                self.agents.append(agent)
                self._cond.notify_all()

    def wait_for(self, n: int, timeout: float = 120.0) -> List[RemoteAgent]:
        with self._cond:
            ok = self._cond.wait_for(lambda: len(self.agents) >= n, timeout)
            if not ok:
                raise TimeoutError(f"only {len(self.agents)}/{n} agents registered")
            return sorted(self.agents, key=lambda a: a.rank)

    def broadcast(self, op: str, timeout: float = 300.0) -> None:
        """Request/ack ``op`` on every agent concurrently."""
        futs = []
        for a in self.agents:
            f: Future = Future()
            futs.append(f)

            def go(a=a, f=f):
                try:
                    f.set_result(a.request(op, timeout=timeout))
                except Exception as e:  # noqa: BLE001
                    f.set_exception(e)
            threading.Thread(target=go, daemon=True).start()
        for f in futs:
            f.result(timeout)

    def close(self) -> None:
        for a in self.agents:
            a.shutdown()
        try:
            self.sock.close()
        except OSError:
            pass


RUNTIME_OPS = ("launch", "kill", "fail", "drop", "reset")


def run_agent(master_host: str, port: int, info: dict, check: Callable[[dict], tuple],
              on_barrier: Optional[Callable[[], None]] = None, on_registered: Optional[Callable[[], None]] = None
              ) -> None:
    """Agent main loop (blocking): register, then serve until shutdown: ``check`` / ``barrier``
    requests, and the runtime messages of the tasks this agent runs itself (``agent_runtime``:
    their checks call ``check({"devices": ...})`` on this process's GPU)."""
    from dcos_commons_amd.mesos.agent_runtime import AgentRuntime

    s = socket.create_connection((master_host, port), timeout=120)
    s.settimeout(None)
    s.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
    conn = _Conn(s)
    conn.send(dict(info, op="register", id=0))
    ack = conn.recv()
    if not ack or ack.get("op") != "registered":
        raise ConnectionError("agent registration rejected")
    if on_registered is not None:
        on_registered()

    def report(reports):
        try:
            conn.send({"op": "status", "id": 0, "reports": reports})
        except OSError as e:
            LOGGER.warning("agent status reports lost: %s", e)
    runtime = AgentRuntime(report, lambda devices: bool(check({"devices": devices})[0]),
                           name=f"agent-runtime-{info.get('rank', 0)}")
    try:
        while True:
            msg = conn.recv()
            if msg is None or msg.get("op") == "shutdown":
                break
            op, rid = msg.get("op"), msg.get("id")
            if op in RUNTIME_OPS:
                runtime.handle(msg)
            elif op == "check":
                try:
                    ok, detail = check(msg)
                except Exception as e:  # noqa: BLE001
                    LOGGER.exception("check failed")
                    ok, detail = False, str(e)
                conn.send({"op": "result", "id": rid, "ok": bool(ok), "detail": detail})
            elif op == "barrier":
                conn.send({"op": "result", "id": rid, "ok": True})
                if on_barrier is not None:
                    on_barrier()
            else:
                conn.send({"op": "result", "id": rid, "ok": False, "detail": f"unknown op {op}"})
    finally:
        runtime.shutdown()
        conn.close()
