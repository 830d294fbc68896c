"""Mesos v1 scheduler HTTP API in front of a ``LocalMaster``.

SURVEY §2.10/§2.11: the reference talks to a real Mesos master through the v1 HTTP adapter; this
module provides the master side of the same wire contract (``POST /api/v1/scheduler``: SUBSCRIBE
answered with a chunked RecordIO ``Event`` stream + ``Mesos-Stream-Id``, every other ``Call``
answered ``202``) so that ``V1HttpSchedulerDriver`` runs end-to-end without Mesos, and so the
cluster can run as its own process (``python -m dcos_commons_amd.mesos.http_master``).

Semantics kept from Mesos: calls must carry the stream id of the framework's current
subscription (``400`` otherwise); a re-SUBSCRIBE with the same FrameworkID fails over (the old
stream receives ``ERROR`` and is closed); a dropped stream disconnects the framework (its offers
are rescinded, tasks keep running until the failover timeout); ``redirect_to`` makes this
instance behave as a non-leading master (``307``). Binds 127.0.0.1 unless told otherwise.
"""
from __future__ import annotations

import argparse
import json
import logging
import queue
import select
import socket
import sys
import threading
import time
import uuid
from http.server import BaseHTTPRequestHandler
from typing import Dict, List, Optional

from dcos_commons_amd.mesos import protos as P
from dcos_commons_amd.mesos import recordio
from dcos_commons_amd.mesos.http_driver import JSON, PROTOBUF, SCHEDULER_PATH, STREAM_ID_HEADER, decode_message, \
    encode_message
from dcos_commons_amd.mesos.local_master import TERMINAL, LocalMaster, gpu_agent_specs
from dcos_commons_amd.utils.http_server import QuietThreadingHTTPServer

LOGGER = logging.getLogger(__name__)
_CLOSE = object()
_PEER_POLL_S = 0.25


class _EventSink:
    """Scheduler-shaped object the LocalMaster delivers to; turns callbacks into v1 Events."""

    def __init__(self, sub: "_Subscription"):
        self.sub = sub

    def registered(self, driver, framework_id, master_info) -> None:
        ev = P.Event(type=P.Event.SUBSCRIBED)
        ev.subscribed.framework_id.CopyFrom(framework_id)
        ev.subscribed.heartbeat_interval_seconds = self.sub.heartbeat_s
        ev.subscribed.master_info.CopyFrom(master_info)
        self.sub.put(ev)

    def resource_offers(self, driver, offers) -> None:
        ev = P.Event(type=P.Event.OFFERS)
        ev.offers.offers.extend(offers)
        self.sub.put(ev)

    def offer_rescinded(self, driver, offer_id) -> None:
        ev = P.Event(type=P.Event.RESCIND)
        ev.rescind.offer_id.CopyFrom(offer_id)
        self.sub.put(ev)

    def status_update(self, driver, status) -> None:
        ev = P.Event(type=P.Event.UPDATE)
        ev.update.status.CopyFrom(status)
        self.sub.put(ev)

    def error(self, driver, message: str) -> None:
        ev = P.Event(type=P.Event.ERROR)
        ev.error.message = message
        self.sub.put(ev)


class _Subscription:
    """Plays the ``driver`` role towards LocalMaster for one SUBSCRIBE stream."""

    def __init__(self, heartbeat_s: float, content_type: str):
        self.stream_id = str(uuid.uuid4())
        self.heartbeat_s = heartbeat_s
        self.content_type = content_type
        self.scheduler = _EventSink(self)
        self.queue: "queue.Queue" = queue.Queue()
        self._framework_id: Optional[str] = None
        self.closed = threading.Event()
        self.acknowledged: List[bytes] = []

    def _deliver(self, fn) -> None:
        if not self.closed.is_set():
            fn(self.scheduler)

    def put(self, ev) -> None:
        if not self.closed.is_set():
            self.queue.put(ev)

    def close(self) -> None:
        if not self.closed.is_set():
            self.closed.set()
            self.queue.put(_CLOSE)


def apply_call(m: LocalMaster, fid: str, call: P.Call, sub) -> int:
    """Applies one v1 scheduler ``Call`` of framework ``fid`` (already authenticated to its
    subscription ``sub``) to the master: 202, or 400 for a call type a scheduler may not send.
    Shared by the HTTP front end and the framed stream front end (``mesos.stream_api``)."""
    t = call.type
    if t == P.Call.ACCEPT:
        refuse = call.accept.filters.refuse_seconds if call.accept.HasField("filters") else 5.0
        m.accept(fid, [o.value for o in call.accept.offer_ids], list(call.accept.operations), refuse)
    elif t == P.Call.DECLINE:
        refuse = call.decline.filters.refuse_seconds if call.decline.HasField("filters") else 5.0
        m.decline(fid, [o.value for o in call.decline.offer_ids], refuse)
    elif t == P.Call.REVIVE:
        m.revive(fid)
    elif t == P.Call.SUPPRESS:
        m.suppress(fid)
    elif t == P.Call.KILL:
        m.kill(fid, call.kill.task_id.value)
    elif t == P.Call.RECONCILE:
        statuses = []
        for task in call.reconcile.tasks:
            s = P.TaskStatus()
            s.task_id.CopyFrom(task.task_id)
            if task.HasField("agent_id"):
                s.agent_id.CopyFrom(task.agent_id)
            statuses.append(s)
        m.reconcile(fid, statuses)
    elif t == P.Call.ACKNOWLEDGE:
        sub.acknowledged.append(call.acknowledge.uuid)
    elif t == P.Call.TEARDOWN:
        m.teardown(fid)
    elif t in (P.Call.MESSAGE, P.Call.REQUEST, P.Call.SHUTDOWN):
        pass
    else:
        return 400
    return 202


class HttpMaster:
    def __init__(self, master: LocalMaster, host: str = "127.0.0.1", port: int = 0,
                 heartbeat_s: float = 15.0, redirect_to: Optional[str] = None):
        self.master = master
        self.heartbeat_s = heartbeat_s
        self.redirect_to = redirect_to
        self.subscriptions: Dict[str, _Subscription] = {}
        self._lock = threading.Lock()
        self.calls: Dict[str, int] = {}
        facade = self

        class Handler(_Handler):
            owner = facade

        self.httpd = QuietThreadingHTTPServer((host, port), Handler)
        self.httpd.daemon_threads = True
        self._thread: Optional[threading.Thread] = None

    @property
    def port(self) -> int:
        return self.httpd.server_address[1]

    @property
    def url(self) -> str:
        return f"http://{self.httpd.server_address[0]}:{self.port}"

    def start(self) -> "HttpMaster":
        self._thread = threading.Thread(target=self.httpd.serve_forever, name="http-master", daemon=True)
        self._thread.start()
        return self

    def stop(self) -> None:
        with self._lock:
            subs = list(self.subscriptions.values())
        for s in subs:
            s.close()
        if getattr(self, "_zk", None) is not None:
            self._zk.close()
        self.httpd.shutdown()
        self.httpd.server_close()

    def register_in_zk(self, connect: str, path: str = "/mesos"):
        """Publishes this master as ``<path>/json.info_<seq>`` (ephemeral), like a Mesos leader."""
        from dcos_commons_amd.storage import zookeeper as Z

        client = Z.ZkClient(connect).start()
        client.ensure_path(path)
        host, port = self.httpd.server_address[:2]
        info = {"id": self.master.master_info.id, "hostname": host, "port": port,
                "address": {"hostname": host, "ip": host, "port": port}}
        client.create(path + "/json.info_", json.dumps(info).encode(), ephemeral=True, sequence=True)
        self._zk = client
        return client

    def drop_streams(self) -> None:
        """Closes every event stream (simulates a master failover / network cut)."""
        with self._lock:
            subs = list(self.subscriptions.values())
        for s in subs:
            s.close()

    # -- call handling ------------------------------------------------------------------
    def _count(self, call_type: int) -> None:
        name = P.Call.Type.Name(call_type)
        with self._lock:
            self.calls[name] = self.calls.get(name, 0) + 1

    def subscribe(self, call: P.Call, content_type: str) -> _Subscription:
        sub = _Subscription(self.heartbeat_s, content_type)
        info = call.subscribe.framework_info
        fid = info.id.value if info.HasField("id") else ""
        with self._lock:
            # unbind the old stream now: when its handler notices the close it must not disconnect
            # the framework, which by then belongs to this new subscription
            old = self.subscriptions.pop(fid, None) if fid else None
        if old is not None:
            old.scheduler.error(None, "Framework failed over")
            old.close()
        self._count(call.type)
        self.master.subscribe(sub, info)
        return sub

    def bind(self, sub: _Subscription) -> None:
        with self._lock:
            self.subscriptions[sub._framework_id] = sub

    def unbind(self, sub: _Subscription) -> None:
        fid = sub._framework_id
        with self._lock:
            current = self.subscriptions.get(fid) is sub
            if current:
                del self.subscriptions[fid]
        if current and fid:
            self.master.disconnect(fid)

    def handle(self, call: P.Call, stream_id: Optional[str]) -> int:
        fid = call.framework_id.value
        with self._lock:
            sub = self.subscriptions.get(fid)
        if sub is None or stream_id != sub.stream_id:
            return 400
        self._count(call.type)
        code = apply_call(self.master, fid, call, sub)
        if call.type == P.Call.TEARDOWN:
            with self._lock:
                self.subscriptions.pop(fid, None)
            sub.close()
        return code

    def state(self) -> dict:
        def do():
            agents = []
            for aid, a in self.master.agents.items():
                agents.append({"id": aid, "hostname": a.spec.hostname,
                               "tasks": {tid: P.TaskState.Name(t.status.state) for tid, t in a.tasks.items()
                                         if t.status.state not in TERMINAL}})
            return {"frameworks": sorted(self.master.frameworks), "agents": agents}
        out = self.master.call(do)
        with self._lock:
            out["calls"] = dict(self.calls)
        return out


class _Handler(BaseHTTPRequestHandler):
    protocol_version = "HTTP/1.1"
    owner: HttpMaster = None

    def log_message(self, fmt, *args):  # route through logging
        LOGGER.debug("%s " + fmt, self.address_string(), *args)

    def setup(self):
        super().setup()
        # events go out as they happen, one small write each: without TCP_NODELAY an event
        # written while the previous one is unacknowledged waits for the scheduler's delayed ACK
        self.connection.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)

    def _reply(self, status: int, body: bytes = b"", ctype: str = "text/plain") -> None:
        self.send_response(status)
        self.send_header("Content-Type", ctype)
        self.send_header("Content-Length", str(len(body)))
        self._headers_buffer.append(b"\r\n" + body)   # status line, headers and body in one write
        self.flush_headers()

    def do_GET(self):  # noqa: N802
        if self.path in ("/health", "/master/health"):
            self._reply(200)
        elif self.path in ("/state", "/master/state"):
            self._reply(200, json.dumps(self.owner.state()).encode(), JSON)
        else:
            self._reply(404)

    def do_POST(self):  # noqa: N802
        n = int(self.headers.get("Content-Length") or 0)
        body = self.rfile.read(n) if n else b""
        if self.path != SCHEDULER_PATH:
            self._reply(404)
            return
        if self.owner.redirect_to:
            self.send_response(307)
            self.send_header("Location", self.owner.redirect_to + SCHEDULER_PATH)
            self.send_header("Content-Length", "0")
            self.end_headers()
            return
        ctype = (self.headers.get("Content-Type") or JSON).split(";")[0].strip()
        if ctype not in (JSON, PROTOBUF):
            self._reply(415, b"unsupported content type")
            return
        accept = (self.headers.get("Accept") or ctype).split(";")[0].strip()
        accept = accept if accept in (JSON, PROTOBUF) else ctype
        try:
            call = decode_message(P.Call, body, ctype)
        except Exception as e:  # noqa: BLE001
            self._reply(400, f"Failed to parse body: {e}".encode())
            return
        if call.type == P.Call.SUBSCRIBE:
            self._stream(call, accept)
            return
        status = self.owner.handle(call, self.headers.get(STREAM_ID_HEADER))
        self._reply(status, b"" if status == 202 else b"Call rejected: missing or stale Mesos-Stream-Id")

    def _peer_closed(self) -> bool:
        """True only on evidence that the scheduler went away: EOF, reset or a poll error.

        ``poll`` (not ``select``) so that descriptors >= FD_SETSIZE work in a master that holds
        many sockets; the peek is non-blocking, and "nothing to read" means the peer is alive."""
        try:
            p = select.poll()
            p.register(self.connection.fileno(), select.POLLIN | select.POLLPRI)
            events = p.poll(0)
        except (OSError, ValueError):  # fileno() of a closed socket
            return True
        if not events:
            return False
        mask = events[0][1]
        if mask & (select.POLLERR | select.POLLNVAL):
            return True
        try:
            return self.connection.recv(1, socket.MSG_PEEK | socket.MSG_DONTWAIT) == b""
        except (BlockingIOError, InterruptedError):
            return False
        except OSError:
            return True

    def _stream(self, call: P.Call, accept: str) -> None:
        sub = self.owner.subscribe(call, accept)
        self.send_response(200)
        self.send_header("Content-Type", accept)
        self.send_header(STREAM_ID_HEADER, sub.stream_id)
        self.send_header("Transfer-Encoding", "chunked")
        self.end_headers()
        bound = False
        try:
            idle_s = 0.0
            while True:
                try:
                    ev = sub.queue.get(timeout=_PEER_POLL_S)
                    idle_s = 0.0
                except queue.Empty:
                    # a scheduler that died closes its connection: notice it now, like Mesos does,
                    # instead of at the next write
                    if self._peer_closed():
                        break
                    idle_s += _PEER_POLL_S
                    if idle_s < sub.heartbeat_s:
                        continue
                    idle_s = 0.0
                    ev = P.Event(type=P.Event.HEARTBEAT)
                if ev is _CLOSE:
                    break
                if not bound and ev.type == P.Event.SUBSCRIBED:
                    self.owner.bind(sub)
                    bound = True
                rec = recordio.encode(encode_message(ev, accept))
                self.wfile.write(b"%x\r\n%s\r\n" % (len(rec), rec))
                self.wfile.flush()
            self.wfile.write(b"0\r\n\r\n")
            self.wfile.flush()
        except (BrokenPipeError, ConnectionResetError, OSError):
            pass
        finally:
            sub.close()
            if bound:
                self.owner.unbind(sub)
            self.close_connection = True


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description="Local Mesos-compatible master (v1 scheduler HTTP API)")
    ap.add_argument("--host", default="127.0.0.1")
    ap.add_argument("--port", type=int, default=5050)
    ap.add_argument("--agents", type=int, default=3)
    ap.add_argument("--cpus", type=float, default=8.0)
    ap.add_argument("--mem", type=float, default=32768.0)
    ap.add_argument("--disk", type=float, default=65536.0)
    ap.add_argument("--gpus", default="0",
                    help="GPUs per agent, or 'auto' to split this node's discovered GPUs between the agents")
    ap.add_argument("--allocation-interval", type=float, default=1.0)
    ap.add_argument("--heartbeat", type=float, default=15.0)
    args = ap.parse_args(argv)
    logging.basicConfig(level=logging.INFO, format="%(asctime)s %(levelname)s %(name)s: %(message)s")
    lm = LocalMaster(allocation_interval_s=args.allocation_interval)
    for spec in gpu_agent_specs(args.agents, args.gpus if args.gpus == "auto" else int(args.gpus),
                                lambda i: f"agent-{i}.local", cpus=args.cpus, mem=args.mem, disk=args.disk):
        lm.add_agent(spec)
    hm = HttpMaster(lm, args.host, args.port, heartbeat_s=args.heartbeat).start()
    print(f"master listening on {hm.url}", flush=True)
    try:
        while True:
            time.sleep(3600)
    except KeyboardInterrupt:
        pass
    hm.stop()
    lm.shutdown()
    return 0


if __name__ == "__main__":
    sys.exit(main())
