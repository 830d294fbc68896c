"""The v1 scheduler API's messages over one persistent framed socket.

The v1 HTTP API (``http_driver`` / ``http_master``) wraps every ``Call`` in an HTTP request and
the ``Event`` stream in chunked RecordIO. Between processes of one node (the bench's scheduler and
its stand-in master) most of its cost is Python's HTTP machinery, not the messages. This transport
keeps the messages and their semantics and drops the HTTP layer, the way the reference's V0
driver talks to the master over libprocess messages rather than over HTTP requests:

* one TCP connection per subscription; every frame is a 4-byte big-endian length plus a
  serialized protobuf;
* scheduler -> master: ``Call`` frames, the first of which must be ``SUBSCRIBE``; later calls
  need no stream id (the connection is the stream) and get no answer (a v1 call is answered
  ``202`` before it is applied anyway);
* master -> scheduler: ``Event`` frames. The driver hands every ``UPDATE`` that arrived in one
  read to the scheduler together (``status_updates``), as ``V1HttpSchedulerDriver`` does;
* the connection closing is the stream ending: the master disconnects the framework (failover
  semantics as in ``HttpMaster``), the driver reports ``disconnected``.

``StreamSchedulerDriver("host:port", ...)`` is the scheduler side (``SDK_MESOS_MASTER=
mesos-stream://host:port``); ``StreamMaster(local_master)`` serves a ``LocalMaster``.
"""
from __future__ import annotations

import contextlib
import logging
import socket
import struct
import threading
from typing import Dict, Iterator, List, Optional

from dcos_commons_amd.mesos import protos as P
from dcos_commons_amd.mesos.http_driver import MesosCallError, V1HttpSchedulerDriver
from dcos_commons_amd.mesos.http_master import apply_call

LOGGER = logging.getLogger(__name__)
SCHEME = "mesos-stream://"
_LEN = struct.Struct(">I")
MAX_FRAME = 64 << 20


def frame(payload: bytes) -> bytes:
    return _LEN.pack(len(payload)) + payload


class FrameReader:
    """Reads length-prefixed frames; ``batches()`` yields every frame that one ``recv`` completed,
    together, so a reader that fell behind processes what queued up in one go."""

    def __init__(self, sock: socket.socket, bufsize: int = 1 << 16):
        self.sock = sock
        self.bufsize = bufsize
        self._buf = bytearray()

    def batches(self) -> Iterator[List[bytes]]:
        while True:
            data = self.sock.recv(self.bufsize)
            if not data:
                return
            self._buf += data
            out = self._complete()
            if out:
                yield out

    def ready(self) -> List[bytes]:
        """The complete frames that have arrived by now, without blocking (a reader that waited
        before handling its batch picks up what queued up meanwhile). An end of stream seen here
        is seen again by the next blocking read."""
        while True:
            try:
                data = self.sock.recv(self.bufsize, socket.MSG_DONTWAIT)
            except (BlockingIOError, InterruptedError):
                break
            if not data:
                break
            self._buf += data
            if len(data) < self.bufsize:
                break
        return self._complete()

    def _complete(self) -> List[bytes]:
        buf = self._buf
        out = []
        pos = 0
        while len(buf) - pos >= 4:
            (n,) = _LEN.unpack_from(buf, pos)
            if n > MAX_FRAME:
                raise OSError(f"frame of {n} bytes exceeds the {MAX_FRAME}-byte limit")
            if len(buf) - pos - 4 < n:
                break
            out.append(bytes(buf[pos + 4:pos + 4 + n]))
            pos += 4 + n
        if pos:
            del buf[:pos]
        return out


def _nodelay(sock: socket.socket) -> None:
    try:
        sock.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
    except OSError:
        pass


# -- master side ---------------------------------------------------------------------------
class _Sink:
    """Scheduler-shaped object the LocalMaster delivers to: each callback becomes one ``Event``
    frame, written on the master's own thread (a local socket write of a few hundred bytes)."""

    def __init__(self, sub: "_StreamSubscription"):
        self.sub = sub

    def registered(self, driver, framework_id, master_info) -> None:
        # bound under its framework id before SUBSCRIBED goes out (a re-SUBSCRIBE then fails it over)
        self.sub.on_registered(framework_id.value)
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


_CORK = threading.local()


@contextlib.contextmanager
def corked():
    """Events put on this thread's subscriptions inside the block are written at its end, one
    write per connection (``LocalMaster.batch_delivery``: a runtime report's STARTING, RUNNING and
    readiness reach the scheduler in one read instead of three)."""
    pending = getattr(_CORK, "pending", None)
    if pending is not None:      # nested: the outer block writes
        yield
        return
    _CORK.pending = pending = {}
    try:
        yield
    finally:
        _CORK.pending = None
        for sub, frames in pending.values():
            sub.write(b"".join(frames))


class _StreamSubscription:
    """Plays the ``driver`` role towards LocalMaster for one connection."""

    def __init__(self, sock: socket.socket, heartbeat_s: float):
        self.sock = sock
        self.heartbeat_s = heartbeat_s
        self.scheduler = _Sink(self)
        self._framework_id: Optional[str] = None   # set by LocalMaster.subscribe
        self._wlock = threading.Lock()
        self.closed = threading.Event()
        self.acknowledged: List[bytes] = []
        self.torn_down = False
        self.on_registered = lambda framework_id: None

    def _deliver(self, fn) -> None:
        if not self.closed.is_set():
            fn(self.scheduler)

    def put(self, ev: P.Event) -> None:
        if self.closed.is_set():
            return
        data = frame(ev.SerializeToString())
        pending = getattr(_CORK, "pending", None)
        if pending is not None:
            pending.setdefault(id(self), (self, []))[1].append(data)
            return
        self.write(data)

    def write(self, data: bytes) -> None:
        if self.closed.is_set() or not data:
            return
        try:
            with self._wlock:
                self.sock.sendall(data)
        except OSError:
            self.close()

    def close(self) -> None:
        if self.closed.is_set():
            return
        self.closed.set()
        try:
            self.sock.shutdown(socket.SHUT_RDWR)
        except OSError:
            pass


class StreamMaster:
    """Serves a ``LocalMaster`` to ``StreamSchedulerDriver``s (binds 127.0.0.1 by default: the
    link carries no authentication)."""

    def __init__(self, master, host: str = "127.0.0.1", port: int = 0, heartbeat_s: float = 15.0):
        self.master = master
        self.heartbeat_s = heartbeat_s
        self.sock = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
        self.sock.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
        self.sock.bind((host, port))
        self.sock.listen(64)
        self._lock = threading.Lock()
        self.subscriptions: Dict[str, _StreamSubscription] = {}
        self._all: List[_StreamSubscription] = []
        self.calls: Dict[str, int] = {}
        self._thread = threading.Thread(target=self._accept_loop, name="stream-master", daemon=True)

    @property
    def port(self) -> int:
        return self.sock.getsockname()[1]

    @property
    def address(self) -> str:
        return f"{self.sock.getsockname()[0]}:{self.port}"

    def start(self) -> "StreamMaster":
        self.master.batch_delivery = corked
        self._thread.start()
        return self

    def set_master(self, master) -> None:
        """Serves ``master`` from now on; every open subscription (of the old one) is closed."""
        self.drop_streams()
        self.master = master
        master.batch_delivery = corked

    def drop_streams(self) -> None:
        with self._lock:
            subs, self._all = list(self._all), []
            self.subscriptions.clear()
        for s in subs:
            s.close()

    def stop(self) -> None:
        self.drop_streams()
        try:
            self.sock.close()
        except OSError:
            pass

    def _accept_loop(self) -> None:
        while True:
            try:
                conn, _ = self.sock.accept()
            except OSError:
                return
            _nodelay(conn)
            threading.Thread(target=self._serve, args=(conn,), name="stream-master-conn", daemon=True).start()

    def _count(self, t: int) -> None:
        name = P.Call.Type.Name(t)
        with self._lock:
            self.calls[name] = self.calls.get(name, 0) + 1

    def _serve(self, conn: socket.socket) -> None:
        reader = FrameReader(conn)
        sub: Optional[_StreamSubscription] = None
        master = self.master
        try:
            for batch in reader.batches():
                for data in batch:
                    call = P.Call.FromString(data)
                    if sub is None:
                        if call.type != P.Call.SUBSCRIBE:
                            return
                        sub = self._subscribe(conn, call)
                        master = self.master
                        continue
                    fid = sub._framework_id
                    if not fid or (call.framework_id.value and call.framework_id.value != fid):
                        LOGGER.warning("dropping %s: not from the subscribed framework", P.Call.Type.Name(call.type))
                        continue
                    self._count(call.type)
                    if apply_call(master, fid, call, sub) != 202:
                        LOGGER.warning("dropping call %s: not a scheduler call", P.Call.Type.Name(call.type))
                    if call.type == P.Call.TEARDOWN:
                        sub.torn_down = True
                        with self._lock:
                            if self.subscriptions.get(fid) is sub:
                                del self.subscriptions[fid]
                        return
        except (OSError, ValueError) as e:
            LOGGER.debug("stream connection ended: %s", e)
        finally:
            if sub is not None:
                fid = sub._framework_id
                with self._lock:
                    current = fid and self.subscriptions.get(fid) is sub
                    if current:
                        del self.subscriptions[fid]
                    if sub in self._all:
                        self._all.remove(sub)
                if current and not sub.torn_down and master is self.master:
                    master.disconnect(fid)
                sub.close()
            try:
                conn.close()
            except OSError:
                pass

    def _subscribe(self, conn: socket.socket, call: P.Call) -> _StreamSubscription:
        sub = _StreamSubscription(conn, self.heartbeat_s)
        info = call.subscribe.framework_info
        fid = info.id.value if info.HasField("id") else ""
        with self._lock:
            old = self.subscriptions.pop(fid, None) if fid else None
            self._all.append(sub)
        if old is not None:
            old.scheduler.error(None, "Framework failed over")
            old.close()
        self._count(call.type)

        def bind(framework_id: str) -> None:
            with self._lock:
                self.subscriptions[framework_id] = sub
        sub.on_registered = bind
        self.master.subscribe(sub, info)
        return sub


# -- scheduler side ------------------------------------------------------------------------
def _with_fid(call: P.Call, fid: Optional[str]) -> P.Call:
    if fid:
        call.framework_id.value = fid
    return call


class StreamSchedulerDriver(V1HttpSchedulerDriver):
    """``SchedulerDriver`` over the framed stream: the callbacks, acknowledgements and update
    batching of ``V1HttpSchedulerDriver``, its HTTP transport replaced by one socket. A call is
    one frame written by the caller's thread (no sender thread: the write does not wait for an
    answer, so the caller never blocks on the master)."""

    def __init__(self, address: str, scheduler, framework_info: P.FrameworkInfo, connect_timeout_s: float = 10.0,
                 reconnect: bool = False, **_ignored):
        if address.startswith(SCHEME):
            address = address[len(SCHEME):]
        host, _, port = address.rstrip("/").rpartition(":")
        self.address = (host or "127.0.0.1", int(port))
        super().__init__(f"http://{host or '127.0.0.1'}:{port}", scheduler, framework_info,
                         connect_timeout_s=connect_timeout_s, reconnect=reconnect, async_calls=False)
        self._sock: Optional[socket.socket] = None
        self._wlock = threading.Lock()

    def _stream_loop(self) -> None:
        backoff = self.backoff_s
        while not self._stopped.is_set():
            reason = "event stream ended"
            try:
                sock = socket.create_connection(self.address, timeout=self.connect_timeout_s)
                sock.settimeout(None)
                _nodelay(sock)
                with self._wlock:
                    self._sock = sock
                    sock.sendall(frame(self._subscribe_call().SerializeToString()))
                self.stream_id = "stream"
                backoff = self.backoff_s
                reader = FrameReader(sock)
                for batch in reader.batches():
                    if self._stopped.is_set():
                        break
                    events = [P.Event.FromString(data) for data in batch]
                    gate = self._status_gate
                    if gate is not None and any(ev.type == P.Event.UPDATE for ev in events):
                        # a status waits for a running offer cycle (FrameworkScheduler's gate);
                        # what arrived meanwhile joins this batch, so it is handled in one go
                        if gate():
                            events.extend(P.Event.FromString(data) for data in reader.ready())
                    updates: List[P.TaskStatus] = []
                    for ev in events:
                        if ev.type == P.Event.UPDATE:
                            updates.append(ev.update.status)
                            continue
                        if updates:
                            self._on_updates(updates)
                            updates = []
                        self._on_event(ev)
                    if updates:
                        self._on_updates(updates)
            except (OSError, ValueError) as e:
                reason = f"{type(e).__name__}: {e}"
            self.stream_id = None
            self._subscribed.clear()
            self._close_stream()
            if self._stopped.is_set() or self._tearing_down:
                self._stopped.set()
                return
            LOGGER.warning("Lost Mesos event stream (%s)", reason)
            if self._subscribed_once and not self.reconnect:
                self._call_scheduler("disconnected")
                self.exit_status = 5
                self._stopped.set()
                return
            self._stopped.wait(backoff)
            backoff = min(backoff * 2, self.max_backoff_s)

    def _send(self, call: P.Call) -> None:
        self._send_now(call)

    def _send_now(self, call: P.Call) -> None:
        if self._framework_id:
            call.framework_id.value = self._framework_id
        data = frame(call.SerializeToString())
        with self._wlock:
            sock = self._sock
            if sock is None or self.stream_id is None:
                raise MesosCallError(0, f"not subscribed; dropping {P.Call.Type.Name(call.type)}")
            try:
                sock.sendall(data)
            except OSError as e:
                raise MesosCallError(0, str(e)) from e

    def _acknowledge_all(self, statuses: List[P.TaskStatus]) -> None:
        """A batch's ACKNOWLEDGEs leave in one write: one frame per call, so the master reads
        them as one batch (its reader hands every frame of a read over together)."""
        calls = [c for c in map(self._ack_call, statuses) if c is not None]
        if len(calls) < 2:
            for c in calls:
                self._send_quiet(c)
            return
        fid = self._framework_id
        data = b"".join(frame(_with_fid(c, fid).SerializeToString()) for c in calls)
        with self._wlock:
            sock = self._sock
            if sock is None or self.stream_id is None:
                LOGGER.warning("ACKNOWLEDGE of %d update(s) dropped: not subscribed", len(calls))
                return
            try:
                sock.sendall(data)
            except OSError as e:
                LOGGER.warning("ACKNOWLEDGE of %d update(s) failed: %s", len(calls), e)

    def _send_quiet(self, call: P.Call) -> None:
        try:
            self._send_now(call)
        except MesosCallError as e:
            LOGGER.warning("ACKNOWLEDGE of %s failed: %s", call.acknowledge.task_id.value, e)

    def flush(self, timeout_s: float = 10.0) -> bool:
        return True

    def _close_stream(self) -> None:
        with self._wlock:
            sock, self._sock = self._sock, None
        if sock is not None:
            try:
                sock.shutdown(socket.SHUT_RDWR)
            except OSError:
                pass
            sock.close()
