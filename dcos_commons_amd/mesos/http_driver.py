"""Mesos v1 scheduler HTTP API driver.

Reference: the SDK builds a ``MesosToSchedulerDriverAdapter`` (external mesos-http-adapter 0.4.1)
in ``framework/SchedulerDriverFactory.java:80-158`` and uses the V1 API by default
(``SchedulerConfig.java:583``). This is a from-scratch implementation of the same contract:

* one long-lived ``SUBSCRIBE`` POST whose response is a RecordIO stream of ``Event``s, read on a
  dedicated thread which invokes the scheduler callbacks in stream order;
* every other ``Call`` is a separate POST carrying the ``Mesos-Stream-Id`` header and answered with
  ``202 Accepted``; calls come from several scheduler threads (offer processor, task killer,
  reconcilers) so each thread keeps its own keep-alive connection;
* implicit acknowledgements: after ``status_update`` returns, updates that carry a ``uuid`` are
  ACKNOWLEDGEd (the adapter's default);
* UPDATE events read from the stream together (the scheduler fell behind while a previous one was
  stored) go to ``scheduler.status_updates`` in one call when the scheduler has it, so they are
  persisted in one transaction; each is still acknowledged only after that call returns;
* ``307 Temporary Redirect`` follows the leading master; ``503`` (no leader yet) backs off;
* heartbeats: the stream is considered dead after ``heartbeat_misses`` intervals of silence.

Loss of the stream calls ``scheduler.disconnected`` (the SDK then exits, ``ProcessExit
DISCONNECTED``) unless ``reconnect`` is set, in which case the driver resubscribes with its
FrameworkID and calls ``scheduler.reregistered`` (the adapter's failover behaviour).

Wire formats: ``application/x-protobuf`` (default; binary-compatible with the Mesos bindings, as
``protos`` is built from the v1 .proto) or ``application/json``.
"""
from __future__ import annotations

import base64
import collections
import http.client
import json
import logging
import socket
import threading
import time
import urllib.parse
from typing import Callable, Iterable, List, Optional

from dcos_commons_amd.framework.driver import SchedulerDriver
from dcos_commons_amd.mesos import protos as P
from dcos_commons_amd.mesos import recordio

LOGGER = logging.getLogger(__name__)

PROTOBUF = "application/x-protobuf"
JSON = "application/json"
SCHEDULER_PATH = "/api/v1/scheduler"
STREAM_ID_HEADER = "Mesos-Stream-Id"


class MesosCallError(RuntimeError):
    def __init__(self, status: int, body: str):
        super().__init__(f"Mesos call failed: HTTP {status}: {body[:200]}")
        self.status = status
        self.body = body


def encode_message(msg, content_type: str) -> bytes:
    if content_type == PROTOBUF:
        return msg.SerializeToString()
    return json.dumps(P.to_json(msg), separators=(",", ":")).encode("utf-8")


def decode_message(cls, data: bytes, content_type: str):
    if content_type == PROTOBUF:
        m = cls()
        m.ParseFromString(data)
        return m
    return P.from_json(cls, json.loads(data.decode("utf-8")))


class V1HttpSchedulerDriver(SchedulerDriver):
    def __init__(self, master_url: str, scheduler, framework_info: P.FrameworkInfo,
                 credential: Optional[P.Credential] = None, content_type: str = PROTOBUF,
                 implicit_acknowledgements: bool = True, reconnect: bool = False,
                 heartbeat_misses: int = 5, connect_timeout_s: float = 10.0,
                 backoff_s: float = 0.5, max_backoff_s: float = 10.0, token_provider=None,
                 async_calls: bool = False):
        if content_type not in (PROTOBUF, JSON):
            raise ValueError(f"unsupported content type {content_type}")
        self.master_url = master_url.rstrip("/")
        self.scheduler = scheduler
        self.framework_info = P.FrameworkInfo()
        self.framework_info.CopyFrom(framework_info)
        self.credential = credential
        # side-channel auth: a principal-only credential plus a DC/OS IAM token per call
        self.token_provider = token_provider
        self.content_type = content_type
        self.implicit_acknowledgements = implicit_acknowledgements
        self.reconnect = reconnect
        self.heartbeat_misses = heartbeat_misses
        self.connect_timeout_s = connect_timeout_s
        self.backoff_s = backoff_s
        self.max_backoff_s = max_backoff_s
        self.stream_id: Optional[str] = None
        self.master_info: Optional[P.MasterInfo] = None
        self._framework_id: Optional[str] = framework_info.id.value if framework_info.HasField("id") else None
        self._subscribed_once = False
        self._stopped = threading.Event()
        self._subscribed = threading.Event()
        self._thread: Optional[threading.Thread] = None
        self._stream_conn: Optional[http.client.HTTPConnection] = None
        self._local = threading.local()
        self._conns: List[http.client.HTTPConnection] = []
        self._conns_lock = threading.Lock()
        self.exit_status = 0
        self._tearing_down = False
        # async_calls: calls are POSTed in submission order by one sender thread and the caller
        # returns at once, like the reference's libprocess-backed driver (a call's outcome is
        # logged, not raised). The offer thread then does not wait for an ACCEPT's HTTP round trip,
        # nor the event stream for an ACKNOWLEDGE's before it reads the next event.
        self.async_calls = async_calls
        self._outbox: "collections.deque[P.Call]" = collections.deque()
        self._outbox_cond = threading.Condition()
        self._in_flight = 0
        self._sender: Optional[threading.Thread] = None
        self._status_gate: Optional[Callable[[], bool]] = None

    # -- lifecycle ---------------------------------------------------------------------
    @property
    def framework_id(self) -> Optional[str]:
        return self._framework_id

    def start(self) -> None:
        if self._thread is not None:
            return
        self._thread = threading.Thread(target=self._stream_loop, name="mesos-v1-stream", daemon=True)
        self._thread.start()

    def run(self) -> int:
        self.start()
        self._stopped.wait()
        return self.exit_status

    def join(self, timeout: Optional[float] = None) -> bool:
        return self._stopped.wait(timeout)

    def wait_subscribed(self, timeout: Optional[float] = None) -> bool:
        return self._subscribed.wait(timeout)

    def stop(self, failover: bool = True) -> None:
        if self._stopped.is_set():
            return
        self.flush()
        if not failover and self._framework_id and self.stream_id and not self._tearing_down:
            try:
                self._send_now(P.Call(type=P.Call.TEARDOWN))
            except Exception as e:  # noqa: BLE001
                LOGGER.warning("TEARDOWN on stop failed: %s", e)
        self._stopped.set()
        self._close_stream()
        with self._conns_lock:
            for c in self._conns:
                c.close()
            self._conns.clear()

    # -- SchedulerDriver calls ---------------------------------------------------------
    def accept_offers(self, offer_ids: Iterable[P.OfferID], operations: Iterable[P.Offer.Operation],
                      filters: Optional[P.Filters] = None) -> None:
        call = P.Call(type=P.Call.ACCEPT)
        call.accept.offer_ids.extend(offer_ids)
        call.accept.operations.extend(operations)
        if filters is not None:
            call.accept.filters.CopyFrom(filters)
        self._send(call)

    def decline_offer(self, offer_id: P.OfferID, filters: Optional[P.Filters] = None) -> None:
        self.decline_offers([offer_id], filters)

    def decline_offers(self, offer_ids, filters: Optional[P.Filters] = None) -> None:
        call = P.Call(type=P.Call.DECLINE)
        call.decline.offer_ids.extend(offer_ids)
        if filters is not None:
            call.decline.filters.CopyFrom(filters)
        self._send(call)

    def kill_task(self, task_id: P.TaskID, agent_id: Optional[P.AgentID] = None) -> None:
        call = P.Call(type=P.Call.KILL)
        call.kill.task_id.CopyFrom(task_id)
        if agent_id is not None:
            call.kill.agent_id.CopyFrom(agent_id)
        self._send(call)

    def reconcile_tasks(self, statuses: List[P.TaskStatus]) -> None:
        call = P.Call(type=P.Call.RECONCILE)
        for s in statuses:
            t = call.reconcile.tasks.add()
            t.task_id.CopyFrom(s.task_id)
            if s.HasField("agent_id"):
                t.agent_id.CopyFrom(s.agent_id)
        self._send(call)

    def revive_offers(self) -> None:
        self._send(P.Call(type=P.Call.REVIVE))

    def suppress_offers(self) -> None:
        self._send(P.Call(type=P.Call.SUPPRESS))

    def acknowledge_status_update(self, status: P.TaskStatus) -> None:
        call = self._ack_call(status)
        if call is not None:
            self._send(call)

    def send_framework_message(self, executor_id: P.ExecutorID, agent_id: P.AgentID, data: bytes) -> None:
        call = P.Call(type=P.Call.MESSAGE)
        call.message.executor_id.CopyFrom(executor_id)
        call.message.agent_id.CopyFrom(agent_id)
        call.message.data = data
        self._send(call)

    def teardown(self) -> None:
        # the master ends the event stream in answer: that is not a disconnection
        self._tearing_down = True
        self.flush()
        self._send_now(P.Call(type=P.Call.TEARDOWN))

    # -- transport ---------------------------------------------------------------------
    def _headers(self, accept: str) -> dict:
        h = {"Content-Type": self.content_type, "Accept": accept, "Connection": "keep-alive"}
        if self.token_provider is not None:
            try:
                tok = self.token_provider()
            except Exception as e:  # noqa: BLE001 -- IAM outage, bad credential, parse error...
                # status 0 = transport failure: SUBSCRIBE retries with backoff, calls retry below
                raise MesosCallError(0, f"auth token refresh failed: {type(e).__name__}: {e}") from e
            h["Authorization"] = "token=" + (tok.value if hasattr(tok, "value") else str(tok))
        elif self.credential is not None and self.credential.principal:
            token = f"{self.credential.principal}:{self.credential.secret or ''}".encode("utf-8")
            h["Authorization"] = "Basic " + base64.b64encode(token).decode("ascii")
        return h

    def _new_conn(self, timeout: Optional[float]) -> http.client.HTTPConnection:
        u = urllib.parse.urlsplit(self.master_url)
        cls = http.client.HTTPSConnection if u.scheme == "https" else http.client.HTTPConnection
        return cls(u.hostname, u.port or (443 if u.scheme == "https" else 80), timeout=timeout)

    def _thread_conn(self) -> http.client.HTTPConnection:
        conn = getattr(self._local, "conn", None)
        if conn is None or getattr(self._local, "url", None) != self.master_url:
            conn = self._new_conn(self.connect_timeout_s)
            self._local.conn, self._local.url = conn, self.master_url
            with self._conns_lock:
                self._conns.append(conn)
        return conn

    def _send(self, call: P.Call) -> None:
        if not self.async_calls:
            self._send_now(call)
            return
        with self._outbox_cond:
            self._outbox.append(call)
            if self._sender is None:
                self._sender = threading.Thread(target=self._send_loop, name="mesos-v1-calls", daemon=True)
                self._sender.start()
            self._outbox_cond.notify()

    def _send_loop(self) -> None:
        while True:
            with self._outbox_cond:
                while not self._outbox:
                    if self._stopped.is_set():
                        return
                    self._outbox_cond.wait(0.5)
                call = self._outbox.popleft()
                self._in_flight += 1
            try:
                self._send_now(call)
            except Exception as e:  # noqa: BLE001 -- the caller has moved on: report, keep sending
                LOGGER.error("Mesos %s call failed: %s", P.Call.Type.Name(call.type), e)
            finally:
                with self._outbox_cond:
                    self._in_flight -= 1
                    self._outbox_cond.notify_all()

    def flush(self, timeout_s: float = 10.0) -> bool:
        """Waits until every call submitted so far has been sent (async mode); True if it was."""
        if not self.async_calls:
            return True
        deadline = time.monotonic() + timeout_s
        with self._outbox_cond:
            while self._outbox or self._in_flight:
                left = deadline - time.monotonic()
                if left <= 0 or self._sender is None or not self._sender.is_alive():
                    return False
                self._outbox_cond.wait(min(left, 0.05))
        return True

    def _send_now(self, call: P.Call) -> None:
        if self._framework_id:
            call.framework_id.value = self._framework_id
        if self.stream_id is None:
            raise MesosCallError(0, f"not subscribed; dropping {P.Call.Type.Name(call.type)}")
        body = encode_message(call, self.content_type)
        backoff = self.backoff_s
        for attempt in range(3):
            conn = self._thread_conn()
            try:
                headers = self._headers(self.content_type)
            except MesosCallError as e:
                if attempt == 2 or self._stopped.is_set():
                    raise
                LOGGER.warning("%s: retrying %s in %.1fs", e, P.Call.Type.Name(call.type), backoff)
                self._stopped.wait(backoff)
                backoff = min(backoff * 2, self.max_backoff_s)
                continue
            headers[STREAM_ID_HEADER] = self.stream_id
            try:
                conn.request("POST", SCHEDULER_PATH, body=body, headers=headers)
                resp = conn.getresponse()
                data = resp.read()
            except (OSError, http.client.HTTPException) as e:
                conn.close()
                self._local.conn = None
                if attempt == 2 or self._stopped.is_set():
                    raise MesosCallError(0, str(e)) from e
                continue
            if resp.status in (200, 202):
                return
            raise MesosCallError(resp.status, data.decode("utf-8", "replace"))

    def _close_stream(self) -> None:
        conn, self._stream_conn = self._stream_conn, None
        if conn is not None:
            try:
                if conn.sock is not None:
                    conn.sock.shutdown(socket.SHUT_RDWR)
            except OSError:
                pass
            conn.close()

    def _subscribe_call(self) -> P.Call:
        call = P.Call(type=P.Call.SUBSCRIBE)
        info = call.subscribe.framework_info
        info.CopyFrom(self.framework_info)
        if self._framework_id:
            info.id.value = self._framework_id
            call.framework_id.value = self._framework_id
        return call

    def _open_stream(self):
        """POSTs SUBSCRIBE (following redirects); returns the streaming response."""
        for _ in range(5):
            conn = self._new_conn(self.connect_timeout_s)
            self._stream_conn = conn
            body = encode_message(self._subscribe_call(), self.content_type)
            conn.request("POST", SCHEDULER_PATH, body=body, headers=self._headers(self.content_type))
            resp = conn.getresponse()
            if resp.status == 200:
                self.stream_id = resp.getheader(STREAM_ID_HEADER)
                if not self.stream_id:
                    raise MesosCallError(200, "SUBSCRIBE response carried no Mesos-Stream-Id")
                return resp
            data = resp.read().decode("utf-8", "replace")
            conn.close()
            if resp.status == 307:
                loc = resp.getheader("Location") or ""
                if loc.startswith("//"):
                    loc = urllib.parse.urlsplit(self.master_url).scheme + ":" + loc
                u = urllib.parse.urlsplit(loc)
                self.master_url = f"{u.scheme}://{u.netloc}"
                LOGGER.info("Redirected to leading master %s", self.master_url)
                continue
            raise MesosCallError(resp.status, data)
        raise MesosCallError(307, "too many redirects")

    def _stream_loop(self) -> None:
        backoff = self.backoff_s
        while not self._stopped.is_set():
            try:
                resp = self._open_stream()
                backoff = self.backoff_s
                self._consume(resp)
                reason = "event stream ended"
            except MesosCallError as e:
                if e.status in (400, 401, 403):
                    LOGGER.error("SUBSCRIBE rejected: %s", e)
                    self._call_scheduler("error", str(e))
                    self.exit_status = 1
                    self._stopped.set()
                    return
                reason = str(e)
            except (OSError, http.client.HTTPException, recordio.RecordIOError) as e:
                reason = f"{type(e).__name__}: {e}"
            except Exception as e:  # noqa: BLE001 -- e.g. stop() closed the response mid-read
                if not self._stopped.is_set():
                    raise
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

    def _consume(self, resp) -> None:
        dec = recordio.Decoder()
        # a chunked stream is de-chunked here from the socket's buffered reader: every event that
        # has arrived is decoded in one pass (http.client returns one chunk per read)
        chunks = recordio.ChunkedDecoder() if resp.chunked else None
        read = resp.fp.read1 if chunks is not None else resp.read1
        while not self._stopped.is_set():
            try:
                data = read(65536)
            except socket.timeout:
                raise OSError("missed heartbeats") from None
            if not data:
                return
            if chunks is not None:
                data = chunks.feed(data)
            updates: List[P.TaskStatus] = []
            for rec in dec.feed(data):
                ev = decode_message(P.Event, rec, self.content_type)
                if ev.type == P.Event.UPDATE:
                    # updates read together are handed over together (order kept): a scheduler
                    # that fell behind stores them in one transaction instead of one each
                    updates.append(ev.update.status)
                    continue
                if updates:
                    self._on_updates(updates)
                    updates = []
                self._on_event(ev)
            if updates:
                self._on_updates(updates)
            if chunks is not None and chunks.done:
                return

    def set_status_gate(self, gate: Optional[Callable[[], bool]]) -> None:
        """``gate()`` runs on the event thread before each status callback and may block it (the
        framework's offer-cycle gate; True when it did); the thread holds no lock of the
        scheduler's there."""
        self._status_gate = gate

    def _on_updates(self, statuses: List[P.TaskStatus]) -> None:
        gate = self._status_gate
        if gate is not None:
            gate()
        if len(statuses) == 1 or getattr(self.scheduler, "status_updates", None) is None:
            for status in statuses:
                self._on_update(status)
            return
        self._call_scheduler("status_updates", statuses)
        if self.implicit_acknowledgements:
            self._acknowledge_all(statuses)

    def _on_update(self, status: P.TaskStatus) -> None:
        self._call_scheduler("status_update", status)
        if self.implicit_acknowledgements:
            self._acknowledge(status)

    def _acknowledge(self, status: P.TaskStatus) -> None:
        try:
            self.acknowledge_status_update(status)
        except MesosCallError as e:
            LOGGER.warning("ACKNOWLEDGE of %s failed: %s", status.task_id.value, e)

    def _acknowledge_all(self, statuses: List[P.TaskStatus]) -> None:
        """The ACKNOWLEDGEs of a batch of updates (one call each over HTTP)."""
        for status in statuses:
            self._acknowledge(status)

    @staticmethod
    def _ack_call(status: P.TaskStatus) -> Optional[P.Call]:
        if not status.uuid or not status.HasField("agent_id"):
            return None
        call = P.Call(type=P.Call.ACKNOWLEDGE)
        call.acknowledge.agent_id.CopyFrom(status.agent_id)
        call.acknowledge.task_id.CopyFrom(status.task_id)
        call.acknowledge.uuid = status.uuid
        return call

    def _call_scheduler(self, name: str, *args) -> None:
        fn = getattr(self.scheduler, name, None)
        if fn is None:
            return
        try:
            fn(self, *args)
        except Exception:  # noqa: BLE001
            LOGGER.exception("Scheduler callback %s failed", name)

    def _on_event(self, ev: P.Event) -> None:
        t = ev.type
        if t == P.Event.SUBSCRIBED:
            sub = ev.subscribed
            self._framework_id = sub.framework_id.value
            self.master_info = sub.master_info if sub.HasField("master_info") else None
            hb = sub.heartbeat_interval_seconds or 15.0
            if self._stream_conn is not None and self._stream_conn.sock is not None:
                self._stream_conn.sock.settimeout(hb * self.heartbeat_misses)
            again = self._subscribed_once
            self._subscribed_once = True
            self._subscribed.set()
            if again:
                self._call_scheduler("reregistered", self.master_info)
            else:
                self._call_scheduler("registered", P.FrameworkID(value=self._framework_id), self.master_info)
        elif t == P.Event.OFFERS:
            self._call_scheduler("resource_offers", list(ev.offers.offers))
        elif t == P.Event.RESCIND:
            self._call_scheduler("offer_rescinded", ev.rescind.offer_id)
        elif t == P.Event.UPDATE:
            self._on_updates([ev.update.status])
        elif t == P.Event.MESSAGE:
            m = ev.message
            self._call_scheduler("framework_message", m.executor_id, m.agent_id, m.data)
        elif t == P.Event.FAILURE:
            f = ev.failure
            if f.HasField("executor_id"):
                self._call_scheduler("executor_lost", f.executor_id, f.agent_id, f.status)
            else:
                self._call_scheduler("agent_lost", f.agent_id)
        elif t == P.Event.ERROR:
            self._call_scheduler("error", ev.error.message)
        elif t == P.Event.HEARTBEAT:
            pass
        else:
            LOGGER.debug("Ignoring event type %s", t)


def resolve_master_url(url: str, timeout_s: float = 10.0) -> str:
    """``http(s)://host:port`` as is; ``zk://hosts/path`` -> the leading master's v1 endpoint.

    Mesos masters publish ephemeral-sequential ``json.info_<seq>`` nodes (MasterInfo as JSON)
    under the ZK path; the lowest sequence number is the leader (how libmesos' detector, used by
    the reference's ``zk://master.mesos:2181/mesos`` driver URL, finds it).
    """
    if not url.startswith("zk://"):
        return url
    from dcos_commons_amd.storage import zookeeper as Z

    rest = url[len("zk://"):]
    hosts, _, path = rest.partition("/")
    client = Z.ZkClient(hosts, connect_timeout_s=timeout_s).start()
    try:
        deadline = time.monotonic() + timeout_s
        while True:
            infos = sorted(c for c in client.get_children("/" + path) if c.startswith("json.info_"))
            if infos:
                data, _ = client.get(f"/{path}/{infos[0]}")
                info = json.loads((data or b"{}").decode("utf-8"))
                addr = info.get("address") or {}
                host = addr.get("hostname") or addr.get("ip") or info.get("hostname")
                port = addr.get("port") or info.get("port") or 5050
                return f"http://{host}:{port}"
            if time.monotonic() > deadline:
                raise MesosCallError(503, f"no leading master registered under {url}")
            time.sleep(0.1)
    finally:
        client.close()
