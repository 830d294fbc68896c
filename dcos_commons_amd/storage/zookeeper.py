"""A minimal ZooKeeper client speaking the native jute wire protocol.

The reference stores all scheduler state in ZooKeeper through Apache Curator
(sdk/.../curator/CuratorPersister.java, CuratorLocker.java). No ZooKeeper library exists in this
image, so this module implements the subset of the protocol the SDK needs, from the wire format up:

* framing: 4-byte big-endian length + jute record; ``ConnectRequest``/``ConnectResponse``
  handshake carrying session id/password/timeout; session re-attach on reconnect;
* requests: create (ephemeral/sequential flags, ACLs), delete, exists, getData, setData,
  getChildren, sync, multi (check/create/delete/setData, atomic), auth (digest), ping, close;
* one reader thread matches replies to requests by xid and dispatches watch notifications;
  a ping is sent every ``session_timeout/3`` of idle time;
* connect strings ``host1:port1,host2:port2[/chroot]`` with round-robin failover.

Errors surface as ``ZkError`` subclasses keyed by the ZooKeeper error code (``NoNodeError``,
``NodeExistsError``, ``BadVersionError``, ``NotEmptyError``, ``ConnectionLossError`` ...).
"""
from __future__ import annotations

import logging
import random
import socket
import struct
import threading
import time
from concurrent.futures import Future
from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional, Sequence, Tuple

LOGGER = logging.getLogger(__name__)

# -- op codes / xids / flags ---------------------------------------------------------------
OP_NOTIFICATION = 0
OP_CREATE = 1
OP_DELETE = 2
OP_EXISTS = 3
OP_GET_DATA = 4
OP_SET_DATA = 5
OP_GET_ACL = 6
OP_SET_ACL = 7
OP_GET_CHILDREN = 8
OP_SYNC = 9
OP_PING = 11
OP_GET_CHILDREN2 = 12
OP_CHECK = 13
OP_MULTI = 14
OP_AUTH = 100
OP_SET_WATCHES = 101
OP_CLOSE = -11
OP_ERROR = -1

XID_NOTIFICATION = -1
XID_PING = -2
XID_AUTH = -4
XID_SET_WATCHES = -8

EPHEMERAL = 1
SEQUENCE = 2

PERM_READ, PERM_WRITE, PERM_CREATE, PERM_DELETE, PERM_ADMIN = 1, 2, 4, 8, 16
PERM_ALL = 31

# watcher event types / states
EVENT_NONE, EVENT_CREATED, EVENT_DELETED, EVENT_DATA_CHANGED, EVENT_CHILD_CHANGED = -1, 1, 2, 3, 4
STATE_DISCONNECTED, STATE_SYNC_CONNECTED, STATE_AUTH_FAILED, STATE_EXPIRED = 0, 3, 4, -112


# -- errors --------------------------------------------------------------------------------
class ZkError(Exception):
    code = -1

    def __init__(self, message: str = "", path: str = ""):
        super().__init__(f"{type(self).__name__}({self.code}) {path} {message}".strip())
        self.path = path


def _err(name: str, code: int):
    return type(name, (ZkError,), {"code": code})


SystemError_ = _err("SystemZkError", -1)
RuntimeInconsistencyError = _err("RuntimeInconsistencyError", -2)
DataInconsistencyError = _err("DataInconsistencyError", -3)
ConnectionLossError = _err("ConnectionLossError", -4)
MarshallingError = _err("MarshallingError", -5)
UnimplementedError = _err("UnimplementedError", -6)
OperationTimeoutError = _err("OperationTimeoutError", -7)
BadArgumentsError = _err("BadArgumentsError", -8)
NoNodeError = _err("NoNodeError", -101)
NoAuthError = _err("NoAuthError", -102)
BadVersionError = _err("BadVersionError", -103)
NoChildrenForEphemeralsError = _err("NoChildrenForEphemeralsError", -108)
NodeExistsError = _err("NodeExistsError", -110)
NotEmptyError = _err("NotEmptyError", -111)
SessionExpiredError = _err("SessionExpiredError", -112)
InvalidAclError = _err("InvalidAclError", -114)
AuthFailedError = _err("AuthFailedError", -115)

ERRORS: Dict[int, type] = {c.code: c for c in (
    SystemError_, RuntimeInconsistencyError, DataInconsistencyError, ConnectionLossError, MarshallingError,
    UnimplementedError, OperationTimeoutError, BadArgumentsError, NoNodeError, NoAuthError, BadVersionError,
    NoChildrenForEphemeralsError, NodeExistsError, NotEmptyError, SessionExpiredError, InvalidAclError,
    AuthFailedError)}


def error_for(code: int, path: str = "") -> ZkError:
    return ERRORS.get(code, SystemError_)(path=path)


class TransactionError(ZkError):
    """A multi() was rolled back; ``results`` holds the per-op error codes (0 = would have succeeded)."""
    code = -2

    def __init__(self, results: List[int], failed: ZkError):
        super().__init__(f"transaction failed: {failed}", failed.path)
        self.results = results
        self.failed = failed


# -- jute codec ----------------------------------------------------------------------------
class Writer:
    def __init__(self):
        self.parts: List[bytes] = []

    def int(self, v: int) -> "Writer":
        self.parts.append(struct.pack(">i", v))
        return self

    def long(self, v: int) -> "Writer":
        self.parts.append(struct.pack(">q", v))
        return self

    def bool(self, v: bool) -> "Writer":
        self.parts.append(b"\x01" if v else b"\x00")
        return self

    def buffer(self, v: Optional[bytes]) -> "Writer":
        if v is None:
            return self.int(-1)
        self.int(len(v))
        self.parts.append(bytes(v))
        return self

    def string(self, v: Optional[str]) -> "Writer":
        return self.buffer(None if v is None else v.encode("utf-8"))

    def acls(self, acls: Sequence["ACL"]) -> "Writer":
        self.int(len(acls))
        for a in acls:
            self.int(a.perms).string(a.scheme).string(a.id)
        return self

    def strings(self, items: Sequence[str]) -> "Writer":
        self.int(len(items))
        for s in items:
            self.string(s)
        return self

    def raw(self, b: bytes) -> "Writer":
        self.parts.append(b)
        return self

    def bytes(self) -> bytes:
        return b"".join(self.parts)


class Reader:
    def __init__(self, data: bytes, pos: int = 0):
        self.data = data
        self.pos = pos

    def _take(self, n: int) -> bytes:
        if self.pos + n > len(self.data):
            raise MarshallingError("truncated record")
        b = self.data[self.pos:self.pos + n]
        self.pos += n
        return b

    def int(self) -> int:
        return struct.unpack(">i", self._take(4))[0]

    def long(self) -> int:
        return struct.unpack(">q", self._take(8))[0]

    def bool(self) -> bool:
        return self._take(1) != b"\x00"

    def buffer(self) -> Optional[bytes]:
        n = self.int()
        return None if n < 0 else self._take(n)

    def string(self) -> Optional[str]:
        b = self.buffer()
        return None if b is None else b.decode("utf-8")

    def acls(self) -> List["ACL"]:
        return [ACL(self.int(), self.string(), self.string()) for _ in range(self.int())]

    def strings(self) -> List[str]:
        n = self.int()
        return [] if n < 0 else [self.string() for _ in range(n)]

    def remaining(self) -> int:
        return len(self.data) - self.pos


@dataclass
class ACL:
    perms: int
    scheme: str
    id: str


OPEN_ACL_UNSAFE = [ACL(PERM_ALL, "world", "anyone")]
CREATOR_ALL_ACL = [ACL(PERM_ALL, "auth", "")]
READ_ACL_UNSAFE = [ACL(PERM_READ, "world", "anyone")]


@dataclass
class Stat:
    czxid: int = 0
    mzxid: int = 0
    ctime: int = 0
    mtime: int = 0
    version: int = 0
    cversion: int = 0
    aversion: int = 0
    ephemeral_owner: int = 0
    data_length: int = 0
    num_children: int = 0
    pzxid: int = 0

    def write(self, w: Writer) -> Writer:
        return (w.long(self.czxid).long(self.mzxid).long(self.ctime).long(self.mtime).int(self.version)
                .int(self.cversion).int(self.aversion).long(self.ephemeral_owner).int(self.data_length)
                .int(self.num_children).long(self.pzxid))

    @classmethod
    def read(cls, r: Reader) -> "Stat":
        return cls(r.long(), r.long(), r.long(), r.long(), r.int(), r.int(), r.int(), r.long(), r.int(), r.int(),
                   r.long())


@dataclass
class WatchedEvent:
    type: int
    state: int
    path: str


# -- transaction ops -----------------------------------------------------------------------
@dataclass
class Create:
    path: str
    data: Optional[bytes] = None
    acl: List[ACL] = field(default_factory=lambda: list(OPEN_ACL_UNSAFE))
    flags: int = 0
    op = OP_CREATE

    def write(self, w: Writer, chroot: str) -> None:
        w.string(chroot + self.path).buffer(self.data).acls(self.acl).int(self.flags)


@dataclass
class Delete:
    path: str
    version: int = -1
    op = OP_DELETE

    def write(self, w: Writer, chroot: str) -> None:
        w.string(chroot + self.path).int(self.version)


@dataclass
class SetData:
    path: str
    data: Optional[bytes]
    version: int = -1
    op = OP_SET_DATA

    def write(self, w: Writer, chroot: str) -> None:
        w.string(chroot + self.path).buffer(self.data).int(self.version)


@dataclass
class Check:
    path: str
    version: int = -1
    op = OP_CHECK

    def write(self, w: Writer, chroot: str) -> None:
        w.string(chroot + self.path).int(self.version)


def parse_connect_string(hosts: str) -> Tuple[List[Tuple[str, int]], str]:
    chroot = ""
    if "/" in hosts:
        hosts, chroot = hosts.split("/", 1)
        chroot = "/" + chroot.strip("/") if chroot.strip("/") else ""
    out = []
    for h in hosts.split(","):
        h = h.strip()
        if not h:
            continue
        host, _, port = h.rpartition(":") if ":" in h else (h, "", "2181")
        out.append((host or h, int(port or 2181)))
    if not out:
        raise ValueError(f"no ZooKeeper hosts in {hosts!r}")
    return out, chroot


# -- client --------------------------------------------------------------------------------
class ZkClient:
    def __init__(self, hosts: str, session_timeout_ms: int = 10000, connect_timeout_s: float = 10.0,
                 auth: Optional[List[Tuple[str, bytes]]] = None, default_acl: Optional[List[ACL]] = None):
        self.servers, self.chroot = parse_connect_string(hosts)
        random.shuffle(self.servers)
        self.session_timeout_ms = session_timeout_ms
        self.connect_timeout_s = connect_timeout_s
        self.auth = list(auth or [])
        self.default_acl = list(default_acl or OPEN_ACL_UNSAFE)
        self.session_id = 0
        self.session_passwd = b"\x00" * 16
        self.negotiated_timeout_ms = session_timeout_ms
        self.last_zxid = 0
        self._sock: Optional[socket.socket] = None
        self._send_lock = threading.Lock()
        self._state_lock = threading.Lock()
        self._xid = 0
        self._pending: Dict[int, Tuple[Future, int]] = {}
        self._watchers: Dict[Tuple[str, str], List[Callable[[WatchedEvent], None]]] = {}
        self._closed = threading.Event()
        self._connected = threading.Event()
        self._reader: Optional[threading.Thread] = None
        self._pinger: Optional[threading.Thread] = None
        self._last_send = time.monotonic()
        self._server_idx = 0
        self.expired = False

    # -- connection management ---------------------------------------------------------
    def start(self) -> "ZkClient":
        self._connect()
        self._pinger = threading.Thread(target=self._ping_loop, name="zk-ping", daemon=True)
        self._pinger.start()
        return self

    def _connect(self) -> None:
        deadline = time.monotonic() + self.connect_timeout_s
        last: Optional[BaseException] = None
        while time.monotonic() < deadline and not self._closed.is_set():
            host, port = self.servers[self._server_idx % len(self.servers)]
            self._server_idx += 1
            try:
                sock = socket.create_connection((host, port), timeout=max(0.1, deadline - time.monotonic()))
                sock.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
                req = (Writer().int(0).long(self.last_zxid).int(self.session_timeout_ms).long(self.session_id)
                       .buffer(self.session_passwd).bool(False).bytes())
                sock.sendall(struct.pack(">i", len(req)) + req)
                resp = Reader(_recv_frame(sock))
                resp.int()  # protocol version
                timeout = resp.int()
                sid = resp.long()
                passwd = resp.buffer() or b""
                if timeout <= 0:
                    sock.close()
                    self.expired = True
                    raise SessionExpiredError("session expired on reconnect")
                self.negotiated_timeout_ms, self.session_id, self.session_passwd = timeout, sid, passwd
                sock.settimeout(None)
                self._sock = sock
                self._connected.set()
                self._reader = threading.Thread(target=self._read_loop, args=(sock,), name="zk-reader", daemon=True)
                self._reader.start()
                for scheme, cred in self.auth:
                    self._add_auth(scheme, cred)
                self._restore_watches()
                LOGGER.debug("Connected to ZooKeeper %s:%d session 0x%x", host, port, sid)
                return
            except SessionExpiredError:
                raise
            except (OSError, ZkError) as e:
                last = e
                time.sleep(0.05)
        raise ConnectionLossError(f"unable to connect to {self.servers}: {last}")

    def close(self) -> None:
        if self._closed.is_set():
            return
        if self._connected.is_set():
            try:
                self._submit(OP_CLOSE, b"", timeout=2.0)
            except ZkError:
                pass
        self._closed.set()
        self._drop_connection()

    def _drop_connection(self) -> None:
        self._connected.clear()
        sock, self._sock = self._sock, None
        if sock is not None:
            try:
                sock.shutdown(socket.SHUT_RDWR)
            except OSError:
                pass
            sock.close()
        with self._state_lock:
            pending, self._pending = self._pending, {}
        for fut, _ in pending.values():
            if not fut.done():
                fut.set_exception(ConnectionLossError("connection lost"))

    def _read_loop(self, sock: socket.socket) -> None:
        try:
            while True:
                r = Reader(_recv_frame(sock))
                xid, zxid, err = r.int(), r.long(), r.int()
                if zxid > 0:
                    self.last_zxid = zxid
                if xid == XID_NOTIFICATION:
                    self._dispatch_watch(WatchedEvent(r.int(), r.int(), self._strip(r.string() or "")))
                    continue
                if xid in (XID_PING, XID_AUTH, XID_SET_WATCHES):
                    if xid == XID_AUTH and err:
                        LOGGER.error("ZooKeeper auth failed: %d", err)
                    continue
                with self._state_lock:
                    entry = self._pending.pop(xid, None)
                if entry is None:
                    continue
                fut, _op = entry
                if err:
                    fut.set_exception(error_for(err))
                else:
                    fut.set_result(r)
        except (OSError, ZkError):
            pass
        if sock is self._sock:
            self._drop_connection()
            self._dispatch_all(WatchedEvent(EVENT_NONE, STATE_DISCONNECTED, ""))
            if not self._closed.is_set():
                threading.Thread(target=self._reconnect, name="zk-reconnect", daemon=True).start()

    def _reconnect(self) -> None:
        try:
            self._connect()
            self._dispatch_all(WatchedEvent(EVENT_NONE, STATE_SYNC_CONNECTED, ""))
        except SessionExpiredError:
            LOGGER.error("ZooKeeper session 0x%x expired", self.session_id)
            self._dispatch_all(WatchedEvent(EVENT_NONE, STATE_EXPIRED, ""))
        except ZkError as e:
            LOGGER.error("ZooKeeper reconnect failed: %s", e)

    def _ping_loop(self) -> None:
        while not self._closed.wait(0.05):
            if not self._connected.is_set():
                continue
            if time.monotonic() - self._last_send > self.negotiated_timeout_ms / 3000.0:
                try:
                    self._send_frame(Writer().int(XID_PING).int(OP_PING).bytes())
                except (OSError, ConnectionLossError):
                    pass  # the connection dropped between the check and the send: the reader reconnects

    def _send_frame(self, payload: bytes) -> None:
        with self._send_lock:
            sock = self._sock
            if sock is None:
                raise ConnectionLossError("not connected")
            sock.sendall(struct.pack(">i", len(payload)) + payload)
            self._last_send = time.monotonic()

    def _add_auth(self, scheme: str, cred: bytes) -> None:
        self._send_frame(Writer().int(XID_AUTH).int(OP_AUTH).int(0).string(scheme).buffer(cred).bytes())

    def _restore_watches(self) -> None:
        """Re-arms server-side watches after a reconnect (SetWatches, xid -8)."""
        with self._state_lock:
            keys = list(self._watchers)
        if not keys:
            return
        by_kind = {k: [self._p(p) for (kind, p) in keys if kind == k] for k in ("data", "exists", "child")}
        w = Writer().int(XID_SET_WATCHES).int(OP_SET_WATCHES).long(self.last_zxid)
        w.strings(by_kind["data"]).strings(by_kind["exists"]).strings(by_kind["child"])
        self._send_frame(w.bytes())

    def add_auth(self, scheme: str, cred: bytes) -> None:
        self.auth.append((scheme, cred))
        if self._connected.is_set():
            self._add_auth(scheme, cred)

    # -- request plumbing ---------------------------------------------------------------
    def _submit(self, op: int, body: bytes, timeout: Optional[float] = None) -> Reader:
        if self._closed.is_set():
            raise ConnectionLossError("client closed")
        if not self._connected.wait(self.connect_timeout_s):
            raise ConnectionLossError("not connected")
        fut: Future = Future()
        with self._state_lock:
            self._xid = (self._xid + 1) & 0x7FFFFFFF or 1
            xid = self._xid
            self._pending[xid] = (fut, op)
        try:
            self._send_frame(Writer().int(xid).int(op).raw(body).bytes())
        except OSError as e:
            with self._state_lock:
                self._pending.pop(xid, None)
            raise ConnectionLossError(str(e)) from e
        try:
            return fut.result(timeout if timeout is not None else self.negotiated_timeout_ms / 1000.0 * 2)
        except TimeoutError:
            raise OperationTimeoutError("request timed out") from None

    def _p(self, path: str) -> str:
        if not path.startswith("/"):
            raise BadArgumentsError("path must be absolute", path)
        if self.chroot:
            return self.chroot if path == "/" else self.chroot + path
        return path

    def _strip(self, path: str) -> str:
        if self.chroot and path.startswith(self.chroot):
            return path[len(self.chroot):] or "/"
        return path

    def _call(self, op: int, w: Writer, path: str) -> Reader:
        try:
            return self._submit(op, w.bytes())
        except ZkError as e:
            if not e.path:
                e.path = path
                e.args = (f"{type(e).__name__}({e.code}) {path}",)
            raise

    # -- watches ------------------------------------------------------------------------
    def _register(self, kind: str, path: str, watch) -> None:
        if watch is not None:
            with self._state_lock:
                self._watchers.setdefault((kind, path), []).append(watch)

    def _dispatch_watch(self, ev: WatchedEvent) -> None:
        kinds = {EVENT_CREATED: ("exists", "data"), EVENT_DELETED: ("exists", "data", "child"),
                 EVENT_DATA_CHANGED: ("exists", "data"), EVENT_CHILD_CHANGED: ("child",)}.get(ev.type, ())
        fns = []
        with self._state_lock:
            for k in kinds:
                fns.extend(self._watchers.pop((k, ev.path), []))
        for fn in fns:
            try:
                fn(ev)
            except Exception:  # noqa: BLE001
                LOGGER.exception("watch callback failed")

    def _dispatch_all(self, ev: WatchedEvent) -> None:
        """Session-level events go to every outstanding watcher (they stay registered)."""
        with self._state_lock:
            fns = [fn for lst in self._watchers.values() for fn in lst]
        for fn in fns:
            try:
                fn(ev)
            except Exception:  # noqa: BLE001
                LOGGER.exception("watch callback failed")

    # -- API ----------------------------------------------------------------------------
    def create(self, path: str, data: Optional[bytes] = None, acl: Optional[List[ACL]] = None,
               ephemeral: bool = False, sequence: bool = False, make_parents: bool = False) -> str:
        if make_parents:
            parent = path.rsplit("/", 1)[0]
            if parent:
                self.ensure_path(parent)
        flags = (EPHEMERAL if ephemeral else 0) | (SEQUENCE if sequence else 0)
        w = Writer().string(self._p(path)).buffer(data).acls(acl or self.default_acl).int(flags)
        return self._strip(self._call(OP_CREATE, w, path).string())

    def ensure_path(self, path: str) -> None:
        cur = ""
        for part in [p for p in path.split("/") if p]:
            cur += "/" + part
            if self.exists(cur) is None:
                try:
                    self.create(cur)
                except NodeExistsError:
                    pass

    def delete(self, path: str, version: int = -1, recursive: bool = False) -> None:
        if recursive:
            for child in self.get_children(path):
                self.delete(path.rstrip("/") + "/" + child, recursive=True)
        self._call(OP_DELETE, Writer().string(self._p(path)).int(version), path)

    def exists(self, path: str, watch: Optional[Callable[[WatchedEvent], None]] = None) -> Optional[Stat]:
        self._register("exists", path, watch)
        try:
            return Stat.read(self._call(OP_EXISTS, Writer().string(self._p(path)).bool(watch is not None), path))
        except NoNodeError:
            return None

    def get(self, path: str, watch=None) -> Tuple[Optional[bytes], Stat]:
        r = self._call(OP_GET_DATA, Writer().string(self._p(path)).bool(watch is not None), path)
        data = r.buffer()
        stat = Stat.read(r)
        self._register("data", path, watch)
        return data, stat

    def set(self, path: str, data: Optional[bytes], version: int = -1) -> Stat:
        return Stat.read(self._call(OP_SET_DATA, Writer().string(self._p(path)).buffer(data).int(version), path))

    def get_children(self, path: str, watch=None) -> List[str]:
        r = self._call(OP_GET_CHILDREN, Writer().string(self._p(path)).bool(watch is not None), path)
        self._register("child", path, watch)
        return r.strings()

    def sync(self, path: str = "/") -> None:
        self._call(OP_SYNC, Writer().string(self._p(path)), path)

    def multi(self, ops: Sequence) -> List:
        """Runs ``ops`` atomically. Returns per-op results (created path / Stat / None)."""
        w = Writer()
        for op in ops:
            w.int(op.op).bool(False).int(-1)
            op.write(w, self.chroot)
        w.int(-1).bool(True).int(-1)
        r = self._call(OP_MULTI, w, ops[0].path if ops else "/")
        results: List = []
        codes: List[int] = []
        failed: Optional[ZkError] = None
        while True:
            typ, done, err = r.int(), r.bool(), r.int()
            if done:
                break
            if typ == OP_CREATE:
                results.append(self._strip(r.string()))
                codes.append(0)
            elif typ == OP_SET_DATA:
                results.append(Stat.read(r))
                codes.append(0)
            elif typ in (OP_DELETE, OP_CHECK):
                results.append(None)
                codes.append(0)
            elif typ == OP_ERROR:
                code = r.int()
                codes.append(code)
                results.append(None)
                if code not in (0, -2) and failed is None:  # -2: rolled back because another op failed
                    failed = error_for(code, ops[len(codes) - 1].path)
            else:
                raise MarshallingError(f"unexpected multi result type {typ}")
        if failed is not None:
            raise TransactionError(codes, failed)
        return results


def _recv_exact(sock: socket.socket, n: int) -> bytes:
    buf = bytearray()
    while len(buf) < n:
        chunk = sock.recv(n - len(buf))
        if not chunk:
            raise ConnectionLossError("connection closed by peer")
        buf += chunk
    return bytes(buf)


def _recv_frame(sock: socket.socket, max_len: int = 16 << 20) -> bytes:
    (n,) = struct.unpack(">i", _recv_exact(sock, 4))
    if n < 0 or n > max_len:
        raise MarshallingError(f"bad frame length {n}")
    return _recv_exact(sock, n)


def digest_acl(user: str, password: str, perms: int = PERM_ALL) -> ACL:
    """ACL entry for the ``digest`` scheme: id = user:base64(sha1(user:password))."""
    import base64
    import hashlib

    h = base64.b64encode(hashlib.sha1(f"{user}:{password}".encode("utf-8")).digest()).decode("ascii")
    return ACL(perms, "digest", f"{user}:{h}")
