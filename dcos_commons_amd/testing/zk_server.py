"""A single-node ZooKeeper server speaking the jute wire protocol, for tests and local runs.

It exists so ``storage.zookeeper.ZkClient`` / ``ZooKeeperPersister`` / ``ZkLocker`` are exercised
over a real socket with real ZooKeeper semantics (the reference tests Curator against Curator's
``TestingServer``: sdk/scheduler/src/test/java/.../curator/CuratorPersisterTest.java). Implemented:
sessions (create, re-attach with password, expiry after the negotiated timeout without a
connection, close), ephemeral and sequential nodes, versions and ``cversion``, NoNode/NodeExists/
NotEmpty/BadVersion, atomic ``multi`` (all-or-nothing with per-op error results), data/exists/child
watches (one-shot, delivered to the owning session's live connection; re-armed by SetWatches),
digest authentication and ACL enforcement for read/write/create/delete.

Run standalone: ``python -m dcos_commons_amd.testing.zk_server --port 2181`` (binds 127.0.0.1).
"""
from __future__ import annotations

import argparse
import base64
import copy
import hashlib
import logging
import os
import socket
import socketserver
import struct
import sys
import threading
import time
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Set, Tuple

from dcos_commons_amd.storage import zookeeper as Z
from dcos_commons_amd.storage.zookeeper import ACL, Reader, Stat, Writer

LOGGER = logging.getLogger(__name__)


@dataclass
class _Node:
    data: Optional[bytes]
    acl: List[ACL]
    stat: Stat
    children: Set[str] = field(default_factory=set)
    seq: int = 0


@dataclass
class _Session:
    sid: int
    passwd: bytes
    timeout_ms: int
    conn: Optional["_Conn"] = None
    last_seen: float = field(default_factory=time.monotonic)
    auth: Set[Tuple[str, str]] = field(default_factory=set)
    closed: bool = False


class _Err(Exception):
    def __init__(self, code: int):
        super().__init__(code)
        self.code = code


class ZkServer:
    def __init__(self, host: str = "127.0.0.1", port: int = 0, min_session_timeout_ms: int = 200,
                 max_session_timeout_ms: int = 60000):
        self.lock = threading.RLock()
        self.zxid = 0
        root = _Node(None, list(Z.OPEN_ACL_UNSAFE), Stat())
        self.nodes: Dict[str, _Node] = {"/": root}
        self.sessions: Dict[int, _Session] = {}
        self.ephemerals: Dict[int, Set[str]] = {}
        # watches: (kind, path) -> set of session ids; kind in {"data", "exists", "child"}
        self.watches: Dict[Tuple[str, str], Set[int]] = {}
        self.min_timeout = min_session_timeout_ms
        self.max_timeout = max_session_timeout_ms
        self._next_sid = int.from_bytes(os.urandom(4), "big") << 24
        srv = self

        class Handler(socketserver.BaseRequestHandler):
            def handle(self):
                _Conn(srv, self.request).serve()

        class TCP(socketserver.ThreadingTCPServer):
            allow_reuse_address = True
            daemon_threads = True

        self.tcp = TCP((host, port), Handler)
        self._stop = threading.Event()
        self._threads: List[threading.Thread] = []

    @property
    def port(self) -> int:
        return self.tcp.server_address[1]

    @property
    def connect_string(self) -> str:
        return f"127.0.0.1:{self.port}"

    def start(self) -> "ZkServer":
        for target, name in ((self.tcp.serve_forever, "zk-server"), (self._expiry_loop, "zk-expiry")):
            t = threading.Thread(target=target, name=name, daemon=True)
            t.start()
            self._threads.append(t)
        return self

    def stop(self) -> None:
        self._stop.set()
        self.tcp.shutdown()
        self.tcp.server_close()
        with self.lock:
            conns = [s.conn for s in self.sessions.values() if s.conn is not None]
        for c in conns:
            c.close()

    def drop_connections(self) -> None:
        """Cuts every client connection (sessions survive until they time out)."""
        with self.lock:
            conns = [s.conn for s in self.sessions.values() if s.conn is not None]
        for c in conns:
            c.close()

    def expire_session(self, sid: int) -> None:
        with self.lock:
            s = self.sessions.get(sid)
            if s is not None:
                self._end_session(s)
        if s is not None and s.conn is not None:
            s.conn.close()

    # -- sessions -----------------------------------------------------------------------
    def _expiry_loop(self) -> None:
        while not self._stop.wait(0.05):
            now = time.monotonic()
            with self.lock:
                dead = [s for s in self.sessions.values()
                        if s.conn is None and now - s.last_seen > s.timeout_ms / 1000.0]
                for s in dead:
                    LOGGER.debug("expiring session 0x%x", s.sid)
                    self._end_session(s)

    def _end_session(self, s: _Session) -> None:
        s.closed = True
        self.sessions.pop(s.sid, None)
        for path in sorted(self.ephemerals.pop(s.sid, set()), key=len, reverse=True):
            if path in self.nodes:
                self._delete(path)
        for ws in self.watches.values():
            ws.discard(s.sid)

    def connect(self, conn: "_Conn", timeout_ms: int, sid: int, passwd: bytes) -> Optional[_Session]:
        timeout_ms = max(self.min_timeout, min(self.max_timeout, timeout_ms))
        with self.lock:
            if sid:
                s = self.sessions.get(sid)
                if s is None or s.passwd != passwd:
                    return None
                if s.conn is not None and s.conn is not conn:
                    s.conn.close()
                s.conn, s.timeout_ms, s.last_seen = conn, timeout_ms, time.monotonic()
                return s
            self._next_sid += 1
            s = _Session(self._next_sid, os.urandom(16), timeout_ms, conn)
            self.sessions[s.sid] = s
            return s

    def disconnect(self, conn: "_Conn") -> None:
        with self.lock:
            s = conn.session
            if s is not None and s.conn is conn:
                s.conn = None
                s.last_seen = time.monotonic()

    # -- tree helpers -------------------------------------------------------------------
    @staticmethod
    def _parent(path: str) -> str:
        p = path.rsplit("/", 1)[0]
        return p or "/"

    @staticmethod
    def _validate(path: Optional[str]) -> str:
        if not path or not path.startswith("/") or (len(path) > 1 and path.endswith("/")) or "//" in path:
            raise _Err(-8)
        return path

    def _check_acl(self, s: _Session, node: _Node, perm: int) -> None:
        for a in node.acl:
            if not a.perms & perm:
                continue
            if a.scheme == "world" and a.id == "anyone":
                return
            if (a.scheme, a.id) in s.auth:
                return
        raise _Err(-102)

    def _trigger(self, kind: str, path: str, ev_type: int) -> None:
        sids = self.watches.pop((kind, path), set())
        for sid in sids:
            s = self.sessions.get(sid)
            if s is not None and s.conn is not None:
                s.conn.notify(ev_type, path)

    def _fire(self, path: str, ev_type: int) -> None:
        if ev_type == Z.EVENT_CREATED:
            self._trigger("exists", path, ev_type)
            self._trigger("child", self._parent(path), Z.EVENT_CHILD_CHANGED)
        elif ev_type == Z.EVENT_DELETED:
            for kind in ("exists", "data", "child"):
                self._trigger(kind, path, ev_type)
            self._trigger("child", self._parent(path), Z.EVENT_CHILD_CHANGED)
        elif ev_type == Z.EVENT_DATA_CHANGED:
            self._trigger("exists", path, ev_type)
            self._trigger("data", path, ev_type)

    def _create(self, s: _Session, path: str, data: Optional[bytes], acl: List[ACL], flags: int) -> str:
        self._validate(path)
        parent_path = self._parent(path)
        parent = self.nodes.get(parent_path)
        if parent is None:
            raise _Err(-101)
        self._check_acl(s, parent, Z.PERM_CREATE)
        if parent.stat.ephemeral_owner:
            raise _Err(-108)
        if flags & Z.SEQUENCE:
            path = f"{path}{parent.stat.cversion:010d}"
        if path in self.nodes:
            raise _Err(-110)
        if not acl:
            raise _Err(-114)
        resolved = []
        for a in acl:  # "auth" scheme expands to the session's authenticated identities
            if a.scheme == "auth":
                if not s.auth:
                    raise _Err(-114)
                resolved.extend(ACL(a.perms, sch, ident) for sch, ident in sorted(s.auth))
            else:
                resolved.append(a)
        self.zxid += 1
        now = int(time.time() * 1000)
        st = Stat(czxid=self.zxid, mzxid=self.zxid, ctime=now, mtime=now, pzxid=self.zxid,
                  data_length=len(data or b""), ephemeral_owner=s.sid if flags & Z.EPHEMERAL else 0)
        self.nodes[path] = _Node(data, resolved, st)
        parent.children.add(path.rsplit("/", 1)[1])
        parent.stat.cversion += 1
        parent.stat.num_children = len(parent.children)
        parent.stat.pzxid = self.zxid
        if flags & Z.EPHEMERAL:
            self.ephemerals.setdefault(s.sid, set()).add(path)
        self._fire(path, Z.EVENT_CREATED)
        return path

    def _delete(self, path: str) -> None:
        node = self.nodes.pop(path)
        parent = self.nodes[self._parent(path)]
        parent.children.discard(path.rsplit("/", 1)[1])
        self.zxid += 1
        parent.stat.cversion += 1
        parent.stat.num_children = len(parent.children)
        parent.stat.pzxid = self.zxid
        if node.stat.ephemeral_owner:
            self.ephemerals.get(node.stat.ephemeral_owner, set()).discard(path)
        self._fire(path, Z.EVENT_DELETED)

    def _checked_delete(self, s: _Session, path: str, version: int) -> None:
        self._validate(path)
        if path == "/":
            raise _Err(-8)
        node = self.nodes.get(path)
        if node is None:
            raise _Err(-101)
        self._check_acl(s, self.nodes[self._parent(path)], Z.PERM_DELETE)
        if version != -1 and node.stat.version != version:
            raise _Err(-103)
        if node.children:
            raise _Err(-111)
        self._delete(path)

    def _set(self, s: _Session, path: str, data: Optional[bytes], version: int) -> Stat:
        node = self.nodes.get(self._validate(path))
        if node is None:
            raise _Err(-101)
        self._check_acl(s, node, Z.PERM_WRITE)
        if version != -1 and node.stat.version != version:
            raise _Err(-103)
        self.zxid += 1
        node.data = data
        node.stat.version += 1
        node.stat.mzxid = self.zxid
        node.stat.mtime = int(time.time() * 1000)
        node.stat.data_length = len(data or b"")
        self._fire(path, Z.EVENT_DATA_CHANGED)
        return copy.copy(node.stat)

    def _check(self, path: str, version: int) -> None:
        node = self.nodes.get(self._validate(path))
        if node is None:
            raise _Err(-101)
        if version != -1 and node.stat.version != version:
            raise _Err(-103)

    # -- request dispatch ---------------------------------------------------------------
    def handle(self, s: _Session, op: int, r: Reader) -> Tuple[int, bytes]:
        """Returns (error code, response body)."""
        with self.lock:
            s.last_seen = time.monotonic()
            try:
                return 0, self._handle(s, op, r)
            except _Err as e:
                return e.code, b""

    def _handle(self, s: _Session, op: int, r: Reader) -> bytes:
        w = Writer()
        if op == Z.OP_PING:
            return b""
        if op == Z.OP_CREATE:
            path, data, acl, flags = r.string(), r.buffer(), r.acls(), r.int()
            return w.string(self._create(s, path, data, acl, flags)).bytes()
        if op == Z.OP_DELETE:
            self._checked_delete(s, r.string(), r.int())
            return b""
        if op == Z.OP_EXISTS:
            path, watch = self._validate(r.string()), r.bool()
            node = self.nodes.get(path)
            if watch:
                self.watches.setdefault(("exists" if node is None else "data", path), set()).add(s.sid)
            if node is None:
                raise _Err(-101)
            return node.stat.write(w).bytes()
        if op == Z.OP_GET_DATA:
            path, watch = self._validate(r.string()), r.bool()
            node = self.nodes.get(path)
            if node is None:
                raise _Err(-101)
            self._check_acl(s, node, Z.PERM_READ)
            if watch:
                self.watches.setdefault(("data", path), set()).add(s.sid)
            return node.stat.write(w.buffer(node.data)).bytes()
        if op == Z.OP_SET_DATA:
            path, data, version = r.string(), r.buffer(), r.int()
            return self._set(s, path, data, version).write(w).bytes()
        if op in (Z.OP_GET_CHILDREN, Z.OP_GET_CHILDREN2):
            path, watch = self._validate(r.string()), r.bool()
            node = self.nodes.get(path)
            if node is None:
                raise _Err(-101)
            self._check_acl(s, node, Z.PERM_READ)
            if watch:
                self.watches.setdefault(("child", path), set()).add(s.sid)
            w.strings(sorted(node.children))
            if op == Z.OP_GET_CHILDREN2:
                node.stat.write(w)
            return w.bytes()
        if op == Z.OP_GET_ACL:
            node = self.nodes.get(self._validate(r.string()))
            if node is None:
                raise _Err(-101)
            return node.stat.write(w.acls(node.acl)).bytes()
        if op == Z.OP_SYNC:
            return w.string(r.string()).bytes()
        if op == Z.OP_CHECK:
            self._check(r.string(), r.int())
            return b""
        if op == Z.OP_MULTI:
            return self._multi(s, r)
        if op == Z.OP_SET_WATCHES:
            r.long()
            for kind in ("data", "exists", "child"):
                for path in r.strings():
                    self.watches.setdefault((kind, path), set()).add(s.sid)
            return b""
        raise _Err(-6)

    def _multi(self, s: _Session, r: Reader) -> bytes:
        ops = []
        while True:
            typ, done, _err = r.int(), r.bool(), r.int()
            if done:
                break
            if typ == Z.OP_CREATE:
                ops.append((typ, (r.string(), r.buffer(), r.acls(), r.int())))
            elif typ == Z.OP_DELETE:
                ops.append((typ, (r.string(), r.int())))
            elif typ == Z.OP_SET_DATA:
                ops.append((typ, (r.string(), r.buffer(), r.int())))
            elif typ == Z.OP_CHECK:
                ops.append((typ, (r.string(), r.int())))
            else:
                raise _Err(-8)
        # Snapshot for rollback; watches fire only if the whole transaction commits.
        saved = (copy.deepcopy(self.nodes), self.zxid, copy.deepcopy(self.ephemerals), copy.deepcopy(self.watches))
        pending_notes: List[Tuple[int, str]] = []
        real_trigger = self._trigger
        self._trigger = lambda kind, path, ev: pending_notes.append((kind, path, ev))  # type: ignore
        results: List[Tuple[int, object]] = []
        failed_at = -1
        try:
            for i, (typ, args) in enumerate(ops):
                try:
                    if typ == Z.OP_CREATE:
                        results.append((typ, self._create(s, *args)))
                    elif typ == Z.OP_DELETE:
                        self._checked_delete(s, *args)
                        results.append((typ, None))
                    elif typ == Z.OP_SET_DATA:
                        results.append((typ, self._set(s, *args)))
                    else:
                        self._check(*args)
                        results.append((typ, None))
                except _Err as e:
                    failed_at = i
                    results.append((Z.OP_ERROR, e.code))
                    break
        finally:
            self._trigger = real_trigger  # type: ignore
        w = Writer()
        if failed_at >= 0:
            self.nodes, self.zxid, self.ephemerals, self.watches = saved
            for i in range(len(ops)):
                code = 0 if i < failed_at else (results[failed_at][1] if i == failed_at else -2)
                w.int(Z.OP_ERROR).bool(False).int(code).int(code)
        else:
            for kind, path, ev in pending_notes:
                real_trigger(kind, path, ev)
            for typ, res in results:
                w.int(typ).bool(False).int(0)
                if typ == Z.OP_CREATE:
                    w.string(res)
                elif typ == Z.OP_SET_DATA:
                    res.write(w)
        return w.int(-1).bool(True).int(-1).bytes()

    def add_auth(self, s: _Session, scheme: str, cred: bytes) -> bool:
        if scheme != "digest":
            return False
        user, _, pw = cred.decode("utf-8").partition(":")
        h = base64.b64encode(hashlib.sha1(f"{user}:{pw}".encode("utf-8")).digest()).decode("ascii")
        with self.lock:
            s.auth.add(("digest", f"{user}:{h}"))
        return True


class _Conn:
    def __init__(self, server: ZkServer, sock: socket.socket):
        self.server = server
        self.sock = sock
        # as ZooKeeper's server does (NIOServerCnxnFactory: tcpNoDelay): replies to pipelined
        # requests and watch events go out back to back, not behind the client's delayed ACK
        try:
            sock.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
        except OSError:
            pass
        self.session: Optional[_Session] = None
        self.send_lock = threading.Lock()
        self.closed = False

    def close(self) -> None:
        self.closed = True
        try:
            self.sock.shutdown(socket.SHUT_RDWR)
        except OSError:
            pass

    def send(self, payload: bytes) -> None:
        with self.send_lock:
            try:
                self.sock.sendall(struct.pack(">i", len(payload)) + payload)
            except OSError:
                self.closed = True

    def notify(self, ev_type: int, path: str) -> None:
        self.send(Writer().int(Z.XID_NOTIFICATION).long(-1).int(0)
                  .int(ev_type).int(Z.STATE_SYNC_CONNECTED).string(path).bytes())

    def serve(self) -> None:
        try:
            r = Reader(Z._recv_frame(self.sock))
            r.int()  # protocol version
            r.long()  # last zxid seen
            timeout, sid, passwd = r.int(), r.long(), r.buffer() or b""
            s = self.server.connect(self, timeout, sid, passwd)
            if s is None:  # expired / unknown session
                self.send(Writer().int(0).int(0).long(0).buffer(b"\x00" * 16).bool(False).bytes())
                return
            self.session = s
            self.send(Writer().int(0).int(s.timeout_ms).long(s.sid).buffer(s.passwd).bool(False).bytes())
            while not self.closed:
                r = Reader(Z._recv_frame(self.sock))
                xid, op = r.int(), r.int()
                if op == Z.OP_AUTH:
                    r.int()
                    ok = self.server.add_auth(s, r.string(), r.buffer() or b"")
                    self.send(Writer().int(Z.XID_AUTH).long(self.server.zxid).int(0 if ok else -115).bytes())
                    continue
                if op == Z.OP_CLOSE:
                    with self.server.lock:
                        self.server._end_session(s)
                    self.send(Writer().int(xid).long(self.server.zxid).int(0).bytes())
                    return
                err, body = self.server.handle(s, op, r)
                self.send(Writer().int(xid).long(self.server.zxid).int(err).raw(body).bytes())
        except (OSError, Z.ZkError):
            pass
        finally:
            self.server.disconnect(self)
            try:
                self.sock.close()
            except OSError:
                pass


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description="single-node ZooKeeper-protocol server (testing)")
    ap.add_argument("--host", default="127.0.0.1")
    ap.add_argument("--port", type=int, default=2181)
    args = ap.parse_args(argv)
    logging.basicConfig(level=logging.INFO)
    srv = ZkServer(args.host, args.port).start()
    print(f"zookeeper listening on {srv.connect_string}", flush=True)
    try:
        while True:
            time.sleep(3600)
    except KeyboardInterrupt:
        srv.stop()
    return 0


if __name__ == "__main__":
    sys.exit(main())
