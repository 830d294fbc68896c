"""ZooKeeper wire conformance of ``storage/zookeeper.ZkClient`` against the jute record layouts of
the ZooKeeper protocol (``zookeeper.jute``: ConnectRequest/Response, RequestHeader, ReplyHeader,
CreateRequest, SetDataRequest, GetDataRequest, MultiHeader, Stat, WatcherEvent, ErrorResult).

The other ZooKeeper tests run the client against this repository's own jute server
(``testing/zk_server.py``), so a mistake made the same way on both sides would pass them. Here the
server is a script: every frame the client sends is compared with bytes packed by hand from the
protocol's record definitions (independent of the client's ``Writer``), and the replies it parses
are canned frames in the same layout. No real ZooKeeper exists in this image; this pins the
reference's storage backend (Curator over ZooKeeper, ``curator/CuratorPersister.java``) at the
protocol level.
"""
import socket
import struct
import threading

import pytest

from dcos_commons_amd.storage import zookeeper as Z


def i32(v):
    return struct.pack(">i", v)


def i64(v):
    return struct.pack(">q", v)


def boolean(v):
    return b"\x01" if v else b"\x00"


def ustring(s):
    if s is None:
        return i32(-1)
    b = s.encode()
    return i32(len(b)) + b


def buffer(b):
    return i32(-1) if b is None else i32(len(b)) + b


def frame(payload):
    return i32(len(payload)) + payload


OPEN_ACL = i32(1) + i32(31) + ustring("world") + ustring("anyone")   # vector<ACL>: one world:anyone ALL


def stat(version=0, data_length=0):
    # Stat: czxid mzxid ctime mtime (long) version cversion aversion (int) ephemeralOwner (long)
    # dataLength numChildren (int) pzxid (long): 68 bytes
    return i64(5) + i64(6) + i64(1000) + i64(2000) + i32(version) + i32(0) + i32(0) + i64(0) + \
        i32(data_length) + i32(0) + i64(7)


class ScriptedServer:
    """Accepts one client; answers the handshake, then one scripted reply per request frame."""

    def __init__(self, replies):
        self.sock = socket.socket()
        self.sock.bind(("127.0.0.1", 0))
        self.sock.listen(1)
        self.port = self.sock.getsockname()[1]
        self.replies = list(replies)      # callables: request payload -> list of reply payloads
        self.frames = []                  # every frame the client sent (payload, without length)
        self.conn = None
        self.thread = threading.Thread(target=self._serve, daemon=True)
        self.thread.start()

    def _recv(self, n):
        buf = b""
        while len(buf) < n:
            chunk = self.conn.recv(n - len(buf))
            if not chunk:
                raise EOFError
            buf += chunk
        return buf

    def _serve(self):
        self.conn, _ = self.sock.accept()
        try:
            while True:
                (n,) = struct.unpack(">i", self._recv(4))
                payload = self._recv(n)
                self.frames.append(payload)
                if len(self.frames) == 1:
                    # ConnectResponse: protocolVersion, timeOut, sessionId, passwd, readOnly
                    self.conn.sendall(frame(i32(0) + i32(4000) + i64(0x1234) + buffer(b"p" * 16) + boolean(False)))
                    continue
                (xid, op) = struct.unpack(">ii", payload[:8])
                if xid == Z.XID_PING:
                    continue
                reply = self.replies.pop(0) if self.replies else (lambda p: [i32(xid) + i64(9) + i32(0)])
                for out in reply(payload):
                    self.conn.sendall(frame(out))
        except (EOFError, OSError):
            pass

    def close(self):
        for s in (self.conn, self.sock):
            try:
                if s is not None:
                    s.close()
            except OSError:
                pass


def reply(body=b"", err=0, zxid=9):
    def make(payload):
        (xid,) = struct.unpack(">i", payload[:4])
        return [i32(xid) + i64(zxid) + i32(err) + body]
    return make


@pytest.fixture
def scripted():
    servers = []

    def start(*replies):
        srv = ScriptedServer(replies)
        servers.append(srv)
        client = Z.ZkClient(f"127.0.0.1:{srv.port}", session_timeout_ms=4000).start()
        servers.append(client)
        return srv, client
    yield start
    for s in servers:
        if isinstance(s, Z.ZkClient):
            s._closed.set()
            s._drop_connection()
        else:
            s.close()


def test_handshake_is_a_jute_connect_request(scripted):
    srv, client = scripted()
    # ConnectRequest: protocolVersion, lastZxidSeen, timeOut, sessionId, passwd (16 zero bytes), readOnly
    assert srv.frames[0] == i32(0) + i64(0) + i32(4000) + i64(0) + buffer(b"\x00" * 16) + boolean(False)
    assert client.session_id == 0x1234 and client.negotiated_timeout_ms == 4000
    assert client.session_passwd == b"p" * 16


def test_create_set_get_delete_requests_and_replies(scripted):
    srv, client = scripted(reply(ustring("/a")), reply(stat(version=1, data_length=2)),
                           reply(buffer(b"yz") + stat(version=1, data_length=2)), reply(),
                           reply(err=-101))
    assert client.create("/a", b"x") == "/a"
    st = client.set("/a", b"yz")
    assert (st.version, st.data_length, st.mzxid, st.pzxid) == (1, 2, 6, 7)
    data, st = client.get("/a")
    assert data == b"yz" and st.version == 1
    client.delete("/a", version=1)
    with pytest.raises(Z.NoNodeError):
        client.get("/missing")
    sent = srv.frames[1:]
    # RequestHeader(xid, type) + CreateRequest(path, data, acl, flags)
    assert sent[0] == i32(1) + i32(Z.OP_CREATE) + ustring("/a") + buffer(b"x") + OPEN_ACL + i32(0)
    # SetDataRequest(path, data, version)
    assert sent[1] == i32(2) + i32(Z.OP_SET_DATA) + ustring("/a") + buffer(b"yz") + i32(-1)
    # GetDataRequest(path, watch)
    assert sent[2] == i32(3) + i32(Z.OP_GET_DATA) + ustring("/a") + boolean(False)
    # DeleteRequest(path, version)
    assert sent[3] == i32(4) + i32(Z.OP_DELETE) + ustring("/a") + i32(1)
    assert sent[4] == i32(5) + i32(Z.OP_GET_DATA) + ustring("/missing") + boolean(False)


def test_ephemeral_sequential_flags_and_null_data(scripted):
    srv, client = scripted(reply(ustring("/lock/n-0000000003")))
    assert client.create("/lock/n-", None, ephemeral=True, sequence=True) == "/lock/n-0000000003"
    # flags: EPHEMERAL=1 | SEQUENCE=2; null data is a buffer of length -1
    assert srv.frames[1] == i32(1) + i32(Z.OP_CREATE) + ustring("/lock/n-") + i32(-1) + OPEN_ACL + i32(3)


def test_multi_request_and_results(scripted):
    results = (i32(Z.OP_SET_DATA) + boolean(False) + i32(0) + stat(version=4) +
               i32(Z.OP_CREATE) + boolean(False) + i32(0) + ustring("/b") +
               i32(-1) + boolean(True) + i32(-1))
    srv, client = scripted(reply(results))
    out = client.multi([Z.SetData("/a", b"1", 3), Z.Create("/b", b"2")])
    assert out[0].version == 4 and out[1] == "/b"
    # MultiHeader(type, done, err) before each op, then the end marker {-1, true, -1}
    expected = (i32(1) + i32(Z.OP_MULTI) +
                i32(Z.OP_SET_DATA) + boolean(False) + i32(-1) + ustring("/a") + buffer(b"1") + i32(3) +
                i32(Z.OP_CREATE) + boolean(False) + i32(-1) + ustring("/b") + buffer(b"2") + OPEN_ACL + i32(0) +
                i32(-1) + boolean(True) + i32(-1))
    assert srv.frames[1] == expected


def test_failed_multi_reports_the_failing_op(scripted):
    # per-op ErrorResult: the failing op carries its code, the others -2 (RuntimeInconsistency: rolled back)
    results = (i32(Z.OP_ERROR) + boolean(False) + i32(-101) + i32(-101) +
               i32(Z.OP_ERROR) + boolean(False) + i32(-2) + i32(-2) +
               i32(-1) + boolean(True) + i32(-1))
    srv, client = scripted(reply(results))   # the header carries OK: the ErrorResults say what failed
    with pytest.raises(Z.TransactionError) as e:
        client.multi([Z.Check("/gone", 0), Z.SetData("/a", b"1")])
    assert isinstance(e.value.failed, Z.NoNodeError) and e.value.results == [-101, -2]
    # CheckVersionRequest(path, version) inside the multi
    assert srv.frames[1] == (i32(1) + i32(Z.OP_MULTI) +
                             i32(Z.OP_CHECK) + boolean(False) + i32(-1) + ustring("/gone") + i32(0) +
                             i32(Z.OP_SET_DATA) + boolean(False) + i32(-1) + ustring("/a") + buffer(b"1") + i32(-1) +
                             i32(-1) + boolean(True) + i32(-1))


def test_watch_notification_is_a_watcher_event(scripted):
    fired = []
    got = threading.Event()

    def data_and_notification(payload):
        (xid,) = struct.unpack(">i", payload[:4])
        # the reply, then a notification: ReplyHeader(xid=-1, zxid, err=0) + WatcherEvent(type, state, path)
        return [i32(xid) + i64(9) + i32(0) + buffer(b"v") + stat(),
                i32(Z.XID_NOTIFICATION) + i64(-1) + i32(0) + i32(Z.EVENT_DATA_CHANGED) +
                i32(Z.STATE_SYNC_CONNECTED) + ustring("/w")]

    srv, client = scripted(data_and_notification)

    def watcher(ev):
        fired.append((ev.type, ev.state, ev.path))
        got.set()
    data, _ = client.get("/w", watch=watcher)
    assert data == b"v"
    assert srv.frames[1] == i32(1) + i32(Z.OP_GET_DATA) + ustring("/w") + boolean(True)
    assert got.wait(5) and fired == [(Z.EVENT_DATA_CHANGED, Z.STATE_SYNC_CONNECTED, "/w")]


def test_chroot_is_prefixed_on_the_wire_and_stripped_from_results(scripted):
    srv = ScriptedServer([reply(ustring("/root/x"))])
    client = Z.ZkClient(f"127.0.0.1:{srv.port}/root", session_timeout_ms=4000).start()
    try:
        assert client.create("/x", b"") == "/x"
        assert srv.frames[1] == i32(1) + i32(Z.OP_CREATE) + ustring("/root/x") + buffer(b"") + OPEN_ACL + i32(0)
    finally:
        client._closed.set()
        client._drop_connection()
        srv.close()
