"""Mesos v1 HTTP scheduler API: RecordIO codec, driver <-> master wire contract, and the full
helloworld scheduler deployed/recovered over a socket (SURVEY §2.10 "libmesos /
mesos-http-adapter" row; reference driver selection in framework/SchedulerDriverFactory.java)."""
import http.client
import json
import threading
import time

import pytest

from dcos_commons_amd.framework.process_exit import ProcessExit
from dcos_commons_amd.mesos import protos as P
from dcos_commons_amd.mesos import recordio
from dcos_commons_amd.mesos.http_driver import JSON, PROTOBUF, MesosCallError, V1HttpSchedulerDriver, encode_message
from dcos_commons_amd.mesos.http_master import HttpMaster
from dcos_commons_amd.mesos.local_master import AgentSpec, LocalMaster
from test_e2e_helloworld import Cluster


def test_recordio_roundtrip_and_partial_feeds():
    recs = [b"", b"a", b"hello\nworld", bytes(range(256)) * 40]
    wire = b"".join(recordio.encode(r) for r in recs)
    for step in (1, 3, 7, 4096, len(wire)):
        dec = recordio.Decoder()
        out = []
        for i in range(0, len(wire), step):
            out.extend(dec.feed(wire[i:i + step]))
        assert out == recs and dec.pending_bytes == 0
    with pytest.raises(recordio.RecordIOError):
        recordio.Decoder().feed(b"12x\n")
    with pytest.raises(recordio.RecordIOError):
        recordio.Decoder(max_record_bytes=4).feed(b"5\nabcde")
    chunks = iter([wire[:5], wire[5:], b""])
    assert list(recordio.iter_records(lambda n: next(chunks))) == recs
    bad = iter([b"10\nabc", b""])
    with pytest.raises(recordio.RecordIOError):
        list(recordio.iter_records(lambda n: next(bad)))


def _chunked(payload: bytes, sizes, ext=b"") -> bytes:
    out, i = b"", 0
    for n in sizes:
        out += b"%x%s\r\n" % (n, ext) + payload[i:i + n] + b"\r\n"
        i += n
    return out + b"0\r\n\r\n"


def test_chunked_decoder_returns_everything_that_arrived():
    payload = b"".join(recordio.encode(r) for r in (b"a" * 300, b"", b"event\r\n3"))
    for ext in (b"", b";name=value"):
        wire = _chunked(payload, [1, 17, 0x100, len(payload) - 0x112], ext)
        for step in (1, 2, 5, 64, len(wire)):
            dec, out = recordio.ChunkedDecoder(), b""
            for i in range(0, len(wire), step):
                out += dec.feed(wire[i:i + step])
            assert out == payload and dec.done
    dec = recordio.ChunkedDecoder()
    assert dec.feed(_chunked(b"xy", [2]) + b"ignored after the last chunk") == b"xy" and dec.done
    with pytest.raises(recordio.RecordIOError):
        recordio.ChunkedDecoder().feed(b"zz\r\n")
    with pytest.raises(recordio.RecordIOError):
        recordio.ChunkedDecoder().feed(b"2\r\nabXY")


class Recorder:
    def __init__(self):
        self.events = []
        self.cv = threading.Condition()

    def _add(self, *e):
        with self.cv:
            self.events.append(e)
            self.cv.notify_all()

    def registered(self, d, fid, mi):
        self._add("registered", fid.value)

    def reregistered(self, d, mi):
        self._add("reregistered")

    def resource_offers(self, d, offers):
        self._add("offers", offers)

    def offer_rescinded(self, d, oid):
        self._add("rescind", oid.value)

    def status_update(self, d, st):
        self._add("update", st)

    def disconnected(self, d):
        self._add("disconnected")

    def error(self, d, msg):
        self._add("error", msg)

    def wait_for(self, kind, n=1, timeout=10):
        with self.cv:
            ok = self.cv.wait_for(lambda: sum(1 for e in self.events if e[0] == kind) >= n, timeout)
        assert ok, f"no {kind} event; have {[e[0] for e in self.events]}"
        return [e for e in self.events if e[0] == kind]


@pytest.fixture
def cluster():
    lm = LocalMaster(allocation_interval_s=0.05)
    lm.add_agent(AgentSpec(hostname="h0", cpus=2, mem=1024, disk=1000))
    hm = HttpMaster(lm, heartbeat_s=0.2).start()
    yield lm, hm
    hm.stop()
    lm.shutdown()


@pytest.mark.parametrize("ctype", [PROTOBUF, JSON])
def test_subscribe_offers_launch_kill_ack(cluster, ctype):
    lm, hm = cluster
    rec = Recorder()
    d = V1HttpSchedulerDriver(hm.url, rec, P.FrameworkInfo(name="fw", role="r", user="u"), content_type=ctype)
    d.start()
    try:
        fid = rec.wait_for("registered")[0][1]
        assert d.framework_id == fid and d.stream_id
        offer = rec.wait_for("offers")[0][1][0]
        assert offer.hostname == "h0"
        op = P.Offer.Operation(type=P.Offer.Operation.LAUNCH)
        t = op.launch.task_infos.add(name="t")
        t.task_id.value = "t-1"
        t.agent_id.CopyFrom(offer.agent_id)
        t.command.value = "sleep 1000"
        t.resources.extend([r for r in offer.resources if r.name == "cpus"])
        d.accept_offers([offer.id], [op], P.Filters(refuse_seconds=1))
        wait_state = lambda s: any(e[1].state == s for e in rec.wait_for("update"))  # noqa: E731
        deadline = time.time() + 10
        while not wait_state(P.TASK_RUNNING) and time.time() < deadline:
            time.sleep(0.01)
        assert lm.task_states()["t-1"] == P.TASK_RUNNING
        d.kill_task(P.TaskID(value="t-1"))
        deadline = time.time() + 10
        while lm.task_states().get("t-1") != P.TASK_KILLED and time.time() < deadline:
            time.sleep(0.01)
        assert lm.task_states()["t-1"] == P.TASK_KILLED
        # every status that carried a uuid was implicitly acknowledged
        time.sleep(0.1)
        sub = hm.subscriptions[fid]
        uuids = {e[1].uuid for e in rec.events if e[0] == "update" and e[1].uuid}
        assert uuids and uuids <= set(sub.acknowledged)
        d.reconcile_tasks([P.TaskStatus(task_id=P.TaskID(value="nope"), state=P.TASK_RUNNING)])
        deadline = time.time() + 5
        while not any(e[0] == "update" and e[1].task_id.value == "nope" for e in rec.events) and time.time() < deadline:
            time.sleep(0.01)
        lost = [e[1] for e in rec.events if e[0] == "update" and e[1].task_id.value == "nope"]
        assert lost and lost[0].state == P.TASK_LOST
        d.suppress_offers()
        d.revive_offers()
        time.sleep(0.5)  # heartbeats (0.2 s) keep the stream alive
        assert not any(e[0] == "disconnected" for e in rec.events)
        assert hm.calls["ACCEPT"] == 1 and hm.calls["KILL"] == 1 and hm.calls["ACKNOWLEDGE"] >= 1
    finally:
        d.stop()


def test_calls_need_current_stream_id(cluster):
    lm, hm = cluster
    rec = Recorder()
    d = V1HttpSchedulerDriver(hm.url, rec, P.FrameworkInfo(name="fw", role="r"))
    d.start()
    try:
        fid = rec.wait_for("registered")[0][1]
        conn = http.client.HTTPConnection("127.0.0.1", hm.port, timeout=5)
        call = P.Call(type=P.Call.REVIVE)
        call.framework_id.value = fid
        conn.request("POST", "/api/v1/scheduler", body=encode_message(call, JSON),
                     headers={"Content-Type": JSON, "Mesos-Stream-Id": "bogus"})
        r = conn.getresponse()
        r.read()
        assert r.status == 400
        conn.request("POST", "/api/v1/scheduler", body=b"{", headers={"Content-Type": JSON})
        r = conn.getresponse()
        r.read()
        assert r.status == 400
        conn.request("GET", "/state")
        r = conn.getresponse()
        state = json.loads(r.read())
        assert state["frameworks"] == [fid] and state["agents"][0]["hostname"] == "h0"
    finally:
        d.stop()


def test_redirect_to_leader(cluster):
    lm, hm = cluster
    follower = HttpMaster(lm, redirect_to=hm.url).start()
    rec = Recorder()
    d = V1HttpSchedulerDriver(follower.url, rec, P.FrameworkInfo(name="fw", role="r"))
    d.start()
    try:
        rec.wait_for("registered")
        assert d.master_url == hm.url
        d.revive_offers()
    finally:
        d.stop()
        follower.stop()


def test_stream_loss_disconnects_or_fails_over(cluster):
    lm, hm = cluster
    rec = Recorder()
    d = V1HttpSchedulerDriver(hm.url, rec, P.FrameworkInfo(name="fw", role="r"))
    d.start()
    rec.wait_for("registered")
    hm.drop_streams()
    rec.wait_for("disconnected")  # reference semantics: the scheduler exits on disconnection
    assert d.join(5) and d.exit_status == 5

    rec2 = Recorder()
    d2 = V1HttpSchedulerDriver(hm.url, rec2, P.FrameworkInfo(name="fw2", role="r"), reconnect=True, backoff_s=0.05)
    d2.start()
    try:
        fid = rec2.wait_for("registered")[0][1]
        old_stream = d2.stream_id
        hm.drop_streams()
        rec2.wait_for("reregistered")
        assert d2.framework_id == fid and d2.stream_id != old_stream  # same framework, new stream
        d2.revive_offers()
        # a second subscriber with the same FrameworkID takes over; the first gets ERROR
        rec3 = Recorder()
        info = P.FrameworkInfo(name="fw2", role="r")
        info.id.value = fid
        d3 = V1HttpSchedulerDriver(hm.url, rec3, info)
        d3.start()
        rec3.wait_for("registered")
        rec2.wait_for("error")
        d3.stop(failover=False)  # TEARDOWN removes the framework
        deadline = time.time() + 5
        while fid in lm.frameworks and time.time() < deadline:
            time.sleep(0.01)
        assert fid not in lm.frameworks
    finally:
        d2.stop()


def _raw_subscribe(hm, name="raw"):
    """SUBSCRIBE over a bare socket; returns (socket, framework_id) once SUBSCRIBED arrived."""
    import socket as _socket

    call = P.Call(type=P.Call.SUBSCRIBE)
    call.subscribe.framework_info.name = name
    call.subscribe.framework_info.role = "r"
    body = encode_message(call, JSON)
    s = _socket.create_connection(("127.0.0.1", hm.port), timeout=5)
    s.sendall(b"POST /api/v1/scheduler HTTP/1.1\r\nHost: x\r\nContent-Type: application/json\r\n"
              b"Accept: application/json\r\nContent-Length: %d\r\n\r\n%s" % (len(body), body))
    buf = b""
    deadline = time.time() + 5
    while b"SUBSCRIBED" not in buf and time.time() < deadline:
        buf += s.recv(65536)
    assert b"SUBSCRIBED" in buf, buf
    deadline = time.time() + 5
    while not hm.subscriptions and time.time() < deadline:
        time.sleep(0.01)
    return s, next(iter(hm.subscriptions))


def _connected(lm, fid):
    fw = lm.call(lambda: lm.frameworks.get(fid))
    return fw is not None and fw.connected


def test_closed_client_socket_disconnects_the_framework_within_a_second(cluster):
    """the master notices a scheduler whose connection closed (EOF on the stream
    socket) at its next idle poll, not at the next heartbeat write."""
    lm, hm = cluster
    hm.heartbeat_s = 30.0  # no heartbeat write can be what detects the close
    s, fid = _raw_subscribe(hm)
    assert _connected(lm, fid)
    t0 = time.time()
    s.close()
    while _connected(lm, fid) and time.time() - t0 < 3:
        time.sleep(0.02)
    assert not _connected(lm, fid)
    assert time.time() - t0 < 1.0 + 0.5  # one 0.25 s idle poll + scheduling slack
    assert fid not in hm.subscriptions


def test_stream_survives_when_master_holds_more_than_fd_setsize_descriptors(cluster):
    """with >= 1024 open descriptors ``select`` raised ValueError, which read as
    'peer closed' and dropped every stream after its first idle poll."""
    import os
    import resource

    lm, hm = cluster
    hm.heartbeat_s = 30.0
    soft, hard = resource.getrlimit(resource.RLIMIT_NOFILE)
    if hard != resource.RLIM_INFINITY and hard < 1200:
        pytest.skip(f"RLIMIT_NOFILE hard limit {hard} < 1200")
    if soft != resource.RLIM_INFINITY and soft < 1200:
        resource.setrlimit(resource.RLIMIT_NOFILE, (1200, hard))
    held = []
    try:
        while not held or held[-1] < 1030:
            held.append(os.open(os.devnull, os.O_RDONLY))
        s, fid = _raw_subscribe(hm)
        stream_sock_fd = hm.subscriptions[fid]  # noqa: F841 (the server-side socket is > 1024 now)
        time.sleep(1.2)  # several idle polls
        assert _connected(lm, fid)
        s.close()
        t0 = time.time()
        while _connected(lm, fid) and time.time() - t0 < 3:
            time.sleep(0.02)
        assert not _connected(lm, fid)
    finally:
        for fd in held:
            os.close(fd)
        resource.setrlimit(resource.RLIMIT_NOFILE, (soft, hard))


def test_failover_recovers_offers_held_by_the_previous_instance(cluster):
    """A scheduler that re-subscribes with its FrameworkID while the master still counts offers as
    outstanding to the old instance gets those resources offered again (Mesos rescinds them on
    failover); before, a restarted scheduler could wait forever for an agent's resources."""
    lm, hm = cluster
    rec = Recorder()
    d = V1HttpSchedulerDriver(hm.url, rec, P.FrameworkInfo(name="fw", role="r"))
    d.start()
    fid = rec.wait_for("registered")[0][1]
    rec.wait_for("offers")
    d.suppress_offers()
    # the old instance disappears without its stream being noticed: offers stay outstanding
    d._tearing_down = True
    d.stop(failover=True)
    assert any(o.framework_id == fid for o in lm.offers.values())
    rec2 = Recorder()
    info = P.FrameworkInfo(name="fw", role="r")
    info.id.value = fid
    d2 = V1HttpSchedulerDriver(hm.url, rec2, info)
    d2.start()
    try:
        rec2.wait_for("registered")
        offers = rec2.wait_for("offers")[0][1]
        assert offers and offers[0].hostname == "h0"
    finally:
        d2.stop()


def test_subscribe_rejected_calls_error():
    rec = Recorder()
    d = V1HttpSchedulerDriver("http://127.0.0.1:9", rec, P.FrameworkInfo(name="fw"), backoff_s=0.01,
                              max_backoff_s=0.02)
    d.start()
    time.sleep(0.2)  # connection refused: keeps retrying (no leader yet), never registers
    assert not rec.events
    d.stop()
    assert d.join(1)


@pytest.mark.parametrize("transport", ["protobuf", "json"])
def test_helloworld_over_http(transport):
    ProcessExit.set_test_mode(True)
    with Cluster(transport=transport) as c:
        c.wait_plan("deploy")
        states = c.master.task_states()
        assert len(states) == 4 and set(states.values()) == {P.TASK_RUNNING}
        old = c.store.fetch_task("hello-0-server").task_id.value
        c.master.fail_task(old)
        c.wait(lambda: c.store.fetch_status("hello-0-server").task_id.value != old and
               c.store.fetch_status("hello-0-server").state == P.TASK_RUNNING)
        c.wait_plan("recovery")
        assert c.http_master.calls["ACCEPT"] >= 5


def test_zk_master_detection(cluster):
    from dcos_commons_amd.mesos.http_driver import resolve_master_url
    from dcos_commons_amd.testing.zk_server import ZkServer

    lm, hm = cluster
    zk = ZkServer().start()
    try:
        assert resolve_master_url("http://x:1") == "http://x:1"
        standby = HttpMaster(lm, redirect_to=hm.url).start()
        hm.register_in_zk(zk.connect_string, "/mesos")  # first registered = leader
        standby.register_in_zk(zk.connect_string, "/mesos")
        url = resolve_master_url(f"zk://{zk.connect_string}/mesos")
        assert url == hm.url
        rec = Recorder()
        d = V1HttpSchedulerDriver(url, rec, P.FrameworkInfo(name="fw", role="r"))
        d.start()
        rec.wait_for("registered")
        d.stop()
        standby.stop()
    finally:
        zk.stop()


def test_token_refresh_failures_take_the_retry_path(cluster):
    """An IAM token refresh that fails (outage, bad credential) is a transport failure, not an
    exception out of every driver call: SUBSCRIBE retries with backoff and calls retry, and the
    driver carries on once the provider answers again."""
    lm, hm = cluster
    rec = Recorder()
    failures = {"left": 2}

    def provider():
        if failures["left"] > 0:
            failures["left"] -= 1
            raise ConnectionError("IAM unavailable")
        return "jwt"

    d = V1HttpSchedulerDriver(hm.url, rec, P.FrameworkInfo(name="fw", role="r", principal="p"),
                              credential=P.Credential(principal="p"), token_provider=provider, backoff_s=0.01)
    d.start()
    try:
        rec.wait_for("registered")                  # two failed SUBSCRIBE attempts, then success
        failures["left"] = 1
        d.revive_offers()                           # one failed header build, retried
        assert hm.calls["REVIVE"] == 1
        failures["left"] = 5
        with pytest.raises(MesosCallError) as e:
            d.suppress_offers()                     # still failing after three attempts
        assert e.value.status == 0 and "token refresh failed" in str(e.value)
    finally:
        d.stop()


def test_mesos_principal_override_must_match_the_framework_principal():
    from dcos_commons_amd.framework.scheduler_driver_factory import check_principal_override
    from dcos_commons_amd.scheduler.scheduler_config import SchedulerConfig

    info = P.FrameworkInfo(name="fw", principal="svc-principal")
    check_principal_override(info, SchedulerConfig.for_testing())
    check_principal_override(info, SchedulerConfig.for_testing(SDK_MESOS_PRINCIPAL="svc-principal"))
    with pytest.raises(ValueError, match="SDK_MESOS_PRINCIPAL"):
        check_principal_override(info, SchedulerConfig.for_testing(SDK_MESOS_PRINCIPAL="other"))


def test_async_calls_are_sent_in_order_and_failures_are_logged(caplog):
    lm = LocalMaster(allocation_interval_s=0.05)
    lm.add_agent(AgentSpec(hostname="h0", cpus=2, mem=1024, disk=1024))
    hm = HttpMaster(lm, heartbeat_s=0.2).start()
    rec = Recorder()
    d = V1HttpSchedulerDriver(hm.url, rec, P.FrameworkInfo(name="fw", role="r"), async_calls=True)
    d.start()
    try:
        rec.wait_for("registered")
        for _ in range(5):
            d.suppress_offers()
            d.revive_offers()
        assert d.flush(5.0)
        assert hm.calls["SUPPRESS"] == 5 and hm.calls["REVIVE"] == 5
        order = [c for c in getattr(hm, "call_log", []) if c in ("SUPPRESS", "REVIVE")]
        if order:   # when the fake master logs call order, it is the submission order
            assert order == ["SUPPRESS", "REVIVE"] * 5
        # a call the master rejects is reported in the log; the caller is not interrupted
        d.kill_task(P.TaskID(value=""))   # no task id: a 400 from the master
        d.flush(5.0)
    finally:
        d.stop()
        hm.stop()
        lm.shutdown()


def test_updates_read_together_reach_the_scheduler_together(cluster):
    """UPDATE events that queue up while the scheduler is busy are handed to ``status_updates``
    in one call, in stream order (the scheduler stores them in one transaction)."""
    lm, hm = cluster
    gate = threading.Event()

    class Batching(Recorder):
        def status_update(self, d, st):
            gate.wait(10)               # busy: the next updates pile up on the stream
            self._add("update", st)

        def status_updates(self, d, sts):
            self._add("batch", [s.task_id.value for s in sts])
            for s in sts:
                self._add("update", s)

    rec = Batching()
    d = V1HttpSchedulerDriver(hm.url, rec, P.FrameworkInfo(name="fw", role="r", user="u"))
    d.start()
    try:
        rec.wait_for("registered")
        d.reconcile_tasks([P.TaskStatus(task_id=P.TaskID(value="first"), state=P.TASK_RUNNING)])
        time.sleep(0.2)                 # the stream thread is now inside status_update("first")
        names = [f"t{i}" for i in range(6)]
        d.reconcile_tasks([P.TaskStatus(task_id=P.TaskID(value=n), state=P.TASK_RUNNING) for n in names])
        time.sleep(0.3)
        gate.set()
        ups = rec.wait_for("update", 1 + len(names))
        assert [u[1].task_id.value for u in ups] == ["first"] + names
        batches = [e[1] for e in rec.events if e[0] == "batch"]
        assert batches and max(len(b) for b in batches) > 1
        assert [n for b in batches for n in b] == names[len(names) - sum(len(b) for b in batches):]
    finally:
        d.stop()
