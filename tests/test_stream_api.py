"""``mesos.stream_api``: the v1 scheduler messages over one framed socket, and
``mesos.agent_runtime``: agents that run their own tasks' lifecycle.

Covered: frame parsing across partial reads and several frames per read; a scheduler deploys,
restarts and replaces a helloworld pod through ``StreamSchedulerDriver`` against a ``LocalMaster``
served by ``StreamMaster``, with agents whose lifecycle runs in an ``AgentRuntime`` (the statuses
the scheduler sees are the ones the in-process lifecycle produces, readiness included); a
failed-over subscription is closed; a dropped connection disconnects the framework; the runtime's
reports (checks that fail then pass, kill, injected failure, drop, reset).
"""
import socket
import struct
import threading
import time

import pytest

from dcos_commons_amd.mesos import protos as P
from dcos_commons_amd.mesos.agent_runtime import AgentRuntime
from dcos_commons_amd.mesos.local_master import AgentSpec, LocalMaster
from dcos_commons_amd.mesos.stream_api import FrameReader, StreamMaster, StreamSchedulerDriver, frame


def test_frames_split_and_coalesced():
    a, b = socket.socketpair()
    try:
        payloads = [b"x" * 3, b"", b"y" * 70000, b"z"]
        data = b"".join(frame(p) for p in payloads)
        reader = FrameReader(b, bufsize=4096)
        got = []

        def feed():
            for i in range(0, len(data), 997):          # torn at arbitrary points
                a.sendall(data[i:i + 997])
            a.shutdown(socket.SHUT_WR)
        t = threading.Thread(target=feed)
        t.start()
        for batch in reader.batches():
            got.extend(batch)
        t.join()
        assert got == payloads
    finally:
        a.close()
        b.close()


def test_oversized_frame_is_refused():
    a, b = socket.socketpair()
    a.sendall(struct.pack(">I", 1 << 30))
    with pytest.raises(OSError):
        next(FrameReader(b).batches())
    a.close()
    b.close()


class _RuntimeLink:
    """In-process stand-in for an agent link: master -> runtime messages are handed over directly,
    the runtime's reports go to ``LocalMaster.runtime_reports``."""

    def __init__(self, master: LocalMaster, check=None):
        self.master = master
        self.aid = None
        self.sent = []
        self.runtime = AgentRuntime(lambda reps: master.runtime_reports(self.aid, reps), check)

    def send(self, msg):
        self.sent.append(msg["op"])
        self.runtime.handle(msg)


def _runtime_master(n=1, check=None):
    master = LocalMaster(allocation_interval_s=0.05)
    links = []
    for i in range(n):
        link = _RuntimeLink(master, check)
        spec = AgentSpec(hostname=f"agent-{i}", cpus=8, mem=32768, disk=65536, gpus=1, gpu_devices=[i])
        link.aid = master.add_agent(spec, runtime=link)
        links.append(link)
    return master, links


def test_scheduler_over_the_stream_with_agent_run_tasks():
    """DeployBench's cycle (deploy, TASK_FAILED restart, pod replace) through the framed stream,
    every pod's lifecycle and readiness check run by its agent's runtime."""
    from dcos_commons_amd.benchmarks import deploy_bench as DB

    master, links = _runtime_master(2, check=lambda devices: True)
    stream = StreamMaster(master).start()

    class Cluster:
        def driver(self, sched, info):
            return StreamSchedulerDriver(stream.address, sched, info)

        def placement(self):
            return master.placement()

        def fail_task(self, tid):
            master.fail_task(tid)

        def shutdown(self):
            pass

    bench = DB.DeployBench(2, timeout_s=20, allocation_interval_s=0.05)
    bench._make_master = lambda: Cluster()
    try:
        r = bench.run_cycle()
        assert r.deploy_s > 0 and r.mttr_restart_s > 0 and r.mttr_replace_s > 0
        assert sorted(p["task"] for p in bench.last_placement) == ["hello-0-server", "hello-1-server"]
        # the master sent launches and the kill to the agents; the agents ran the checks
        assert all("launch" in link.sent for link in links)
        assert sum(link.runtime.checks for link in links) >= 4   # 2 deploys + restart + replace
        assert stream.calls.get("ACCEPT", 0) >= 2 and stream.calls.get("ACKNOWLEDGE", 0) >= 6
    finally:
        stream.stop()
        master.shutdown()


class _Sched:
    def __init__(self):
        self.events = []
        self.registered_ev = threading.Event()
        self.disconnected_ev = threading.Event()

    def registered(self, driver, fid, info):
        self.events.append(("registered", fid.value))
        self.registered_ev.set()

    def resource_offers(self, driver, offers):
        self.events.append(("offers", len(offers)))

    def error(self, driver, message):
        self.events.append(("error", message))

    def disconnected(self, driver):
        self.disconnected_ev.set()


def test_failover_closes_the_old_subscription_and_a_dropped_stream_disconnects():
    master = LocalMaster(allocation_interval_s=0.05)
    master.add_agent(AgentSpec(hostname="a"))
    stream = StreamMaster(master).start()
    try:
        s1 = _Sched()
        info = P.FrameworkInfo(name="svc", user="nobody", roles=["svc-role"])
        d1 = StreamSchedulerDriver(stream.address, s1, info)
        d1.start()
        assert s1.registered_ev.wait(5)
        fid = d1.framework_id
        info2 = P.FrameworkInfo()
        info2.CopyFrom(info)
        info2.id.value = fid
        s2 = _Sched()
        d2 = StreamSchedulerDriver(stream.address, s2, info2)
        d2.start()
        assert s2.registered_ev.wait(5)
        assert s1.disconnected_ev.wait(5)                 # the failed-over stream ended
        assert ("error", "Framework failed over") in s1.events
        assert d2.framework_id == fid
        # the new stream's connection drops: the master disconnects the framework
        d2._close_stream()
        deadline = time.time() + 5
        while time.time() < deadline and master.frameworks[fid].connected:
            time.sleep(0.01)
        assert not master.frameworks[fid].connected
    finally:
        stream.stop()
        master.shutdown()


def test_runtime_reports_checks_kill_fail_drop_and_reset():
    reports = []
    got = threading.Event()
    results = iter([False, True])

    def report(reps):
        reports.extend(reps)
        got.set()

    rt = AgentRuntime(report, check=lambda devices: next(results))
    try:
        rt.handle({"op": "launch", "task": "t1", "name": "hello-0-server", "devices": [0],
                   "check": {"delay": 0.0, "interval": 0.05}, "timing": {}})
        deadline = time.time() + 5
        while time.time() < deadline and not any(r["event"] == "ready" for r in reports):
            time.sleep(0.01)
        assert [r["event"] for r in reports] == ["starting", "running", "check_failed", "ready"]
        reports.clear()
        rt.handle({"op": "kill", "task": "t1"})
        assert reports == [{"task": "t1", "event": "exited", "state": 4, "message": "Task killed by scheduler"}]
        reports.clear()
        rt.handle({"op": "launch", "task": "t2", "devices": [], "check": None, "timing": {}})
        rt.handle({"op": "fail", "task": "t2", "state": 3, "message": "boom", "reason": 1})
        assert [r["event"] for r in reports] == ["starting", "running", "exited"]
        assert reports[-1]["state"] == 3 and reports[-1]["message"] == "boom"
        reports.clear()
        rt.handle({"op": "launch", "task": "t3", "devices": [], "check": None, "timing": {"finish_after": 0.05}})
        rt.handle({"op": "drop", "task": "t3"})
        rt.handle({"op": "launch", "task": "t4", "devices": [], "check": {"delay": 0.05, "interval": 1}, "timing": {}})
        rt.handle({"op": "reset"})
        time.sleep(0.2)
        # t3 was dropped before it finished and t4 reset before its check: nothing more from either
        assert [r["event"] for r in reports] == ["starting", "running", "starting", "running"]
        assert rt.live_tasks == []
    finally:
        rt.shutdown()


def test_master_with_agent_runtimes_reports_what_its_own_lifecycle_would():
    """The same launch, once with the master's in-process lifecycle and once with an agent runtime:
    the framework sees the same sequence of states and check results."""
    def run(with_runtime):
        seen = []
        done = threading.Event()
        master = LocalMaster(allocation_interval_s=0.05)
        spec = AgentSpec(hostname="a", gpus=1, gpu_devices=[0])
        if with_runtime:
            link = _RuntimeLink(master, check=lambda d: True)
            link.aid = master.add_agent(spec, runtime=link)
        else:
            master.add_agent(spec)

        class S:
            def registered(self, d, fid, info):
                pass

            def resource_offers(self, d, offers):
                o = offers[0]
                t = P.TaskInfo(name="hello-0-server")
                t.task_id.value = "task-1"
                t.agent_id.CopyFrom(o.agent_id)
                t.command.value = "true"
                r = t.resources.add(name="gpus", type=P.Value.SCALAR)
                r.scalar.value = 1
                t.check.type = P.CheckInfo.COMMAND
                t.check.command.command.value = "true"
                t.check.delay_seconds = 0      # Mesos' default is 15 s
                op = P.Offer.Operation(type=P.Offer.Operation.LAUNCH)
                op.launch.task_infos.add().CopyFrom(t)
                d.accept_offers([o.id], [op])
                d.suppress_offers()

            def status_update(self, d, st):
                exit_code = st.check_status.command.exit_code if st.check_status.command.HasField("exit_code") else None
                seen.append((P.TaskState.Name(st.state), exit_code, [l.value for l in st.labels.labels]))
                if exit_code == 0:
                    done.set()
        from dcos_commons_amd.mesos.local_master import LocalSchedulerDriver

        drv = LocalSchedulerDriver(master, S(), P.FrameworkInfo(name="f", roles=["*"]))
        drv.start()
        assert done.wait(5)
        master.shutdown()
        return seen
    assert run(True) == run(False) == [("TASK_STARTING", None, ["0"]), ("TASK_RUNNING", None, ["0"]),
                                       ("TASK_RUNNING", 0, ["0"])]


@pytest.mark.gpu
def test_agent_runtime_gates_readiness_on_the_hip_probe():
    """The split topology's agent side on an MI355X: every pod's readiness check runs the fused HIP
    probe (``ops.readiness``) on the agent's device, from the agent's runtime; the scheduler gets
    the result over the framed stream."""
    from dcos_commons_amd import ops
    from dcos_commons_amd.benchmarks import deploy_bench as DB
    from dcos_commons_amd.benchmarks.runner import gpu_check_runner

    probe = gpu_check_runner()
    ran = []

    def check(devices):
        ran.append(list(devices))
        return probe(None, devices)
    master, links = _runtime_master(2, check=check)
    # both agents own device 0 of this box (their AgentSpec names device i; map them onto 0)
    for link in links:
        link.runtime._check = lambda devices: check([0])
    stream = StreamMaster(master).start()

    class Cluster:
        def driver(self, sched, info):
            return StreamSchedulerDriver(stream.address, sched, info)

        def placement(self):
            return master.placement()

        def fail_task(self, tid):
            master.fail_task(tid)

        def shutdown(self):
            pass

    bench = DB.DeployBench(2, timeout_s=60, allocation_interval_s=0.05)
    bench._make_master = lambda: Cluster()
    try:
        r = bench.run_cycle()
        assert r.deploy_s > 0 and len(ran) >= 4 and all(d == [0] for d in ran)
        assert ops.lib() is not None        # the in-tree HIP extension served the checks
    finally:
        stream.stop()
        master.shutdown()


def test_runtime_reports_running_before_a_check_unless_checks_are_fast(monkeypatch):
    """STARTING / RUNNING leave before the first check; once this agent's checks finish within
    the report window they leave together with the check's result; after a slow check they go
    first again."""
    monkeypatch.setenv("SDK_AGENT_REPORT_WINDOW_MS", "50")
    reports = []
    delay = {"s": 0.0}

    def check(devices):
        time.sleep(delay["s"])
        return True
    rt = AgentRuntime(lambda reps: reports.append([r["event"] for r in reps]), check)
    try:
        def launch(tid):
            reports.clear()
            rt.handle({"op": "launch", "task": tid, "name": tid, "devices": [0], "check": {"delay": 0, "interval": 1},
                       "timing": {}})
            return list(reports)
        assert launch("t1") == [["starting", "running"], ["ready"]]          # nothing known yet: RUNNING first
        assert launch("t2") == [["starting", "running", "ready"]]            # fast checks: one report
        delay["s"] = 0.08
        assert launch("t3") == [["starting", "running", "ready"]]            # looked fast; this one was slow
        delay["s"] = 0.0
        assert launch("t4") == [["starting", "running"], ["ready"]]          # after a slow check: RUNNING first
    finally:
        rt.shutdown()
    monkeypatch.delenv("SDK_AGENT_REPORT_WINDOW_MS")       # the default: RUNNING always first
    rt = AgentRuntime(lambda reps: reports.append([r["event"] for r in reps]), lambda d: True)
    try:
        for tid in ("a", "b"):
            reports.clear()
            rt.handle({"op": "launch", "task": tid, "name": tid, "devices": [0], "check": {"delay": 0, "interval": 1},
                       "timing": {}})
            assert reports == [["starting", "running"], ["ready"]]
    finally:
        rt.shutdown()


def test_ready_returns_what_arrived_without_blocking():
    a, b = socket.socketpair()
    try:
        reader = FrameReader(b)
        assert reader.ready() == []                       # nothing yet: no wait
        a.sendall(frame(b"one") + frame(b"two") + frame(b"thr")[:5])
        time.sleep(0.05)
        assert reader.ready() == [b"one", b"two"]         # the torn third frame stays buffered
        a.sendall(frame(b"thr")[5:])
        a.shutdown(socket.SHUT_WR)
        assert next(reader.batches()) == [b"thr"]
    finally:
        a.close()
        b.close()


def test_corked_events_leave_in_one_write_per_connection():
    from dcos_commons_amd.mesos.stream_api import _StreamSubscription, corked

    a, b = socket.socketpair()
    c, d = socket.socketpair()
    try:
        s1, s2 = _StreamSubscription(a, 15.0), _StreamSubscription(c, 15.0)
        writes = []
        for s in (s1, s2):
            orig = s.write
            s.write = lambda data, orig=orig, s=s: (writes.append((s, len(data))), orig(data))
        ev = P.Event(type=P.Event.HEARTBEAT)
        with corked():
            s1.put(ev)
            s2.put(ev)
            with corked():          # nested blocks write with the outermost
                s1.put(ev)
            assert writes == []
        assert sorted((id(s), n) for s, n in writes) == sorted([(id(s1), 2 * len(frame(ev.SerializeToString()))),
                                                              (id(s2), len(frame(ev.SerializeToString())))])
        s1.put(ev)                  # uncorked: written at once
        assert len(writes) == 3
    finally:
        for x in (a, b, c, d):
            x.close()
