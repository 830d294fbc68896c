"""Master <-> remote-agent link used by the multi-rank bench (``parallel.agent_link``): agents
register over loopback TCP, serve checks and barriers, and report a disconnect to pending requests.
Both the blocking check runner and the asynchronous one (``run_async``, the result delivered from
the link's reader thread) are exercised, including through ``LocalMaster``'s readiness path."""
import threading
import time

from dcos_commons_amd.mesos import protos as P
from dcos_commons_amd.mesos.local_master import AgentSpec, LocalMaster, TaskBehavior, TaskTiming
from dcos_commons_amd.parallel import agent_link


def _agent(server, rank, results):
    def check(msg):
        results.append(msg["name"])
        return msg["name"] != "bad", "synthetic"
    t = threading.Thread(target=agent_link.run_agent, args=("127.0.0.1", server.port,
                                                            {"rank": rank, "hostname": f"h{rank}", "devices": [0]},
                                                            check), daemon=True)
    t.start()
    return t


def _info(name):
    t = P.TaskInfo(name=name)
    t.task_id.value = name + "__id"
    return t


def test_blocking_and_async_checks():
    server = agent_link.AgentLinkServer()
    seen = []
    th = _agent(server, 1, seen)
    try:
        (remote,) = server.wait_for(1, timeout=10)
        runner = agent_link.RemoteCheckRunner(remote)
        assert runner(_info("good"), [0]) is True
        assert runner(_info("bad"), [0]) is False
        got = []
        ev = threading.Event()
        runner.run_async(_info("good"), [0], lambda ok: (got.append(ok), ev.set()))
        assert ev.wait(5) and got == [True]
        server.broadcast("barrier", timeout=5)
        assert seen == ["good", "bad", "good"]
    finally:
        server.close()
    th.join(5)


def test_async_check_reports_failure_when_the_agent_goes_away():
    server = agent_link.AgentLinkServer()
    th = _agent(server, 1, [])
    (remote,) = server.wait_for(1, timeout=10)
    got = []
    ev = threading.Event()
    remote.shutdown()              # the agent leaves before it answers
    th.join(5)
    time.sleep(0.1)
    remote.run_check_async(_info("late"), [0], lambda ok: (got.append(ok), ev.set()))
    assert ev.wait(5) and got == [False]
    server.close()


def test_local_master_readiness_through_an_async_remote_runner():
    server = agent_link.AgentLinkServer()
    seen = []
    th = _agent(server, 1, seen)
    master = None
    try:
        (remote,) = server.wait_for(1, timeout=10)
        master = LocalMaster(allocation_interval_s=0.05, behavior=TaskBehavior(TaskTiming()))
        master.add_agent(AgentSpec(hostname="h1", cpus=4, mem=4096, disk=4096),
                         check_runner=agent_link.RemoteCheckRunner(remote))
        # the async path is chosen: no pool thread blocks while the remote check runs
        assert hasattr(master.agents[next(iter(master.agents))].check_runner, "run_async")
    finally:
        if master is not None:
            master.shutdown()
        server.close()
    th.join(5)
