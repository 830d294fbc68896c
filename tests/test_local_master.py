"""LocalMaster behaviours the local DC/OS stand-in relies on, checked without a cluster:
hierarchical-role offers, task addresses per network, mount disks added to a running agent."""
import threading

from dcos_commons_amd.mesos import protos as P
from dcos_commons_amd.mesos.local_master import AgentSpec, LocalMaster, LocalSchedulerDriver


class _Sink:
    def __init__(self):
        self.offers = []
        self.got = threading.Event()

    def resource_offers(self, driver, offers):
        self.offers.extend(offers)
        self.got.set()

    def __getattr__(self, name):
        return lambda *a, **kw: None


def _framework(master, roles):
    info = P.FrameworkInfo(name="fw", user="nobody")
    if len(roles) > 1:
        info.roles.extend(roles)
        info.capabilities.add(type=P.FrameworkInfo.Capability.MULTI_ROLE)
    else:
        info.role = roles[0]
    sink = _Sink()
    driver = LocalSchedulerDriver(master, sink, info)
    driver.start()
    assert sink.got.wait(5)
    return driver, sink


def test_static_reservations_are_offered_to_sub_roles():
    m = LocalMaster(allocation_interval_s=0.05)
    try:
        m.add_agent(AgentSpec(hostname="10.0.0.1", pre_reserved=(("slave_public", "cpus", 2.0),)))
        _, sink = _framework(m, ["slave_public/svc-role", "svc-role"])
        cpus = [r for r in sink.offers[0].resources if r.name == "cpus"]
        static = [r for r in cpus if r.reservations]
        unreserved = [r for r in cpus if not r.reservations]
        # the slave_public reservation goes to the sub-role that can refine it
        assert static and static[0].allocation_info.role == "slave_public/svc-role"
        assert unreserved and unreserved[0].allocation_info.role in ("slave_public/svc-role", "svc-role")
        # a framework of an unrelated role is never allocated it
        other = type("Fw", (), {"roles": {"other-role"}})()
        assert LocalMaster._alloc_role(other, "slave_public") is None
        assert LocalMaster._alloc_role(other, "*") == "other-role"
    finally:
        m.shutdown()


def test_task_addresses_follow_the_network():
    m = LocalMaster(allocation_interval_s=0.05)
    try:
        aid = m.add_agent(AgentSpec(hostname="10.0.0.7"))
        agent = m.agents[aid]
        host = agent.task_networks(None)
        assert [(n.name, n.ip_addresses[0].ip_address) for n in host] == [("", "10.0.0.7")]
        c = P.ContainerInfo(type=P.ContainerInfo.MESOS)
        ni = c.network_infos.add(name="dcos")
        ni.labels.labels.add(key="k", value="v")
        (overlay,) = agent.task_networks(c)
        assert overlay.name == "dcos" and overlay.ip_addresses[0].ip_address.startswith("9.0.")
        assert overlay.labels.labels[0].key == "k"
        b = P.ContainerInfo(type=P.ContainerInfo.MESOS)
        b.network_infos.add(name="mesos-bridge")
        (bridge,) = agent.task_networks(b)
        assert bridge.name == "mesos-bridge" and bridge.ip_addresses[0].ip_address == "10.0.0.7"
        # non-IP hostnames fall back to the loopback address
        other = m.agents[m.add_agent(AgentSpec(hostname="agent-b"))]
        assert other.task_networks(None)[0].ip_addresses[0].ip_address == "127.0.0.1"
    finally:
        m.shutdown()


def test_mount_disks_added_to_a_running_agent():
    m = LocalMaster(allocation_interval_s=0.05)
    try:
        aid = m.add_agent(AgentSpec(hostname="10.0.0.1", mount_disks=(("/dcos/volume0", 100.0),)))
        m.add_mount_disks(aid, [("/dcos/volume1", 200.0, "xfs")])
        disks = {r.disk.source.mount.root: r for r in m.agent_resources(aid) if r.HasField("disk")
                 and r.disk.source.type == P.Resource.DiskInfo.Source.MOUNT}
        assert disks["/dcos/volume0"].scalar.value == 100.0 and not disks["/dcos/volume0"].disk.source.profile
        assert disks["/dcos/volume1"].scalar.value == 200.0 and disks["/dcos/volume1"].disk.source.profile == "xfs"
        assert len(m.agents[aid].spec.mount_disks) == 2
    finally:
        m.shutdown()


def test_zero_delay_lifecycle_steps_run_inline_on_the_dispatcher_only():
    """``_after``: due now and on the dispatcher thread, a task's next lifecycle step runs in
    place (STARTING -> RUNNING -> check submission without queueing behind other tasks);
    anything else is scheduled on the dispatcher."""
    m = LocalMaster(allocation_interval_s=60)
    try:
        order = []
        m.call(lambda: (m._after(0, order.append, "inline"), order.append("after-call")))
        assert order == ["inline", "after-call"]          # ran in place, before the caller continued
        done = threading.Event()
        m._after(0, lambda: (order.append("scheduled"), done.set()))   # from a foreign thread
        assert done.wait(5) and order[-1] == "scheduled"
        late = threading.Event()
        m.call(lambda: m._after(0.05, late.set))            # a positive delay is always scheduled
        assert not late.is_set() and late.wait(5)
    finally:
        m.shutdown()


def test_inline_checks_run_on_each_agents_own_thread():
    """an inline readiness check (one native HIP call) runs on its agent's check
    thread, not the master's event thread, so a slow probe on one GPU neither stalls the master
    nor serializes the other agents' checks."""
    import time

    from dcos_commons_amd.benchmarks.deploy_bench import DeployBench

    seen = {}

    def runner(name, delay):
        def run(task_info, devices):
            t0 = time.perf_counter()
            if delay and name not in seen:
                time.sleep(delay)
            seen.setdefault(name, (threading.current_thread().name, t0, time.perf_counter()))
            return True
        run.inline = True
        return run

    bench = DeployBench(2, agent_runners=[runner("slow", 0.3), runner("fast", 0.0)], allocation_interval_s=0.05)
    bench.run_cycle()
    (slow_thread, slow_start, slow_end), (fast_thread, _, fast_end) = seen["slow"], seen["fast"]
    assert slow_thread.startswith("check-") and fast_thread.startswith("check-") and slow_thread != fast_thread
    assert fast_end < slow_end       # the other agent's check did not wait behind the slow probe
