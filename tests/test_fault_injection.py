"""Fault injection against the live scheduler on the in-process master.

The reference injects faults only in its DC/OS integration tests (pkill, iptables partitions,
agent shutdown, master/ZK kills: testing/sdk_cmd.py, sdk_agents.py, helloworld/tests/
test_zzzrecovery.py) and in simulation ticks. Here the fake master's injectors drive the same
situations in-process: a lost ACCEPT, offer rescinds mid-deploy, an agent partition that heals,
an agent marked gone by the operator, a scheduler crash + restart (resume from the persister),
and a task the master forgot while the scheduler was down.
"""
import os
import threading
import time

import pytest

from dcos_commons_amd.mesos import protos as P
from dcos_commons_amd.mesos.local_master import AgentSpec, LocalMaster, LocalSchedulerDriver
from dcos_commons_amd.scheduler.scheduler_builder import SchedulerBuilder
from dcos_commons_amd.scheduler.scheduler_config import SchedulerConfig
from dcos_commons_amd.scheduler.scheduler_runner import SchedulerRunner
from dcos_commons_amd.specification.yaml.mappers import ServiceSpecGenerator
from dcos_commons_amd.specification.yaml.raw import RawServiceSpec
from dcos_commons_amd.storage.mem_persister import MemPersister
from dcos_commons_amd.testing import profiles

pytestmark = pytest.mark.usefixtures("sched_profile")

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SPECS = os.path.join(ROOT, "frameworks", "helloworld", "specs")
ENV = dict(FRAMEWORK_NAME="hello-world", FRAMEWORK_PRINCIPAL="hw-principal", FRAMEWORK_USER="nobody",
           HELLO_COUNT="2", HELLO_PLACEMENT='[["hostname", "UNIQUE"]]', HELLO_CPUS="0.1", HELLO_MEM="252",
           HELLO_DISK="25", SLEEP_DURATION="1000", WORLD_COUNT="2", WORLD_PLACEMENT='[["hostname", "UNIQUE"]]',
           WORLD_CPUS="0.2", WORLD_MEM="512", WORLD_DISK="25", WORLD_READINESS_CHECK_INTERVAL="5",
           WORLD_READINESS_CHECK_DELAY="0", WORLD_READINESS_CHECK_TIMEOUT="10")


class Chaos:
    def __init__(self, agents=3, **cfg):
        overrides = {"PORT_API": "0", "SDK_OFFER_WAIT_S": "0.2", "SDK_LAUNCH_RECONCILE_S": "0.3"}
        overrides.update(profiles.ACTIVE)    # the suite's flag profile; the test's own flags win
        overrides.update(cfg)
        self.cfg = SchedulerConfig.for_testing(**overrides)
        self.raw = RawServiceSpec.new_builder(os.path.join(SPECS, "svc.yml")).set_env(ENV).build()
        self.spec = ServiceSpecGenerator(self.raw, self.cfg, SPECS, ENV).build()
        self.master = LocalMaster(allocation_interval_s=0.05)
        self.agent_ids = [self.master.add_agent(AgentSpec(hostname=f"host-{i}", cpus=4, mem=8192, disk=20000))
                          for i in range(agents)]
        self.persister = MemPersister()
        self.runner = None

    def start(self):
        self.runner = SchedulerRunner(SchedulerBuilder(self.spec, self.cfg, self.persister).set_plans_from(self.raw),
                                      driver_factory=lambda s, i: LocalSchedulerDriver(self.master, s, i))
        self.runner.run(block=False)
        self.api = self.runner.framework_runner.api_server.router
        self.store = self.runner.scheduler.state_store
        return self

    def crash(self):
        """Scheduler process dies: the driver fails over (tasks keep running), nothing else."""
        self.runner.stop()
        self.runner = None

    def __enter__(self):
        return self.start()

    def __exit__(self, *exc):
        if self.runner is not None:
            self.runner.stop()
        self.master.shutdown()

    def wait(self, pred, timeout=20.0, what="condition"):
        t0 = time.time()
        while time.time() - t0 < timeout:
            if pred():
                return
            time.sleep(0.005)
        raise AssertionError(f"{what} not reached in {timeout}s")

    def plan_code(self, name):
        return self.api.get(f"/v1/plans/{name}").status

    def wait_plan(self, name, timeout=20.0):
        self.wait(lambda: self.plan_code(name) == 200, timeout, f"plan {name} COMPLETE")

    def task_id(self, name):
        t = self.store.fetch_task(name)
        return t.task_id.value if t is not None else None

    def state(self, name):
        s = self.store.fetch_status(name)
        return s.state if s is not None else None

    def agent_of(self, name):
        return self.store.fetch_task(name).agent_id.value

    def running_ids(self):
        return {tid for tid, st in self.master.task_states().items() if st == P.TASK_RUNNING}


# Flags a test depends on are set explicitly: the suite runs under both flag profiles
# (tests/conftest.py ``sched_profile``), and these behaviours exist only with the flag on.
UNKNOWN_AS_LOST = dict(SDK_UNKNOWN_AS_LOST="true")   # UNKNOWN recovered as LOST; the never-launched rule
# a lost ACCEPT is recovered by the launch watchdog's reconciliation AND the handling of its answer
WATCHDOG = dict(SDK_LAUNCH_RECONCILE_S="0.3", **UNKNOWN_AS_LOST)


def test_lost_accept_is_reconciled_and_relaunched():
    with Chaos(**WATCHDOG) as c:
        c.master.drop_next_accepts(1)
        c.wait_plan("deploy", 30)
        assert c.master.dropped_accepts == 1
        # every stored task is the one the master is running
        for name in ("hello-0-server", "hello-1-server", "world-0-server", "world-1-server"):
            assert c.task_id(name) in c.running_ids()
        assert c.runner.scheduler.launch_watchdog.watched() == set()


def test_lost_accept_stalls_without_the_watchdog():
    """Reference behaviour: a lost ACCEPT leaves its step STARTING until a restart. The restart's
    reconciliation answers TASK_UNKNOWN (partition-aware framework): only with UNKNOWN handled as
    LOST does that recover it (under the reference's handling it stays STAGING for good, see
    test_task_forgotten_reference_behaviour_never_recovers)."""
    with Chaos(SDK_LAUNCH_RECONCILE_S="0", **UNKNOWN_AS_LOST) as c:
        c.master.drop_next_accepts(1)
        time.sleep(1.5)
        assert c.plan_code("deploy") == 202
        assert c.state("hello-0-server") == P.TASK_STAGING
        c.crash()
        c.start()                        # explicit reconciliation at re-registration recovers it
        c.wait_plan("deploy", 30)


def test_offer_rescinds_during_deploy():
    """An ACCEPT naming an offer rescinded meanwhile is refused (TASK_DROPPED, INVALID_OFFERS).
    For a pod's first launch its reservations were never made; the never-launched rule
    (UNKNOWN_AS_LOST) relaunches it with a fresh footprint. Without it the step waits for those
    reservations forever, as the reference's does: under the reference flags this deploy stalled in
    about one run in four."""
    with Chaos(**UNKNOWN_AS_LOST) as c:
        stop = threading.Event()

        def rescinder():
            while not stop.is_set():
                c.master.rescind_offers()
                time.sleep(0.03)
        t = threading.Thread(target=rescinder, daemon=True)
        t.start()
        try:
            time.sleep(0.3)
        finally:
            stop.set()
            t.join()
        c.wait_plan("deploy", 30)
        assert len(c.running_ids()) == 4


def _volume_ids(c, name):
    return sorted(r.disk.persistence.id for r in c.store.fetch_task(name).resources if r.disk.persistence.id)


def test_agent_partition_heals_and_pod_relaunches_in_place():
    """UNREACHABLE starts a TRANSIENT recovery; its kill cannot reach the agent (the master
    answers UNREACHABLE and keeps the resources). When the agent returns, the recovery kills
    the stale task and relaunches the pod in place: same agent, same persistent volume."""
    with Chaos() as c:
        c.wait_plan("deploy")
        tid = c.task_id("hello-0-server")
        aid = c.agent_of("hello-0-server")
        vols = _volume_ids(c, "hello-0-server")
        c.master.lose_agent(aid)
        c.wait(lambda: c.state("hello-0-server") == P.TASK_UNREACHABLE, what="UNREACHABLE")
        c.wait(lambda: c.plan_code("recovery") == 202, what="recovery in progress")
        time.sleep(0.3)
        assert c.task_id("hello-0-server") == tid          # nothing can move while partitioned
        c.master.reconnect_agent(aid)
        c.wait(lambda: c.task_id("hello-0-server") != tid and c.state("hello-0-server") == P.TASK_RUNNING,
               what="relaunched in place")
        c.wait_plan("recovery")
        assert c.agent_of("hello-0-server") == aid
        assert _volume_ids(c, "hello-0-server") == vols
        assert c.master.task_states()[tid] == P.TASK_KILLED


def test_agent_gone_by_operator_is_replaced_elsewhere():
    with Chaos(agents=4) as c:
        c.wait_plan("deploy")
        old_agent = c.agent_of("world-0-server")
        old_tid = c.task_id("world-0-server")
        c.master.gone_by_operator(old_agent)
        c.wait(lambda: c.task_id("world-0-server") != old_tid and c.state("world-0-server") == P.TASK_RUNNING,
               what="world-0 replaced")
        c.wait_plan("recovery")
        assert c.agent_of("world-0-server") != old_agent
        assert c.task_id("world-0-server") in c.running_ids()


def test_scheduler_restart_resumes_without_relaunch():
    with Chaos() as c:
        c.wait_plan("deploy")
        before = {n: c.task_id(n) for n in ("hello-0-server", "hello-1-server", "world-0-server", "world-1-server")}
        launches = c.master.accept_calls
        c.crash()
        c.start()
        c.wait_plan("deploy")
        after = {n: c.task_id(n) for n in before}
        assert after == before
        time.sleep(0.3)
        # re-registration reconciles; nothing was relaunched
        assert set(before.values()) <= c.running_ids()
        assert c.master.accept_calls - launches <= 1   # at most an idle reservation-GC accept


def test_task_forgotten_while_scheduler_down_is_recovered():
    with Chaos(**UNKNOWN_AS_LOST) as c:
        c.wait_plan("deploy")
        tid = c.task_id("world-1-server")
        c.crash()
        c.master.forget_task(tid)
        c.start()
        c.wait(lambda: c.task_id("world-1-server") != tid and c.state("world-1-server") == P.TASK_RUNNING,
               timeout=30, what="world-1 relaunched")
        c.wait_plan("recovery", 30)


def test_task_forgotten_reference_behaviour_never_recovers():
    """With SDK_UNKNOWN_AS_LOST=false the TASK_UNKNOWN reply is stored and nothing recovers it."""
    with Chaos(SDK_UNKNOWN_AS_LOST="false") as c:
        c.wait_plan("deploy")
        tid = c.task_id("world-1-server")
        c.crash()
        c.master.forget_task(tid)
        c.start()
        c.wait(lambda: c.state("world-1-server") == P.TASK_UNKNOWN, what="TASK_UNKNOWN stored")
        time.sleep(0.5)
        assert c.task_id("world-1-server") == tid


def _restart_pod_with_lost_accept(c, pod):
    """Restart ``pod`` in place while its relaunch ACCEPT is lost in transit."""
    c.master.drop_next_accepts(1)
    assert c.api.post(f"/v1/pod/{pod}/restart").status == 200
    c.wait(lambda: c.master.dropped_accepts == 1, what="relaunch ACCEPT dropped")


def test_lost_accept_on_in_place_relaunch_keeps_the_volume():
    """the relaunch of a pod that already owns reservations and a persistent
    volume must stay TRANSIENT when its ACCEPT is lost (the watchdog's reconciliation answers
    LOST/UNKNOWN): same agent, same volume, never marked permanently failed."""
    from dcos_commons_amd.offer.taskdata.labels import TaskLabelReader

    with Chaos(**WATCHDOG) as c:
        c.wait_plan("deploy")
        name = "hello-0-server"
        tid, aid, vols = c.task_id(name), c.agent_of(name), _volume_ids(c, name)
        assert vols
        assert TaskLabelReader(c.store.fetch_task(name)).is_launch_new_footprint()   # first launch
        _restart_pod_with_lost_accept(c, "hello-0")
        c.wait(lambda: c.task_id(name) != tid and c.state(name) == P.TASK_RUNNING
               and c.task_id(name) in c.running_ids(), timeout=30, what="hello-0 relaunched")
        info = c.store.fetch_task(name)
        assert not TaskLabelReader(info).is_permanently_failed()
        assert not TaskLabelReader(info).is_launch_new_footprint()                   # in-place relaunch
        assert c.agent_of(name) == aid
        assert _volume_ids(c, name) == vols


def _stage_relaunch(c, name, new_footprint):
    """Write-ahead state of a relaunch whose ACCEPT never reached the master."""
    from dcos_commons_amd.offer.taskdata.labels import TaskLabelWriter

    info = P.TaskInfo()
    info.CopyFrom(c.store.fetch_task(name))
    info.task_id.value = info.task_id.value + "-relaunch"
    TaskLabelWriter(info).set_launch_new_footprint(new_footprint).apply()
    c.store.store_tasks([info])
    staging = P.TaskStatus(state=P.TASK_STAGING)
    staging.task_id.CopyFrom(info.task_id)
    c.store.store_status(name, staging)
    return info


def _master_reply(info, state, reason):
    st = P.TaskStatus(state=state, source=P.TaskStatus.SOURCE_MASTER, reason=reason)
    st.task_id.CopyFrom(info.task_id)
    return st


def test_never_launched_rule_applies_only_to_a_new_footprint():
    """The never-launched rule (TASK_DROPPED/REASON_INVALID_OFFERS or reconciliation LOST on the
    write-ahead STAGING status) re-footprints a first launch, and never an in-place relaunch."""
    from dcos_commons_amd.offer.taskdata.labels import TaskLabelReader

    cases = [(P.TASK_DROPPED, P.TaskStatus.REASON_INVALID_OFFERS),
             (P.TASK_LOST, P.TaskStatus.REASON_RECONCILIATION)]
    with Chaos(**WATCHDOG) as c:
        c.wait_plan("deploy")
        sched = c.runner.scheduler
        for state, reason in cases:
            # relaunch in place: reservations exist, the task must stay transiently failed
            info = _stage_relaunch(c, "world-0-server", new_footprint=False)
            sched.process_status_update(_master_reply(info, state, reason))
            assert not TaskLabelReader(c.store.fetch_task("world-0-server")).is_permanently_failed()
        # first footprint: the reservations were never made, so it is re-footprinted
        info = _stage_relaunch(c, "world-1-server", new_footprint=True)
        sched.process_status_update(_master_reply(info, P.TASK_DROPPED, P.TaskStatus.REASON_INVALID_OFFERS))
        assert TaskLabelReader(c.store.fetch_task("world-1-server")).is_permanently_failed()


def test_lost_accept_of_a_new_resource_set_next_to_a_running_executor_is_relaunched():
    """the first launch of a sidecar task (its own ``sidecar-res`` resource set) next to
    a running server, with its ACCEPT lost. The pod's first footprint (the server's deploy) already
    reserved ``sidecar-res`` (the new-footprint pipeline reserves every resource set of the pod, as
    the reference's does), so this launch is not a new footprint: the watchdog's reconciliation
    answers LOST, the task is relaunched in place on those reservations and the sidecar plan
    completes; the server and its executor are never touched."""
    from dcos_commons_amd.mesos.local_master import TaskBehavior, TaskTiming
    from dcos_commons_amd.offer.resources import get_resource_ids
    from dcos_commons_amd.offer.taskdata.labels import TaskLabelReader

    env = dict(ENV, HELLO_COUNT="1")
    cfg = SchedulerConfig.for_testing(PORT_API="0", SDK_OFFER_WAIT_S="0.2", SDK_LAUNCH_RECONCILE_S="0.3")
    raw = RawServiceSpec.new_builder(os.path.join(SPECS, "sidecar.yml")).set_env(env).build()
    spec = ServiceSpecGenerator(raw, cfg, SPECS, env).build()
    once = TaskTiming(finish_after_s=0.05)
    master = LocalMaster(allocation_interval_s=0.05,
                         behavior=TaskBehavior(overrides={"backup": once, "verify": once}))
    master.add_agent(AgentSpec(hostname="host-0", cpus=4, mem=8192, disk=20000))
    runner = SchedulerRunner(SchedulerBuilder(spec, cfg, MemPersister()).set_plans_from(raw),
                             driver_factory=lambda s, i: LocalSchedulerDriver(master, s, i))
    runner.run(block=False)
    try:
        api = runner.framework_runner.api_server.router
        store = runner.scheduler.state_store

        def wait(pred, what, timeout=20.0):
            t0 = time.time()
            while time.time() - t0 < timeout:
                if pred():
                    return
                time.sleep(0.005)
            raise AssertionError(f"{what} not reached in {timeout}s")

        wait(lambda: api.get("/v1/plans/deploy").status == 200, "deploy COMPLETE")
        server = store.fetch_task("hello-0-server")
        server_tid = server.task_id.value
        reserved_at_deploy = sorted(get_resource_ids(store.fetch_task("hello-0-backup").resources))
        assert reserved_at_deploy  # stored with an empty TaskID by the first footprint
        master.drop_next_accepts(1)
        assert api.post("/v1/plans/sidecar/start", body={}).status == 200
        wait(lambda: master.dropped_accepts == 1, "backup ACCEPT dropped")
        wait(lambda: api.get("/v1/plans/sidecar").status == 200, "sidecar plan COMPLETE")
        backup = store.fetch_task("hello-0-backup")
        assert not TaskLabelReader(backup).is_permanently_failed()
        assert store.fetch_status("hello-0-backup").state == P.TASK_FINISHED
        # the server and its executor were never touched
        assert store.fetch_task("hello-0-server").task_id.value == server_tid
        assert master.task_states()[server_tid] == P.TASK_RUNNING
        assert backup.executor.executor_id.value == server.executor.executor_id.value
        assert not TaskLabelReader(backup).is_launch_new_footprint()
        assert sorted(get_resource_ids(backup.resources)) == reserved_at_deploy
    finally:
        runner.stop()
        master.shutdown()
