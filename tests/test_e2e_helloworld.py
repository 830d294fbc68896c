"""End-to-end: helloworld deploys on the in-process Mesos master, recovers and answers the API.

Mirrors the reference's helloworld ServiceTest flow (frameworks/helloworld/src/test/java/com/
mesosphere/sdk/helloworld/scheduler/ServiceTest.java) but against a live offer loop.
"""
import os
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

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SPECS = os.path.join(ROOT, "frameworks", "helloworld", "specs")


def hello_env(hello=2, world=2):
    return dict(FRAMEWORK_NAME="hello-world", FRAMEWORK_PRINCIPAL="hw-principal", FRAMEWORK_USER="nobody",
                HELLO_COUNT=str(hello), HELLO_PLACEMENT='[["hostname", "UNIQUE"]]', HELLO_CPUS="0.1",
                HELLO_MEM="252", HELLO_DISK="25", HELLO_GPUS="1", SLEEP_DURATION="1000", WORLD_COUNT=str(world),
                WORLD_PLACEMENT='[["hostname", "UNIQUE"]]', WORLD_CPUS="0.2", WORLD_MEM="512", WORLD_DISK="25",
                WORLD_READINESS_CHECK_INTERVAL="5", WORLD_READINESS_CHECK_DELAY="0",
                WORLD_READINESS_CHECK_TIMEOUT="10", GPU_PROBE_CMD="true")


# every live-scheduler test runs under the scheduler defaults and with every deviation off
pytestmark = pytest.mark.usefixtures("sched_profile")


class Cluster:
    def __init__(self, spec_file="svc.yml", agents=3, gpus=0, env=None, transport="local", **cfg):
        self.env = env or hello_env()
        overrides = {"PORT_API": "0", "SDK_OFFER_WAIT_S": "0.5"}
        from dcos_commons_amd.testing import profiles

        overrides.update(profiles.ACTIVE)    # the suite's flag profile; the test's own flags win
        overrides.update(cfg)
        self.cfg = SchedulerConfig.for_testing(**overrides)
        raw = RawServiceSpec.new_builder(os.path.join(SPECS, spec_file)).set_env(self.env).build()
        self.spec = ServiceSpecGenerator(raw, self.cfg, SPECS, self.env).build()
        self.master = LocalMaster(allocation_interval_s=0.05)
        self.agent_ids = [self.master.add_agent(AgentSpec(hostname=f"host-{i}", cpus=4, mem=8192, disk=20000,
                                                          gpus=gpus)) for i in range(agents)]
        self.persister = MemPersister()
        self.http_master = None
        if transport == "local":
            factory = lambda s, i: LocalSchedulerDriver(self.master, s, i)  # noqa: E731
        else:  # the Mesos v1 HTTP API, over a socket, in json or protobuf
            from dcos_commons_amd.mesos.http_driver import JSON, PROTOBUF, V1HttpSchedulerDriver
            from dcos_commons_amd.mesos.http_master import HttpMaster

            self.http_master = HttpMaster(self.master, heartbeat_s=1.0).start()
            ctype = JSON if transport == "json" else PROTOBUF
            factory = lambda s, i: V1HttpSchedulerDriver(self.http_master.url, s, i, content_type=ctype)  # noqa: E731
        self.runner = SchedulerRunner(SchedulerBuilder(self.spec, self.cfg, self.persister).set_plans_from(raw),
                                      driver_factory=factory)

    def __enter__(self):
        self.runner.run(block=False)
        self.api = self.runner.framework_runner.api_server.router
        self.store = self.runner.scheduler.state_store
        return self

    def __exit__(self, *exc):
        self.runner.stop()
        if self.http_master is not None:
            self.http_master.stop()
        self.master.shutdown()

    def wait(self, pred, timeout=20.0, what="condition"):
        t0 = time.time()
        while time.time() - t0 < timeout:
            if pred():
                return
            time.sleep(0.005)
        raise AssertionError(f"{what} not reached in {timeout}s")

    def wait_plan(self, name, code=200, timeout=20.0):
        self.wait(lambda: self.api.get(f"/v1/plans/{name}").status == code, timeout)


def test_helloworld_deploys_serially_and_reports_complete():
    with Cluster() as c:
        c.wait_plan("deploy")
        plan = c.api.get("/v1/plans/deploy").json()
        assert plan["status"] == "COMPLETE"
        assert [p["name"] for p in plan["phases"]] == ["hello", "world"]
        assert [s["name"] for s in plan["phases"][0]["steps"]] == ["hello-0:[server]", "hello-1:[server]"]
        states = c.master.task_states()
        assert len(states) == 4 and set(states.values()) == {P.TASK_RUNNING}
        # one pod per host (hostname:UNIQUE) for each pod type
        hosts = {}
        for info in c.store.fetch_tasks():
            hosts.setdefault(info.name.split("-")[0], set()).add(
                next(l.value for l in info.labels.labels if l.key == "offer_hostname"))
        assert len(hosts["hello"]) == 2 and len(hosts["world"]) == 2
        assert c.api.get("/v1/health").status == 200
        assert sorted(c.api.get("/v1/pod").json()) == ["hello-0", "hello-1", "world-0", "world-1"]


def test_restart_and_replace_recover():
    # the last check (stale reservations released while the scheduler goes idle) needs the MI355X
    # reservation GC on every offer: the reference GCs only offers it leaves unused, and the offer
    # carrying the replaced pod's reservations is the one its replacement launches on
    with Cluster(SDK_RESERVATION_GC_ALL_OFFERS="true") as c:
        c.wait_plan("deploy")
        old = c.store.fetch_task("hello-0-server").task_id.value
        c.master.fail_task(old)
        c.wait(lambda: (c.store.fetch_status("hello-0-server") or P.TaskStatus()).task_id.value not in ("", old)
               and c.store.fetch_status("hello-0-server").state == P.TASK_RUNNING)
        c.wait_plan("recovery")
        old = c.store.fetch_task("world-1-server").task_id.value
        r = c.api.post("/v1/pod/world-1/replace")
        assert r.status == 200 and r.json() == {"pod": "world-1", "tasks": ["world-1-server"]}
        c.wait(lambda: (c.store.fetch_status("world-1-server") or P.TaskStatus()).task_id.value not in ("", old)
               and c.store.fetch_status("world-1-server").state == P.TASK_RUNNING)
        c.wait_plan("recovery")
        # the replaced pod got fresh reservations; the old ones were released
        for aid in c.agent_ids:
            ids = {next((l.value for l in r.reservations[-1].labels.labels if l.key == "resource_id"), None)
                   for r in c.master.reserved_resources(aid)}
            live = set()
            for info in c.store.fetch_tasks():
                for res in list(info.resources) + list(info.executor.resources):
                    for l in res.reservations[-1].labels.labels if len(res.reservations) else []:
                        if l.key == "resource_id":
                            live.add(l.value)
            c.wait(lambda aid=aid, live=live: {next((l.value for l in r.reservations[-1].labels.labels
                                                      if l.key == "resource_id"), None)
                                                for r in c.master.reserved_resources(aid)} <= live)


def test_gpu_pods_get_one_device_each():
    env = hello_env(hello=3, world=0)
    with Cluster("gpu.yml", agents=3, gpus=1, env=env) as c:
        c.wait_plan("deploy")
        devices = []
        for info in c.store.fetch_tasks():
            gp = [r for r in info.resources if r.name == "gpus"]
            assert gp and gp[0].scalar.value == 1.0
            st = c.store.fetch_status(info.name)
            devices.append(next(l.value for l in st.labels.labels if l.key == "gpu_devices"))
        assert devices == ["0", "0", "0"]  # each agent owns device 0 of its own node


def test_plan_interrupt_and_continue_via_api():
    env = hello_env(hello=2, world=1)
    with Cluster(env=env) as c:
        c.wait_plan("deploy")
        assert c.api.post("/v1/plans/deploy/interrupt").status == 208  # already complete
        assert c.api.post("/v1/plans/nope/continue").status == 404
        r = c.api.post("/v1/plans/deploy/restart?phase=world")
        assert r.status == 200
        c.wait_plan("deploy")


@pytest.mark.parametrize("profile", ["mi355x", "reference"])
def test_bench_cycle_cpu(profile):
    from dcos_commons_amd.benchmarks.deploy_bench import DeployBench

    res = DeployBench(2, profile=profile, allocation_interval_s=0.05, timeout_s=60).run_cycle()
    assert res.deploy_s < 10 and res.mttr_restart_s < 15 and res.mttr_replace_s < 15
    # BASELINE.md's window starts at SUBSCRIBED, inside the headline's (which starts at construction)
    assert 0 < res.deploy_from_subscribed_s < res.deploy_s
