"""Multi-service scheduler: two helloworld services behind one framework (reference:
scheduler/multi/{MultiServiceEventClientTest,MultiServiceManagerTest,ServiceStoreTest,
ParallelFootprintDisciplineTest}; helloworld ServiceTest.testDefaultDeploymentWithNamespace)."""
import os
import time

import pytest

from dcos_commons_amd.framework.framework_config import FrameworkConfig
from dcos_commons_amd.mesos import protos as P
from dcos_commons_amd.mesos.local_master import AgentSpec, LocalMaster, LocalSchedulerDriver
from dcos_commons_amd.scheduler.mesos_event_client import ClientStatusResponse
from dcos_commons_amd.scheduler.multi import (
    DisciplineSelectionStore,
    MultiServiceEventClient,
    MultiServiceManager,
    MultiServiceRunner,
    ParallelFootprintDiscipline,
    ServiceStore,
)
from dcos_commons_amd.scheduler.scheduler_builder import SchedulerBuilder
from dcos_commons_amd.scheduler.scheduler_config import SchedulerConfig
from dcos_commons_amd.specification.yaml.mappers import ServiceSpecGenerator
from dcos_commons_amd.specification.yaml.raw import RawServiceSpec
from dcos_commons_amd.storage.mem_persister import MemPersister
from test_e2e_helloworld import hello_env

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SVC = os.path.join(ROOT, "frameworks", "helloworld", "specs", "svc.yml")
FC = FrameworkConfig(framework_name="multi-fw", role="multi-fw-role", principal="multi-fw-principal")


def build_service(name, persister, cfg, hello=1, world=1):
    env = hello_env(hello=hello, world=world)
    env["FRAMEWORK_NAME"] = name
    raw = RawServiceSpec.new_builder(SVC).set_env(env).build()
    spec = ServiceSpecGenerator(raw, cfg, os.path.dirname(SVC), env).set_multi_service_framework_config(FC).build()
    return SchedulerBuilder(spec, cfg, persister).set_plans_from(raw).enable_multi_service(FC.framework_name).build()


def wait(pred, timeout=20):
    t0 = time.time()
    while time.time() - t0 < timeout:
        if pred():
            return
        time.sleep(0.01)
    raise AssertionError("timeout")


def test_two_services_deploy_under_one_framework():
    cfg = SchedulerConfig.for_testing(PORT_API="0", SDK_OFFER_WAIT_S="0.5")
    persister = MemPersister()
    manager = MultiServiceManager()
    a = build_service("hello-a", persister, cfg)
    b = build_service("/path/to/hello-b", persister, cfg)
    manager.put_service(a).put_service(b)
    client = MultiServiceEventClient(FC.framework_name, cfg, manager, persister)
    master = LocalMaster(allocation_interval_s=0.05)
    for i in range(4):
        master.add_agent(AgentSpec(hostname=f"h{i}", cpus=4, mem=8192, disk=20000))
    runner = MultiServiceRunner(cfg, FC, persister, client, driver_factory=lambda s, i: LocalSchedulerDriver(master, s, i))
    runner.run(block=False)
    api = runner.framework_runner.api_server.router
    try:
        wait(lambda: api.get("/v1/service/hello-a/plans/deploy").status == 200 and
             api.get("/v1/service/path.to.hello-b/plans/deploy").status == 200)
        assert api.get("/v1/health").status == 200
        assert api.get("/v1/service").json() == ["/path/to/hello-b", "hello-a"]
        assert api.get("/v1/service/nope/plans").status == 404
        assert sorted(api.get("/v1/service/hello-a/pod").json()) == ["hello-0", "world-0"]
        # state is namespaced per service
        assert len(persister.get_children("Services/hello-a/Tasks")) == 2
        assert len(persister.get_children("Services/path__to__hello-b/Tasks")) == 2
        states = master.task_states()
        assert len(states) == 4 and set(states.values()) == {P.TASK_RUNNING}
        # task IDs carry the sanitized service name, which routes statuses back to the owner
        names = sorted(tid.split("__")[0] for tid in states)
        assert names == ["hello-a", "hello-a", "path.to.hello-b", "path.to.hello-b"]
        # pod restart through the delegated API recovers in the right service
        old = b.state_store.fetch_task("world-0-server").task_id.value
        assert api.post("/v1/service/path.to.hello-b/pod/world-0/restart").status == 200
        wait(lambda: (b.state_store.fetch_status("world-0-server") or P.TaskStatus()).task_id.value not in ("", old)
             and b.state_store.fetch_status("world-0-server").state == P.TASK_RUNNING)
        # reservations are labelled with their service namespace
        ns = set()
        for aid in master.agents:
            for r in master.reserved_resources(aid):
                ns.update(l.value for l in r.reservations[-1].labels.labels if l.key == "namespace")
        assert ns == {"hello-a", "/path/to/hello-b"}
    finally:
        runner.stop()
        master.shutdown()


def test_uninstall_one_service_releases_its_reservations():
    cfg = SchedulerConfig.for_testing(PORT_API="0", SDK_OFFER_WAIT_S="0.5")
    persister = MemPersister()
    manager = MultiServiceManager()
    store = ServiceStore(persister, lambda ctx: build_service(ctx.decode(), persister, cfg))
    a = store.put(b"hello-a")
    b = store.put(b"hello-b")
    manager.put_service(a).put_service(b)
    client = MultiServiceEventClient(FC.framework_name, cfg, manager, persister,
                                     uninstall_callback=store.uninstall_callback())
    master = LocalMaster(allocation_interval_s=0.05)
    for i in range(3):
        master.add_agent(AgentSpec(hostname=f"h{i}", cpus=4, mem=8192, disk=20000))
    runner = MultiServiceRunner(cfg, FC, persister, client, driver_factory=lambda s, i: LocalSchedulerDriver(master, s, i))
    runner.run(block=False)
    api = runner.framework_runner.api_server.router
    try:
        wait(lambda: api.get("/v1/health").status == 200)
        manager.uninstall_service("hello-a")
        wait(lambda: manager.get_service("hello-a") is None)
        # hello-a's tasks were killed and its reservations released; its state and context are gone
        wait(lambda: not any(tid.startswith("hello-a__") and st == P.TASK_RUNNING for tid, st in master.task_states().items()))

        def a_reservations():
            out = 0
            for aid in master.agents:
                for r in master.reserved_resources(aid):
                    if any(l.key == "namespace" and l.value == "hello-a" for l in r.reservations[-1].labels.labels):
                        out += 1
            return out
        wait(lambda: a_reservations() == 0)
        assert store.get("hello-a") is None and store.get("hello-b") == b"hello-b"
        with pytest.raises(Exception):
            persister.get_children("Services/hello-a")
        assert api.get("/v1/service/hello-b/plans/deploy").status == 200
        # the service list survives a scheduler restart
        assert [s.service_spec.name for s in store.recover()] == ["hello-b"]
    finally:
        runner.stop()
        master.shutdown()


def test_parallel_footprint_discipline_limits_reserving_services():
    store = DisciplineSelectionStore(MemPersister())
    d = ParallelFootprintDiscipline(1, store)
    d.update_services({"a", "b"})
    fp = ClientStatusResponse.footprint(True)
    assert d.update_service_status("a", fp)
    assert not d.update_service_status("b", fp)  # only one may grow its footprint
    assert d.update_service_status("b", ClientStatusResponse.launching(False))
    assert d.update_service_status("a", ClientStatusResponse.idle())  # a finished reserving
    assert d.update_service_status("b", fp)
    d.update_services({"b"})  # selection is persisted when the service set is refreshed
    assert store.fetch_selected_services() == frozenset({"b"})
    d2 = ParallelFootprintDiscipline(1, DisciplineSelectionStore(store.persister))
    d2.update_services({"a", "b"})
    assert d2.selected == {"b"}  # recovered from SelectedServices
    with pytest.raises(ValueError):
        ParallelFootprintDiscipline(0, store)


def test_manager_rejects_sanitized_name_collisions():
    cfg = SchedulerConfig.for_testing(PORT_API="0")
    m = MultiServiceManager()
    p = MemPersister()
    m.put_service(build_service("/a/b", p, cfg))
    with pytest.raises(ValueError):
        m.put_service(build_service("a.b", p, cfg))


def test_service_store_context_limit():
    cfg = SchedulerConfig.for_testing(PORT_API="0")
    p = MemPersister()
    store = ServiceStore(p, lambda ctx: build_service("svc", p, cfg))
    with pytest.raises(ValueError):
        store.put(b"x" * (100 * 1024 + 1))
    assert store.recover() == []
