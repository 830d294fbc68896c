"""hello-world entry modes, scenarios and customizers (reference: frameworks/helloworld/src/main/
java/.../scheduler/{Main,Scenario,ReversePhasesCustomizer,DecommissionCustomizer,
ExampleMultiServiceResource}.java and helloworld's CustomStepsTest / ServiceTest)."""
import json
import time

import pytest

from dcos_commons_amd.mesos import protos as P
from dcos_commons_amd.mesos.local_master import AgentSpec, LocalMaster, LocalSchedulerDriver
from dcos_commons_amd.models import helloworld as H
from dcos_commons_amd.scheduler.scheduler_config import SchedulerConfig
from dcos_commons_amd.storage.mem_persister import MemPersister
from dcos_commons_amd.testing import Expect, Send
from test_sim_helloworld import ENV, default_deployment_ticks, runner


def test_scenario_parsing():
    assert H.get_scenarios({}) == [H.Scenario.YAML]
    assert H.get_scenarios({"SCENARIOS": "java, custom_plan"}) == [H.Scenario.JAVA, H.Scenario.CUSTOM_PLAN]
    with pytest.raises(ValueError) as e:
        H.get_scenarios({"SCENARIOS": "nope"})
    assert "Expected one of" in str(e.value)


def test_reverse_phases_customizer():
    def check(sim):
        plan = sim.scheduler.get_plan("deploy")
        world = next(p for p in plan.get_children() if p.get_name() == "world")
        assert [s.get_name() for s in world.get_children()] == ["world-1:[server]", "world-0:[server]"]

    r = runner().set_builder_customizer(lambda b: H.customize(b, None, [H.Scenario.CUSTOM_PLAN]))
    r.run([Send.register(), Expect.that(check, "world steps reversed")])


def test_decommission_customizer_prepends_step():
    first = runner().run(default_deployment_ticks())

    def check(sim):
        plan = sim.scheduler.get_plan("decommission")
        assert plan is not None
        names = [[s.get_name() for s in ph.get_children()] for ph in plan.get_children()]
        assert names and all(n[0] == H.CUSTOM_DECOMMISSION_STEP_NAME for n in names), names

    second = (runner(WORLD_COUNT="1").set_state(first.persister)
              .set_builder_customizer(lambda b: H.customize(b, None, [H.Scenario.CUSTOM_DECOMMISSION])))
    second.run([Send.register(), Expect.that(check, "custom step first in each decommission phase")])


def test_multi_region_scenario_sets_region_constraint():
    from dcos_commons_amd.scheduler.scheduler_builder import SchedulerBuilder

    b = H.customize(SchedulerBuilder.__new__(SchedulerBuilder), None, [H.Scenario.MULTI_REGION])
    assert b.region_awareness_enabled


class _Live:
    def __init__(self, agents=3):
        self.master = LocalMaster(allocation_interval_s=0.05)
        for i in range(agents):
            self.master.add_agent(AgentSpec(hostname=f"h{i}", cpus=8, mem=16384, disk=100000))
        self.cfg = SchedulerConfig.for_testing(PORT_API="0", SDK_OFFER_WAIT_S="0.5")
        self.persister = MemPersister()
        self.runner = None

    def start(self, args, env):
        self.runner = H.run(args, env=env, scheduler_config=self.cfg, persister=self.persister, block=False,
                            driver_factory=lambda s, i: LocalSchedulerDriver(self.master, s, i))
        return self.runner.framework_runner.api_server.router

    def wait(self, pred, timeout=20):
        t0 = time.time()
        while time.time() - t0 < timeout:
            if pred():
                return
            time.sleep(0.01)
        raise AssertionError("timeout")

    def stop(self):
        if self.runner is not None:
            self.runner.stop()
        self.master.shutdown()


def test_java_scenario_deploys_code_defined_service():
    live = _Live()
    try:
        api = live.start([], dict(SCENARIOS="JAVA", HELLO_COUNT="2", HELLO_CPUS="0.5"))
        live.wait(lambda: api.get("/v1/plans/deploy").status == 200)
        assert sorted(api.get("/v1/pod").json()) == ["hello-0", "hello-1"]
        assert set(live.master.task_states().values()) == {P.TASK_RUNNING}
    finally:
        live.stop()


def test_single_and_static_multi_yaml_modes():
    live = _Live()
    try:
        api = live.start(["svc"], dict(ENV))
        live.wait(lambda: api.get("/v1/plans/deploy").status == 200)
        assert len(live.master.task_states()) == 3
    finally:
        live.stop()
    live = _Live(agents=4)
    env = dict(ENV, FRAMEWORK_NAME="multi-hello")
    try:
        api = live.start(["svc,svc"], env)
        # the same YAML twice renders the same service name -> rejected as a duplicate? No: the
        # second overwrites the first in the manager; one service answers under /v1/service
        live.wait(lambda: api.get("/v1/service").status == 200)
        names = api.get("/v1/service").json()
        assert names == ["multi-hello"]
        live.wait(lambda: api.get("/v1/service/multi-hello/plans/deploy").status == 200)
    finally:
        live.stop()


def test_dynamic_multi_service_add_list_uninstall_and_recover():
    live = _Live(agents=4)
    env = dict(ENV, FRAMEWORK_NAME="dyn-hello", HELLO_COUNT="1", WORLD_COUNT="1")
    try:
        api = live.start([], env)
        assert "svc" in api.get("/v1/multi/yaml").json()
        r = api.post("/v1/multi/svc-a?yaml=svc", {"FRAMEWORK_NAME": "svc-a"})
        assert r.status == 200 and r.json() == {"name": "svc-a", "yaml": "svc"}
        assert api.post("/v1/multi/bad?yaml=nope", {}).status == 400
        r = api.post("/v1/multi/svc-b?yaml=svc", {"FRAMEWORK_NAME": "svc-b"})
        assert r.status == 200
        live.wait(lambda: api.get("/v1/service/svc-a/plans/deploy").status == 200 and
                  api.get("/v1/service/svc-b/plans/deploy").status == 200)
        listed = {e["service"]: e for e in api.get("/v1/multi").json()}
        assert listed["svc-a"] == {"service": "svc-a", "uninstall": False, "yaml": "svc"}
        assert api.dispatch("DELETE", "/v1/multi/svc-a").status == 200
        live.wait(lambda: "svc-a" not in api.get("/v1/service").json())
        assert not any(t.startswith("svc-a__") and s == P.TASK_RUNNING for t, s in live.master.task_states().items())
    finally:
        live.stop()
    # a restarted scheduler recovers the remaining service from the ServiceStore
    live2 = _Live(agents=4)
    live2.persister = live.persister
    try:
        api = live2.start([], env)
        assert api.get("/v1/service").json() == ["svc-b"]
        assert [e["service"] for e in api.get("/v1/multi").json()] == ["svc-b"]
    finally:
        live2.stop()


def test_example_resource_context_roundtrip():
    ctx = H.ExampleMultiServiceResource.serialize("n", "svc", {"B": "2", "A": "1"})
    assert json.loads(ctx) == {"name": "n", "yaml": "svc", "params": [{"key": "A", "value": "1"},
                                                                     {"key": "B", "value": "2"}]}
