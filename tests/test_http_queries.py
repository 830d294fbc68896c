"""Unit tests of the /v1 query layer against fixed state (no running scheduler).

Mirrors the reference's query and endpoint suites under sdk/scheduler/src/test/java/com/
mesosphere/sdk/http/: PlansQueriesTest (plan/phase/step commands and their 200/208/400/404
answers), PodQueriesTest (pod grouping, override-aware task states, pause/restart/replace),
StateQueriesTest (framework ID, properties, files, zones, cache refresh), ConfigQueriesTest
(400/404/500 mapping), HealthResourceTest (service status codes by plan state) and
ArtifactQueriesTest / EndpointsQueriesTest. Everything goes through the same Router the HTTP
server uses, so the status codes are the wire ones.
"""
import json
import uuid

import pytest

from dcos_commons_amd.framework import driver as driver_mod
from dcos_commons_amd.framework import task_killer
from dcos_commons_amd.http import resources as R
from dcos_commons_amd.http.api import Router
from dcos_commons_amd.mesos import protos as P
from dcos_commons_amd.offer.common_id_utils import to_sanitized_service_name_from_id, to_task_id, to_task_name
from dcos_commons_amd.offer.taskdata.labels import TaskLabelWriter
from dcos_commons_amd.scheduler.plan import backoff as B
from dcos_commons_amd.scheduler.plan.deployment_step import DeploymentStep
from dcos_commons_amd.scheduler.plan.elements import DefaultPhase, DefaultPlan
from dcos_commons_amd.scheduler.plan.managers import DefaultPlanCoordinator, DefaultPlanManager
from dcos_commons_amd.scheduler.plan.pod_instance_requirement import PodInstanceRequirement
from dcos_commons_amd.scheduler.plan.status import Status
from dcos_commons_amd.scheduler.plan.strategy import CanaryStrategy, ParallelStrategy, SerialStrategy
from dcos_commons_amd.scheduler.scheduler_config import SchedulerConfig
from dcos_commons_amd.specification.specs import PodInstance
from dcos_commons_amd.specification.yaml import mappers
from dcos_commons_amd.specification.yaml.raw import RawServiceSpec
from dcos_commons_amd.state.config_store import ConfigStoreException
from dcos_commons_amd.state.framework_store import FrameworkStore
from dcos_commons_amd.state.goal_state_override import GoalStateOverride, OverrideProgress, OverrideStatus
from dcos_commons_amd.state.state_store import StateStore, StateStoreException
from dcos_commons_amd.storage.mem_persister import MemPersister
from dcos_commons_amd.storage.persister import PersisterException, Reason
from dcos_commons_amd.storage.persister_cache import PersisterCache

SERVICE = "test-service"


class RecordingDriver(driver_mod.SchedulerDriver):
    def __init__(self):
        self.killed = []

    def kill_task(self, task_id):
        self.killed.append(task_id.value)


@pytest.fixture(autouse=True)
def quiet_killer():
    """TaskKiller without its background re-kill thread, against a recording driver."""
    task_killer.reset(executor_enabled=False)
    d = RecordingDriver()
    prev = driver_mod.get_instance()
    driver_mod.set_driver(d)
    yield d
    driver_mod.set_driver(prev)
    task_killer.reset(executor_enabled=True)


# ---------------------------------------------------------------------------------------
# pods (PodQueriesTest)


def _task(name, pod_type=None, index=None, tid_name=None):
    t = P.TaskInfo(name=name)
    t.task_id.CopyFrom(to_task_id(SERVICE, tid_name or name))
    t.agent_id.value = "test-agent-id"
    if pod_type is not None:
        w = TaskLabelWriter(t)
        w.set_type(pod_type)
        w.set_index(index)
        w.apply()
    return t


def _status(info, state):
    st = P.TaskStatus(state=state)
    st.task_id.CopyFrom(info.task_id)
    return st


NO_POD = _task("test-task-name")
P0 = {c: _task(f"test-0-{c}", "test", 0, c) for c in "abcd"}
P1 = {c: _task(f"test-1-{c}", "test", 1, c) for c in "ab"}
P2A = _task("test-2-a", "test", 2, "a")


@pytest.fixture
def pod_store():
    st = StateStore(MemPersister(), repair=False)
    st.store_tasks([NO_POD, *P0.values(), *P1.values(), P2A])
    for info, state in ((NO_POD, P.TASK_RUNNING), (P0["a"], P.TASK_RUNNING), (P0["b"], P.TASK_STAGING),
                        (P0["c"], P.TASK_RUNNING), (P1["a"], P.TASK_FINISHED), (P1["b"], P.TASK_RUNNING),
                        (P2A, P.TASK_FINISHED)):
        st.store_status(info.name, _status(info, state))  # test-0-d has no status
    return st


def pods_router(store, failure_setter=None):
    return Router([R.PodResource(store, config_store=None, service_name=SERVICE, failure_setter=failure_setter)])


def test_pod_names_sort_instances_and_list_podless_tasks_last(pod_store):
    r = pods_router(pod_store).get("/v1/pod")
    assert r.status == 200 and r.json() == ["test-0", "test-1", "test-2", "UNKNOWN_POD_test-task-name"]


def test_all_pod_statuses_follow_goal_overrides(pod_store):
    ov = pod_store.store_goal_override_status
    ov("test-0-b", GoalStateOverride.NONE.new_status(OverrideProgress.IN_PROGRESS))
    ov("test-0-c", GoalStateOverride.PAUSED.new_status(OverrideProgress.PENDING))
    ov("test-1-b", GoalStateOverride.NONE.new_status(OverrideProgress.IN_PROGRESS))
    ov("test-task-name", GoalStateOverride.PAUSED.new_status(OverrideProgress.COMPLETE))
    body = pods_router(pod_store).get("/v1/pod/status").json()
    assert set(body) == {"service", "pods"} and body["service"] == SERVICE
    test, unknown = body["pods"]
    assert test["name"] == "test" and [i["name"] for i in test["instances"]] == ["test-0", "test-1", "test-2"]

    def states(inst):
        return [(t["name"], t.get("status")) for t in inst["tasks"]]
    i0, i1, i2 = test["instances"]
    assert states(i0) == [("test-0-a", "RUNNING"), ("test-0-b", "STARTING"), ("test-0-c", "PAUSING"),
                          ("test-0-d", None)]
    assert set(i0["tasks"][3]) == {"id", "name"}  # no status key without a TaskStatus
    assert states(i1) == [("test-1-a", "FINISHED"), ("test-1-b", "STARTING")]
    assert states(i2) == [("test-2-a", "FINISHED")]
    for t in i0["tasks"]:
        tid = P.TaskID(value=t["id"])
        assert to_sanitized_service_name_from_id(tid) == SERVICE
        assert to_task_name(tid) == t["name"][len("test-0-"):]
    assert unknown["name"] == "UNKNOWN_POD"
    assert unknown["instances"] == [{"name": "UNKNOWN_POD-0", "tasks": [
        {"id": NO_POD.task_id.value, "name": "test-task-name", "status": "PAUSED"}]}]


def test_one_pod_status_and_not_found(pod_store):
    pod_store.store_goal_override_status("test-1-b", GoalStateOverride.PAUSED.new_status(OverrideProgress.IN_PROGRESS))
    router = pods_router(pod_store)
    r = router.get("/v1/pod/test-1/status")
    assert r.status == 200
    assert r.json() == {"name": "test-1", "tasks": [
        {"id": P1["a"].task_id.value, "name": "test-1-a", "status": "FINISHED"},
        {"id": P1["b"].task_id.value, "name": "test-1-b", "status": "PAUSING"}]}
    assert router.get("/v1/pod/aaa/status").status == 404


def test_pod_info_pairs_each_task_with_its_status(pod_store):
    router = pods_router(pod_store)
    r = router.get("/v1/pod/test-1/info")
    assert r.status == 200
    body = r.json()
    assert [e["info"]["name"] for e in body] == ["test-1-a", "test-1-b"]
    assert [e["status"]["state"] for e in body] == ["TASK_FINISHED", "TASK_RUNNING"]
    assert router.get("/v1/pod/test-0/info").json()[3]["status"] is None  # test-0-d
    assert router.get("/v1/pod/aaa/info").status == 404


def test_pause_entire_pod(pod_store, quiet_killer):
    r = pods_router(pod_store).post("/v1/pod/test-0/pause")
    assert r.status == 200 and r.json() == {"pod": "test-0", "tasks": [f"test-0-{c}" for c in "abcd"]}
    for c in "abcd":
        assert pod_store.fetch_goal_override_status(f"test-0-{c}") == \
            GoalStateOverride.PAUSED.new_status(OverrideProgress.PENDING)
    assert sorted(quiet_killer.killed) == sorted(P0[c].task_id.value for c in "abcd")


def test_pause_unknown_pod_changes_nothing(pod_store, quiet_killer):
    assert pods_router(pod_store).post("/v1/pod/aaa/pause").status == 404
    assert all(pod_store.fetch_goal_override_status(n) == OverrideStatus.INACTIVE for n in pod_store.fetch_task_names())
    assert quiet_killer.killed == []


def test_pause_selected_tasks_with_or_without_pod_prefix(pod_store, quiet_killer):
    r = pods_router(pod_store).post("/v1/pod/test-0/pause", json.dumps(["a", "test-0-c"]))
    assert r.status == 200 and r.json() == {"pod": "test-0", "tasks": ["test-0-a", "test-0-c"]}
    paused = GoalStateOverride.PAUSED.new_status(OverrideProgress.PENDING)
    assert pod_store.fetch_goal_override_status("test-0-a") == paused
    assert pod_store.fetch_goal_override_status("test-0-c") == paused
    assert pod_store.fetch_goal_override_status("test-0-b") != paused
    assert pod_store.fetch_goal_override_status("test-0-d") != paused
    assert sorted(quiet_killer.killed) == sorted([P0["a"].task_id.value, P0["c"].task_id.value])


def test_pause_with_an_unknown_task_is_404_and_changes_nothing(pod_store, quiet_killer):
    r = pods_router(pod_store).post("/v1/pod/test-0/pause", json.dumps(["a", "test-0-c", "e"]))
    assert r.status == 404
    paused = GoalStateOverride.PAUSED.new_status(OverrideProgress.PENDING)
    assert all(pod_store.fetch_goal_override_status(f"test-0-{c}") != paused for c in "abcd")
    assert quiet_killer.killed == []


def test_pause_rejects_a_malformed_task_list(pod_store):
    assert pods_router(pod_store).post("/v1/pod/test-0/pause", "[not json").status == 400


def test_resume_sets_the_none_override(pod_store):
    r = pods_router(pod_store).post("/v1/pod/test-1/resume")
    assert r.status == 200
    assert pod_store.fetch_goal_override_status("test-1-a") == GoalStateOverride.NONE.new_status(
        OverrideProgress.PENDING)


@pytest.mark.parametrize("action", ["restart", "replace"])
def test_restart_or_replace_unknown_pod(pod_store, quiet_killer, action):
    calls = []
    r = pods_router(pod_store, lambda cs, ss, infos: calls.append(infos)).post(f"/v1/pod/aaa/{action}")
    assert r.status == 404 and calls == [] and quiet_killer.killed == []


@pytest.mark.parametrize("pod,tasks", [("test-0", P0), ("test-1", P1)])
def test_restart_kills_every_task_without_marking_failures(pod_store, quiet_killer, pod, tasks):
    calls = []
    r = pods_router(pod_store, lambda cs, ss, infos: calls.append(infos)).post(f"/v1/pod/{pod}/restart")
    assert r.status == 200 and r.json() == {"pod": pod, "tasks": [t.name for t in tasks.values()]}
    assert sorted(quiet_killer.killed) == sorted(t.task_id.value for t in tasks.values())
    assert calls == []


@pytest.mark.parametrize("pod,tasks", [("test-0", P0), ("test-1", P1)])
def test_replace_marks_the_pod_failed_once_then_kills(pod_store, quiet_killer, pod, tasks):
    calls = []
    router = pods_router(pod_store, lambda cs, ss, infos: calls.append([i.name for i in infos]))
    r = router.post(f"/v1/pod/{pod}/replace")
    assert r.status == 200 and r.json()["tasks"] == [t.name for t in tasks.values()]
    assert calls == [[t.name for t in tasks.values()]]
    assert sorted(quiet_killer.killed) == sorted(t.task_id.value for t in tasks.values())


def test_restart_clears_launch_backoff(pod_store):
    B.set_instance(B.ExponentialBackoff(2.0, 60, 300))
    try:
        name = to_task_name(P1["a"].task_id)
        B.get_instance().add_delay(name)
        assert B.get_instance().get_delay(name) is not None
        pods_router(pod_store).post("/v1/pod/test-1/restart")
        assert B.get_instance().get_delay(name) is None
    finally:
        B.set_instance(None)


def test_default_failure_setter_skips_unlaunched_stub_tasks():
    class Boom:
        def fetch(self, *_):
            raise AssertionError("a stub task must not be resolved to a pod")
    stub = P.TaskInfo(name="test-0-x")
    R.set_pods_permanently_failed(Boom(), StateStore(MemPersister(), repair=False), [stub])


# ---------------------------------------------------------------------------------------
# plans (PlansQueriesTest)


class TStep:
    """A plain step whose state flags are set directly (the reference mocks Step)."""

    def __init__(self, name):
        self._id = uuid.uuid4()
        self.name = name
        self.flags = dict(complete=False, pending=False, running=False, interrupted=False)
        self.calls = []

    def get_id(self):
        return self._id

    def get_name(self):
        return self.name

    def get_display_status(self):
        return "PENDING"

    def get_message(self):
        return ""

    def is_complete(self):
        return self.flags["complete"]

    def is_pending(self):
        return self.flags["pending"]

    def force_complete(self):
        self.calls.append("forceComplete")

    def restart(self):
        self.calls.append("restart")

    def proceed(self):
        self.calls.append("proceed")


class TStrategy:
    def __init__(self):
        self.interrupts = 0

    def get_name(self):
        return "serial"

    def interrupt(self):
        self.interrupts += 1


class TParent:
    def __init__(self, name, children):
        self._id = uuid.uuid4()
        self.name = name
        self.children = children
        self.strategy = TStrategy()
        self.flags = dict(complete=False, pending=False, running=False, interrupted=False, errors=False)
        self.calls = []
        self.parameters = None

    def get_id(self):
        return self._id

    def get_name(self):
        return self.name

    def get_children(self):
        return self.children

    def get_strategy(self):
        return self.strategy

    def get_status(self):
        return Status.COMPLETE if self.flags["complete"] else Status.IN_PROGRESS

    def get_errors(self):
        return ["err"] if self.flags["errors"] else []

    def has_errors(self):
        return self.flags["errors"]

    def is_complete(self):
        return self.flags["complete"]

    def is_pending(self):
        return self.flags["pending"]

    def is_running(self):
        return self.flags["running"]

    def is_interrupted(self):
        return self.flags["interrupted"]

    def proceed(self):
        self.calls.append("proceed")

    def interrupt(self):
        self.calls.append("interrupt")

    def restart(self):
        self.calls.append("restart")

    def force_complete(self):
        self.calls.append("forceComplete")

    def update_parameters(self, params):
        self.parameters = params


class TPlanManager:
    def __init__(self, plan):
        self.plan = plan

    def get_plan(self):
        return self.plan


@pytest.fixture
def plan_env():
    step = TStep("test-step")
    phase = TParent("test-phase", [step])
    plan = TParent("test-plan", [phase])
    router = Router([R.PlansResource([TPlanManager(plan)])])
    return router, plan, phase, step


def _cmd(r, cmd):
    assert r.status == 200, (r.status, r.body)
    assert r.json()["message"].startswith(f"Received cmd: {cmd}")


def test_plans_list(plan_env):
    router, plan, _, _ = plan_env
    assert router.get("/v1/plans").json() == ["test-plan"]


@pytest.mark.parametrize("complete,errors,code", [(True, False, 200), (False, True, 417), (True, True, 417),
                                                  (False, False, 202)])
def test_plan_info_status_code(plan_env, complete, errors, code):
    router, plan, _, _ = plan_env
    plan.flags.update(complete=complete, errors=errors)
    r = router.get("/v1/plans/test-plan")
    assert r.status == code
    assert r.json()["phases"][0]["steps"][0]["name"] == "test-step"


def test_plan_info_unknown(plan_env):
    assert plan_env[0].get("/v1/plans/bad-name").status == 404


def test_continue_plan_and_phase_by_id_or_name(plan_env):
    router, plan, phase, _ = plan_env
    _cmd(router.post("/v1/plans/test-plan/continue"), "continue")
    assert plan.calls == ["proceed"]
    _cmd(router.post(f"/v1/plans/test-plan/continue?phase={phase.get_id()}"), "continue")
    _cmd(router.post("/v1/plans/test-plan/continue?phase=test-phase"), "continue")
    assert phase.calls == ["proceed", "proceed"]


def test_continue_unknown(plan_env):
    router = plan_env[0]
    assert router.post("/v1/plans/bad-name/continue").status == 404
    assert router.post("/v1/plans/test-plan/continue?phase=bad-name").status == 404
    assert router.post("/v1/plans/bad-name/continue?phase=test-phase").status == 404


@pytest.mark.parametrize("flag", ["running", "complete"])
def test_continue_already_running_or_complete_is_208(plan_env, flag):
    router, plan, phase, _ = plan_env
    plan.flags[flag] = phase.flags[flag] = True
    assert router.post("/v1/plans/test-plan/continue").status == 208
    assert router.post("/v1/plans/test-plan/continue?phase=test-phase").status == 208
    assert plan.calls == [] and phase.calls == []


def test_interrupt_plan_and_phase(plan_env):
    router, plan, phase, _ = plan_env
    _cmd(router.post("/v1/plans/test-plan/interrupt"), "interrupt")
    assert plan.calls == ["interrupt"]
    _cmd(router.post(f"/v1/plans/test-plan/interrupt?phase={phase.get_id()}"), "interrupt")
    _cmd(router.post("/v1/plans/test-plan/interrupt?phase=test-phase"), "interrupt")
    assert phase.strategy.interrupts == 2


def test_interrupt_unknown(plan_env):
    router = plan_env[0]
    assert router.post("/v1/plans/bad-name/interrupt").status == 404
    assert router.post("/v1/plans/test-plan/interrupt?phase=bad-name").status == 404


def test_interrupt_already_interrupted_or_complete_is_208(plan_env):
    router, plan, phase, _ = plan_env
    plan.flags["interrupted"] = True
    assert router.post("/v1/plans/test-plan/interrupt").status == 208
    plan.flags["interrupted"], phase.flags["interrupted"] = False, True
    assert router.post("/v1/plans/test-plan/interrupt?phase=test-phase").status == 208
    phase.flags["interrupted"] = False
    plan.flags["complete"] = True
    assert router.post("/v1/plans/test-plan/interrupt").status == 208
    plan.flags["complete"], phase.flags["complete"] = False, True
    assert router.post("/v1/plans/test-plan/interrupt?phase=test-phase").status == 208


def test_force_complete_step_by_id_and_name(plan_env):
    router, _, phase, step = plan_env
    _cmd(router.post(f"/v1/plans/test-plan/forceComplete?phase={phase.get_id()}&step={step.get_id()}"),
         "forceComplete")
    _cmd(router.post("/v1/plans/test-plan/forceComplete?phase=test-phase&step=test-step"), "forceComplete")
    assert step.calls == ["forceComplete", "forceComplete"]


def test_force_complete_unknown_touches_nothing(plan_env):
    router, _, _, step = plan_env
    assert router.post("/v1/plans/bad-name/forceComplete?phase=test-phase&step=test-step").status == 404
    assert router.post(f"/v1/plans/test-plan/forceComplete?phase={uuid.uuid4()}&step={uuid.uuid4()}").status == 404
    assert router.post("/v1/plans/test-plan/forceComplete?phase=bad-phase&step=bad-step").status == 404
    assert step.calls == []


def test_force_complete_already_complete_is_208(plan_env):
    router, _, phase, step = plan_env
    step.flags["complete"] = True
    assert router.post(f"/v1/plans/test-plan/forceComplete?phase={phase.get_id()}&step={step.get_id()}").status \
        == 208


def test_force_complete_plan_or_phase(plan_env):
    router, plan, phase, _ = plan_env
    _cmd(router.post("/v1/plans/test-plan/forceComplete"), "forceComplete")
    _cmd(router.post("/v1/plans/test-plan/forceComplete?phase=test-phase"), "forceComplete")
    assert plan.calls == ["forceComplete"] and phase.calls == ["forceComplete"]


def test_force_complete_argument_errors(plan_env):
    router = plan_env[0]
    assert router.post("/v1/plans/test-plan/forceComplete?step=test-step").status == 400  # step without phase
    assert router.post("/v1/plans/None/forceComplete?step=test-step").status == 404


def test_restart_step_proceeds_then_restarts(plan_env):
    router, _, phase, step = plan_env
    _cmd(router.post(f"/v1/plans/test-plan/restart?phase={phase.get_id()}&step={step.get_id()}"), "restart")
    _cmd(router.post("/v1/plans/test-plan/restart?phase=test-phase&step=test-step"), "restart")
    assert step.calls == ["proceed", "restart", "proceed", "restart"]


def test_restart_unknown_and_pending(plan_env):
    router, _, _, step = plan_env
    assert router.post("/v1/plans/bad-name/restart?phase=test-phase&step=test-step").status == 404
    assert router.post(f"/v1/plans/test-plan/restart?phase={uuid.uuid4()}&step={uuid.uuid4()}").status == 404
    assert router.post("/v1/plans/test-plan/restart?phase=bad-phase&step=bad-step").status == 404
    assert step.calls == []
    step.flags["pending"] = True
    assert router.post("/v1/plans/test-plan/restart?phase=test-phase&step=test-step").status == 208


def test_restart_plan_or_phase(plan_env):
    router, plan, phase, _ = plan_env
    _cmd(router.post("/v1/plans/test-plan/restart"), "restart")
    assert plan.calls == ["proceed", "restart"]
    _cmd(router.post("/v1/plans/test-plan/restart?phase=test-phase"), "restart")
    assert phase.calls == ["proceed", "restart"]
    assert router.post("/v1/plans/test-plan/restart?phase=bad-phase").status == 404
    assert router.post("/v1/plans/bad-plan/restart").status == 404
    assert router.post("/v1/plans/test-plan/restart?step=non-null").status == 400


def test_start_proceeds_and_restarts_only_a_complete_plan(plan_env):
    router, plan, _, _ = plan_env
    r = router.post("/v1/plans/test-plan/start", {"SOME_ENVVAR": "val"})
    assert r.status == 200 and plan.calls == ["proceed"] and plan.parameters == {"SOME_ENVVAR": "val"}
    plan.calls.clear()
    plan.flags["complete"] = True
    assert router.post("/v1/plans/test-plan/start", {}).status == 200
    assert plan.calls == ["restart", "proceed"]


@pytest.mark.parametrize("body", [{"not-an-envvar": "v"}, {"1ABC": "v"}, "[1, 2]", "{bad"])
def test_start_rejects_invalid_parameters(plan_env, body):
    router, plan, _, _ = plan_env
    assert router.post("/v1/plans/test-plan/start", body).status == 400
    assert plan.calls == []


def test_stop_interrupts_and_restarts(plan_env):
    router, plan, _, _ = plan_env
    _cmd(router.post("/v1/plans/test-plan/stop"), "stop")
    assert plan.calls == ["interrupt", "restart"]
    assert router.post("/v1/plans/bad-plan/stop").status == 404


# ---------------------------------------------------------------------------------------
# state (StateQueriesTest)


class FailingFrameworkStore:
    def fetch_framework_id(self):
        raise StateStoreException(Reason.STORAGE_ERROR, "hi")


def state_router(state_store=None, framework_store=None):
    p = MemPersister()
    return Router([R.StateResource(framework_store or FrameworkStore(p), state_store or StateStore(p, repair=False))])


def test_framework_id_present_missing_and_failing():
    p = MemPersister()
    fs = FrameworkStore(p)
    router = Router([R.StateResource(fs, StateStore(p, repair=False))])
    assert router.get("/v1/state/frameworkId").status == 404
    fs.store_framework_id(P.FrameworkID(value="aoeu-asdf"))
    r = router.get("/v1/state/frameworkId")
    assert r.status == 200 and r.json() == ["aoeu-asdf"]
    assert state_router(framework_store=FailingFrameworkStore()).get("/v1/state/frameworkId").status == 500


def test_property_keys_and_values():
    st = StateStore(MemPersister(), repair=False)
    router = state_router(st)
    assert router.get("/v1/state/properties").json() == []
    st.store_property("hi", b"1")
    st.store_property("hey", b"hello this is a property")
    assert sorted(router.get("/v1/state/properties").json()) == ["hey", "hi"]
    r = router.get("/v1/state/properties/hey")
    assert r.status == 200 and r.body == "hello this is a property"  # the deserializer's string, as-is
    assert router.get("/v1/state/properties/missing").status == 404


class FailingProps(StateStore):
    def fetch_property_keys(self):
        raise StateStoreException(Reason.STORAGE_ERROR, "hi")

    def fetch_property(self, key):
        raise StateStoreException(Reason.STORAGE_ERROR, "hi")

    def store_property(self, key, value):
        raise StateStoreException(Reason.STORAGE_ERROR, "Failed to store")


def test_property_storage_failures_are_500():
    router = state_router(FailingProps(MemPersister(), repair=False))
    assert router.get("/v1/state/properties").status == 500
    assert router.get("/v1/state/properties/foo").status == 500
    assert router.put("/v1/state/files/test-file", "test data").status == 500


def test_files_put_get_list_and_limits():
    st = StateStore(MemPersister(), repair=False)
    router = state_router(st)
    assert router.put("/v1/state/files/test-file", "test data").status == 200
    r = router.get("/v1/state/files/test-file")
    assert r.status == 200 and r.body == "test data"
    assert st.fetch_property("file-test-file") == b"test data"
    assert router.get("/v1/state/files").body == "[test-file]"
    assert router.get("/v1/state/files/nope").status == 404
    big = "test data" * (1024 // len("test data") * 100)
    r = router.put("/v1/state/files/test-file", big)
    assert r.status == 400 and r.body == "Stream exceeds 1024 byte size limit"
    boundary = "XyZ"
    body = (f"--{boundary}\r\nContent-Disposition: form-data; name=\"file\"; filename=\"f\"\r\n\r\n"
            f"multi part data\r\n--{boundary}--\r\n")
    r = router.put("/v1/state/files/mp", body, {"Content-Type": f"multipart/form-data; boundary={boundary}"})
    assert r.status == 200 and router.get("/v1/state/files/mp").body == "multi part data"


def _zoned(name, zone):
    t = P.TaskInfo(name=name)
    t.task_id.CopyFrom(to_task_id(SERVICE, name))
    t.agent_id.value = "ignored"
    v = t.command.environment.variables.add()
    v.name, v.value = "ZONE", zone
    return t


def test_task_zones_by_name_and_by_ip():
    st = StateStore(MemPersister(), repair=False)
    t = _zoned("test-task-name", "us-west-2a")
    st.store_tasks([t, _task("plain-task")])
    s = _status(t, P.TASK_UNKNOWN)
    s.container_status.network_infos.add().ip_addresses.add(ip_address="10.0.0.7")
    st.store_status(t.name, s)
    router = state_router(st)
    assert router.get("/v1/state/zone/tasks").json() == {"test-task-name": "us-west-2a"}
    assert router.get("/v1/state/zone/tasks/test-task-name").body == "us-west-2a"
    assert router.get("/v1/state/zone/tasks/plain-task").status == 404
    assert router.get("/v1/state/zone/test/10.0.0.7").body == "us-west-2a"
    assert router.get("/v1/state/zone/test/10.0.0.8").status == 404


class FailingCache(PersisterCache):
    def refresh(self):
        raise PersisterException(Reason.STORAGE_ERROR, "hi")


def test_refresh_needs_a_cache_and_reports_failures():
    cached = StateStore(PersisterCache(MemPersister()), repair=False)
    r = state_router(cached).put("/v1/state/refresh")
    assert r.status == 200 and r.json() == {"message": "Received cmd: refresh"}
    assert state_router(StateStore(MemPersister(), repair=False)).put("/v1/state/refresh").status == 409
    assert state_router(StateStore(FailingCache(MemPersister()), repair=False)).put("/v1/state/refresh").status \
        == 500


# ---------------------------------------------------------------------------------------
# configurations (ConfigQueriesTest)


class StringConfig:
    def __init__(self, s):
        self.s = s

    def to_dict(self):
        return {"value": self.s}


class FakeConfigStore:
    def __init__(self, ids=(), configs=None, target=None, fail=None):
        self.ids = list(ids)
        self.configs = dict(configs or {})
        self.target = target
        self.fail = fail or {}

    def _maybe_fail(self, op):
        if op in self.fail:
            raise ConfigStoreException(self.fail[op], op)

    def list(self):
        self._maybe_fail("list")
        return self.ids

    def fetch(self, cid):
        self._maybe_fail("fetch")
        if cid not in self.configs:
            raise ConfigStoreException(Reason.NOT_FOUND, str(cid))
        return self.configs[cid]

    def get_target_config(self):
        self._maybe_fail("target")
        if self.target is None:
            raise ConfigStoreException(Reason.NOT_FOUND, "no target")
        return self.target


ID1, ID2 = uuid.uuid4(), uuid.uuid4()


def cfg_router(store):
    return Router([R.ConfigResource(store)])


def test_config_ids_and_failure():
    assert cfg_router(FakeConfigStore([ID1, ID2])).get("/v1/configurations").json() == [str(ID1), str(ID2)]
    assert cfg_router(FakeConfigStore(fail={"list": Reason.STORAGE_ERROR})).get("/v1/configurations").status == 500


def test_config_by_id():
    store = FakeConfigStore(configs={ID1: StringConfig("one")})
    router = cfg_router(store)
    r = router.get(f"/v1/configurations/{ID1}")
    assert r.status == 200 and r.json() == {"value": "one"}
    assert router.get("/v1/configurations/hello").status == 400
    assert router.get(f"/v1/configurations/{ID2}").status == 404
    failing = cfg_router(FakeConfigStore(fail={"fetch": Reason.STORAGE_ERROR}))
    assert failing.get(f"/v1/configurations/{ID1}").status == 500


def test_target_id():
    r = cfg_router(FakeConfigStore(target=ID2)).get("/v1/configurations/targetId")
    assert r.status == 200 and r.json() == [str(ID2)]
    assert cfg_router(FakeConfigStore()).get("/v1/configurations/targetId").status == 404
    assert cfg_router(FakeConfigStore(fail={"target": Reason.STORAGE_ERROR})).get(
        "/v1/configurations/targetId").status == 500


def test_target_config():
    r = cfg_router(FakeConfigStore(configs={ID2: StringConfig("one")}, target=ID2)).get("/v1/configurations/target")
    assert r.status == 200 and r.json() == {"value": "one"}
    assert cfg_router(FakeConfigStore()).get("/v1/configurations/target").status == 404
    assert cfg_router(FakeConfigStore(fail={"target": Reason.STORAGE_ERROR})).get(
        "/v1/configurations/target").status == 500
    # the target ID exists but its config does not: data that should be there is missing -> 500
    assert cfg_router(FakeConfigStore(target=ID2)).get("/v1/configurations/target").status == 500
    assert cfg_router(FakeConfigStore(configs={ID2: StringConfig("one")}, target=ID2,
                                      fail={"fetch": Reason.STORAGE_ERROR})).get(
        "/v1/configurations/target").status == 500


# ---------------------------------------------------------------------------------------
# health (HealthResourceTest)


HW_SPEC = """\
name: svc
pods:
  hello:
    count: 1
    tasks:
      hello:
        goal: RUNNING
        cmd: echo hello
        cpus: 1.0
        memory: 1000
  world:
    count: 1
    tasks:
      world:
        goal: RUNNING
        cmd: echo world
        cpus: 1.0
        memory: 1000
"""


@pytest.fixture(scope="module")
def hw_spec():
    raw = RawServiceSpec.from_string(HW_SPEC)
    return mappers.ServiceSpecGenerator(raw, SchedulerConfig.for_testing(), "/tmp", {}).build()


def _steps(spec, store, pod, statuses):
    pi = PodInstance(spec.pod(pod), 0)
    req = PodInstanceRequirement(pi, [pod])
    return [DeploymentStep(f"{pod}-step-{i}", req, store).update_initial_status(s) for i, s in enumerate(statuses)]


def _health(spec, deploy_phases, other_plans=(), registered=True, deploy_interrupted=False, phase_strategy=None):
    p = MemPersister()
    fs = FrameworkStore(p)
    if registered:
        fs.store_framework_id(P.FrameworkID(value="fw-id"))
    store = StateStore(p, repair=False)
    phases = []
    for name, pod, statuses in deploy_phases:
        steps = _steps(spec, store, pod, statuses)
        strategy = phase_strategy(steps) if phase_strategy else SerialStrategy()
        phases.append(DefaultPhase(name, steps, strategy))
    deploy = DefaultPlan("deploy", phases, SerialStrategy())
    pms = [DefaultPlanManager.create_interrupted(deploy) if deploy_interrupted else
           DefaultPlanManager.create_proceeding(deploy)]
    recovery_present = False
    for plan_name, pod, statuses in other_plans:
        recovery_present |= plan_name == "recovery"
        phase = DefaultPhase(f"{plan_name}-phase", _steps(spec, store, pod, statuses), SerialStrategy())
        pms.append(DefaultPlanManager.create_proceeding(DefaultPlan(plan_name, [phase], SerialStrategy())))
    if not recovery_present:
        pms.append(DefaultPlanManager.create_proceeding(DefaultPlan("recovery", [], SerialStrategy())))
    return R.HealthResource(DefaultPlanCoordinator(pms), fs)


C, S_ = Status.COMPLETE, Status


@pytest.mark.parametrize("registered,expected_not", [(False, None), (True, "INITIALIZING")])
def test_health_initializing_until_registered(hw_spec, registered, expected_not):
    res = _health(hw_spec, [("hello-deploy", "hello", [S_.PENDING]),
                            ("world-deploy", "world", [S_.PENDING, S_.PENDING])], registered=registered)
    code, _ = res.evaluate()
    if expected_not is None:
        assert code == "INITIALIZING"
    else:
        assert code != expected_not


def test_health_error_creating_service(hw_spec):
    p = MemPersister()
    fs = FrameworkStore(p)
    fs.store_framework_id(P.FrameworkID(value="fw-id"))
    store = StateStore(p, repair=False)
    hello = _steps(hw_spec, store, "hello", [S_.ERROR])[0]
    hello.add_error("Added test error.")
    deploy = DefaultPlan("deploy", [DefaultPhase("hello-deploy", [hello], SerialStrategy()),
                                    DefaultPhase("world-deploy", _steps(hw_spec, store, "world", [S_.PENDING] * 2),
                                                 SerialStrategy())], SerialStrategy())
    coord = DefaultPlanCoordinator([DefaultPlanManager.create_proceeding(deploy),
                                    DefaultPlanManager.create_proceeding(DefaultPlan("recovery", [], SerialStrategy()))])
    code, body = R.HealthResource(coord, fs).evaluate(verbose=True)
    assert code == "ERROR_CREATING_SERVICE" and body["value"] == 500
    assert any("Status Code 500 is TRUE" in reason for reason in body["reasons"])


@pytest.mark.parametrize("hello,world,expected", [
    ([S_.PREPARED, S_.PENDING], [S_.STARTING] * 3, "DEPLOYING_PENDING"),   # pessimistic: pending wins
    ([S_.STARTING, S_.STARTED], [C] * 3, "DEPLOYING_STARTING"),
    ([C, C], [C] * 3, "RUNNING"),
])
def test_health_deploy_states(hw_spec, hello, world, expected):
    res = _health(hw_spec, [("hello-deploy", "hello", hello), ("world-deploy", "world", world)])
    code, body = res.evaluate()
    assert code == expected and body["value"] == R.SERVICE_STATUS[expected][0]
    assert res.health().status == R.SERVICE_STATUS[expected][0]


@pytest.mark.parametrize("plans,expected", [
    ([("recovery", "world", [S_.PREPARED, S_.PENDING, S_.STARTED])], "RECOVERING_PENDING"),
    ([("recovery", "world", [S_.STARTING, C, C])], "RECOVERING_STARTING"),
    ([("backup-s3", "world", [S_.PENDING, S_.STARTED, C])], "BACKING_UP"),
    ([("restore-s3", "world", [S_.PENDING, S_.STARTED, C])], "RESTORING"),
    # recovery outranks a running restore
    ([("recovery", "world", [S_.STARTING, C, C]), ("restore-s3", "world", [S_.PENDING, S_.STARTED, C])],
     "RECOVERING_STARTING"),
])
def test_health_recovery_backup_restore(hw_spec, plans, expected):
    res = _health(hw_spec, [("hello-deploy", "hello", [C, C]), ("world-deploy", "world", [C, C, C])], plans)
    assert res.evaluate()[0] == expected


@pytest.mark.parametrize("post", [SerialStrategy, ParallelStrategy])
def test_health_canary_waiting_for_the_user(hw_spec, post):
    res = _health(hw_spec, [("hello-deploy", "hello", [C, C, C, C, S_.WAITING]),
                            ("world-deploy", "world", [C, C, C])],
                  deploy_interrupted=True, phase_strategy=lambda steps: CanaryStrategy(post(), steps))
    code, body = res.evaluate(verbose=True)
    assert code == "DEPLOYING_WAITING_USER" and body["value"] == 207
    assert len(body["reasons"]) == 10


def test_health_verbose_lists_every_check(hw_spec):
    res = _health(hw_spec, [("hello-deploy", "hello", [C]), ("world-deploy", "world", [C])])
    r = Router([res]).get("/v1/health?verbose=true")
    assert r.status == 200 and r.json()["value"] == 200
    assert [x.split(".")[0] for x in r.json()["reasons"]] == [
        "Priority 1", "Priority 1", "Priority 2", "Priority 1", "Priority 2", "Priority 3", "Priority 4",
        "Priority 5", "Priority 5", "Priority 6"]
    assert "reasons" not in Router([res]).get("/v1/health").json()


# ---------------------------------------------------------------------------------------
# artifacts (ArtifactQueriesTest) and endpoints (EndpointsQueriesTest)


ART_SPEC = """\
name: svc
pods:
  pod:
    count: 1
    tasks:
      task:
        goal: RUNNING
        cmd: ./run
        cpus: 0.1
        memory: 32
        configs:
          conf:
            template: tmpl.mustache
            dest: conf.out
"""


def test_artifact_template_lookup(tmp_path):
    (tmp_path / "tmpl.mustache").write_text("hello {{WHO}}")
    raw = RawServiceSpec.from_string(ART_SPEC)
    spec = mappers.ServiceSpecGenerator(raw, SchedulerConfig.for_testing(), str(tmp_path), {}).build()
    store = FakeConfigStore(configs={ID1: spec})
    router = Router([R.ArtifactResource(store)])
    r = router.get(f"/v1/artifacts/template/{ID1}/pod/task/conf")
    assert r.status == 200 and r.body == "hello {{WHO}}"
    assert router.get("/v1/artifacts/template/not-a-uuid/pod/task/conf").status == 400
    assert router.get(f"/v1/artifacts/template/{ID2}/pod/task/conf").status == 404
    for bad in ("nope/task/conf", "pod/nope/conf", "pod/task/nope"):
        assert router.get(f"/v1/artifacts/template/{ID1}/{bad}").status == 404
    failing = Router([R.ArtifactResource(FakeConfigStore(fail={"fetch": Reason.STORAGE_ERROR}))])
    assert failing.get(f"/v1/artifacts/template/{ID1}/pod/task/conf").status == 500


def _discovered(name, host, ports, ips=(), vip=None):
    t = P.TaskInfo(name=name)
    t.task_id.CopyFrom(to_task_id(SERVICE, name))
    t.agent_id.value = "a"
    w = TaskLabelWriter(t)
    w.set_type("pod")
    w.set_index(0)
    off = P.Offer(hostname=host)
    w.set_hostname(off)
    w.apply()
    t.discovery.visibility = P.DiscoveryInfo.FRAMEWORK
    t.discovery.name = name
    for pname, num in ports:
        p = t.discovery.ports.ports.add(name=pname, number=num, protocol="tcp")
        p.visibility = P.DiscoveryInfo.EXTERNAL
        if vip:
            lab = p.labels.labels.add()
            lab.key, lab.value = "VIP_" + str(uuid.uuid4()), vip
    st = _status(t, P.TASK_RUNNING)
    for ip in ips:
        st.container_status.network_infos.add().ip_addresses.add(ip_address=ip)
    return t, st


def test_endpoints_list_and_detail():
    store = StateStore(MemPersister(), repair=False)
    t1, s1 = _discovered("pod-0-task", "host-1", [("http", 8080)], vip="web:80")
    t2, s2 = _discovered("pod-1-task", "host-2", [("http", 8081)], ips=["10.0.0.2"])
    store.store_tasks([t1, t2])
    store.store_status(t1.name, s1)
    store.store_status(t2.name, s2)
    res = R.EndpointsResource(store, SERVICE, SchedulerConfig.for_testing(), {"custom": lambda: "custom-value"})
    router = Router([res])
    assert router.get("/v1/endpoints").json() == ["custom", "http"]
    e = router.get("/v1/endpoints/http").json()
    assert e["address"] == ["host-1:8080", "10.0.0.2:8081"]
    assert e["dns"] == [f"pod-0-task.{SERVICE}.autoip.dcos.thisdcos.directory:8080",
                        f"pod-1-task.{SERVICE}.autoip.dcos.thisdcos.directory:8081"]
    assert e["vip"] == f"web.{SERVICE}.l4lb.thisdcos.directory:80"
    r = router.get("/v1/endpoints/custom")
    assert r.status == 200 and r.body == "custom-value"
    assert router.get("/v1/endpoints/nope").status == 404
