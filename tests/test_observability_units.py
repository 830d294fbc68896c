"""Metrics, debug trackers, offer history and HTTP helper units.

Mirrors sdk/scheduler/src/test/java/com/mesosphere/sdk/metrics/{MetricsTest,PlanReporterTest}.java,
debug/{OfferOutcomeTrackerV2Test,PlansTrackerTest,TaskStatusesTrackerTest,
TaskReservationsTrackerTest}.java, offer/history/OfferOutcomeTrackerTest.java and
http/{EndpointUtilsTest,RequestUtilsTest,ResponseUtilsTest}.java, http/types/PlanInfoTest.java.
"""
import io
import json
import textwrap
import time
import types

import pytest

import testutils as U
from dcos_commons_amd import metrics as M
from dcos_commons_amd.debug import PlansTracker, TaskReservationsTracker, TaskStatusesTracker
from dcos_commons_amd.http import endpoint_utils as E
from dcos_commons_amd.http.api import json_ok, read_data, to_json_text
from dcos_commons_amd.http.resources import plan_info
from dcos_commons_amd.mesos import protos as P
from dcos_commons_amd.offer.history import OfferOutcome, OfferOutcomeTracker, OfferOutcomeTrackerV2
from dcos_commons_amd.offer.recommendations import LaunchOfferRecommendation, StoreTaskInfoRecommendation
from dcos_commons_amd.offer.taskdata.labels import TaskLabelWriter
from dcos_commons_amd.scheduler.plan.deployment_step import DeploymentStep
from dcos_commons_amd.scheduler.plan.elements import DefaultPhase, DefaultPlan
from dcos_commons_amd.scheduler.plan.managers import DefaultPlanCoordinator, DefaultPlanManager
from dcos_commons_amd.scheduler.plan.pod_instance_requirement import PodInstanceRequirement
from dcos_commons_amd.scheduler.plan.status import Status
from dcos_commons_amd.scheduler.plan.strategy import SerialStrategy
from dcos_commons_amd.scheduler.scheduler_config import SchedulerConfig
from dcos_commons_amd.specification.specs import PodInstance
from dcos_commons_amd.specification.yaml import mappers
from dcos_commons_amd.specification.yaml.raw import RawServiceSpec
from dcos_commons_amd.state.framework_store import FrameworkStore
from dcos_commons_amd.state.state_store import StateStore
from dcos_commons_amd.storage.mem_persister import MemPersister

CFG = SchedulerConfig.for_testing()


# ---------------------------------------------------------------------------------------
# Metrics


@pytest.mark.parametrize("fn,name,n", [
    (M.increment_received_offers, M.RECEIVED_OFFERS, 5),
    (M.increment_processed_offers, M.PROCESSED_OFFERS, 5),
    (M.increment_declines_short, M.DECLINE_SHORT, 5),
    (M.increment_declines_long, M.DECLINE_LONG, 5),
])
def test_counted_increments(fn, name, n):
    before = M.REGISTRY.counter(name)
    fn(n)
    assert M.REGISTRY.counter(name) - before == n


@pytest.mark.parametrize("fn,name", [(M.increment_revives, M.REVIVES),
                                     (M.increment_revive_throttles, M.REVIVE_THROTTLES)])
def test_single_increments(fn, name):
    before = M.REGISTRY.counter(name)
    fn()
    assert M.REGISTRY.counter(name) - before == 1


def test_process_offers_timer():
    before = M.REGISTRY.timer(M.PROCESS_OFFERS).count
    M.process_offers_timer().stop()
    assert M.REGISTRY.timer(M.PROCESS_OFFERS).count - before == 1


def test_suppression_gauge():
    M.increment_suppresses()
    assert M.REGISTRY.to_json()["gauges"][M.IS_SUPPRESSED]["value"] is True
    M.not_suppressed()
    assert M.REGISTRY.to_json()["gauges"][M.IS_SUPPRESSED]["value"] is False


def test_task_statuses():
    for state, name in ((P.TASK_RUNNING, "task_status.task_running"), (P.TASK_LOST, "task_status.task_lost")):
        before = M.REGISTRY.counter(name)
        M.record_status(P.TaskStatus(state=state, task_id=U.TASK_ID))
        assert M.REGISTRY.counter(name) - before == 1


def _task_info():
    t = P.TaskInfo(name=U.TASK_NAME)
    t.task_id.CopyFrom(U.TASK_ID)
    t.agent_id.CopyFrom(U.AGENT_ID)
    return t


def _executor():
    e = P.ExecutorInfo()
    e.executor_id.value = "executor"
    return e


def test_launches_are_counted_by_operation():
    rec = LaunchOfferRecommendation(U.empty_offer(), _task_info(), _executor())
    before = M.REGISTRY.counter("operation.launch_group")
    M.increment_recommendations([rec, rec, rec])
    assert M.REGISTRY.counter("operation.launch_group") - before == 3


def test_task_info_updates_are_not_counted():
    rec = StoreTaskInfoRecommendation(U.empty_offer(), _task_info(), _executor())
    before = dict(M.REGISTRY.counters)
    M.increment_recommendations([rec, rec, rec])
    assert M.REGISTRY.counters == before


@pytest.mark.parametrize("status,value", [
    (Status.ERROR, -1), (Status.COMPLETE, 0), (Status.WAITING, 1), (Status.PENDING, 1), (Status.PREPARED, 2),
    (Status.IN_PROGRESS, 2), (Status.STARTED, 2), (Status.STARTING, 2),
])
def test_plan_gauge_values(status, value):
    M.update_plan_status(None, "gauge-values", status)
    assert M.REGISTRY.to_json()["gauges"]["plan_status.gauge-values"]["value"] == value


@pytest.mark.parametrize("namespace,name", [(None, "plan_status.nonamespace"),
                                            ("namespace", "plan_status.namespace.nonamespace")])
def test_plan_status_gauge_is_created_then_updated(namespace, name):
    M.REGISTRY.gauges.pop(name, None)
    M.update_plan_status(namespace, "nonamespace", Status.ERROR)
    assert M.REGISTRY.to_json()["gauges"][name]["value"] == -1
    M.update_plan_status(namespace, "nonamespace", Status.IN_PROGRESS)
    assert M.REGISTRY.to_json()["gauges"][name]["value"] == 2


def test_prometheus_export_names():
    M.increment_received_offers(1)
    text = M.REGISTRY.to_prometheus()
    assert "# TYPE offers_received counter" in text and "offers_process_count" in text


class _StubPlan:
    def __init__(self, name, status):
        self.name, self.status = name, status

    def get_name(self):
        return self.name

    def get_status(self):
        return self.status


def test_plan_reporter_scrapes_every_manager():
    managers = [types.SimpleNamespace(get_plan=lambda: _StubPlan("plan1", Status.ERROR)),
                types.SimpleNamespace(get_plan=lambda: _StubPlan("plan2", Status.COMPLETE))]
    reporter = M.PlanReporter(None, managers, period_s=0.01)
    deadline = time.time() + 5
    while not reporter.has_scraped and time.time() < deadline:
        time.sleep(0.005)
    reporter.stop()
    gauges = M.REGISTRY.to_json()["gauges"]
    assert gauges["plan_status.plan1"]["value"] == -1 and gauges["plan_status.plan2"]["value"] == 0


# ---------------------------------------------------------------------------------------
# Offer outcome history (v1 ring, v2 summary)


def _outcome(passed):
    return OfferOutcome("instance-name", passed, P.Offer(), "an outcome")


def _outcomes(tracker):
    out = tracker.to_json()["outcomes"]
    for o in out:
        assert all(o.get(k) is not None for k in ("timestamp", "pod-instance-name", "outcome", "explanation",
                                                   "offer"))
    return [o["outcome"] for o in out]


def test_outcomes_newest_first():
    t = OfferOutcomeTracker()
    for passed in (True, False, True, False, False):
        t.track(_outcome(passed))
    assert _outcomes(t) == ["fail", "fail", "pass", "fail", "pass"]


def test_outcomes_evicted_at_capacity():
    t = OfferOutcomeTracker(2)
    t.track(_outcome(True))
    t.track(_outcome(False))
    assert _outcomes(t) == ["fail", "pass"]
    t.track(_outcome(True))
    assert _outcomes(t) == ["pass", "fail"]


def test_outcome_html_escapes():
    t = OfferOutcomeTracker()
    t.track(OfferOutcome("<pod>", False, P.Offer(), "a < b\nsecond line"))
    page = t.to_html()
    assert "&lt;pod&gt;" in page and "a &lt; b" in page and "<td>FAIL</td>" in page


def test_outcome_details_render_lazily():
    calls = []
    o = OfferOutcome("p", True, P.Offer(), lambda: calls.append(1) or "rendered")
    assert calls == []
    assert o.details == "rendered" and o.details == "rendered" and calls == [1]


def test_v2_summary_counts_agents_and_reasons():
    t = OfferOutcomeTrackerV2()
    for passed in (True, False, True, False, False):
        t.summary.add_offer(_outcome(passed))
    for agent in ("foo", "foo", "bar"):
        t.summary.add_failure_agent(agent)
    for reason in ("insufficientCpu", "insufficientCpu", "insufficientMem"):
        t.summary.add_failure_reason(reason)
    j = t.to_json()
    assert (j["acceptedCount"], j["rejectedCount"]) == (2, 3)
    assert j["rejectedAgents"] == {"foo": 2, "bar": 1}
    assert j["failureReasons"] == {"insufficientCpu": 2, "insufficientMem": 1}


# ---------------------------------------------------------------------------------------
# Debug trackers


def _pod(name):
    text = f"""\
        name: helloworld
        scheduler:
          principal: {U.PRINCIPAL}
        pods:
          {name}:
            count: 1
            tasks:
              {name}:
                goal: RUNNING
                cmd: echo {name}
                cpus: 1.0
                memory: 1000
        """
    return mappers.ServiceSpecGenerator(RawServiceSpec.from_string(textwrap.dedent(text)), CFG, "/tmp", {}) \
        .build().pods[0]


@pytest.fixture
def deploy():
    persister = MemPersister()
    FrameworkStore(persister).store_framework_id(U.FRAMEWORK_ID)
    store = StateStore(persister)
    hello = PodInstanceRequirement(PodInstance(_pod("hello"), 0), ["hello"])
    world = PodInstanceRequirement(PodInstance(_pod("world"), 0), ["world"])
    steps = [DeploymentStep("hello-step", hello, store).update_initial_status(Status.COMPLETE),
             DeploymentStep("world-step-1", world, store).update_initial_status(Status.IN_PROGRESS),
             DeploymentStep("world-step-2", world, store).update_initial_status(Status.PENDING)]
    plan = DefaultPlan("deploy", [DefaultPhase("hello-deploy", steps[:1], SerialStrategy()),
                                  DefaultPhase("world-deploy", steps[1:], SerialStrategy())], SerialStrategy())
    coordinator = DefaultPlanCoordinator([DefaultPlanManager.create_proceeding(plan)])
    return coordinator, store


TOPOLOGY = [{"name": "deploy", "type": "plan", "children": [
    {"name": "hello-deploy", "type": "phase", "children": [{"name": "hello-step", "type": "step", "children": None}]},
    {"name": "world-deploy", "type": "phase", "children": [
        {"name": "world-step-1", "type": "step", "children": None},
        {"name": "world-step-2", "type": "step", "children": None}]}]}]


def test_plans_tracker_unfiltered(deploy):
    j = PlansTracker(*deploy).get_json()
    assert j["schedulerState"] == "DEPLOYING" and j["activePlans"] == ["deploy"]
    plan, = j["plans"]
    assert (plan["name"], plan["strategy"], plan["status"]) == ("deploy", "serial", "IN_PROGRESS")
    assert (plan["totalSteps"], plan["completedSteps"]) == (3, 1)
    assert [(p["name"], p["strategy"], p["status"]) for p in plan["phases"]] == [
        ("hello-deploy", "serial", "COMPLETE"), ("world-deploy", "serial", "IN_PROGRESS")]
    assert [[(s["name"], s["status"], s["errors"]) for s in p["steps"]] for p in plan["phases"]] == [
        [("hello-step", "COMPLETE", [])],
        [("world-step-1", "IN_PROGRESS", []), ("world-step-2", "PENDING", [])]]
    assert j["serviceTopology"] == TOPOLOGY


def test_plans_tracker_filtered(deploy):
    tracker = PlansTracker(*deploy)
    assert "invalid-input" in tracker.get_json("invalid-plan-name")
    assert "invalid-input" in tracker.get_json("deploy", "invalid-phase-name")
    assert "invalid-input" in tracker.get_json("deploy", "hello-deploy", "invalid-step-name")
    assert "invalid-input" in tracker.get_json(None, None, "hello-step")  # step without its parents
    j = tracker.get_json("deploy", "hello-deploy", "hello-step")
    assert j["schedulerState"] == "DEPLOYING" and j["activePlans"] == ["deploy"]
    plan, = j["plans"]
    assert (plan["totalSteps"], plan["completedSteps"]) == (3, 1)  # roll-ups ignore the filter
    phase, = plan["phases"]
    assert phase["name"] == "hello-deploy" and [s["name"] for s in phase["steps"]] == ["hello-step"]
    assert j["serviceTopology"] == TOPOLOGY  # the topology is always complete


def test_task_statuses_tracker(deploy):
    coordinator, store = deploy
    for pod, state in (("hello", P.TASK_FINISHED), ("world", P.TASK_RUNNING)):
        info = P.TaskInfo(name=f"{pod}-0-{pod}")
        info.task_id.CopyFrom(U.to_task_id("helloworld", info.name))
        info.agent_id.value = "proto-field-required"
        store.store_tasks([info])
        store.store_status(info.name, P.TaskStatus(task_id=info.task_id, state=state))
    j = TaskStatusesTracker(coordinator, store).get_json()
    plan, = j
    assert plan["name"] == "deploy" and [p["name"] for p in plan["phases"]] == ["hello-deploy", "world-deploy"]
    hello, world = plan["phases"]
    assert [s["name"] for s in hello["steps"]] == ["hello-step"]
    assert [s["name"] for s in world["steps"]] == ["world-step-1", "world-step-2"]
    assert hello["steps"][0]["taskStatus"][0]["taskStatus"] == "TASK_FINISHED"
    assert world["steps"][0]["taskStatus"][0]["taskStatus"] == "TASK_RUNNING"
    assert TaskStatusesTracker(coordinator, store).get_json("deploy", "world-deploy", "world-step-2")[0][
        "phases"][0]["steps"][0]["name"] == "world-step-2"


def _task_on(name, host, resources):
    t = U.get_task_info(list(resources), name=name)
    TaskLabelWriter(t).set_hostname(P.Offer(hostname=host)).apply()
    return t


def test_task_reservations_tracker():
    store = StateStore(MemPersister())
    store.store_tasks([
        _task_on("Task_A", "host-1", [U.reserved_ports(123, 234, "resource-1"), U.reserved_cpus(1.0, "resource-3"),
                                      U.reserved_cpus(2.0, "resource-5")]),
        _task_on("Task_B", "host-2", [U.reserved_root_volume(999.0, "resource-2", "resource-2"),
                                      U.reserved_cpus(1.0, "resource-4"), U.reserved_cpus(3.0, "resource-6")]),
        _task_on("Task_C", "host-2", [U.reserved_cpus(4.0, "resource-7"), U.reserved_ports(456, 456, "resource-8")]),
    ])
    j = TaskReservationsTracker(store).get_json()
    assert j == {"host-1": ["resource-1", "resource-3", "resource-5"],
                 "host-2": ["resource-2", "resource-4", "resource-6", "resource-7", "resource-8"]}


# ---------------------------------------------------------------------------------------
# EndpointUtils


CONFIG = types.SimpleNamespace(api_server_port=lambda: 1234, autoip_tld=lambda: "autoip.tld",
                               vip_tld=lambda: "vip.tld", marathon_name=lambda: "test-marathon")


def test_to_endpoint():
    assert E.to_endpoint("foo", 5) == "foo:5"


@pytest.mark.parametrize("svc,expected", [
    ("svc", "task.svc.autoip.tld:5"), ("/path/to/svc", "task.pathtosvc.autoip.tld:5"),
    ("path/to/svc", "task.pathtosvc.autoip.tld:5"), ("path/to/svc.with.dots", "task.pathtosvc-with-dots.autoip.tld:5"),
])
def test_auto_ip_endpoint(svc, expected):
    assert E.to_auto_ip_endpoint(svc, "task", 5, CONFIG) == expected


@pytest.mark.parametrize("vip", ["vip", "/vip"])
@pytest.mark.parametrize("svc,expected", [
    ("svc", "vip.svc.vip.tld:5"), ("/path/to/svc", "vip.pathtosvc.vip.tld:5"),
    ("path/to/svc", "vip.pathtosvc.vip.tld:5"), ("path/to/svc.with.dots", "vip.pathtosvc.with.dots.vip.tld:5"),
])
def test_vip_endpoint(vip, svc, expected):
    assert E.to_vip_endpoint(svc, CONFIG, vip, 5) == expected


@pytest.mark.parametrize("svc,expected", [
    ("svc", "svc.test-marathon.autoip.tld"), ("/svc", "svc.test-marathon.autoip.tld"),
    ("path/to/svc", "svc-to-path.test-marathon.autoip.tld"), ("/path/to/svc", "svc-to-path.test-marathon.autoip.tld"),
    ("path/to/svc.with.dots", "svc-with-dots-to-path.test-marathon.autoip.tld"),
    ("/path/to/svc.with.dots", "svc-with-dots-to-path.test-marathon.autoip.tld"),
])
def test_scheduler_auto_ip(svc, expected):
    assert E.to_scheduler_auto_ip_hostname(svc, CONFIG) == expected
    assert E.to_scheduler_auto_ip_endpoint(svc, CONFIG) == expected + ":1234"


# ---------------------------------------------------------------------------------------
# RequestUtils.readData


LIMIT = 8
EXCEED, MATCH, UNDER = b"123456789", b"12345678", b"1234567"


class UntouchableStream:
    def read(self, *a):
        raise AssertionError("the stream must not be read")


def test_read_null_stream():
    with pytest.raises(ValueError, match="Missing payload"):
        read_data(None, None, LIMIT)


@pytest.mark.parametrize("limit", [0, -1])
@pytest.mark.parametrize("data", [EXCEED, MATCH])
def test_read_without_a_limit(limit, data):
    assert read_data(io.BytesIO(data), len(data), limit) == data


def test_declared_size_over_the_limit_fails_before_reading():
    with pytest.raises(ValueError, match="Stream exceeds 8 byte size limit"):
        read_data(UntouchableStream(), len(EXCEED), LIMIT)


@pytest.mark.parametrize("declared", [len(MATCH), None])
def test_stream_over_the_limit_fails_whatever_was_declared(declared):
    with pytest.raises(ValueError):
        read_data(io.BytesIO(EXCEED), declared, LIMIT)


@pytest.mark.parametrize("data", [MATCH, UNDER])
@pytest.mark.parametrize("declared_delta", [0, -1, None, "neg"])
def test_streams_within_the_limit_pass(data, declared_delta):
    declared = None if declared_delta is None else (-1 if declared_delta == "neg" else len(data) + declared_delta)
    assert read_data(io.BytesIO(data), declared, LIMIT) == data


# ---------------------------------------------------------------------------------------
# ResponseUtils (org.json layout)


@pytest.mark.parametrize("value,text", [
    ([], "[]"), (["hello"], '["hello"]'), (["hello", "hi"], '[\n  "hello",\n  "hi"\n]'),
    ({}, "{}"), ({"hello": "hi"}, '{"hello": "hi"}'),
    ({"hello": "hi", "hey": ["hello"]}, '{\n  "hello": "hi",\n  "hey": ["hello"]\n}'),
    ({"hello": "hi", "hey": ["hello", "hey"]}, '{\n  "hello": "hi",\n  "hey": [\n    "hello",\n    "hey"\n  ]\n}'),
])
def test_json_layout(value, text):
    assert to_json_text(value) == text
    r = json_ok(value)
    assert r.status == 200 and r.payload().decode() == text
    assert json.loads(text) == value


# ---------------------------------------------------------------------------------------
# PlanInfo


class _Step:
    def __init__(self, name, display, message):
        import uuid

        self.id, self.name, self.display, self.message = uuid.uuid4(), name, display, message

    def get_id(self):
        return self.id

    def get_name(self):
        return self.name

    def get_display_status(self):
        return self.display

    def get_message(self):
        return self.message


def test_plan_info_layout():
    steps = [_Step("step-0", "PENDING", "hi"), _Step("step-1", "ERROR", "hey")]
    phase0 = types.SimpleNamespace(get_id=lambda: "p0", get_name=lambda: "phase-0", get_status=lambda: Status.PENDING,
                                   get_strategy=SerialStrategy, get_children=lambda: steps)
    phase1 = types.SimpleNamespace(get_id=lambda: "p1", get_name=lambda: "phase-1",
                                   get_status=lambda: Status.COMPLETE, get_strategy=SerialStrategy,
                                   get_children=lambda: [])
    plan = types.SimpleNamespace(get_children=lambda: [phase0, phase1], get_errors=lambda: ["err0", "err1"],
                                 get_status=lambda: Status.WAITING, get_strategy=SerialStrategy)
    info = plan_info(plan)
    assert info["errors"] == ["err0", "err1"] and info["status"] == "WAITING" and info["strategy"] == "serial"
    p0, p1 = info["phases"]
    assert (p0["id"], p0["name"], p0["status"], len(p0["steps"])) == ("p0", "phase-0", "PENDING", 2)
    assert [(s["id"], s["name"], s["message"], s["status"]) for s in p0["steps"]] == [
        (str(steps[0].id), "step-0", "hi", "PENDING"), (str(steps[1].id), "step-1", "hey", "ERROR")]
    assert (p1["id"], p1["name"], p1["status"], p1["steps"]) == ("p1", "phase-1", "COMPLETE", [])


def test_plan_status_is_read_before_its_phases():
    """A phase that completes while the view is built shows COMPLETE under an IN_PROGRESS plan."""
    state = {"done": False}
    phase = types.SimpleNamespace(get_id=lambda: "p", get_name=lambda: "phase-0",
                                  get_status=lambda: Status.COMPLETE if state["done"] else Status.IN_PROGRESS,
                                  get_strategy=SerialStrategy, get_children=lambda: [])

    def plan_status():
        s = phase.get_status()
        state["done"] = True  # the phase finishes right after the plan's status was taken
        return s

    plan = types.SimpleNamespace(get_children=lambda: [phase], get_errors=lambda: [], get_status=plan_status,
                                 get_strategy=SerialStrategy)
    info = plan_info(plan)
    assert info["status"] == "IN_PROGRESS" and info["phases"][0]["status"] == "COMPLETE"
