"""Plan engine units: plan managers, strategies, phases, the plan scheduler, the step factory and
the plan coordinator.

Mirrors the reference's scheduler/plan suites (sdk/scheduler/src/test/java/com/mesosphere/sdk/
scheduler/plan/{DefaultPlanManagerTest,DefaultPhaseTest,PlanSchedulerTest,DefaultStepFactoryTest,
DefaultPlanCoordinatorTest,RandomRecoveryStrategyTest}.java and strategy/{SerialStrategyTest,
ParallelStrategyTest,CanaryStrategyTest}.java): phase/plan status roll-up from steps, interrupt
and proceed, dirty assets of interrupted plans, canary proceeds (serial, parallel, 3-step,
interrupts ignored while canarying, completed steps skipped, dirty canary steps held back), the
step factory's initial status from stored tasks (readiness, FINISH/ONCE goals) and its
resource-set / DNS-prefix validation, and the coordinator keeping two plans off one pod.
"""
import textwrap
import uuid

import pytest

import testutils as U
from dcos_commons_amd.framework import driver, task_killer
from dcos_commons_amd.http.endpoint_utils import template_url_factory
from dcos_commons_amd.mesos import protos as P
from dcos_commons_amd.offer.common_id_utils import to_task_id
from dcos_commons_amd.offer.evaluate.offer_evaluator import OfferEvaluator
from dcos_commons_amd.offer.taskdata.labels import TaskLabelWriter
from dcos_commons_amd.scheduler.plan.elements import AbstractStep, DefaultPhase, DefaultPlan
from dcos_commons_amd.scheduler.plan.factories import DefaultPhaseFactory, DefaultStepFactory, DeployPlanFactory
from dcos_commons_amd.scheduler.plan.managers import DefaultPlanCoordinator, DefaultPlanManager
from dcos_commons_amd.scheduler.plan.plan_scheduler import PlanScheduler
from dcos_commons_amd.scheduler.plan.pod_instance_requirement import PodInstanceRequirement
from dcos_commons_amd.scheduler.plan.status import Status
from dcos_commons_amd.scheduler.plan.strategy import CanaryStrategy, ParallelStrategy, RandomStrategy, SerialStrategy
from dcos_commons_amd.scheduler.scheduler_config import SchedulerConfig
from dcos_commons_amd.specification.specs import GoalState, PodInstance, loopback_check
from dcos_commons_amd.specification.yaml import mappers
from dcos_commons_amd.specification.yaml.raw import RawServiceSpec
from dcos_commons_amd.state.config_store import ConfigStore
from dcos_commons_amd.state.framework_store import FrameworkStore
from dcos_commons_amd.state.state_store import StateStore
from dcos_commons_amd.storage.mem_persister import MemPersister
from dcos_commons_amd.testing.harness import RecordingDriver

CFG = SchedulerConfig.for_testing()


class TestStep(AbstractStep):
    """scheduler/plan/TestStep.java: start() prepares; an offer outcome prepares or starts."""

    __test__ = False

    def __init__(self, name="test-step", req=None):
        super().__init__(name)
        self.req = req
        self.recommendations = None
        self.updates = []
        self.parameters = []

    def start(self):
        self.set_status(Status.PREPARED)

    def get_pod_instance_requirement(self):
        return self.req

    def update_offer_status(self, recommendations):
        self.recommendations = list(recommendations)
        self.set_status(Status.STARTING if recommendations else Status.PREPARED)

    def update(self, status):
        self.updates.append(status)

    def update_parameters(self, parameters):
        self.parameters.append(dict(parameters))

    def restart(self):
        self.set_status(Status.PENDING)

    def force_complete(self):
        self.set_status(Status.COMPLETE)


def _spec(pods_yaml, name=U.SERVICE_NAME):
    text = f"name: {name}\nscheduler:\n  principal: {U.PRINCIPAL}\npods:\n" + textwrap.indent(
        textwrap.dedent(pods_yaml), "  ")
    return mappers.ServiceSpecGenerator(RawServiceSpec.from_string(text), CFG, "/tmp", {}).build()


def _pod(type_="pod-type", count=1, tasks=("task0",), goal="RUNNING", resource_set=None, dns=None,
         cpus=1.0, mem=1000.0, disk=1500.0):
    """TestPodFactory: each task has cpus/mem and a ROOT volume (its own resource set unless one is
    named), optionally a DNS prefix."""
    body = f"{type_}:\n  count: {count}\n"
    if resource_set is not None:
        body += (f"  resource-sets:\n    {resource_set}:\n      cpus: {cpus}\n      memory: {mem}\n"
                 f"      volume:\n        path: {U.CONTAINER_PATH}\n        type: ROOT\n        size: {int(disk)}\n")
    body += "  tasks:\n"
    for t in tasks:
        body += f"    {t}:\n      goal: {goal}\n      cmd: echo {t}\n"
        if resource_set is not None:
            body += f"      resource-set: {resource_set}\n"
        else:
            body += (f"      cpus: {cpus}\n      memory: {mem}\n      volume:\n        path: {U.CONTAINER_PATH}\n"
                     f"        type: ROOT\n        size: {int(disk)}\n")
        if dns is not None:
            body += f"      discovery:\n        prefix: {dns}\n"
    return body


def _req(pod_spec, index=0, tasks=None):
    return PodInstanceRequirement(PodInstance(pod_spec, index), tasks or [t.name for t in pod_spec.tasks])


# ---------------------------------------------------------------------------------------
# DefaultPlanManager


POD_SPECS = [_spec(_pod(f"type{i}")).pods[0] for i in range(5)]
REQS = [_req(p) for p in POD_SPECS]


def _two_phase_plan(step0, step1):
    return DefaultPlan("test-plan", [DefaultPhase("phase-0", [step0], SerialStrategy()),
                                     DefaultPhase("phase-1", [step1], SerialStrategy())], SerialStrategy())


@pytest.fixture
def pm():
    first, second = TestStep("step-0", REQS[0]), TestStep("step-1", REQS[1])
    plan = _two_phase_plan(first, second)
    return first, second, plan, DefaultPlanManager.create_proceeding(plan)


def _complete(phase):
    for s in phase.get_children():
        s.force_complete()


def test_current_phase_advances(pm):
    first, second, plan, manager = pm
    assert manager.get_candidates([])[0] is plan.get_children()[0].get_children()[0]
    _complete(plan.get_children()[0])
    assert manager.get_candidates([])[0] is plan.get_children()[1].get_children()[0]
    _complete(plan.get_children()[1])
    assert manager.get_candidates([]) == []


def test_phase_status_follows_its_step(pm):
    first, _, plan, _ = pm
    phase = plan.get_children()[0]
    assert phase.get_status() == Status.PENDING
    first.set_status(Status.PREPARED)
    assert phase.get_status() == Status.IN_PROGRESS
    first.set_status(Status.COMPLETE)
    assert phase.get_status() == Status.COMPLETE


def test_empty_plan_is_complete_even_interrupted():
    manager = DefaultPlanManager.create_interrupted(DefaultPlan("test-plan", [], SerialStrategy()))
    assert manager.get_plan().get_status() == Status.COMPLETE


def test_plan_status_roll_up(pm):
    first, second, plan, manager = pm
    assert manager.get_plan().get_status() == Status.PENDING
    first.set_status(Status.ERROR)
    assert manager.get_plan().get_status() == Status.ERROR
    first.set_status(Status.WAITING)
    assert manager.get_plan().get_status() == Status.WAITING
    first.set_status(Status.PREPARED)
    assert manager.get_plan().get_status() == Status.IN_PROGRESS
    first.force_complete()
    second.set_status(Status.STARTING)
    assert manager.get_plan().get_status() == Status.IN_PROGRESS
    _complete(plan.get_children()[0])
    assert manager.get_plan().get_status() == Status.IN_PROGRESS
    _complete(plan.get_children()[1])
    assert manager.get_plan().get_status() == Status.COMPLETE


def test_is_complete(pm):
    _, _, plan, manager = pm
    assert not manager.get_plan().is_complete()
    _complete(plan.get_children()[0])
    assert not manager.get_plan().is_complete()
    _complete(plan.get_children()[1])
    assert manager.get_plan().is_complete()


def test_plan_interrupt_proceed(pm):
    _, _, plan, _ = pm
    assert not plan.is_interrupted()
    plan.interrupt()
    assert plan.is_interrupted()
    plan.proceed()
    assert not plan.is_interrupted()


def test_restart_and_force_complete(pm):
    first = pm[0]
    assert first.is_pending()
    first.set_status(Status.COMPLETE)
    first.restart()
    assert first.is_pending()
    first.set_status(Status.PREPARED)
    first.restart()
    assert first.is_pending()
    first.force_complete()
    assert first.is_complete()
    first.set_status(Status.PREPARED)
    first.force_complete()
    assert first.is_complete()


def test_abstract_step_restart_and_force_complete():
    """The base step (DeploymentStep's parent) behaves as TestStep does."""
    step = AbstractStep("plain")
    step.set_status(Status.STARTING)
    step.restart()
    assert step.is_pending()
    step.force_complete()
    assert step.is_complete()


def test_plan_update_and_parameters_reach_steps():
    step = TestStep("s")
    plan = DefaultPlan("test-plan", [DefaultPhase("phase-0", [step], SerialStrategy())], SerialStrategy())
    assert step.updates == []
    plan.update(U.generate_status(U.TASK_ID, P.TASK_RUNNING))
    assert len(step.updates) == 1
    plan.update_parameters({"PARAM1": "value1"})
    assert step.parameters == [{"PARAM1": "value1"}]


def _waiting_plan(st0, st1):
    s0, s1 = TestStep("test-step-0", REQS[0]), TestStep("test-step-1", REQS[1])
    phase = DefaultPhase("phase-1", [s0, s1], SerialStrategy())
    plan = DefaultPlan("test-plan", [phase], SerialStrategy())
    s0.set_status(st0)
    s1.set_status(st1)
    return phase, plan, DefaultPlanManager.create_interrupted(plan)


def test_all_prepared_steps_are_dirty():
    _, plan, manager = _waiting_plan(Status.PREPARED, Status.PREPARED)
    assert manager.get_plan().get_status() == Status.WAITING
    manager.get_plan().proceed()
    assert manager.get_plan().get_status() == Status.IN_PROGRESS
    assert manager.get_dirty_assets() == {REQS[0], REQS[1]}


def test_only_prepared_step_is_dirty():
    _, plan, manager = _waiting_plan(Status.PENDING, Status.PREPARED)
    assert manager.get_plan().get_status() == Status.WAITING
    plan.proceed()
    assert manager.get_plan().get_status() == Status.IN_PROGRESS
    assert manager.get_dirty_assets() == {REQS[1]}


def test_interrupted_plan_still_reports_dirty_assets():
    phase, plan, manager = _waiting_plan(Status.COMPLETE, Status.PREPARED)
    assert not phase.is_interrupted()
    assert manager.get_plan().get_status() == Status.WAITING
    assert manager.get_dirty_assets() == {REQS[1]}
    manager.get_plan().proceed()
    assert manager.get_plan().get_status() == Status.IN_PROGRESS


# ---------------------------------------------------------------------------------------
# Serial / Parallel / Random strategies


class FakeStep(AbstractStep):
    """A Mockito-style step whose pending/complete answers are set directly."""

    def __init__(self, name, req=None, complete=False):
        super().__init__(name)
        self.req = req
        self.set_status(Status.COMPLETE if complete else Status.PENDING)

    def get_pod_instance_requirement(self):
        return self.req

    def complete(self):
        self.set_status(Status.COMPLETE)


@pytest.fixture
def fakes():
    return [FakeStep(f"step{i}", REQS[i]) for i in range(3)]


def test_serial_execution(fakes):
    st = SerialStrategy()
    for i in range(3):
        assert st.get_candidates(fakes, []) == [fakes[i]]
        fakes[i].complete()
    assert st.get_candidates(fakes, []) == []


def test_serial_proceed_interrupt():
    st = SerialStrategy()
    phase = DefaultPhase("phase-0", [TestStep(), TestStep()], st)
    s0, s1 = phase.get_children()
    st.interrupt()
    assert st.get_candidates(phase.get_children(), []) == []
    st.proceed()
    assert st.get_candidates(phase.get_children(), [])[0] is s0
    st.interrupt()
    assert st.get_candidates(phase.get_children(), []) == []
    s0.set_status(Status.COMPLETE)
    assert st.get_candidates(phase.get_children(), []) == []
    st.proceed()
    assert st.get_candidates(phase.get_children(), [])[0] is s1
    s1.set_status(Status.COMPLETE)
    assert st.get_candidates(phase.get_children(), []) == []


def test_serial_middle_complete(fakes):
    st = SerialStrategy()
    assert st.get_candidates(fakes, []) == [fakes[0]]
    fakes[1].complete()
    assert st.get_candidates(fakes, []) == [fakes[0]]
    fakes[0].complete()
    assert st.get_candidates(fakes, []) == [fakes[2]]


def test_parallel_execution(fakes):
    st = ParallelStrategy()
    assert len(st.get_candidates(fakes, [])) == 3
    fakes[0].complete()
    assert len(st.get_candidates(fakes, [])) == 2
    fakes[1].complete()
    assert st.get_candidates(fakes, []) == [fakes[2]]
    fakes[2].complete()
    assert st.get_candidates(fakes, []) == []


def test_parallel_proceed_interrupt():
    st = ParallelStrategy()
    s0, s1 = TestStep(), TestStep()
    assert set(st.get_candidates([s0, s1], [])) == {s0, s1}
    st.interrupt()
    assert st.get_candidates([s0, s1], []) == []
    st.proceed()
    assert set(st.get_candidates([s0, s1], [])) == {s0, s1}
    s0.set_status(Status.COMPLETE)
    assert st.get_candidates([s0, s1], []) == [s1]
    st.interrupt()
    assert st.get_candidates([s0, s1], []) == []
    st.proceed()
    assert st.get_candidates([s0, s1], []) == [s1]
    s1.set_status(Status.COMPLETE)
    assert st.get_candidates([s0, s1], []) == []
    st.interrupt()
    assert st.get_candidates([s0, s1], []) == []


@pytest.mark.parametrize("steps,empty", [
    ([], True),
    (["pending"], False),
    (["complete"], True),
    (["pending", "pending"], False),
    (["complete", "complete"], True),
])
def test_random_strategy(steps, empty):
    elements = [FakeStep("mock-step", REQS[0], complete=(s == "complete")) for s in steps]
    cands = RandomStrategy().get_candidates(elements, [])
    assert (cands == []) == empty
    assert len(cands) <= 1


# ---------------------------------------------------------------------------------------
# CanaryStrategy


@pytest.fixture
def canary_steps():
    return [TestStep(f"step{i}", REQS[i]) for i in range(5)]


def _done(*steps):
    for s in steps:
        s.set_status(Status.COMPLETE)


def test_serial_canary(canary_steps):
    s = canary_steps
    st = CanaryStrategy(SerialStrategy(), s)
    assert st.get_candidates(s, []) == []
    st.proceed()
    assert st.get_candidates(s, []) == [s[0]]
    _done(s[0])
    assert st.get_candidates(s, []) == []
    st.proceed()
    assert st.get_candidates(s, []) == [s[1]]
    for i in range(1, 5):
        _done(s[i])
        assert st.get_candidates(s, []) == ([s[i + 1]] if i < 4 else [])
    assert all(x.is_complete() for x in s)


def test_long_serial_canary(canary_steps):
    s = canary_steps
    st = CanaryStrategy(SerialStrategy(), s, 3)
    assert st.get_candidates(s, []) == []
    for i in range(3):
        st.proceed()
        assert st.get_candidates(s, []) == [s[i]]
        _done(s[i])
        if i < 2:
            assert st.get_candidates(s, []) == []
    assert st.get_candidates(s, []) == [s[3]]
    _done(s[3])
    assert st.get_candidates(s, []) == [s[4]]
    _done(s[4])
    assert st.get_candidates(s, []) == []


def test_parallel_canary(canary_steps):
    s = canary_steps
    st = CanaryStrategy(ParallelStrategy(), s)
    assert st.get_candidates(s, []) == []
    st.proceed()
    assert st.get_candidates(s, []) == [s[0]]
    _done(s[0])
    assert st.get_candidates(s, []) == []
    st.proceed()
    assert set(st.get_candidates(s, [])) == set(s[1:])
    _done(s[2], s[4])
    assert set(st.get_candidates(s, [])) == {s[1], s[3]}
    _done(s[1], s[3])
    assert st.get_candidates(s, []) == []


def test_long_parallel_canary(canary_steps):
    s = canary_steps
    st = CanaryStrategy(ParallelStrategy(), s, 3)
    for i in range(2):
        st.proceed()
        assert st.get_candidates(s, []) == [s[i]]
        _done(s[i])
        assert st.get_candidates(s, []) == []
    st.proceed()
    assert set(st.get_candidates(s, [])) == {s[2], s[3], s[4]}
    _done(s[2], s[4])
    assert st.get_candidates(s, []) == [s[3]]
    _done(s[3])
    assert st.get_candidates(s, []) == []


def test_interrupts_are_ignored_while_canarying(canary_steps):
    s = canary_steps
    st = CanaryStrategy(SerialStrategy(), s)
    assert st.get_candidates(s, []) == []
    st.interrupt()  # ignored: no extra proceed needed
    st.proceed()
    assert st.get_candidates(s, []) == [s[0]]
    _done(s[0])
    st.interrupt()  # ignored
    st.proceed()
    assert st.get_candidates(s, []) == [s[1]]
    # past the canary, interrupts reach the serial strategy underneath
    st.interrupt()
    _done(s[1])
    assert st.get_candidates(s, []) == []
    st.proceed()
    assert st.get_candidates(s, []) == [s[2]]
    st.interrupt()
    _done(s[2])
    assert st.get_candidates(s, []) == []
    st.proceed()
    assert st.get_candidates(s, []) == [s[3]]
    _done(s[3])
    assert st.get_candidates(s, []) == [s[4]]
    _done(s[4])
    assert st.get_candidates(s, []) == []


def test_canary_skips_completed_steps(canary_steps):
    s = canary_steps
    _done(s[0], s[2])
    st = CanaryStrategy(SerialStrategy(), s)
    assert st.get_candidates(s, []) == []
    st.proceed()
    assert st.get_candidates(s, []) == [s[1]]
    _done(s[1])
    assert st.get_candidates(s, []) == []
    st.proceed()
    assert st.get_candidates(s, []) == [s[3]]
    _done(s[3])
    assert st.get_candidates(s, []) == [s[4]]
    _done(s[4])
    assert st.get_candidates(s, []) == []


def test_dirty_canary_steps_are_held_back(canary_steps):
    s = canary_steps
    st = CanaryStrategy(SerialStrategy(), s)
    assert st.get_candidates(s, []) == []
    st.proceed()
    for i in range(5):
        if i == 1:
            st.proceed()
        assert st.get_candidates(s, [REQS[i]]) == []
        assert st.get_candidates(s, [r for j, r in enumerate(REQS) if j != i]) == [s[i]]
        _done(s[i])
    assert st.get_candidates(s, []) == []


def test_single_and_empty_canary(canary_steps):
    s = canary_steps
    st = CanaryStrategy(SerialStrategy(), s)
    only = [s[0]]
    assert st.get_candidates(only, []) == []
    st.proceed()
    assert st.get_candidates(only, []) == [s[0]]
    _done(s[0])
    assert st.get_candidates(only, []) == []
    empty = CanaryStrategy(SerialStrategy(), [])
    assert empty.get_candidates([], []) == []
    empty.proceed()
    assert empty.get_candidates([], []) == []


# ---------------------------------------------------------------------------------------
# DefaultPhase


def test_phase_status_serial_vs_canary():
    s1, s2 = FakeStep("a"), FakeStep("b")
    s2.interrupt()  # WAITING
    assert DefaultPhase("serial-phase", [s1, s2], SerialStrategy()).get_status() == Status.PENDING
    s1.interrupt()
    assert DefaultPhase("canary-phase", [s1, s2], CanaryStrategy(SerialStrategy(), [s1, s2])).get_status() \
        == Status.WAITING


# ---------------------------------------------------------------------------------------
# PlanScheduler


class StubEvaluator:
    def __init__(self, recs=()):
        self.recs = list(recs)
        self.calls = []

    def evaluate(self, req, offers, all_tasks=None):
        self.calls.append((req, list(offers)))
        return list(self.recs)


OFFERS = [U.get_offer(offer_id=P.OfferID(value="offerid"), hostname="hello")]


@pytest.fixture
def drv():
    d = RecordingDriver()
    driver.set_driver(d)
    task_killer.reset(executor_enabled=False)
    yield d
    task_killer.reset(executor_enabled=False)
    driver.set_driver(None)


def test_plan_scheduler_skips_non_pending_steps(drv):
    step = TestStep()
    step.set_status(Status.STARTING)
    assert PlanScheduler(StubEvaluator(), StateStore(MemPersister())).resource_offers(OFFERS, [step]) == []
    assert step.get_status() == Status.STARTING


def test_plan_scheduler_prepares_steps_without_requirement(drv):
    step = TestStep()
    assert PlanScheduler(StubEvaluator(), StateStore(MemPersister())).resource_offers(OFFERS, [step]) == []
    assert step.is_prepared()


def test_plan_scheduler_no_recommendations(drv):
    req = _req(_spec(_pod()).pods[0])
    step = TestStep("offer-step", req)
    ev = StubEvaluator()
    assert PlanScheduler(ev, StateStore(MemPersister())).resource_offers(OFFERS, [step]) == []
    assert step.recommendations == []
    assert [c[0] for c in ev.calls] == [req] and ev.calls[0][1] == OFFERS
    assert step.is_prepared()


# ---------------------------------------------------------------------------------------
# DefaultStepFactory


def _factory(pod_yaml):
    spec = _spec(pod_yaml)
    persister = MemPersister()
    state_store = StateStore(persister)
    config_store = ConfigStore(loopback_check(spec), persister)
    config_store.set_target_config(config_store.store(spec))
    return DefaultStepFactory(config_store, state_store), state_store, config_store, PodInstance(spec.pods[0], 0)


def test_step_fails_on_shared_resource_set():
    factory, *_, pi = _factory(_pod(tasks=("t0", "t1"), resource_set=U.RESOURCE_SET_ID))
    step = factory.get_step(pi, ["t0", "t1"])
    assert step.get_status() == Status.ERROR
    assert "same resource set id" in step.get_errors()[0]


def test_step_fails_on_duplicate_dns_prefixes():
    factory, *_, pi = _factory(_pod(tasks=("t0", "t1"), dns="task-prefix"))
    step = factory.get_step(pi, ["t0", "t1"])
    assert step.get_status() == Status.ERROR
    assert "same DNS name" in step.get_errors()[0]


def _stored_task(state_store, name, config_id, readiness=False):
    t = P.TaskInfo(name=name)
    t.task_id.CopyFrom(to_task_id(U.SERVICE_NAME, name))
    t.agent_id.value = "proto-field-required"
    w = TaskLabelWriter(t)
    w.set_target_configuration(config_id)
    if readiness:
        w.set_readiness_check(P.HealthCheck())
    t.labels.CopyFrom(w.to_proto())
    state_store.store_tasks([t])
    return state_store.fetch_task(name)


def _status(info, state, ready=None):
    return U.generate_status(info.task_id, state, ready)


def test_initial_state_of_running_task_depends_on_readiness():
    factory, store, config_store, pi = _factory(_pod(tasks=("test-task-name0",)))
    config_id = uuid.uuid4()
    config_store.set_target_config(config_id)
    name = f"{pi.name}-test-task-name0"
    info = _stored_task(store, name, config_id, readiness=True)
    store.store_status(name, _status(info, P.TASK_RUNNING, ready=False))
    assert not factory.has_reached_goal_state(store.fetch_task(name), GoalState.RUNNING, config_id)
    step = factory.get_step(pi, ["test-task-name0"])
    assert step.is_pending() and not step.is_complete()
    store.store_status(name, _status(info, P.TASK_RUNNING, ready=True))
    assert factory.has_reached_goal_state(store.fetch_task(name), GoalState.RUNNING, config_id)
    step = factory.get_step(pi, ["test-task-name0"])
    assert step.is_complete() and not step.is_pending()


def test_running_task_on_another_config_is_pending():
    factory, store, config_store, pi = _factory(_pod(tasks=("t",)))
    name = f"{pi.name}-t"
    info = _stored_task(store, name, uuid.uuid4())
    store.store_status(name, _status(info, P.TASK_RUNNING))
    assert factory.get_step(pi, ["t"]).is_pending()


@pytest.mark.parametrize("goal", [GoalState.FINISH, GoalState.ONCE])
def test_finished_goal_states_are_reached_by_finishing(goal):
    factory, store, config_store, pi = _factory(_pod(tasks=(U.TASK_NAME,), goal=goal.name))
    config_id = uuid.uuid4()
    config_store.set_target_config(config_id)
    name = f"{pi.name}-{U.TASK_NAME}"
    info = _stored_task(store, name, config_id)
    store.store_status(name, _status(info, P.TASK_RUNNING))
    assert not factory.has_reached_goal_state(store.fetch_task(name), goal, config_id)
    store.store_status(name, _status(info, P.TASK_FINISHED))
    assert factory.has_reached_goal_state(store.fetch_task(name), goal, config_id)
    assert factory.get_step(pi, [U.TASK_NAME]).is_complete()


def test_once_task_finished_on_an_old_config_stays_complete():
    """ONCE ignores the target config (FINISH does not): a finished ONCE task never reruns."""
    factory, store, config_store, pi = _factory(_pod(tasks=("t",), goal="ONCE"))
    name = f"{pi.name}-t"
    info = _stored_task(store, name, uuid.uuid4())
    store.store_status(name, _status(info, P.TASK_FINISHED))
    assert factory.get_step(pi, ["t"]).is_complete()
    factory2, store2, _, pi2 = _factory(_pod(tasks=("t",), goal="FINISH"))
    info2 = _stored_task(store2, name, uuid.uuid4())
    store2.store_status(name, _status(info2, P.TASK_FINISHED))
    assert factory2.get_step(pi2, ["t"]).is_pending()


# ---------------------------------------------------------------------------------------
# DefaultPlanCoordinator


POD_A = _pod("POD-A", 1, ("A",), cpus=1.0, mem=1000.0, disk=1500.0)
POD_B = _pod("POD-B", 2, ("B",), cpus=2.0, mem=2000.0, disk=2500.0)
OTHER_ID = P.OfferID(value="other-offer")


@pytest.fixture
def coord_env(drv):
    persister = MemPersister()
    fs = FrameworkStore(persister)
    fs.store_framework_id(U.FRAMEWORK_ID)
    store = StateStore(persister)
    config_store = ConfigStore(None, persister)
    config_store.set_target_config(uuid.uuid4())
    phase_factory = DefaultPhaseFactory(DefaultStepFactory(config_store, store))
    evaluator = OfferEvaluator(fs, store, U.SERVICE_NAME, uuid.uuid4(), template_url_factory(U.SERVICE_NAME, CFG),
                               CFG)
    return phase_factory, PlanScheduler(evaluator, store)


def _offers(cpus, mem, disk):
    res = [U.unreserved_cpus(cpus), U.unreserved_mem(mem), U.unreserved_disk(disk)]
    return [U.complete_offer(res), U.complete_offer(res, offer_id=OTHER_ID)]


def _offer_ids(recs):
    out = []
    for r in recs:
        if r.offer_id.value not in out:
            out.append(r.offer_id.value)
    return out


def _deploy(phase_factory, pods, name=U.SERVICE_NAME):
    return DeployPlanFactory(phase_factory).get_plan(_spec(pods, name))


def test_coordinator_needs_a_plan_manager():
    with pytest.raises(ValueError):
        DefaultPlanCoordinator([])


def test_one_plan_sufficient_offer(coord_env):
    pf, ps = coord_env
    coord = DefaultPlanCoordinator([DefaultPlanManager.create_proceeding(_deploy(pf, POD_A))])
    assert _offer_ids(ps.resource_offers(_offers(2, 2000, 10000), coord.get_candidates())) == [U.OFFER_ID.value]


def test_pod_instance_requirement_conflicts():
    def multi(pod_type, task, n):
        return _spec(_pod(pod_type, 1, tuple(f"{task}{i}" for i in range(n)),
                          resource_set=None)).pods[0]

    base = _req(multi("POD-A", "A", 2))
    overlap = _req(multi("POD-A", "A", 1))
    different_tasks = _req(multi("POD-A", "AA", 1))
    different_pod = _req(multi("POD-B", "A", 2))
    assert base.conflicts_with(overlap)
    assert not base.conflicts_with(different_tasks)
    assert not base.conflicts_with(different_pod)
    assert base.conflicts_with(base)


def test_interrupted_plan_gets_nothing(coord_env):
    pf, ps = coord_env
    coord = DefaultPlanCoordinator([DefaultPlanManager.create_interrupted(_deploy(pf, POD_A))])
    assert ps.resource_offers(_offers(2, 1, 1), coord.get_candidates()) == []
    assert coord.get_candidates() == []


def test_complete_plan_gets_nothing(coord_env):
    pf, ps = coord_env
    plan = _deploy(pf, POD_A)
    plan.get_children()[0].get_children()[0].force_complete()
    coord = DefaultPlanCoordinator([DefaultPlanManager.create_interrupted(plan)])
    assert ps.resource_offers(_offers(2, 2000, 10000), coord.get_candidates()) == []


def test_insufficient_offer_launches_nothing(coord_env):
    pf, ps = coord_env
    coord = DefaultPlanCoordinator([DefaultPlanManager.create_proceeding(_deploy(pf, POD_A))])
    assert ps.resource_offers(_offers(2, 1, 1), coord.get_candidates()) == []


def test_two_plans_disjoint_assets_use_both_offers(coord_env):
    pf, ps = coord_env
    coord = DefaultPlanCoordinator([DefaultPlanManager.create_proceeding(_deploy(pf, POD_A)),
                                    DefaultPlanManager.create_proceeding(_deploy(pf, POD_B, U.SERVICE_NAME + "-B"))])
    assert _offer_ids(ps.resource_offers(_offers(2, 2000, 10000), coord.get_candidates())) == [
        U.OFFER_ID.value, OTHER_ID.value]


def test_two_plans_same_assets_only_one_launches(coord_env):
    pf, ps = coord_env
    coord = DefaultPlanCoordinator([DefaultPlanManager.create_proceeding(_deploy(pf, POD_A)),
                                    DefaultPlanManager.create_proceeding(_deploy(pf, POD_A, U.SERVICE_NAME + "-B"))])
    assert _offer_ids(ps.resource_offers(_offers(2, 2000, 10000), coord.get_candidates())) == [U.OFFER_ID.value]


def test_two_complete_plans_get_nothing(coord_env):
    pf, ps = coord_env
    a, b = _deploy(pf, POD_A), _deploy(pf, POD_A)
    managers = [DefaultPlanManager.create_interrupted(a), DefaultPlanManager.create_interrupted(b)]
    a.get_children()[0].get_children()[0].force_complete()
    b.get_children()[0].get_children()[0].force_complete()
    assert ps.resource_offers(_offers(2, 2000, 10000), DefaultPlanCoordinator(managers).get_candidates()) == []


def test_earlier_plan_yields_to_a_later_plans_prepared_step(coord_env):
    """Plan A runs first, but plan B's step on the same pod is already PREPARED: the coordinator
    hands A's manager B's dirty assets, so only B's step is offered."""
    pf, ps = coord_env
    a, b = _deploy(pf, POD_A), _deploy(pf, POD_A)
    coord = DefaultPlanCoordinator([DefaultPlanManager.create_proceeding(a), DefaultPlanManager.create_proceeding(b)])
    step_a, step_b = a.get_children()[0].get_children()[0], b.get_children()[0].get_children()[0]
    assert step_a.get_status() == Status.PENDING
    step_b.set_status(Status.PREPARED)
    assert _offer_ids(ps.resource_offers(_offers(2, 2000, 10000), coord.get_candidates())) == [U.OFFER_ID.value]
    assert step_b.get_status() == Status.STARTING
    assert step_a.get_status() == Status.PENDING
