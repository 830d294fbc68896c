"""Scheduler units: explicit reconciliation, new-work detection, the recovery plan manager and the
decommission plan factory.

Mirrors the reference's suites under sdk/scheduler/src/test/java/com/mesosphere/sdk/scheduler/
({ExplicitReconcilerTest,WorkSetTrackerTest}.java, recovery/DefaultRecoveryPlanManagerTest.java,
decommission/DecommissionPlanFactoryTest.java): reconciliation of stored non-terminal tasks with
the 4 s -> x2 backoff and updates that arrive before they are asked for; new work only for steps
not seen in the previous work set; failed tasks recovered in place (or permanently when the failure
monitor or the failed label says so), insufficient offers launching nothing, duplicate failures
keeping one recovery step; decommission phases for pods beyond ``count`` (and pod types no longer
in the spec) ordered highest index first, with stale DECOMMISSIONED overrides cleared.
"""
import uuid

import pytest

import testutils as U
from dcos_commons_amd.framework import driver, task_killer
from dcos_commons_amd.http.endpoint_utils import template_url_factory
from dcos_commons_amd.mesos import protos as P
from dcos_commons_amd.offer.evaluate.offer_evaluator import OfferEvaluator
from dcos_commons_amd.offer.taskdata.labels import TaskLabelWriter
from dcos_commons_amd.scheduler.decommission import (DECOMMISSIONING_STATUS, DecommissionPlanFactory,
                                                     get_pods_to_decommission)
from dcos_commons_amd.scheduler.plan.elements import AbstractStep
from dcos_commons_amd.scheduler.plan.managers import DefaultPlanCoordinator, DefaultPlanManager
from dcos_commons_amd.scheduler.plan.plan_scheduler import PlanScheduler
from dcos_commons_amd.scheduler.plan.pod_instance_requirement import PodInstanceRequirement, RecoveryType
from dcos_commons_amd.scheduler.plan.status import Status
from dcos_commons_amd.scheduler.reconciliation import ExplicitReconciler, WorkSetTracker
from dcos_commons_amd.scheduler.recovery import DefaultRecoveryPlanManager, TestingFailureMonitor
from dcos_commons_amd.scheduler.scheduler_config import SchedulerConfig
from dcos_commons_amd.specification.specs import PodInstance, loopback_check
from dcos_commons_amd.specification.yaml import mappers
from dcos_commons_amd.specification.yaml.raw import RawServiceSpec
from dcos_commons_amd.state.config_store import ConfigStore
from dcos_commons_amd.state.framework_store import FrameworkStore
from dcos_commons_amd.state.goal_state_override import GoalStateOverride, OverrideProgress, OverrideStatus
from dcos_commons_amd.state.state_store import StateStore
from dcos_commons_amd.storage.mem_persister import MemPersister
from dcos_commons_amd.testing.harness import RecordingDriver

CFG = SchedulerConfig.for_testing()


@pytest.fixture
def drv():
    d = RecordingDriver()
    driver.set_driver(d)
    task_killer.reset(executor_enabled=False)
    yield d
    task_killer.reset(executor_enabled=False)
    driver.set_driver(None)


# ---------------------------------------------------------------------------------------
# ExplicitReconciler


def _st(tid, state):
    s = P.TaskStatus(state=state)
    s.task_id.value = tid
    return s


S1 = _st("task-1", P.TASK_RUNNING)
S2 = _st("task-2", P.TASK_LOST)


class StatusStore:
    def __init__(self, statuses=()):
        self.statuses = list(statuses)

    def fetch_statuses(self):
        return list(self.statuses)


class Clock:
    def __init__(self, ms=12345.0):
        self.ms = ms

    def __call__(self):
        return self.ms


def _reconciler(statuses=(), clock=None):
    store = StatusStore(statuses)
    return ExplicitReconciler(store, clock_ms=clock or Clock()), store


def test_reconciler_start_empty(drv):
    r, _ = _reconciler()
    assert r.is_reconciled()
    r.start()
    assert r.is_reconciled() and r.remaining() == set()
    r.reconcile()
    assert drv.reconciles == []


def test_reconciler_start(drv):
    r, _ = _reconciler([S1, S2])
    assert r.is_reconciled()
    r.start()
    assert not r.is_reconciled()
    assert r.remaining() == {"task-1", "task-2"}


def test_reconciler_start_skips_terminal_tasks(drv):
    r, _ = _reconciler([S1, _st("task-3", P.TASK_FINISHED), _st("task-4", P.TASK_KILLED)])
    r.start()
    assert r.remaining() == {"task-1"}


def test_reconciler_start_multiple_times_appends_and_merges(drv):
    r, store = _reconciler([S1])
    r.start()
    assert r.remaining() == {"task-1"}
    store.statuses = [S2]
    r.start()
    assert r.remaining() == {"task-1", "task-2"}
    store.statuses = [S1, S2]
    r.start()
    assert r.remaining() == {"task-1", "task-2"}
    assert not r.is_reconciled()


def test_reconciler_updates_before_reconcile(drv):
    r, _ = _reconciler([S1, S2])
    r.start()
    r.update(S1)
    assert not r.is_reconciled() and r.remaining() == {"task-2"}
    r.update(S1)  # no change
    assert r.remaining() == {"task-2"}
    r.update(S2)
    assert r.is_reconciled() and r.remaining() == set()
    r.reconcile()  # no-op
    assert drv.reconciles == []


def test_reconciler_backoff_sequence(drv):
    clock = Clock()
    r, _ = _reconciler([S1, S2], clock)
    r.start()
    r.reconcile()  # first request: both tasks
    assert r.remaining() == {"task-1", "task-2"}
    r.update(S2)
    r.update(S2)
    assert r.remaining() == {"task-1"}
    r.reconcile()  # too soon: skipped
    assert len(drv.reconciles) == 1
    clock.ms += 30000
    r.reconcile()  # second request: the one left
    assert r.remaining() == {"task-1"}
    r.update(S1)
    assert r.is_reconciled()
    r.reconcile()  # marks reconciliation complete, no driver call
    r.reconcile()  # no-op
    assert [len(c) for c in drv.reconciles] == [2, 1]


def test_reconciler_backoff_doubles_up_to_the_cap(drv):
    clock = Clock(0.0)
    r, _ = _reconciler([S1], clock)
    r.start()
    sent_at = []
    for t in range(0, 200_000, 1000):
        clock.ms = float(t)
        before = len(drv.reconciles)
        r.reconcile()
        if len(drv.reconciles) > before:
            sent_at.append(t)
    # the first request waits the base 4 s, each later one twice the previous wait, capped at 30 s
    assert sent_at[0] == 4000
    gaps = [b - a for a, b in zip(sent_at, sent_at[1:])]
    assert gaps[:3] == [8000, 16000, 30000]
    assert set(gaps[3:]) == {30000}


def test_reconciler_lost_then_running(drv):
    r, _ = _reconciler([S2])
    r.start()
    assert r.remaining() == {"task-2"}
    r.reconcile()
    assert drv.reconciles == [[S2]]
    running = P.TaskStatus()
    running.CopyFrom(S2)
    running.state = P.TASK_RUNNING
    r.update(running)
    r.reconcile()
    assert r.is_reconciled() and r.remaining() == set()


# ---------------------------------------------------------------------------------------
# WorkSetTracker


def _spec(text):
    return mappers.ServiceSpecGenerator(RawServiceSpec.from_string(text), CFG, "/tmp", {}).build()


POD = _spec("name: svc\npods:\n  pod-type:\n    count: 2\n    tasks:\n      test-task-name:\n        goal: RUNNING\n"
            "        cmd: echo\n        cpus: 1\n        memory: 32\n").pods[0]


class NamedStep(AbstractStep):
    def __init__(self, name, req):
        super().__init__(name)
        self.req = req

    def get_pod_instance_requirement(self):
        return self.req


def _steps(index):
    req = PodInstanceRequirement(PodInstance(POD, index), ["test-task-name"])
    return [NamedStep(f"step-{index}", req)]


def test_work_set_new_work():
    t = WorkSetTracker()
    t.update_work_set(_steps(0))
    assert t.has_new_work()


def test_work_set_same_work():
    t = WorkSetTracker()
    t.update_work_set(_steps(0))
    assert t.has_new_work()
    t.update_work_set(_steps(0))
    assert not t.has_new_work()


def test_work_set_same_work_shows_up_later():
    t = WorkSetTracker()
    t.update_work_set(_steps(0))
    assert t.has_new_work()
    t.update_work_set([])
    assert not t.has_new_work()
    t.update_work_set(_steps(0))
    assert t.has_new_work()


def test_work_set_new_work_survives_across_work_sets():
    t = WorkSetTracker()
    t.update_work_set(_steps(0))
    t.update_work_set([])
    assert t.has_new_work()
    assert not t.has_new_work()
    t.update_work_set(_steps(0))
    assert t.has_new_work()
    assert not t.has_new_work()


def test_work_set_additional_new_work():
    t = WorkSetTracker()
    t.update_work_set(_steps(0))
    assert t.has_new_work()
    t.update_work_set(_steps(1))
    assert t.has_new_work()


def test_work_set_empty():
    t = WorkSetTracker()
    t.update_work_set([])
    assert not t.has_new_work()


# ---------------------------------------------------------------------------------------
# DefaultRecoveryPlanManager


RECOVERY_YML = """\
name: "hello-world"
pods:
  test-task-type:
    count: 1
    tasks:
      test-task-name:
        goal: RUNNING
        cmd: "echo 'Hello World'"
        cpus: 1.0
        memory: 1000
"""
TASK_NAME = "test-task-type-0-test-task-name"


class SpyFailureMonitor(TestingFailureMonitor):
    def __init__(self):
        super().__init__()
        self.asked = []

    def has_failed(self, task):
        self.asked.append(task.name)
        return super().has_failed(task)


class StubDeployManager(DefaultPlanManager):
    def __init__(self, candidates=()):
        from dcos_commons_amd.scheduler.plan.elements import DefaultPlan

        super().__init__(DefaultPlan("deploy", []))
        self.candidates = list(candidates)

    def get_candidates(self, dirty_assets):
        return list(self.candidates)


class RecoveryEnv:
    def __init__(self, deploy_candidates=()):
        persister = MemPersister()
        self.framework_store = FrameworkStore(persister)
        self.state_store = StateStore(persister)
        self.spec = _spec(RECOVERY_YML)
        self.config_store = ConfigStore(loopback_check(self.spec), persister)
        target = self.config_store.store(self.spec)
        self.config_store.set_target_config(target)
        base = U.get_task_info([U.unreserved_cpus(1.0), U.unreserved_mem(1000.0)], name=TASK_NAME,
                               task_id=U.to_task_id(U.SERVICE_NAME, TASK_NAME))
        w = TaskLabelWriter(base)
        w.set_target_configuration(target)
        w.set_index(0)
        w.set_type("test-task-type")
        base.labels.CopyFrom(w.to_proto())
        self.task = base
        self.monitor = SpyFailureMonitor()
        self.manager = DefaultRecoveryPlanManager(self.state_store, self.config_store, {TASK_NAME}, self.monitor)
        self.deploy = StubDeployManager(deploy_candidates)
        evaluator = OfferEvaluator(self.framework_store, self.state_store, self.spec.name, target,
                                   template_url_factory(self.spec.name, CFG), CFG)
        self.plan_scheduler = PlanScheduler(evaluator, self.state_store)
        self.coordinator = DefaultPlanCoordinator([self.deploy, self.manager])

    def fail(self, task=None, state=P.TASK_FAILED, store_task=True):
        task = task or self.task
        if store_task:
            self.state_store.store_tasks([task])
        st = U.generate_status(task.task_id, state)
        self.state_store.store_status(task.name, st)
        self.framework_store.store_framework_id(U.FRAMEWORK_ID)
        self.manager.update(st)
        return st

    def offers(self, cpus=1.0, mem=1000.0):
        return self.plan_scheduler.resource_offers(
            [U.complete_offer([U.unreserved_cpus(cpus), U.unreserved_mem(mem)])], self.coordinator.get_candidates())

    def recovery_steps(self):
        return [s for ph in self.manager.get_plan().get_children() for s in ph.get_children()]


def _distinct_offers(recs):
    return {r.offer_id.value for r in recs}


def test_stopped_task_is_relaunched(drv):
    env = RecoveryEnv()
    env.fail()
    assert len(_distinct_offers(env.offers())) == 1
    assert env.recovery_steps()[0].recovery_type == RecoveryType.TRANSIENT


def test_deploy_step_with_a_different_name_does_not_block_recovery(drv):
    other = NamedStep("different-name", None)
    env = RecoveryEnv([other])
    env.fail()
    assert len(_distinct_offers(env.offers())) == 1


def test_failed_task_is_replaced_permanently(drv):
    env = RecoveryEnv()
    env.monitor.set_failed_list(env.task)
    env.fail()
    assert len(_distinct_offers(env.offers())) == 1
    steps = env.recovery_steps()
    assert [s.get_name() for s in steps] == ["test-task-type-0:[test-task-name]"]
    assert steps[0].recovery_type == RecoveryType.PERMANENT
    # the permanent step marks the task failed when it starts
    assert TaskLabelWriter  # labels read back below
    from dcos_commons_amd.scheduler.recovery import is_permanently_failed

    assert is_permanently_failed(env.state_store.fetch_task(TASK_NAME))


def test_failed_task_waits_for_sufficient_resources(drv):
    env = RecoveryEnv()
    env.monitor.set_failed_list(env.task)
    env.fail()
    assert env.offers(cpus=0.5, mem=500.0) == []
    assert [s.get_name() for s in env.recovery_steps()] == ["test-task-type-0:[test-task-name]"]


def test_permanently_failed_label_skips_the_failure_monitor(drv):
    env = RecoveryEnv()
    failed = U.with_failed_flag(env.task)
    env.monitor.set_failed_list(failed)
    env.fail(failed)
    assert len(_distinct_offers(env.offers())) == 1
    assert env.monitor.asked == []


def test_duplicate_failures_keep_one_recovery_step(drv):
    env = RecoveryEnv()
    env.fail(state=P.TASK_RUNNING)
    assert env.manager.get_plan().get_children() == []
    env.fail(state=P.TASK_FAILED, store_task=False)
    env.manager.get_candidates([])
    assert env.recovery_steps()[0].is_pending()
    env.fail(state=P.TASK_FAILED, store_task=False)
    assert len(env.manager.get_plan().get_children()[0].get_children()) == 1


def test_fail_run_fail_keeps_one_pending_step(drv):
    env = RecoveryEnv()
    env.fail(state=P.TASK_RUNNING)
    assert env.manager.get_plan().get_children() == []
    env.fail(state=P.TASK_FAILED, store_task=False)
    env.manager.get_candidates([])
    assert env.recovery_steps()[0].is_pending()
    env.fail(state=P.TASK_RUNNING)
    env.manager.get_candidates([])
    assert env.recovery_steps()[0].is_pending()
    env.fail(state=P.TASK_FAILED, store_task=False)
    assert len(env.recovery_steps()) == 1
    assert env.recovery_steps()[0].is_pending()


def test_recovery_plan_cannot_be_replaced():
    env = RecoveryEnv()
    with pytest.raises(NotImplementedError):
        env.manager.set_plan(env.manager.get_plan())


def test_tasks_outside_the_recoverable_set_are_not_recovered(drv):
    env = RecoveryEnv()
    env.manager.recoverable_task_names = set()
    env.fail()
    assert env.offers() == []
    assert env.manager.get_plan().get_children() == []


# ---------------------------------------------------------------------------------------
# DecommissionPlanFactory


def _decom_task(pod_type, index, task, resource_count):
    name = f"{pod_type}-{index}-{task}"
    t = P.TaskInfo(name=name)
    t.task_id.CopyFrom(U.TASK_ID)
    t.agent_id.CopyFrom(U.AGENT_ID)
    w = TaskLabelWriter(t)
    w.set_type(pod_type)
    w.set_index(index)
    t.labels.CopyFrom(w.to_proto())
    for i in range(resource_count):
        t.resources.append(U.reserved_cpus(5, f"{name}-resource{i}"))
    return t


TASKS = [
    _decom_task("podA", 0, "taskA", 1),  # decommissioned, pending
    _decom_task("podA", 1, "taskA", 2),  # decommissioned, in progress
    _decom_task("podA", 2, "taskA", 3),  # inactive
    _decom_task("podB", 0, "taskA", 1),  # paused, complete
    _decom_task("podB", 0, "taskB", 2),  # decommissioned, pending
    _decom_task("podB", 1, "taskA", 1),  # decommissioned, in progress
    _decom_task("podB", 1, "taskB", 2),  # inactive
    _decom_task("podC", 0, "taskA", 3),  # paused, complete
    _decom_task("podD", 0, "taskA", 3),  # decommissioned, pending (podD/podE are not in the spec)
    _decom_task("podD", 1, "taskA", 1),  # decommissioned, in progress
    _decom_task("podE", 0, "taskA", 2),  # inactive
]
_OVERRIDES = [GoalStateOverride.DECOMMISSIONED.new_status(OverrideProgress.PENDING),
              GoalStateOverride.DECOMMISSIONED.new_status(OverrideProgress.IN_PROGRESS),
              OverrideStatus.INACTIVE,
              GoalStateOverride.PAUSED.new_status(OverrideProgress.COMPLETE)]


class OverrideStore:
    def __init__(self):
        self.overrides = {t.name: _OVERRIDES[i % 4] for i, t in enumerate(TASKS)}
        self.stored = []

    def fetch_tasks(self):
        return list(TASKS)

    fetch_tasks_shared = fetch_tasks

    def fetch_goal_override_status(self, name):
        return self.overrides[name]

    def store_goal_override_status(self, name, status):
        self.stored.append((name, status))


def _pods(**counts):
    import types

    return types.SimpleNamespace(pods=[types.SimpleNamespace(type=t, count=c) for t, c in counts.items()])


def test_no_decommission_clears_stale_bits():
    store = OverrideStore()
    factory = DecommissionPlanFactory(_pods(podA=3, podB=100, podC=1, podD=2, podE=2), store)
    assert factory.get_plan() is None
    assert factory.get_resource_steps() == []
    cleared = {n for n, s in store.stored if s == OverrideStatus.INACTIVE}
    assert cleared == {"podA-0-taskA", "podA-1-taskA", "podB-0-taskB", "podB-1-taskA", "podD-0-taskA",
                       "podD-1-taskA"}
    assert not any(s == DECOMMISSIONING_STATUS for _, s in store.stored)


def _names(phase):
    return [s.get_name() for s in phase.get_children()]


def test_big_plan_construction():
    store = OverrideStore()
    factory = DecommissionPlanFactory(_pods(podA=1, podB=1, podC=1), store)
    cleared = {n for n, s in store.stored if s == OverrideStatus.INACTIVE}
    assert cleared == {"podA-0-taskA", "podB-0-taskB"}
    pending = GoalStateOverride.DECOMMISSIONED.new_status(OverrideProgress.PENDING)
    assert {n for n, s in store.stored if s == pending} == {"podA-2-taskA", "podB-1-taskB", "podE-0-taskA"}
    assert len(factory.get_resource_steps()) == 14
    plan = factory.get_plan()
    assert plan is not None and plan.get_status() == Status.PENDING
    phases = plan.get_children()
    assert [p.get_name() for p in phases] == ["podD-1", "podD-0", "podE-0", "podB-1", "podA-2", "podA-1"]
    assert _names(phases[0]) == ["kill-podD-1-taskA", "unreserve-podD-1-taskA-resource0", "erase-podD-1-taskA"]
    assert _names(phases[1]) == ["kill-podD-0-taskA"] + [f"unreserve-podD-0-taskA-resource{i}" for i in range(3)] + [
        "erase-podD-0-taskA"]
    assert _names(phases[2]) == ["kill-podE-0-taskA", "unreserve-podE-0-taskA-resource0",
                                 "unreserve-podE-0-taskA-resource1", "erase-podE-0-taskA"]
    assert _names(phases[3]) == ["kill-podB-1-taskA", "kill-podB-1-taskB", "unreserve-podB-1-taskA-resource0",
                                 "unreserve-podB-1-taskB-resource0", "unreserve-podB-1-taskB-resource1",
                                 "erase-podB-1-taskA", "erase-podB-1-taskB"]
    assert _names(phases[4]) == ["kill-podA-2-taskA"] + [f"unreserve-podA-2-taskA-resource{i}" for i in range(3)] + [
        "erase-podA-2-taskA"]
    assert _names(phases[5]) == ["kill-podA-1-taskA", "unreserve-podA-1-taskA-resource0",
                                 "unreserve-podA-1-taskA-resource1", "erase-podA-1-taskA"]


def test_pod_ordering():
    pods = get_pods_to_decommission(_pods(podA=1, podB=1, podC=1), TASKS)
    assert [f"{k[1]}-{k[2]}" for k, _ in pods] == ["podD-1", "podD-0", "podE-0", "podB-1", "podA-2", "podA-1"]


def test_decommission_steps_kill_mark_and_erase(drv):
    persister = MemPersister()
    store = StateStore(persister)
    doomed = U.with_labels(U.get_task_info([U.reserved_cpus(1, "rid-1")], name="podA-1-taskA",
                                           task_id=U.to_task_id(U.SERVICE_NAME, "podA-1-taskA")),
                           lambda w: (w.set_type("podA"), w.set_index(1)))
    store.store_tasks([doomed])
    factory = DecommissionPlanFactory(_pods(podA=1), store)
    assert store.fetch_goal_override_status("podA-1-taskA") == \
        GoalStateOverride.DECOMMISSIONED.new_status(OverrideProgress.PENDING)
    kill, unreserve, erase = factory.get_plan().get_children()[0].get_children()
    kill.start()
    assert kill.is_complete()
    assert drv.kills == [doomed.task_id.value]
    assert store.fetch_goal_override_status("podA-1-taskA") == DECOMMISSIONING_STATUS
    unreserve.start()
    assert unreserve.is_prepared()
    unreserve.update_resource_status({"rid-1"})
    assert unreserve.is_complete()
    erase.start()
    assert store.fetch_task("podA-1-taskA") is None
    assert factory.get_plan().is_complete()
