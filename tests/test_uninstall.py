"""Uninstall: the plan factory, UninstallScheduler, UninstallRecorder and the uninstall steps.

Mirrors the reference's scheduler/uninstall suites (sdk/scheduler/src/test/java/com/mesosphere/
sdk/scheduler/uninstall/{UninstallSchedulerTest,ResourceCleanupStepTest,TLSCleanupStepTest,
TaskKillStepTest,UninstallRecorderTest}.java): the initial plan shape (task kills, resources
deduplicated per agent, tasks that are both permanently failed and TASK_ERROR skipped, the
UNKNOWN_AGENT phase), resource steps completing as their reservations come back in offers,
deregistration only after ``unregistered()``, TLS secret cleanup that keeps foreign secrets,
plan customizers and the removal timeout.
"""
import types

import pytest

import testutils as U
from dcos_commons_amd.framework import driver, task_killer
from dcos_commons_amd.mesos import protos as P
from dcos_commons_amd.offer.evaluate.security import TLSArtifactPaths
from dcos_commons_amd.offer.recommendations import (CreateOfferRecommendation, DestroyOfferRecommendation,
                                                    UnreserveOfferRecommendation)
from dcos_commons_amd.offer.resources import get_resource_id
from dcos_commons_amd.scheduler.mesos_event_client import (ClientStatusResponse, OfferResult,
                                                           UnexpectedResult)
from dcos_commons_amd.scheduler.plan.customizer import PlanCustomizer
from dcos_commons_amd.scheduler.plan.status import Status
from dcos_commons_amd.scheduler.scheduler_config import SchedulerConfig
from dcos_commons_amd.scheduler.uninstall import (ResourceCleanupStep, TaskKillStep, TLSCleanupStep,
                                                  UninstallRecorder, UninstallScheduler)
from dcos_commons_amd.state import state_store_utils
from dcos_commons_amd.state.state_store import StateStore
from dcos_commons_amd.storage.mem_persister import MemPersister
from dcos_commons_amd.testing.harness import RecordingDriver

R1, R2, R3, R4 = "resource-1", "resource-2", "resource-3", "resource-4"
RES1 = U.reserved_ports(123, 234, R1)
RES2 = U.reserved_root_volume(999.0, R2, R2)
RES3 = U.reserved_cpus(1.0, R3)
RES4 = U.reserved_cpus(1.0, R4)


def _host1(w):
    w.set_hostname(U.empty_offer(hostname="host-1"))


TASK_A = U.with_labels(U.get_task_info([RES1, RES2, RES3]), _host1)
# permanently failed, no hostname label (UNKNOWN_AGENT phase); shares RES2 with TASK_A on another agent
TASK_B = U.with_failed_flag(U.get_task_info([RES2, RES4], name="task-b",
                                            task_id=U.to_task_id(U.SERVICE_NAME, "task-b")))
# permanently failed on TASK_A's agent: its RES1 is deduplicated against TASK_A's
TASK_C = U.with_labels(U.get_task_info([RES1, RES4], name="task-c", task_id=U.to_task_id(U.SERVICE_NAME, "task-c")),
                       lambda w: (_host1(w), w.set_permanently_failed()))


class FakeSecretsClient:
    def __init__(self, listing=(), fail=False):
        self.listing = list(listing)
        self.fail = fail
        self.list_calls = []
        self.deleted = []

    def list(self, namespace):
        self.list_calls.append(namespace)
        if self.fail:
            raise IOError("secret store unreachable")
        return list(self.listing)

    def delete(self, path):
        self.deleted.append(path)


class Clock:
    def __init__(self):
        self.s = 1234567890

    def __call__(self):
        return self.s * 1000.0


@pytest.fixture
def drv():
    d = RecordingDriver()
    driver.set_driver(d)
    task_killer.reset(executor_enabled=False)
    yield d
    task_killer.reset(executor_enabled=False)
    driver.set_driver(None)


@pytest.fixture
def store():
    s = StateStore(MemPersister())
    s.store_tasks([TASK_A])
    return s


def _spec(pods=()):
    return types.SimpleNamespace(name=U.SERVICE_NAME, pods=list(pods))


def _tls_spec():
    task = types.SimpleNamespace(transport_encryption=[types.SimpleNamespace(name="foo", type="KEYSTORE")])
    return _spec([types.SimpleNamespace(tasks=[task])])


CFG = SchedulerConfig.for_testing(SERVICE_REMOVAL_TIMEOUT_S="60")


def _scheduler(store, spec=None, customizer=None, secrets=None, clock=None, register=True):
    s = UninstallScheduler(spec or _spec(), store, None, CFG, plan_customizer=customizer or PlanCustomizer(),
                           secrets_client=secrets if secrets is not None else FakeSecretsClient(),
                           clock_ms=clock or Clock())
    if register:
        s.registered(False)
    return s


def _plan(s):
    return s.plan_coordinator.get_plan_managers()[0].get_plan()


def _statuses(plan):
    return [st.get_status() for ph in plan.get_children() for st in ph.get_children()]


def _offer(resources=()):
    return U.get_offer(resources, offer_id=P.OfferID(value=U.uuid4_str()))


# ---------------------------------------------------------------------------------------
# UninstallScheduler


def test_empty_offers(drv, store):
    s = _scheduler(store)
    assert s.get_client_status() == ClientStatusResponse.launching(True)
    assert s.offers([]).result == OfferResult.PROCESSED
    assert drv.accepts == [] and drv.declines == []


def test_initial_plan_and_uninstall_bit(drv, store):
    s = _scheduler(store)
    # 1 task kill + 3 unique resources + deregister step
    assert _statuses(_plan(s)) == [Status.PENDING] * 5
    assert state_store_utils.is_uninstalling(store)
    assert [ph.get_name() for ph in _plan(s).get_children()] == [
        "kill-tasks", "unreserve-resources-host-1", "deregister-service"]


def test_initial_plan_task_resource_overlap(drv, store):
    store.store_tasks([TASK_B, TASK_C])
    plan = _plan(_scheduler(store))
    # 3 kills, 2 resources on UNKNOWN_AGENT (TASK_B), 4 deduplicated on host-1 (A + C), deregister
    assert _statuses(plan) == [Status.PENDING] * 10
    names = [ph.get_name() for ph in plan.get_children()]
    assert names == ["kill-tasks", "unreserve-resources-UNKNOWN_AGENT", "unreserve-resources-host-1",
                     "deregister-service"]
    assert {st.resource_id for st in plan.get_children()[1].get_children()} == {R2, R4}
    assert {st.resource_id for st in plan.get_children()[2].get_children()} == {R1, R2, R3, R4}


def test_initial_plan_skips_resources_of_failed_tasks_in_error(drv, store):
    store.store_tasks([TASK_B, TASK_C])
    store.store_status(TASK_B.name, U.generate_status(TASK_B.task_id, P.TASK_ERROR))
    store.store_status(TASK_C.name, U.generate_status(TASK_C.task_id, P.TASK_ERROR))
    s = _scheduler(store)
    assert s.get_client_status() == ClientStatusResponse.launching(True)
    # 3 kills, only TASK_A's 3 resources, deregister
    assert _statuses(_plan(s)) == [Status.PENDING] * 7


def test_uninstall_steps_prepared(drv, store):
    s = _scheduler(store)
    assert s.get_client_status() == ClientStatusResponse.launching(True)
    s.offers([_offer()])
    # resource steps do not depend on the kill step: PREPARED at once
    assert _statuses(_plan(s)) == [Status.COMPLETE, Status.PREPARED, Status.PREPARED, Status.PREPARED,
                                   Status.PENDING]
    assert drv.kills == [TASK_A.task_id.value]


def _expect_unexpected(s, offer):
    resp = s.get_unexpected_resources([offer])
    assert resp.result == UnexpectedResult.PROCESSED
    assert len(resp.offer_resources) == 1
    assert list(resp.offer_resources[0].resources) == list(offer.resources)


def test_uninstall_steps_complete_as_reservations_return(drv, store):
    offer = _offer([RES1, RES2])
    s = _scheduler(store)
    assert s.get_client_status() == ClientStatusResponse.launching(True)
    s.offers([offer])
    _expect_unexpected(s, offer)
    plan = _plan(s)
    assert _statuses(plan) == [Status.COMPLETE, Status.COMPLETE, Status.COMPLETE, Status.PREPARED, Status.PENDING]
    # every uninstall step was a candidate up front: no new work now
    assert s.get_client_status() == ClientStatusResponse.launching(False)
    offer = _offer([RES3])
    s.offers([offer])
    _expect_unexpected(s, offer)
    assert _statuses(plan) == [Status.COMPLETE] * 4 + [Status.PENDING]
    # the returned reservations are erased from the stored TaskInfo
    assert list(store.fetch_task(TASK_A.name).resources) == []


def test_plan_completes_only_after_unregistered(drv, store):
    offer = _offer([RES1, RES2, RES3])
    s = _scheduler(store)
    assert s.get_client_status() == ClientStatusResponse.launching(True)
    s.offers([offer])
    _expect_unexpected(s, offer)
    plan = _plan(s)
    assert _statuses(plan) == [Status.COMPLETE] * 4 + [Status.PENDING]
    assert s.get_client_status() == ClientStatusResponse.launching(True)
    s.offers([_offer()])
    assert _statuses(plan) == [Status.COMPLETE] * 4 + [Status.PREPARED]
    assert s.get_client_status() == ClientStatusResponse.ready_to_remove()
    s.unregistered()
    assert _statuses(plan) == [Status.COMPLETE] * 5
    assert plan.is_complete()


def test_empty_state_has_only_the_deregister_step(drv):
    s = _scheduler(StateStore(MemPersister()))
    plan = _plan(s)
    assert _statuses(plan) == [Status.PENDING]
    assert plan.is_running()
    assert s.get_client_status() == ClientStatusResponse.launching(True)
    s.offers([_offer()])
    assert s.get_client_status() == ClientStatusResponse.ready_to_remove()
    assert _statuses(plan) == [Status.PREPARED]
    assert plan.is_running()
    s.unregistered()
    assert s.get_client_status() == ClientStatusResponse.ready_to_remove()
    assert _statuses(plan) == [Status.COMPLETE]
    assert plan.is_complete()


def test_tls_cleanup_phase_runs_with_the_resource_phases(drv, store):
    secrets = FakeSecretsClient()
    s = _scheduler(store, spec=_tls_spec(), secrets=secrets)
    plan = _plan(s)
    assert [ph.get_name() for ph in plan.get_children()][-2:] == ["tls-cleanup", "deregister-service"]
    assert s.get_client_status() == ClientStatusResponse.launching(True)
    offer = _offer([RES1, RES2, RES3])
    s.offers([offer])
    _expect_unexpected(s, offer)
    # TLS cleanup does not depend on kills/unreserves: it completed in the same cycle
    assert _statuses(plan) == [Status.COMPLETE] * 5 + [Status.PENDING]
    assert secrets.list_calls == [U.SERVICE_NAME]
    assert s.get_client_status() == ClientStatusResponse.launching(True)
    s.offers([_offer()])
    assert _statuses(plan) == [Status.COMPLETE] * 5 + [Status.PREPARED]
    assert s.get_client_status() == ClientStatusResponse.ready_to_remove()
    s.unregistered()
    assert s.get_client_status() == ClientStatusResponse.ready_to_remove()
    assert _statuses(plan) == [Status.COMPLETE] * 6
    assert plan.is_complete()


def test_tls_artifacts_of_an_earlier_config_are_cleaned_too(drv, store):
    """Beyond the reference (UninstallPlanFactory.java:110-115 only looks at the current spec):
    a spec without TLS still gets the cleanup phase when the secret store holds TLS artifacts."""
    paths = TLSArtifactPaths(U.SERVICE_NAME, "pod-type-0-test-task-name", "a-test-hash")
    secrets = FakeSecretsClient(paths.get_all_names("tls-test") + ["unrelated"])
    plan = _plan(_scheduler(store, secrets=secrets))
    assert "tls-cleanup" in [ph.get_name() for ph in plan.get_children()]
    no_tls = _plan(_scheduler(StateStore(MemPersister()), secrets=FakeSecretsClient(["unrelated"])))
    assert "tls-cleanup" not in [ph.get_name() for ph in no_tls.get_children()]


def test_uninstall_plan_customizer(drv, store):
    class Reversing(PlanCustomizer):
        def update_uninstall_plan(self, plan):
            plan.get_children().reverse()
            return plan

    plan = _plan(_scheduler(store, customizer=Reversing(), register=False))
    assert [ph.get_name() for ph in plan.get_children()] == [
        "deregister-service", "unreserve-resources-host-1", "kill-tasks"]


def test_uninstall_timeout(drv, store):
    clock = Clock()
    s = _scheduler(store, clock=clock)
    assert s.get_client_status() == ClientStatusResponse.launching(True)
    clock.s += 60
    assert s.get_client_status() == ClientStatusResponse.launching(False)
    clock.s += 1
    assert s.get_client_status() == ClientStatusResponse.ready_to_remove()


def test_sdk_uninstall_mode_has_no_timeout(drv, store):
    clock = Clock()
    s = UninstallScheduler(_spec(), store, None, SchedulerConfig.for_testing(SDK_UNINSTALL="true",
                                                                             SERVICE_REMOVAL_TIMEOUT_S="60"),
                           secrets_client=FakeSecretsClient(), clock_ms=clock)
    s.registered(False)
    clock.s += 10_000
    assert s.get_client_status() == ClientStatusResponse.launching(True)


def test_offers_wait_for_explicit_reconciliation(drv, store):
    store.store_status(TASK_A.name, U.generate_status(TASK_A.task_id, P.TASK_RUNNING))
    s = _scheduler(store)
    assert drv.reconciles and [st.task_id.value for st in drv.reconciles[0]] == [TASK_A.task_id.value]
    s.get_client_status()
    assert s.offers([_offer()]).result == OfferResult.NOT_READY
    s.task_status(U.generate_status(TASK_A.task_id, P.TASK_RUNNING))
    assert s.offers([_offer()]).result == OfferResult.PROCESSED


def test_unknown_task_status(drv, store):
    from dcos_commons_amd.scheduler.mesos_event_client import TaskStatusResult

    s = _scheduler(store)
    other = U.generate_status(U.to_task_id(U.SERVICE_NAME, "nope"), P.TASK_RUNNING)
    assert s.task_status(other).result == TaskStatusResult.UNKNOWN_TASK
    assert s.task_status(U.generate_status(TASK_A.task_id, P.TASK_KILLED)).result == TaskStatusResult.PROCESSED
    assert store.fetch_status(TASK_A.name).state == P.TASK_KILLED


# ---------------------------------------------------------------------------------------
# ResourceCleanupStep


def test_resource_cleanup_step_start():
    step = ResourceCleanupStep(U.RESOURCE_ID)
    assert step.get_status() == Status.PENDING
    step.start()
    assert step.get_pod_instance_requirement() is None
    assert step.get_status() == Status.PREPARED
    assert step.get_errors() == []


@pytest.mark.parametrize("ids,expected", [
    ({U.RESOURCE_ID}, Status.COMPLETE),
    ({"different-resource-id"}, Status.PREPARED),
    ({U.RESOURCE_ID, "different-resource-id"}, Status.COMPLETE),
])
def test_resource_cleanup_step_update(ids, expected):
    step = ResourceCleanupStep(U.RESOURCE_ID)
    step.start()
    step.update_resource_status(ids)
    assert step.get_status() == expected


# ---------------------------------------------------------------------------------------
# TLSCleanupStep


PATHS = TLSArtifactPaths(U.SERVICE_NAME, f"{U.POD_TYPE}-0-{U.TASK_NAME}", "a-test-hash")


def test_tls_cleanup_secrets_client_error():
    secrets = FakeSecretsClient(fail=True)
    step = TLSCleanupStep(secrets, U.SERVICE_NAME)
    step.start()
    assert secrets.deleted == []
    assert step.has_errors()


def test_tls_cleanup_deletes_every_artifact():
    secrets = FakeSecretsClient(PATHS.get_all_names("tls-test"))
    step = TLSCleanupStep(secrets, U.SERVICE_NAME)
    step.start()
    assert sorted(secrets.deleted) == sorted(f"{U.SERVICE_NAME}/{n}" for n in PATHS.get_all_names("tls-test"))
    assert step.is_complete()


def test_tls_cleanup_keeps_non_tls_secrets():
    others = ["test", "test/nested"]
    secrets = FakeSecretsClient(PATHS.get_all_names("tls-test") + others)
    step = TLSCleanupStep(secrets, U.SERVICE_NAME)
    step.start()
    assert not any(d.endswith(("/test", "/test/nested")) for d in secrets.deleted)
    assert len(secrets.deleted) == len(PATHS.get_all_names("tls-test"))
    assert step.is_complete()


def test_tls_cleanup_without_tls_secrets():
    secrets = FakeSecretsClient(["test", "test/nested"])
    step = TLSCleanupStep(secrets, U.SERVICE_NAME)
    step.start()
    assert secrets.deleted == []
    assert step.is_complete()


# ---------------------------------------------------------------------------------------
# TaskKillStep


def test_task_kill_step(drv):
    tid = P.TaskID(value="task-1")
    step = TaskKillStep(tid)
    step.start()
    assert step.get_pod_instance_requirement() is None
    assert step.get_status() == Status.COMPLETE
    assert drv.kills == ["task-1"]


# ---------------------------------------------------------------------------------------
# UninstallRecorder


class RecordingStore:
    def __init__(self, tasks):
        self.tasks = tasks
        self.stored = []

    def fetch_tasks(self):
        return list(self.tasks)

    def store_tasks(self, tasks):
        self.stored.append(list(tasks))


class RecordingStep:
    def __init__(self):
        self.updates = []

    def update_resource_status(self, ids):
        self.updates.append(set(ids))


@pytest.fixture
def recorder_env():
    task_res = U.reserved_cpus(5, "matching-resource")
    other_res = U.reserved_cpus(5, "other-resource")
    offer = U.get_offer([task_res, other_res])
    task_a, task_b = U.get_task_info([task_res]), U.get_task_info([task_res])
    store = RecordingStore([task_a, task_b, U.get_task_info([])])
    step = RecordingStep()
    return types.SimpleNamespace(rec=UninstallRecorder(store, [step]), store=store, step=step, offer=offer,
                                 task_res=task_res, other_res=other_res, task_a=task_a, task_b=task_b)


def _emptied(t):
    c = P.TaskInfo()
    c.CopyFrom(t)
    del c.resources[:]
    return c


@pytest.mark.parametrize("cls", [DestroyOfferRecommendation, UnreserveOfferRecommendation])
def test_recorder_resource_not_in_any_task(recorder_env, cls):
    e = recorder_env
    e.rec.record_decommission([cls(e.offer, e.other_res)])
    assert e.store.stored == []
    # steps are notified even when no stored task had the resource
    assert e.step.updates == [{get_resource_id(e.other_res)}]


@pytest.mark.parametrize("cls", [DestroyOfferRecommendation, UnreserveOfferRecommendation])
def test_recorder_erases_the_resource_from_tasks(recorder_env, cls):
    e = recorder_env
    e.rec.record_decommission([cls(e.offer, e.task_res)])
    assert e.store.stored == [[_emptied(e.task_a), _emptied(e.task_b)]]
    assert e.step.updates == [{get_resource_id(e.task_res)}]


def test_recorder_ignores_other_recommendations(recorder_env):
    e = recorder_env
    e.rec.record_decommission([CreateOfferRecommendation(e.offer, U.unreserved_cpus(1.0))])
    assert e.store.stored == [] and e.step.updates == []
