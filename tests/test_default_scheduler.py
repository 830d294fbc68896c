"""DefaultScheduler, SchedulerBuilder, AbstractScheduler and SchedulerConfig units.

Mirrors the reference's scheduler suites (sdk/scheduler/src/test/java/com/mesosphere/sdk/scheduler/
{DefaultSchedulerTest,SchedulerBuilderTest,AbstractSchedulerTest,SchedulerConfigTest,
SchedulerRunnerTest}.java): a two-pod service launched step by step (executor + task reservations,
the ROOT volume, LAUNCH_GROUP and the write-ahead TaskInfo, in that order), insufficient offers
leaving the step PREPARED, per-task and per-pod-type config updates re-running only the changed
steps, a config update that waits for reconciliation before killing and relaunching with the
grown reservation, an invalid (shrinking) update keeping the old target, the stored task IP, FINISH
services asking to be uninstalled, unexpected-reservation GC for permanently failed and
decommissioning tasks, region-rule injection and deploy/update plan selection.
"""
import dataclasses
import threading
import textwrap
import types
import uuid

import pytest

import testutils as U
from dcos_commons_amd.dcos import capabilities
from dcos_commons_amd.framework import driver, task_killer
from dcos_commons_amd.framework.env_store import EnvStore
from dcos_commons_amd.mesos import protos as P
from dcos_commons_amd.offer import constants
from dcos_commons_amd.offer.evaluate import placement as pl
from dcos_commons_amd.offer.recommendations import LaunchOfferRecommendation, StoreTaskInfoRecommendation
from dcos_commons_amd.offer.taskdata.labels import TaskLabelWriter
from dcos_commons_amd.scheduler.abstract_scheduler import AbstractScheduler
from dcos_commons_amd.scheduler.decommission import DECOMMISSIONING_STATUS
from dcos_commons_amd.scheduler.mesos_event_client import (ClientStatusResponse, OfferResponse, OfferResult,
                                                           UnexpectedResult)
from dcos_commons_amd.scheduler.plan.customizer import PlanCustomizer
from dcos_commons_amd.scheduler.plan.elements import DefaultPhase, DefaultPlan
from dcos_commons_amd.scheduler.plan.status import Status
from dcos_commons_amd.scheduler.plan.strategy import SerialStrategy
from dcos_commons_amd.scheduler.scheduler_builder import SchedulerBuilder
from dcos_commons_amd.scheduler.scheduler_config import SchedulerConfig
from dcos_commons_amd.specification.specs import GoalState
from dcos_commons_amd.specification.yaml import mappers
from dcos_commons_amd.specification.yaml.raw import RawServiceSpec
from dcos_commons_amd.state import state_store_utils
from dcos_commons_amd.state.framework_store import FrameworkStore
from dcos_commons_amd.state.state_store import StateStore
from dcos_commons_amd.storage.mem_persister import MemPersister
from dcos_commons_amd.testing.harness import RecordingDriver

CFG = SchedulerConfig.for_testing()
TASK_IP = "9.9.9.9"
R, C, LG = P.Offer.Operation.RESERVE, P.Offer.Operation.CREATE, P.Offer.Operation.LAUNCH_GROUP
FULL_LAUNCH = [R, R, R, R, R, R, C, LG, None]  # executor x3, task x3, volume, launch, stored TaskInfo


def _pod(pod_type, count, task, cpus, mem, disk, allow_decommission=False):
    return textwrap.dedent(f"""\
        {pod_type}:
          count: {count}
          allow-decommission: {str(allow_decommission).lower()}
          resource-sets:
            {U.RESOURCE_SET_ID}-{pod_type[-1]}:
              cpus: {cpus}
              memory: {mem}
              volume:
                path: {U.CONTAINER_PATH}
                type: ROOT
                size: {disk}
          tasks:
            {task}:
              goal: RUNNING
              cmd: echo {task}
              resource-set: {U.RESOURCE_SET_ID}-{pod_type[-1]}
        """)


POD_A = _pod("POD-A", 1, "A", 1.0, 1000, 1500)
POD_B = _pod("POD-B", 2, "B", 2.0, 2000, 2500)
UPDATED_POD_A = _pod("POD-A", 1, "A", 2.0, 1000, 1500)
UPDATED_POD_B = _pod("POD-B", 2, "B", 2.0, 4000, 2500)
INVALID_POD_B = _pod("POD-B", 1, "B", 2.0, 2000, 2500)
SCALED_POD_A = _pod("POD-A", 2, "A", 1.0, 1000, 1500)


def service_spec(*pods, goal=None):
    text = f"name: {U.SERVICE_NAME}\nscheduler:\n  principal: {U.PRINCIPAL}\n  user: {U.SERVICE_USER}\n"
    text += "pods:\n" + textwrap.indent("".join(pods), "  ")
    spec = mappers.ServiceSpecGenerator(RawServiceSpec.from_string(text), CFG, "/tmp", {}).build()
    # the service goal is a builder-only field (DefaultServiceSpec.goalState), not a YAML key
    return dataclasses.replace(spec, goal=goal) if goal is not None else spec


@pytest.fixture(autouse=True)
def env():
    saved = capabilities.get_instance()
    capabilities.override_capabilities(capabilities.Capabilities().with_overrides(supports_gpu_resource=False,
                                                                                   supports_domains=True))
    d = RecordingDriver()
    driver.set_driver(d)
    task_killer.reset(executor_enabled=False)
    yield d
    task_killer.reset(executor_enabled=False)
    driver.set_driver(None)
    capabilities.override_capabilities(saved)


class Harness:
    def __init__(self, drv, spec=None):
        self.drv = drv
        self.persister = MemPersister()
        FrameworkStore(self.persister).store_framework_id(U.FRAMEWORK_ID)
        self.scheduler = self.build(spec or service_spec(POD_A, POD_B))

    def build(self, spec, customizer=None):
        b = SchedulerBuilder(spec, CFG, self.persister)
        if customizer is not None:
            b.set_plan_customizer(customizer)
        s = b.build()
        s.registered(False)
        self.scheduler = s
        return s

    def plan(self, name=constants.DEPLOY_PLAN_NAME):
        return next(pm.get_plan() for pm in self.scheduler.plan_coordinator.get_plan_managers()
                    if pm.get_plan().get_name() == name)

    def statuses(self, name=constants.DEPLOY_PLAN_NAME):
        return [s.get_status() for ph in self.plan(name).get_children() for s in ph.get_children()]

    def status_update(self, task_id, state, ip=TASK_IP):
        self.scheduler.task_status(task_status(task_id, state, ip))

    def install_step(self, phase, step, offer, expected_status, new_work):
        assert self.scheduler.get_client_status() == ClientStatusResponse.footprint(new_work)
        st = self.plan().get_children()[phase].get_children()[step]
        assert st.get_status() == expected_status
        resp = self.scheduler.offers([offer])
        for rec in resp.recommendations:
            assert rec.offer_id == offer.id
            assert rec.agent_id == offer.agent_id
        assert op_types(resp.recommendations) == FULL_LAUNCH
        assert st.is_starting()
        tid = launched_task(resp.recommendations).task_id
        self.status_update(tid, P.TASK_RUNNING)
        assert st.is_complete()
        return tid

    def install(self):
        ids = [self.install_step(0, 0, offer_for_a(), Status.PENDING, True),
               self.install_step(1, 0, offer_for_b(), Status.PENDING, True),
               self.install_step(1, 1, offer_for_b(), Status.PENDING, True)]
        assert self.plan().is_complete()
        assert self.statuses() == [Status.COMPLETE] * 3
        assert self.scheduler.plan_coordinator.get_candidates() == []
        store = StateStore(self.persister)
        assert not state_store_utils.get_deployment_was_completed(store)
        assert self.scheduler.get_client_status() == ClientStatusResponse.idle()
        assert state_store_utils.get_deployment_was_completed(store)
        return ids


def task_status(task_id, state, ip=TASK_IP):
    s = P.TaskStatus(state=state)
    s.task_id.CopyFrom(task_id)
    if ip is not None:
        s.container_status.network_infos.add().ip_addresses.add(ip_address=ip)
    return s


def op_types(recs):
    return [r.get_operation().type if r.get_operation() is not None else None for r in recs]


def launched_task(recs):
    launch = next(r for r in recs if isinstance(r, LaunchOfferRecommendation))
    return launch.task_info


def _offer(*resources):
    return U.get_offer(resources, offer_id=P.OfferID(value=str(uuid.uuid4())))


def offer_for_a():
    return _offer(U.unreserved_cpus(1.0 + 0.1), U.unreserved_mem(1000 + 32), U.unreserved_disk(1500 + 256))


def offer_for_b():
    return _offer(U.unreserved_cpus(2.0 + 0.1), U.unreserved_mem(2000 + 32), U.unreserved_disk(2500 + 256))


@pytest.fixture
def h(env):
    return Harness(env)


# ---------------------------------------------------------------------------------------
# DefaultScheduler


def test_empty_offers(h):
    assert h.scheduler.get_client_status() == ClientStatusResponse.footprint(True)
    resp = h.scheduler.offers([])
    assert resp.result == OfferResult.PROCESSED and resp.recommendations == []


def test_launch_a(h):
    h.install_step(0, 0, offer_for_a(), Status.PENDING, True)
    assert h.statuses() == [Status.COMPLETE, Status.PENDING, Status.PENDING]


def test_launch_b(h):
    test_launch_a(h)
    h.install_step(1, 0, offer_for_b(), Status.PENDING, True)
    assert h.statuses() == [Status.COMPLETE, Status.COMPLETE, Status.PENDING]


def test_insufficient_offer_leaves_the_step_prepared(h):
    step = h.plan().get_children()[0].get_children()[0]
    assert step.is_pending()
    assert h.scheduler.get_client_status() == ClientStatusResponse.footprint(True)
    h.scheduler.offers([_offer(U.unreserved_cpus(0.5), U.unreserved_mem(500))])
    assert h.statuses() == [Status.PREPARED, Status.PENDING, Status.PENDING]


@pytest.mark.parametrize("pods,expected", [
    ((UPDATED_POD_A, POD_B), [Status.PENDING, Status.COMPLETE, Status.PENDING]),
    ((POD_A, UPDATED_POD_B), [Status.COMPLETE, Status.PENDING, Status.PENDING]),
    ((SCALED_POD_A, POD_B), [Status.COMPLETE, Status.PENDING, Status.COMPLETE, Status.PENDING]),
])
def test_updates_rerun_only_changed_steps(h, pods, expected):
    test_launch_b(h)
    h.build(service_spec(*pods))
    assert h.statuses() == expected


def _reserved_by(recs):
    return [r for rec in recs if rec.get_operation() is not None and rec.get_operation().type == R
            for r in rec.get_operation().reserve.resources]


def test_launch_and_recovery(h):
    step = h.plan().get_children()[0].get_children()[0]
    assert h.scheduler.get_client_status() == ClientStatusResponse.footprint(True)
    offer1 = offer_for_a()
    resp = h.scheduler.offers([offer1])
    assert len(resp.recommendations) == 9
    assert resp.recommendations[0].offer_id == offer1.id
    tid = launched_task(resp.recommendations).task_id
    h.status_update(tid, P.TASK_RUNNING)
    assert step.is_complete()
    assert h.statuses() == [Status.COMPLETE, Status.PENDING, Status.PENDING]
    h.status_update(tid, P.TASK_KILLED)
    # offers able to recover A-0 and launch B-0, each also carrying stale reservations to clean
    reserved = _reserved_by(resp.recommendations)
    junk = [U.reserved_cpus(1.0, str(uuid.uuid4())), U.reserved_mem(1.0, str(uuid.uuid4()))]
    offer_a = _offer(*(list(offer_for_a().resources) + reserved + junk))
    offer_b = _offer(*(list(offer_for_b().resources) + reserved + junk))
    offer_c = _offer(*(list(offer_for_b().resources) + reserved + junk))
    assert h.scheduler.get_client_status() == ClientStatusResponse.footprint(True)
    resp = h.scheduler.offers([offer_a, offer_b, offer_c])
    used = {r.offer_id.value for r in resp.recommendations}
    assert used == {offer_a.id.value, offer_b.id.value}
    # deploy's B-0 comes first (executor + task reservations and its volume); recovery's in-place
    # relaunch of A-0 reuses its reservations
    assert op_types(resp.recommendations) == [R, R, R, R, R, R, C, LG, None, LG, None]


def test_configuration_update_waits_for_reconciliation(h):
    step = h.plan().get_children()[0].get_children()[0]
    assert h.scheduler.get_client_status() == ClientStatusResponse.footprint(True)
    offer1 = offer_for_a()
    resp = h.scheduler.offers([offer1])
    assert op_types(resp.recommendations) == FULL_LAUNCH
    tid = launched_task(resp.recommendations).task_id
    assert step.is_starting()
    h.status_update(tid, P.TASK_RUNNING)
    assert step.is_complete()
    assert h.plan(constants.RECOVERY_PLAN_NAME).get_children() == []
    launch = launched_task(resp.recommendations)
    launch_rec = next(r for r in resp.recommendations if isinstance(r, LaunchOfferRecommendation))
    expected = list(launch.resources) + list(launch_rec.executor_info.resources)

    # restart with one more cpu for A
    h.drv.reconciles.clear()
    h.build(service_spec(UPDATED_POD_A, POD_B))
    step = h.plan().get_children()[0].get_children()[0]
    assert step.get_status() == Status.PENDING
    extra_cpu = U.unreserved_cpus(1.0)
    insufficient = U.complete_offer([extra_cpu])
    assert h.scheduler.get_client_status() == ClientStatusResponse.footprint(True)
    resp = h.scheduler.offers([insufficient])
    assert resp.result == OfferResult.NOT_READY and resp.recommendations == []
    assert h.drv.kills == []
    assert step.get_status() == Status.PENDING
    # the restarted scheduler asked the master about its one task
    assert [[s.task_id.value for s in call] for call in h.drv.reconciles] == [[tid.value]]
    h.status_update(tid, P.TASK_RUNNING)
    assert h.scheduler.get_client_status() == ClientStatusResponse.footprint(False)
    resp = h.scheduler.offers([insufficient])
    assert resp.result == OfferResult.PROCESSED and resp.recommendations == []
    assert h.drv.kills == [tid.value]
    assert step.get_status() == Status.PREPARED
    h.status_update(tid, P.TASK_KILLED)
    assert step.get_status() == Status.PREPARED
    assert h.plan(constants.RECOVERY_PLAN_NAME).get_children() == []
    assert h.scheduler.get_client_status() == ClientStatusResponse.footprint(False)
    expected_offer = U.complete_offer(expected + [extra_cpu])
    resp = h.scheduler.offers([expected_offer])
    assert resp.result == OfferResult.PROCESSED
    assert op_types(resp.recommendations) == [R, LG, None]  # grow cpus by the delta, relaunch
    assert resp.recommendations[0].offer_id == expected_offer.id
    assert step.is_starting()
    assert h.plan(constants.RECOVERY_PLAN_NAME).get_children() == []
    h.status_update(launched_task(resp.recommendations).task_id, P.TASK_RUNNING)
    assert step.is_complete()


def test_invalid_configuration_update_keeps_the_target(h):
    test_launch_b(h)
    target = h.scheduler.config_store.get_target_config()
    h.build(service_spec(POD_A, INVALID_POD_B))
    assert h.scheduler.config_store.get_target_config() == target
    errors = h.plan().get_errors()
    assert len(errors) == 1 and "Transition: '2' => '1'" in errors[0]


def test_task_ip_is_stored_on_install(h):
    h.install()
    store = StateStore(h.persister)
    assert state_store_utils.get_task_status_from_property(store, "POD-A-0-A") is not None
    assert state_store_utils.get_task_status_from_property(store, "POD-B-0-B") is not None


def _ip(store, name):
    st = state_store_utils.get_task_status_from_property(store, name)
    return st.container_status.network_infos[0].ip_addresses[0].ip_address


def test_task_ip_is_updated_on_status_update(h):
    ids = h.install()
    store = StateStore(h.persister)
    h.scheduler.task_status(task_status(ids[0], P.TASK_STAGING, "1.1.1.1"))
    assert _ip(store, "POD-A-0-A") == "1.1.1.1"


def test_task_ip_is_not_overwritten_by_an_empty_network(h):
    ids = h.install()
    store = StateStore(h.persister)
    update = task_status(ids[0], P.TASK_STAGING, ip=None)
    update.container_status.network_infos.add()
    h.scheduler.task_status(update)
    assert _ip(store, "POD-A-0-A") == TASK_IP


def test_finished_service_asks_to_uninstall_until_recovery_is_needed(env):
    h = Harness(env, service_spec(POD_A, POD_B, goal=GoalState.FINISH))
    assert not h.plan().is_complete()
    assert h.plan(constants.RECOVERY_PLAN_NAME).is_complete()
    assert h.scheduler.get_client_status() == ClientStatusResponse.footprint(True)
    resp = h.scheduler.offers([])
    assert resp.result == OfferResult.PROCESSED and resp.recommendations == []
    # the offer-less cycle above left A-0 PREPARED
    tid = h.install_step(0, 0, offer_for_a(), Status.PREPARED, False)
    h.install_step(1, 0, offer_for_b(), Status.PENDING, True)
    h.install_step(1, 1, offer_for_b(), Status.PENDING, True)
    assert h.plan().is_complete() and h.plan(constants.RECOVERY_PLAN_NAME).is_complete()
    assert h.scheduler.get_client_status() == ClientStatusResponse.ready_to_uninstall()
    h.status_update(tid, P.TASK_FAILED)
    assert h.scheduler.get_client_status() == ClientStatusResponse.launching(True)
    assert h.plan().is_complete()
    assert not h.plan(constants.RECOVERY_PLAN_NAME).is_complete()
    assert h.statuses(constants.RECOVERY_PLAN_NAME) == [Status.PENDING]
    assert h.scheduler.offers([]).result == OfferResult.PROCESSED
    assert h.scheduler.get_client_status() == ClientStatusResponse.launching(False)
    assert not h.plan(constants.RECOVERY_PLAN_NAME).is_complete()


def test_decommission_plan_is_customized(h):
    seen = []

    class Customizer(PlanCustomizer):
        def update_plan(self, plan):
            if plan.is_decommission_plan():
                seen.append(plan.get_name())
            return plan

    test_launch_b(h)
    h.install_step(1, 1, offer_for_b(), Status.PENDING, True)
    assert h.scheduler.get_client_status() == ClientStatusResponse.idle()
    assert h.statuses() == [Status.COMPLETE] * 3
    SchedulerBuilder(service_spec(POD_A, _pod("POD-B", 1, "B", 2.0, 2000, 2500, allow_decommission=True)),
                     CFG, h.persister).set_plan_customizer(Customizer()).build()
    assert seen == [constants.DECOMMISSION_PLAN_NAME]


def _unexpected(h, resources):
    return h.scheduler.get_unexpected_resources([U.get_offer(resources)])


@pytest.mark.parametrize("mark", ["permanently-failed", "decommissioning"])
def test_unexpected_resources_of_failed_or_decommissioning_tasks(h, mark):
    h.install()
    store = StateStore(h.persister)
    info = store.fetch_tasks()[0]
    assert len(info.resources) > 0
    resp = _unexpected(h, info.resources)
    assert resp.result == UnexpectedResult.PROCESSED and resp.offer_resources == []
    if mark == "permanently-failed":
        store.store_tasks([U.with_failed_flag(info)])
    else:
        store.store_goal_override_status(info.name, DECOMMISSIONING_STATUS)
    resp = _unexpected(h, info.resources)
    assert resp.result == UnexpectedResult.PROCESSED
    assert len(resp.offer_resources) == 1
    assert list(resp.offer_resources[0].resources) == list(info.resources)


def test_unexpected_resources_follow_cleared_and_rewritten_tasks(h):
    """The per-task resource-ID memo is keyed on the stored bytes: clearing a task (or storing it
    again without reservations) turns its offered reservations unexpected on the next pass."""
    h.install()
    store = StateStore(h.persister)
    info = store.fetch_tasks()[0]
    assert _unexpected(h, info.resources).offer_resources == []
    bare = P.TaskInfo()
    bare.CopyFrom(info)
    del bare.resources[:]
    store.store_tasks([bare])
    assert list(_unexpected(h, info.resources).offer_resources[0].resources) == list(info.resources)
    store.store_tasks([info])
    assert _unexpected(h, info.resources).offer_resources == []
    store.clear_task(info.name)
    assert list(_unexpected(h, info.resources).offer_resources[0].resources) == list(info.resources)
    assert info.name not in h.scheduler._expected_ids_cache


def test_unexpected_resources_of_unknown_reservations(h):
    h.install()
    stray = U.reserved_cpus(1.0, "not-a-known-resource")
    unreserved = U.unreserved_cpus(1.0)
    resp = _unexpected(h, [stray, unreserved])
    assert [list(o.resources) for o in resp.offer_resources] == [[stray]]


class RecordingRecorder:
    def __init__(self):
        self.recorded = []

    def record(self, recs):
        self.recorded.append(list(recs))

    def record_decommission(self, recs):
        self.recorded.append(list(recs))


class StubPlanScheduler:
    def __init__(self, recs):
        self.recs = recs

    def resource_offers(self, offers, steps, on_step=None):
        return list(self.recs)


def test_all_recommendations_reach_the_recorders(h):
    offer = U.complete_offer([U.unreserved_cpus(3)])
    info = U.get_task_info([U.unreserved_cpus(3)])
    exe = P.ExecutorInfo()
    exe.executor_id.CopyFrom(U.EXECUTOR_ID)
    launch = LaunchOfferRecommendation(offer, info, exe)
    recs = [StoreTaskInfoRecommendation(offer, info, exe), launch,
            StoreTaskInfoRecommendation(offer, info, exe), StoreTaskInfoRecommendation(offer, info, exe)]
    launch_rec, decom_rec = RecordingRecorder(), RecordingRecorder()
    s = h.scheduler
    s.plan_scheduler = StubPlanScheduler(recs)
    s.launch_recorder, s.decommission_recorder = launch_rec, decom_rec
    resp = s.process_offers([], [])
    assert op_types(resp.recommendations) == [None, LG, None, None]
    assert resp.recommendations == recs
    assert launch_rec.recorded == [recs] and decom_rec.recorded == [recs]


def test_unneeded_tasks_are_killed_on_registration(h):
    h.install()
    store = StateStore(h.persister)
    # a labelled task of an unknown pod type would be decommissioned instead: this one has no labels
    orphan = P.TaskInfo(name="gone-0-task")
    orphan.task_id.CopyFrom(U.to_task_id(U.SERVICE_NAME, "gone-0-task"))
    orphan.agent_id.CopyFrom(U.AGENT_ID)
    store.store_tasks([orphan])
    h.drv.kills.clear()
    h.build(service_spec(POD_A, POD_B))
    assert h.drv.kills == [orphan.task_id.value]


# ---------------------------------------------------------------------------------------
# AbstractScheduler


class MinimalScheduler(AbstractScheduler):
    def __init__(self, store):
        coordinator = types.SimpleNamespace(get_plan_managers=lambda: [], get_candidates=lambda: [])
        super().__init__(None, CFG, store, coordinator)

    def registered_with_mesos(self):
        pass

    def get_status(self):
        return ClientStatusResponse.launching(False)

    def process_offers(self, offers, steps):
        return OfferResponse.processed([])

    def process_status_update(self, status):
        name = state_store_utils.fetch_task_info(self.state_store, status).name
        self.state_store.store_status(name, status)


def test_offers_refused_during_reconciliation(env):
    store = StateStore(MemPersister())
    info = P.TaskInfo(name=U.TASK_NAME)
    info.task_id.CopyFrom(U.TASK_ID)
    info.agent_id.CopyFrom(U.AGENT_ID)
    store.store_tasks([info])
    running = U.generate_status(U.TASK_ID, P.TASK_RUNNING)
    store.store_status(U.TASK_NAME, running)
    s = MinimalScheduler(store)
    s.registered(False)
    offers = [_offer(), _offer(), _offer()]
    assert s.offers(offers).result == OfferResult.NOT_READY
    s.task_status(running)
    assert s.offers(offers).result == OfferResult.PROCESSED


# ---------------------------------------------------------------------------------------
# SchedulerBuilder


MINIMAL = service_spec(textwrap.dedent("""\
    hello:
      count: 1
      tasks:
        server:
          goal: RUNNING
          cmd: echo hello
          cpus: 0.1
          memory: 32
    """))


def _built_spec(spec, cfg, single_region=False, caps=None):
    if caps is not None:
        capabilities.override_capabilities(caps)
    b = SchedulerBuilder(spec, cfg, MemPersister())
    if single_region:
        b.with_single_region_constraint()
    return b.build().service_spec


def test_existing_region_rules_are_left_alone():
    from dataclasses import replace

    remote = pl.RegionRuleFactory.require(pl.ExactMatcher.create(U.REMOTE_REGION))
    local = pl.IsLocalRegionRule()
    base = service_spec(_pod("foo-pod", 1, "t", 1.0, 256, 4096), _pod("bar-pod", 1, "t", 1.0, 256, 4096))
    spec = replace(MINIMAL, pods=MINIMAL.pods + (replace(base.pods[0], placement_rule=remote),
                                                 replace(base.pods[1], placement_rule=local)))
    out = _built_spec(spec, CFG, single_region=True)
    assert isinstance(out.pods[0].placement_rule, pl.IsLocalRegionRule)
    assert out.pods[1].placement_rule is remote
    assert out.pods[2].placement_rule is local


@pytest.mark.parametrize("region,single_region,env_flag,expected", [
    (U.REMOTE_REGION, True, None, "RegionRule"),          # enabled in code
    (U.REMOTE_REGION, False, "true", "RegionRule"),       # enabled by ALLOW_REGION_AWARENESS
    (None, True, None, "IsLocalRegionRule"),              # enabled, but no scheduler region
    (U.REMOTE_REGION, False, "false", "IsLocalRegionRule"),  # disabled
    (None, False, "false", "IsLocalRegionRule"),
])
def test_region_rule_injection(region, single_region, env_flag, expected):
    kw = {}
    if region:
        kw["SERVICE_REGION"] = region
    if env_flag:
        kw["ALLOW_REGION_AWARENESS"] = env_flag
    out = _built_spec(MINIMAL, SchedulerConfig.for_testing(**kw), single_region)
    assert type(out.pods[0].placement_rule).__name__ == expected


def test_domains_not_supported_leave_placement_alone():
    caps = capabilities.Capabilities().with_overrides(supports_domains=False)
    out = _built_spec(MINIMAL, SchedulerConfig.for_testing(SERVICE_REGION=U.REMOTE_REGION), caps=caps)
    assert out.pods[0].placement_rule is None


def _deploy_and_update():
    phase = DefaultPhase("p", [], SerialStrategy())
    return [DefaultPlan(constants.DEPLOY_PLAN_NAME, [phase, phase]), DefaultPlan(constants.UPDATE_PLAN_NAME, [phase])]


def test_update_plan_replaces_deploy_after_deployment():
    plans = SchedulerBuilder.select_deploy_plan(_deploy_and_update(), True)
    assert len(plans) == 1
    assert plans[0].is_deploy_plan() and len(plans[0].get_children()) == 1


def test_deploy_plan_kept_during_install():
    plans = SchedulerBuilder.select_deploy_plan(_deploy_and_update(), False)
    assert len(plans) == 1
    assert plans[0].is_deploy_plan() and len(plans[0].get_children()) == 2


# ---------------------------------------------------------------------------------------
# SchedulerConfig / SchedulerRunner


MINIMAL_ENV = {"PACKAGE_NAME": "test-package", "PACKAGE_VERSION": "1.5", "PACKAGE_BUILD_TIME_EPOCH_MS": "1234567890"}


def _cfg(**kw):
    env = dict(MINIMAL_ENV)
    env.update(kw)
    return SchedulerConfig(EnvStore.from_map(env))


def test_uninstall_flag_is_presence_only():
    for v in ("true", "can be set to anything", ""):
        assert _cfg(SDK_UNINSTALL=v).is_uninstall_enabled()
    assert not _cfg().is_uninstall_enabled()


def test_region_awareness_flag():
    assert _cfg().is_region_awareness_enabled()
    assert not _cfg(ALLOW_REGION_AWARENESS="false").is_region_awareness_enabled()
    assert _cfg(ALLOW_REGION_AWARENESS="true").is_region_awareness_enabled()


def test_hostname_customizations():
    c = _cfg()
    assert (c.autoip_tld(), c.vip_tld(), c.marathon_name()) == (
        "autoip.dcos.thisdcos.directory", "l4lb.thisdcos.directory", "marathon")
    c = _cfg(SERVICE_TLD="test.autoip.tld", VIP_TLD="test.vip.tld", MARATHON_NAME="mom-1")
    assert (c.autoip_tld(), c.vip_tld(), c.marathon_name()) == ("test.autoip.tld", "test.vip.tld", "mom-1")


def test_runner_checks_the_schema_version():
    from dcos_commons_amd.scheduler.scheduler_runner import SchedulerRunner

    persister = MemPersister()
    persister.set("SchemaVersion", b"123")
    builder = SchedulerBuilder(MINIMAL, CFG, persister)
    with pytest.raises(Exception, match="123|[Ss]chema"):
        SchedulerRunner.from_scheduler_builder(builder).run()


# ---------------------------------------------------------------------------------------
# Status updates delivered together (the v1 driver hands over every UPDATE it read at once)


class _CountingPersister(MemPersister):
    def __init__(self):
        super().__init__()
        self.writes = 0
        self.fail_many = False

    def set(self, path, data):
        self.writes += 1
        super().set(path, data)

    def set_many(self, path_bytes):
        self.writes += 1
        if self.fail_many and len(path_bytes) > 2:
            from dcos_commons_amd.storage.persister import PersisterException, Reason
            raise PersisterException(Reason.STORAGE_ERROR, "injected")
        super().set_many(path_bytes)


def _installed(drv, persister):
    hh = Harness.__new__(Harness)
    hh.drv, hh.persister = drv, persister
    FrameworkStore(persister).store_framework_id(U.FRAMEWORK_ID)
    hh.build(service_spec(POD_A, POD_B))
    return hh, hh.install()


def _stored(persister):
    store = StateStore(persister)
    return {n: store.fetch_status(n).state for n in store.fetch_task_names()}, \
        {k: store.fetch_property(k) for k in store.fetch_property_keys()}


def test_status_batch_stores_once_and_matches_one_by_one(env):
    one, ids = _installed(env, _CountingPersister())
    batch, ids_b = _installed(env, _CountingPersister())
    seq = [(0, P.TASK_RUNNING), (1, P.TASK_FAILED), (2, P.TASK_RUNNING), (2, P.TASK_KILLED),
           (0, P.TASK_RUNNING)]
    w0 = one.persister.writes
    for i, st in seq:
        one.scheduler.task_status(task_status(ids[i], st))
    assert one.persister.writes - w0 == len(seq)
    w0 = batch.persister.writes
    resps = batch.scheduler.task_statuses([task_status(ids_b[i], st) for i, st in seq])
    assert batch.persister.writes - w0 == 1          # one transaction for the five updates
    assert [r.result.value for r in resps] == ["PROCESSED"] * len(seq)
    states_1, props_1 = _stored(one.persister)
    states_b, props_b = _stored(batch.persister)
    assert states_1 == states_b == {"POD-A-0-A": P.TASK_RUNNING, "POD-B-0-B": P.TASK_FAILED,
                                    "POD-B-1-B": P.TASK_KILLED}
    def norm(props):
        return {k: P.TaskStatus.FromString(v).state if k.endswith(":task-status") else v for k, v in props.items()}
    assert norm(props_1) == norm(props_b)
    assert one.statuses("recovery") == batch.statuses("recovery")
    assert one.statuses() == batch.statuses() == [Status.COMPLETE] * 3


def test_status_batch_checks_each_status_against_the_one_before(env):
    hh, ids = _installed(env, _CountingPersister())
    bogus = P.TaskID(value="POD-A-0-A__not-launched")
    resps = hh.scheduler.task_statuses([task_status(ids[0], P.TASK_FAILED), task_status(ids[0], P.TASK_UNREACHABLE),
                                        task_status(bogus, P.TASK_RUNNING), task_status(ids[1], P.TASK_RUNNING)])
    assert [r.result.value for r in resps] == ["PROCESSED", "PROCESSED", "UNKNOWN_TASK", "PROCESSED"]
    states, _ = _stored(hh.persister)
    # UNREACHABLE after FAILED in the same batch is dropped, as it is when stored one by one
    assert states["POD-A-0-A"] == P.TASK_FAILED and states["POD-B-0-B"] == P.TASK_RUNNING


def test_status_batch_falls_back_to_one_write_each(env):
    hh, ids = _installed(env, _CountingPersister())
    hh.persister.fail_many = True
    w0 = hh.persister.writes
    hh.scheduler.task_statuses([task_status(ids[i], P.TASK_RUNNING) for i in range(3)])
    assert hh.persister.writes - w0 == 1 + 3
    states, _ = _stored(hh.persister)
    assert set(states.values()) == {P.TASK_RUNNING}


# ---------------------------------------------------------------------------------------
# Launch records written behind the evaluation (scheduler.launch_pipeline)


def _pipelined(drv, persister):
    hh = Harness.__new__(Harness)
    hh.drv, hh.persister = drv, persister
    FrameworkStore(persister).store_framework_id(U.FRAMEWORK_ID)
    cfg = SchedulerConfig.for_testing(SDK_PIPELINE_LAUNCH_WRITES="true")
    s = SchedulerBuilder(service_spec(POD_A, POD_B), cfg, persister).build()
    s.registered(False)
    hh.scheduler = s
    return hh


def test_pipelined_launch_is_recorded_before_it_is_sent(env):
    persister = _CountingPersister()
    hh = _pipelined(env, persister)
    sent = []

    def stream(recs):
        # the ACCEPT goes out only once the TaskInfo is durable
        launch = launched_task(recs)
        assert StateStore(persister).fetch_task(launch.name) is not None
        sent.append(op_types(recs))
    hh.scheduler.get_client_status()
    resp = hh.scheduler.offers([offer_for_a()], launch_stream=stream)
    assert resp.streamed and sent == [FULL_LAUNCH]
    assert op_types(resp.recommendations) == FULL_LAUNCH
    # one writer thread serves the scheduler's cycles; it ends when the scheduler closes
    writer = hh.scheduler._pipeline._thread
    assert writer is not None and writer.is_alive()
    hh.scheduler.close()
    assert not writer.is_alive()


def test_pipelined_launch_whose_record_fails_is_dropped(env):
    persister = _CountingPersister()
    hh = _pipelined(env, persister)
    sent = []
    hh.scheduler.get_client_status()

    def failing_set_many(path_bytes):
        from dcos_commons_amd.storage.persister import PersisterException, Reason
        raise PersisterException(Reason.STORAGE_ERROR, "injected")
    persister.set_many = failing_set_many
    resp = hh.scheduler.offers([offer_for_a()], launch_stream=sent.append)
    assert sent == [] and resp.recommendations == []   # the offer is left unused (declined by the cycle)
    hh.scheduler.close()                               # ends the pipeline's writer thread
