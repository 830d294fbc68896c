"""The standard service scheduler.

Reference: sdk/.../scheduler/DefaultScheduler.java:81-585. Wires the plan scheduler, offer
evaluator, launch recorder, decommission recorder, debug trackers and HTTP resources; implements
the status logic (deploy-completion bit, FINISH goal -> uninstall, footprint vs launch), the
unexpected-reservation garbage collector and status-update processing.
"""
from __future__ import annotations

from typing import Dict, Optional

from dcos_commons_amd.framework import task_killer
from dcos_commons_amd.http import endpoint_utils
from dcos_commons_amd.mesos import protos as P
from dcos_commons_amd.offer.evaluate.offer_evaluator import OfferEvaluator
from dcos_commons_amd.offer.history import OfferOutcomeTracker, OfferOutcomeTrackerV2
from dcos_commons_amd.offer.recommendations import LaunchOfferRecommendation
from dcos_commons_amd.offer.resources import get_all_resources, get_resource_id, get_resource_ids
from dcos_commons_amd.offer.taskdata.labels import TaskLabelReader
from dcos_commons_amd.scheduler.abstract_scheduler import AbstractScheduler
from dcos_commons_amd.scheduler.decommission import DECOMMISSIONING_STATUS
from dcos_commons_amd.scheduler.launch_pipeline import LaunchPipeline
from dcos_commons_amd.scheduler.mesos_event_client import (
    ClientStatusResponse,
    OfferResources,
    OfferResponse,
    UnexpectedResourcesResponse,
)
from dcos_commons_amd.scheduler.plan.elements import get_launchable_tasks
from dcos_commons_amd.scheduler.plan.managers import DecommissionPlanManager
from dcos_commons_amd.scheduler.plan.plan_scheduler import PlanScheduler
from dcos_commons_amd.scheduler.plan.pod_instance_requirement import RecoveryType
from dcos_commons_amd.scheduler.plan.status import Status
from dcos_commons_amd.scheduler.recovery import RecoveryStep, is_permanently_failed, set_permanently_failed
from dcos_commons_amd.scheduler.uninstall import UninstallRecorder
from dcos_commons_amd.specification.specs import GoalState
from dcos_commons_amd.state import state_store_utils
from dcos_commons_amd.state.persistent_launch_recorder import PersistentLaunchRecorder


_NEVER_LAUNCHED_STATES = (P.TASK_LOST, P.TASK_DROPPED)
_NEVER_LAUNCHED_REASONS = (P.TaskStatus.REASON_RECONCILIATION, P.TaskStatus.REASON_INVALID_OFFERS)


def _never_launched(info: P.TaskInfo, prev: Optional[P.TaskStatus], status: P.TaskStatus) -> bool:
    """The master reports a task it never saw (dropped ACCEPT, offer gone before the ACCEPT, or
    forgotten) while our only record of it is the write-ahead STAGING status, AND that launch was
    the one meant to create every reservation the task references (``launch_new_footprint``).

    An in-place relaunch (transient recovery, pod restart, config rollout) reuses reservations and
    persistent volumes that exist whether or not its ACCEPT arrived: it never qualifies, so it stays
    a transient LOST and its volumes are kept."""
    return (prev is not None and prev.state == P.TASK_STAGING and prev.task_id.value == status.task_id.value
            and info.task_id.value == status.task_id.value
            and status.source == P.TaskStatus.SOURCE_MASTER and status.state in _NEVER_LAUNCHED_STATES
            and status.reason in _NEVER_LAUNCHED_REASONS and TaskLabelReader(info).is_launch_new_footprint())


def _cfg_pipeline(scheduler_config) -> Optional[bool]:
    fn = getattr(scheduler_config, "pipeline_launch_writes", None)
    return fn() if callable(fn) else None


def _is_working(plan, st: Optional[Status] = None) -> bool:
    st = plan.get_status() if st is None else st
    if st in (Status.PENDING, Status.IN_PROGRESS, Status.PREPARED, Status.STARTED, Status.STARTING):
        return True
    if st in (Status.DELAYED, Status.COMPLETE, Status.ERROR, Status.WAITING):
        return False
    raise ValueError(f"Unsupported status in {plan.get_name()} plan: {st}")


def _is_replacing(recovery_pm) -> bool:
    plan = recovery_pm.get_plan()
    if plan.is_complete():
        return False
    for phase in plan.get_children():
        if phase.is_complete():
            continue
        for step in phase.get_children():
            if not step.is_complete() and isinstance(step, RecoveryStep) and \
                    step.recovery_type == RecoveryType.PERMANENT:
                return True
    return False


class DefaultScheduler(AbstractScheduler):
    def __init__(self, service_spec, scheduler_config, namespace: Optional[str], custom_resources, plan_coordinator,
                 plan_customizer, framework_store, state_store, config_store, template_url_factory=None,
                 custom_endpoint_producers: Optional[Dict] = None, tls_stage_factory=None):
        super().__init__(service_spec, scheduler_config, state_store, plan_coordinator, plan_customizer, namespace)
        self.framework_store = framework_store
        self.config_store = config_store
        self.goal_state = service_spec.goal
        self.custom_resources = list(custom_resources or [])
        self.custom_endpoint_producers = dict(custom_endpoint_producers or {})
        self.launch_recorder = PersistentLaunchRecorder(state_store, service_spec, namespace)
        decom = self._decommission_manager()
        self.decommission_recorder = (UninstallRecorder(state_store, decom.resource_steps)
                                      if decom is not None else None)
        pms = plan_coordinator.get_plan_managers()
        self.deployment_plan_manager = next(pm for pm in pms if pm.get_plan().is_deploy_plan())
        self.recovery_plan_manager = next(pm for pm in pms if pm.get_plan().is_recovery_plan())
        self._deployment_completion_stored = False
        self._expected_ids_cache: Dict[str, tuple] = {}   # task name -> (TaskInfo bytes, resource IDs, perm-failed)
        self._pipeline = None   # LaunchPipeline, False when launch records are written inline
        self.offer_outcome_tracker = None if namespace else OfferOutcomeTracker()
        self.offer_outcome_tracker_v2 = None if namespace else OfferOutcomeTrackerV2()
        if template_url_factory is None:
            template_url_factory = endpoint_utils.template_url_factory(service_spec.name, scheduler_config)
        self.offer_evaluator = OfferEvaluator(
            framework_store, state_store, service_spec.name, config_store.get_target_config(),
            template_url_factory, scheduler_config, namespace, self.offer_outcome_tracker,
            self.offer_outcome_tracker_v2, tls_stage_factory)
        self.plan_scheduler = PlanScheduler(self.offer_evaluator, state_store, namespace)
        self.customize_plans()

    def _decommission_manager(self) -> Optional[DecommissionPlanManager]:
        for pm in self.plan_coordinator.get_plan_managers():
            if pm.get_plan().is_decommission_plan():
                return pm
        return None

    def get_config_store(self):
        return self.config_store

    def get_custom_endpoints(self):
        return self.custom_endpoint_producers

    def get_http_endpoints(self):
        from dcos_commons_amd.http import resources as R

        out = list(self.custom_resources)
        out.append(R.ArtifactResource(self.config_store))
        out.append(R.ConfigResource(self.config_store))
        out.append(R.EndpointsResource(self.state_store, self.service_spec.name, self.scheduler_config,
                                       self.custom_endpoint_producers))
        out.append(R.PlansResource(self.plan_coordinator.get_plan_managers()))
        out.append(R.HealthResource(self.plan_coordinator, self.framework_store))
        out.append(R.PodResource(self.state_store, self.config_store, self.service_spec.name))
        out.append(R.StateResource(self.framework_store, self.state_store))
        out.append(R.DebugResource(self))
        return out

    def registered_with_mesos(self) -> None:
        active = get_launchable_tasks(self.get_plans())
        decom = self._decommission_manager()
        if decom is not None:
            active |= {t.name for t in decom.tasks_to_decommission}
        unneeded = [t for t in self.state_store.fetch_tasks_shared() if t.name not in active]
        if self.scheduler_config.use_legacy_unneeded_task_kills():
            for t in unneeded:
                c = P.TaskInfo()
                c.CopyFrom(t)
                c.task_id.value = ""
                self.state_store.clear_task(t.name)
                self.state_store.store_tasks([c])
            for t in unneeded:
                task_killer.kill_task(t.task_id)
            from dcos_commons_amd.state.goal_state_override import OverrideProgress

            for t in self.state_store.fetch_tasks():
                if self.state_store.fetch_goal_override_status(t.name).progress == OverrideProgress.PENDING:
                    task_killer.kill_task(t.task_id)
        else:
            for t in unneeded:
                task_killer.kill_task(t.task_id)

    def unregistered(self) -> None:
        raise NotImplementedError("Should not have received unregistered call. "
                                  "This is only applicable to UninstallSchedulers")

    def get_status(self) -> ClientStatusResponse:
        pms = self.plan_coordinator.get_plan_managers()
        # each plan's status is an aggregate over all its steps: compute it once per call
        statuses = [pm.get_plan().get_status() for pm in pms]
        all_delayed_or_complete = all(st in (Status.COMPLETE, Status.DELAYED) for st in statuses)
        deploy_st = next((st for pm, st in zip(pms, statuses) if pm is self.deployment_plan_manager), None)
        if deploy_st is None:
            deploy_st = self.deployment_plan_manager.get_plan().get_status()
        deploy_completed = deploy_st == Status.COMPLETE
        if deploy_completed and not self._deployment_completion_stored:
            state_store_utils.set_deployment_was_completed(self.state_store)
            self._deployment_completion_stored = True
        if (self.goal_state == GoalState.FINISH and deploy_completed
                and self.recovery_plan_manager.get_plan().is_complete()):
            return ClientStatusResponse.ready_to_uninstall()
        if all_delayed_or_complete:
            return ClientStatusResponse.idle()
        if not deploy_completed or _is_replacing(self.recovery_plan_manager):
            return ClientStatusResponse.footprint(self.work_set_tracker.has_new_work())
        if any(_is_working(pm.get_plan(), st) for pm, st in zip(pms, statuses)):
            return ClientStatusResponse.launching(self.work_set_tracker.has_new_work())
        return ClientStatusResponse.idle()

    supports_launch_stream = True

    def prewarm(self, stop=lambda: False) -> None:
        """Before the first offers: the offer evaluator's templates for the first candidate step
        of each pod type (``OfferEvaluator.prewarm``), until ``stop()``."""
        if not self.scheduler_config.is_offer_prewarm() or stop():
            return
        seen = set()
        for step in self.plan_coordinator.get_candidates():
            if not step.is_pending():
                continue
            req = step.get_pod_instance_requirement()
            if req is None or req.pod_instance.pod.type in seen:
                continue
            seen.add(req.pod_instance.pod.type)
            if stop() or not self.plan_scheduler.offer_evaluator.prewarm(req, stop):
                return

    def _record(self, recs) -> bool:
        """Write-ahead: persist the launches before anything is sent to the master."""
        try:
            self.launch_recorder.record(recs)
            if self.decommission_recorder is not None:
                self.decommission_recorder.record_decommission(recs)
        except Exception:  # noqa: BLE001
            self.logger.exception("Failed to record offer operations, dropping them")
            return False
        if self.launch_watchdog.enabled:
            for r in recs:
                if isinstance(r, LaunchOfferRecommendation):
                    st = P.TaskStatus(state=P.TASK_STAGING)
                    st.task_id.CopyFrom(r.task_info.task_id)
                    st.agent_id.CopyFrom(r.task_info.agent_id)
                    self.launch_watchdog.launched(st)
        return True

    def process_offers(self, offers, steps, launch_stream=None) -> OfferResponse:
        if launch_stream is None:
            recs = self.plan_scheduler.resource_offers(offers, steps)
            return OfferResponse.processed(recs if self._record(recs) else [])

        # Launch streaming: each step's launch is recorded and sent to the master as soon as the
        # step is matched, so pods launch (and their agents start them) while later steps are
        # still being evaluated, instead of after the whole cycle.
        pipeline = self._launch_pipeline()
        if pipeline is None:
            def on_step(recs):
                if not self._record(recs):
                    return []
                launch_stream(recs)
                return recs
            return OfferResponse.processed(self.plan_scheduler.resource_offers(offers, steps, on_step),
                                           streamed=True)

        # ... and with a remote persister the records are written behind the evaluation
        # (scheduler.launch_pipeline): ACCEPTs still follow their durable record, in step order
        def on_step_pipelined(recs):
            pipeline.submit(recs, launch_stream)
            return recs
        try:
            recs = self.plan_scheduler.resource_offers(offers, steps, on_step_pipelined)
        finally:
            failed = pipeline.drain()
        if failed:
            dropped = {id(r) for batch in failed for r in batch}
            recs = [r for r in recs if id(r) not in dropped]
        return OfferResponse.processed(recs, streamed=True)

    def close(self) -> None:
        """Ends the launch writer thread (scheduler shutdown)."""
        if self._pipeline:
            self._pipeline.close()

    def _launch_pipeline(self):
        if self._pipeline is None:
            on = _cfg_pipeline(self.scheduler_config)
            if on is None:
                on = getattr(self.state_store.persister, "remote", False)
            self._pipeline = LaunchPipeline(self._record) if on else False
        return self._pipeline or None

    def get_unexpected_resources(self, unused_offers) -> UnexpectedResourcesResponse:
        if not any(get_resource_id(r) is not None for offer in unused_offers for r in offer.resources):
            # nothing reserved by this SDK in the leftover offers: no need to load every task to
            # learn which reservations are still expected
            return UnexpectedResourcesResponse.processed([])
        offered = {rid for offer in unused_offers for r in offer.resources
                   for rid in (get_resource_id(r),) if rid is not None}
        try:
            # Only the expected IDs that appear in the offers decide anything, so a task whose
            # reservations are not offered is skipped before its goal override is read; each
            # task's IDs are memoized on its exact stored bytes (an unchanged TaskInfo is not
            # parsed again on every offer cycle).
            keep = set()
            cache = self._expected_ids_cache
            names = self.state_store.fetch_tasks_bytes()
            for name, data in names.items():
                hit = cache.get(name)
                if hit is None or hit[0] != data:
                    t = self.state_store.shared_task(name, data)
                    hit = cache[name] = (data, frozenset(get_resource_ids(get_all_resources(t))),
                                         is_permanently_failed(t))
                _, ids, failed = hit
                if failed or ids.isdisjoint(offered):
                    continue
                if self.state_store.fetch_goal_override_status(name) == DECOMMISSIONING_STATUS:
                    continue
                keep.update(ids)
            if len(cache) > len(names):
                for gone in set(cache) - set(names):
                    del cache[gone]
        except Exception:  # noqa: BLE001
            self.logger.exception("Failed to fetch expected tasks to determine unexpected resources")
            return UnexpectedResourcesResponse.failed([])
        unexpected = []
        for offer in unused_offers:
            o = OfferResources(offer)
            for r in offer.resources:
                rid = get_resource_id(r)
                if rid is not None and rid not in keep:
                    o.add(r)
            if o.resources:
                unexpected.append(o)
        if self.decommission_recorder is not None:
            try:
                self.decommission_recorder.record_cleanup_or_uninstall(unexpected)
            except Exception:  # noqa: BLE001
                self.logger.exception("Failed to record unexpected resources in decommission recorder")
                return UnexpectedResourcesResponse.failed([])
        return UnexpectedResourcesResponse.processed(unexpected)

    def process_status_update(self, status: P.TaskStatus) -> None:
        name, props = self._prepare_status(status)
        self.state_store.store_status(name, status, props)
        self._apply_status(status)

    def _prepare_status(self, status: P.TaskStatus):
        """What storing ``status`` needs: its task's name and the properties written with it."""
        info = state_store_utils.fetch_task_info(self.state_store, status)
        name = info.name
        if (self.unknown_as_lost and status.state in _NEVER_LAUNCHED_STATES
                and status.reason in _NEVER_LAUNCHED_REASONS
                and _never_launched(info, self.state_store.fetch_status(name), status)):
            # A first-footprint launch was recorded (write-ahead) but its ACCEPT never took
            # effect, so the reservations in the stored TaskInfo were never made and an in-place
            # relaunch would wait for them forever. Mark it permanently failed: the step relaunches
            # with a fresh footprint and anything that was reserved is garbage-collected.
            self.logger.warning("Launch of %s never reached the master (%s, %s): relaunching with new reservations",
                                name, P.TaskState.Name(status.state), P.TaskStatus.Reason.Name(status.reason))
            set_permanently_failed(self.state_store, [info])
        # a status carrying IP addresses is also kept as the `<task>:task-status` property
        # (StateStoreUtils.storeTaskStatusAsProperty), written in the same transaction
        props = None
        if status.HasField("container_status") and any(
                len(ni.ip_addresses) > 0 for ni in status.container_status.network_infos):
            props = {name + state_store_utils.PROPERTY_TASK_INFO_SUFFIX: status.SerializeToString()}
        return name, props

    def _apply_status(self, status: P.TaskStatus) -> None:
        for pm in self.plan_coordinator.get_plan_managers():
            pm.update(status)

    def status_reads_history(self, status: P.TaskStatus) -> bool:
        # the never-launched check compares the status with the stored one
        return self.unknown_as_lost and status.state in _NEVER_LAUNCHED_STATES

    def process_status_updates(self, statuses) -> list:
        """Statuses that arrived together: stored in one transaction, then applied to the plans in
        arrival order. Returns each status's error (None when processed)."""
        errors: list = [None] * len(statuses)
        prepared = []
        for i, status in enumerate(statuses):
            try:
                name, props = self._prepare_status(status)
                prepared.append((i, name, props))
            except Exception as e:  # noqa: BLE001
                errors[i] = e
        stored = self.state_store.store_statuses([(name, statuses[i], props) for i, name, props in prepared])
        for (i, _, _), err in zip(prepared, stored):
            if err is not None:
                errors[i] = err
                continue
            try:
                self._apply_status(statuses[i])
            except Exception as e:  # noqa: BLE001
                errors[i] = e
        return errors

    def to_uninstall_scheduler(self):
        from dcos_commons_amd.scheduler.uninstall import UninstallScheduler

        return UninstallScheduler(self.service_spec, self.state_store, self.config_store, self.scheduler_config,
                                  self.plan_customizer, self.namespace, self.framework_store)
