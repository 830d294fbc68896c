"""Service uninstall: kill everything, unreserve everything, deregister.

Reference: sdk/.../scheduler/uninstall/*.java. The uninstall plan is served as ``deploy``:
``kill-tasks`` (parallel) -> ``unreserve-resources-<host>`` (one step per resource_id) ->
optional ``tls-cleanup`` -> ``deregister-service``, gated by a DependencyStrategy
(UninstallPlanFactory.java:42-152). ``UninstallRecorder`` tombstones resource IDs as they are
unreserved (UninstallRecorder.java:24).
"""
from __future__ import annotations

import logging
import time
from typing import Callable, Collection, Dict, List, Optional, Set

from dcos_commons_amd.framework import task_killer
from dcos_commons_amd.mesos import protos as P
from dcos_commons_amd.offer import constants
from dcos_commons_amd.offer.resources import get_all_resources, get_resource_id, get_resource_ids, has_resource_id
from dcos_commons_amd.offer.recommendations import UninstallRecommendation
from dcos_commons_amd.offer.task_utils import has_tasks_with_tls
from dcos_commons_amd.offer.taskdata.labels import TaskException, TaskLabelReader
from dcos_commons_amd.scheduler.mesos_event_client import (
    ClientStatusResponse,
    OfferResources,
    OfferResponse,
    UnexpectedResourcesResponse,
)
from dcos_commons_amd.scheduler.plan.elements import AbstractStep, DefaultPhase, DefaultPlan
from dcos_commons_amd.scheduler.plan.managers import DefaultPlanManager
from dcos_commons_amd.scheduler.plan.status import Status
from dcos_commons_amd.scheduler.plan.strategy import (
    DependencyStrategy,
    DependencyStrategyHelper,
    ParallelStrategy,
    SerialStrategy,
)
from dcos_commons_amd.state import state_store_utils

LOGGER = logging.getLogger(__name__)
TASK_KILL_PHASE = "kill-tasks"
RESOURCE_PHASE_PREFIX = "unreserve-resources-"
TLS_CLEANUP_PHASE = "tls-cleanup"
DEREGISTER_PHASE = "deregister-service"


class UninstallStep(AbstractStep):
    def get_pod_instance_requirement(self):
        return None

    def update_offer_status(self, recommendations) -> None:
        pass

    def get_errors(self):
        return []

    def update(self, status) -> None:
        pass


class TaskKillStep(UninstallStep):
    def __init__(self, task_id: P.TaskID, namespace: Optional[str] = None):
        super().__init__("kill-task-" + task_id.value, namespace)
        self.task_id = task_id

    def start(self) -> None:
        self._set_status(Status.IN_PROGRESS)
        task_killer.kill_task(self.task_id)
        self._set_status(Status.COMPLETE)


class ResourceCleanupStep(UninstallStep):
    def __init__(self, resource_id: str, namespace: Optional[str] = None):
        super().__init__("unreserve-" + resource_id, namespace)
        self.resource_id = resource_id

    def start(self) -> None:
        if self.is_pending():
            self._set_status(Status.PREPARED)

    def update_resource_status(self, uninstalled: Set[str]) -> None:
        if self.resource_id in uninstalled:
            self._set_status(Status.COMPLETE)


class DeregisterStep(UninstallStep):
    def __init__(self, namespace: Optional[str] = None):
        super().__init__("deregister", namespace)

    def start(self) -> None:
        if self.is_pending():
            self._set_status(Status.PREPARED)

    def set_complete(self) -> None:
        self._set_status(Status.COMPLETE)


class TLSCleanupStep(AbstractStep):
    def __init__(self, secrets_client, secrets_namespace: str, namespace: Optional[str] = None):
        super().__init__("tls-cleanup", namespace)
        self.secrets_client = secrets_client
        self.secrets_namespace = secrets_namespace

    def start(self) -> None:
        from dcos_commons_amd.offer.evaluate.security import known_tls_artifacts

        try:
            for path in known_tls_artifacts(self.secrets_client.list(self.secrets_namespace)):
                self.secrets_client.delete(f"{self.secrets_namespace}/{path}")
            self._set_status(Status.COMPLETE)
        except Exception:  # noqa: BLE001
            self.logger.exception("Failed to clean up secrets in namespace %s", self.secrets_namespace)
            self._set_status(Status.ERROR)


def get_resource_ids_by_agent_host(state_store) -> Dict[str, Set[str]]:
    """SchedulerUtils.getResourceIdsByAgentHost."""
    from dcos_commons_amd.scheduler.recovery import is_permanently_failed

    tasks = state_store.fetch_tasks()
    error_ids = {s.task_id.value for s in state_store.fetch_statuses() if s.state == P.TASK_ERROR}
    out: Dict[str, Set[str]] = {}
    for t in tasks:
        if is_permanently_failed(t) and t.task_id.value in error_ids:
            continue
        try:
            host = TaskLabelReader(t).get_hostname()
        except TaskException:
            host = "UNKNOWN_AGENT"
        out.setdefault(host, set()).update(get_resource_ids(get_all_resources(t)))
    return dict(sorted(out.items()))


def _has_tls_artifacts(secrets_client, secrets_namespace: str) -> bool:
    from dcos_commons_amd.offer.evaluate.security import known_tls_artifacts

    try:
        return bool(known_tls_artifacts(secrets_client.list(secrets_namespace)))
    except Exception:  # noqa: BLE001 -- the store is unreachable: keep the reference's spec-only rule
        LOGGER.warning("Could not list the secret store: TLS artifacts of earlier configs may stay behind")
        return False


class UninstallPlanFactory:
    def __init__(self, service_spec, state_store, scheduler_config, namespace: Optional[str] = None,
                 secrets_client=None):
        phases = []
        kill_steps = [TaskKillStep(t.task_id, namespace) for t in state_store.fetch_tasks()]
        phases.append(DefaultPhase(TASK_KILL_PHASE, kill_steps, ParallelStrategy(), []))
        self.resource_cleanup_steps: List[ResourceCleanupStep] = []
        for host, ids in get_resource_ids_by_agent_host(state_store).items():
            steps = [ResourceCleanupStep(rid, namespace) for rid in sorted(ids)]
            self.resource_cleanup_steps.extend(steps)
            phases.append(DefaultPhase(RESOURCE_PHASE_PREFIX + host, list(steps), ParallelStrategy(), []))
        secrets_ns = scheduler_config.secrets_namespace(service_spec.name)
        if secrets_client is not None and (has_tasks_with_tls(service_spec)
                                           or _has_tls_artifacts(secrets_client, secrets_ns)):
            # Unlike the reference (UninstallPlanFactory.java:110-115), artifacts left by an earlier
            # configuration that had TLS turned on are found too: the secret store is listed.
            phases.append(DefaultPhase(TLS_CLEANUP_PHASE, [TLSCleanupStep(secrets_client, secrets_ns, namespace)],
                                       SerialStrategy(), []))
        self.deregister_step = DeregisterStep(namespace)
        dereg = DefaultPhase(DEREGISTER_PHASE, [self.deregister_step], SerialStrategy(), [])
        helper = DependencyStrategyHelper(phases)
        helper.add_element(dereg)
        for ph in phases:
            helper.add_dependency(dereg, ph)
        phases.append(dereg)
        self.plan = DefaultPlan(constants.DEPLOY_PLAN_NAME, phases, DependencyStrategy(helper))


class UninstallRecorder:
    def __init__(self, state_store, resource_steps: Collection[ResourceCleanupStep]):
        self.state_store = state_store
        self.resource_steps = list(resource_steps)

    @staticmethod
    def _filter(resources, remove: Set[str]):
        if len(resources) == 0:
            return None
        any_update = False
        out = []
        for r in resources:
            rid = get_resource_id(r)
            if rid is not None and rid in remove:
                any_update = True
            else:
                out.append(r)
        return out if any_update else None

    def _record(self, ids: Set[str]) -> None:
        updated = []
        for t in self.state_store.fetch_tasks():
            tr = self._filter(t.resources, ids)
            er = self._filter(t.executor.resources, ids)
            if tr is None and er is None:
                continue
            c = P.TaskInfo()
            c.CopyFrom(t)
            if tr is not None:
                del c.resources[:]
                c.resources.extend(tr)
            if er is not None:
                del c.executor.resources[:]
                c.executor.resources.extend(er)
            updated.append(c)
        if updated:
            self.state_store.store_tasks(updated)
        for s in self.resource_steps:
            s.update_resource_status(ids)

    def record_decommission(self, recommendations) -> None:
        ids = set(get_resource_ids([r.resource for r in recommendations if isinstance(r, UninstallRecommendation)]))
        if ids:
            self._record(ids)

    def record_cleanup_or_uninstall(self, offer_resources) -> None:
        self._record({rid for o in offer_resources for rid in get_resource_ids(o.resources)})


class _SinglePlanCoordinator:
    def __init__(self, manager):
        self.manager = manager

    def get_candidates(self):
        return list(self.manager.get_candidates([]))

    def get_plan_managers(self):
        return [self.manager]


class UninstallScheduler:
    """Serves the uninstall plan (as ``deploy``) until the framework can be removed."""

    def __init__(self, service_spec, state_store, config_store, scheduler_config, plan_customizer=None,
                 namespace: Optional[str] = None, framework_store=None, secrets_client=None,
                 clock_ms: Callable[[], float] = lambda: time.time() * 1000):
        from dcos_commons_amd.scheduler.abstract_scheduler import AbstractScheduler

        self._base = AbstractScheduler  # for isinstance-free reuse below
        self.service_spec = service_spec
        self.state_store = state_store
        self.config_store = config_store
        self.scheduler_config = scheduler_config
        self.plan_customizer = plan_customizer
        self.namespace = namespace
        self.framework_store = framework_store
        self.clock_ms = clock_ms
        self.logger = logging.getLogger(__name__ + (f"({namespace})" if namespace else ""))
        if not state_store_utils.is_uninstalling(state_store):
            self.logger.info("Service has been told to uninstall. Marking this in the persistent state store. "
                             "Uninstall cannot be canceled once triggered.")
            state_store_utils.set_uninstalling(state_store)
        has_account = bool(scheduler_config.env.get_optional("DCOS_SERVICE_ACCOUNT_CREDENTIAL", None))
        if secrets_client is None and (has_tasks_with_tls(service_spec) or has_account):
            # UninstallScheduler.java:90-105: TLS secrets are cleaned up with the service account's token
            # (with an account but no TLS in the current spec: artifacts of earlier TLS configs)
            try:
                from dcos_commons_amd.dcos.clients import DcosHttpExecutor, SecretsClient

                secrets_client = SecretsClient(DcosHttpExecutor(scheduler_config.dcos_auth_token_provider()))
            except Exception as e:  # noqa: BLE001
                self.logger.error("Failed to create a secrets store client, TLS artifacts possibly won't be "
                                  "cleaned up from secrets store: %s", e)
        factory = UninstallPlanFactory(service_spec, state_store, scheduler_config, namespace, secrets_client)
        self.recorder = UninstallRecorder(state_store, factory.resource_cleanup_steps)
        self.deregister_step = factory.deregister_step
        self.plan_manager = DefaultPlanManager.create_proceeding(factory.plan)
        if scheduler_config.is_uninstall_enabled():
            self.deadline_ms = None
            self.timeout_s = -1
        else:
            self.timeout_s = scheduler_config.multi_service_removal_timeout_s()
            self.deadline_ms = None if self.timeout_s <= 0 else clock_ms() + self.timeout_s * 1000
        if plan_customizer is not None:
            self.plan_manager.set_plan(plan_customizer.update_uninstall_plan(self.plan_manager.get_plan()))
        self.plan_coordinator = _SinglePlanCoordinator(self.plan_manager)
        from dcos_commons_amd.scheduler.reconciliation import ExplicitReconciler, WorkSetTracker

        self.work_set_tracker = WorkSetTracker(namespace)
        self.reconciler = ExplicitReconciler(state_store, namespace)
        self._candidates = []

    # MesosEventClient
    def registered(self, re_registered: bool) -> None:
        if not re_registered:
            from dcos_commons_amd.scheduler.reconciliation import ExplicitReconciler, WorkSetTracker

            self.work_set_tracker = WorkSetTracker(self.namespace)
            self.reconciler = ExplicitReconciler(self.state_store, self.namespace)
        self.reconciler.start()
        self.reconciler.reconcile()

    def unregistered(self) -> None:
        self.deregister_step.set_complete()

    def get_plans(self):
        return [self.plan_manager.get_plan()]

    def get_client_status(self) -> ClientStatusResponse:
        self._candidates = self.plan_coordinator.get_candidates()
        in_progress = {s for s in self.plan_manager.get_plan().get_children() for s in s.get_children()
                       if s.is_running()}
        self.work_set_tracker.update_work_set(list(self._candidates) + list(in_progress))
        if self.deregister_step.is_running() or self.deregister_step.is_complete():
            return ClientStatusResponse.ready_to_remove()
        if self.deadline_ms is not None and self.clock_ms() > self.deadline_ms:
            self.logger.error("Failed to complete uninstall within %ss timeout, forcing cleanup. Plan was: %s",
                              self.timeout_s, self.plan_manager.get_plan())
            return ClientStatusResponse.ready_to_remove()
        return ClientStatusResponse.launching(self.work_set_tracker.has_new_work())

    def offers(self, offers, launch_stream=None) -> OfferResponse:
        self.reconciler.reconcile()
        if not self.reconciler.is_reconciled():
            return OfferResponse.not_ready([])
        for s in self._candidates:
            s.start()
            if s is self.deregister_step and s.is_running():
                self._recheck = True
        return OfferResponse.processed([])

    def awaiting_reconciliation(self) -> bool:
        return self.reconciler is None or not self.reconciler.is_reconciled()

    def consume_recheck_request(self) -> bool:
        """True once after the deregister step started: the offer loop re-checks the client
        status immediately and tears the framework down without waiting for the next poll."""
        r, self._recheck = getattr(self, "_recheck", False), False
        return r

    def get_unexpected_resources(self, unused_offers) -> UnexpectedResourcesResponse:
        unexpected = [OfferResources(o, [r for r in o.resources if has_resource_id(r)]) for o in unused_offers]
        try:
            self.recorder.record_cleanup_or_uninstall(unexpected)
        except Exception:  # noqa: BLE001
            self.logger.exception("Failed to record unexpected resources")
            return UnexpectedResourcesResponse.failed([])
        return UnexpectedResourcesResponse.processed(unexpected)

    def task_status(self, status):
        from dcos_commons_amd.scheduler.mesos_event_client import TaskStatusResponse
        from dcos_commons_amd.state import state_store_utils as ssu
        from dcos_commons_amd.state.state_store import StateStoreException
        from dcos_commons_amd.storage.persister import Reason

        try:
            name = ssu.fetch_task_info(self.state_store, status).name
            self.state_store.store_status(name, status)
            self.reconciler.update(status)
        except StateStoreException as e:
            if e.reason == Reason.NOT_FOUND:
                return TaskStatusResponse.unknown_task()
            self.logger.warning("Failed to update TaskStatus: %s", e)
        return TaskStatusResponse.processed()

    def get_http_endpoints(self):
        from dcos_commons_amd.http.resources import HealthResource, PlansResource

        return [PlansResource([self.plan_manager]), HealthResource(self.plan_coordinator, None)]

    def get_config_store(self):
        return self.config_store

    def get_custom_endpoints(self):
        return {}
