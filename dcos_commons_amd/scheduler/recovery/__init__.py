"""Failure detection and pod recovery (transient restart / permanent replace).

Reference: sdk/.../scheduler/recovery/*.java:
* ``FailureUtils`` (permanently-failed label), ``RecoveryStep``, ``RecoveryPlanOverrider``;
* ``monitor/*``: ``NeverFailureMonitor`` (default), ``TimedFailureMonitor`` (escalates a stopped
  task to permanent after ``permanent-failure-timeout-mins``), ``TestingFailureMonitor``;
* ``DefaultRecoveryPlanManager`` (DefaultRecoveryPlanManager.java:53-453): regenerates the
  parallel ``recovery`` plan on every ``get_candidates`` -- one phase per failed pod, recovery type
  TRANSIENT / PERMANENT / NONE(mixed), overrider phase substitution, in-progress recoveries kept
  unless the failure escalated TRANSIENT -> PERMANENT, dirty-asset exclusion against other plans.
"""
from __future__ import annotations

import logging
import threading
import time
from typing import Callable, Collection, Dict, List, Optional, Set

from dcos_commons_amd.mesos import protos as P
from dcos_commons_amd.offer import constants, task_utils
from dcos_commons_amd.offer.taskdata.labels import TaskException, TaskLabelReader, TaskLabelWriter
from dcos_commons_amd.scheduler.plan import backoff as backoff_mod
from dcos_commons_amd.scheduler.plan.deployment_step import DeploymentStep
from dcos_commons_amd.scheduler.plan.elements import DefaultPhase, DefaultPlan, asset_conflicts, get_dirty_assets
from dcos_commons_amd.scheduler.plan.managers import PlanManager
from dcos_commons_amd.scheduler.plan.pod_instance_requirement import PodInstanceRequirement, RecoveryType
from dcos_commons_amd.scheduler.plan.strategy import ParallelStrategy
from dcos_commons_amd.utils.logging_utils import get_logger

DEFAULT_RECOVERY_PHASE_NAME = "default"


# -- FailureUtils -----------------------------------------------------------------------------

def is_permanently_failed(task_info: P.TaskInfo) -> bool:
    return TaskLabelReader(task_info).is_permanently_failed()


def set_permanently_failed(state_store, tasks: Collection[P.TaskInfo]) -> None:
    updated = []
    for t in tasks:
        c = P.TaskInfo()
        c.CopyFrom(t)
        TaskLabelWriter(c).set_permanently_failed().apply()
        updated.append(c)
    if updated:
        state_store.store_tasks(updated)


def set_pod_permanently_failed(state_store, pod_instance) -> None:
    set_permanently_failed(state_store, task_utils.get_pod_tasks(pod_instance, state_store.fetch_tasks()))


# -- failure monitors -------------------------------------------------------------------------

class FailureMonitor:
    def has_failed(self, task: P.TaskInfo) -> bool:
        raise NotImplementedError


class NeverFailureMonitor(FailureMonitor):
    def has_failed(self, task):
        return False


class DefaultFailureMonitor(FailureMonitor):
    def has_failed(self, task):
        return is_permanently_failed(task)


class TestingFailureMonitor(FailureMonitor):
    __test__ = False  # not a pytest class

    def __init__(self, *failed: P.TaskInfo):
        self.failed = list(failed)

    def set_failed_list(self, *failed: P.TaskInfo) -> None:
        self.failed = list(failed)

    def has_failed(self, task):
        return any(task == f for f in self.failed)


class TimedFailureMonitor(DefaultFailureMonitor):
    def __init__(self, duration_s: float, state_store, config_store, clock: Callable[[], float] = time.time):
        self.duration_s = duration_s
        self.state_store = state_store
        self.config_store = config_store
        self.clock = clock
        self._first_failure: Dict[str, float] = {}
        self._lock = threading.Lock()

    def has_failed(self, task):
        if super().has_failed(task):
            return True
        with self._lock:
            first = self._first_failure.setdefault(task.task_id.value, self.clock())
        expired = self.clock() > first + self.duration_s
        if expired:
            try:
                pi = task_utils.get_pod_instance(self.config_store, task)
                set_pod_permanently_failed(self.state_store, pi)
            except TaskException:
                logging.getLogger(__name__).exception("Failed to get pod instance to mark as failed.")
        return expired


# -- recovery step / overrider -----------------------------------------------------------------

class RecoveryStep(DeploymentStep):
    def start(self) -> None:
        if self.pod_instance_requirement.recovery_type == RecoveryType.PERMANENT:
            set_pod_permanently_failed(self.state_store, self.pod_instance_requirement.pod_instance)

    @property
    def recovery_type(self) -> RecoveryType:
        return self.pod_instance_requirement.recovery_type

    def get_message(self) -> str:
        return f"{super().get_message()} RecoveryType: {self.recovery_type.name}"


class RecoveryPlanOverrider:
    """Returns a replacement phase for a recovery requirement, or None to use the default."""

    def override(self, requirement: PodInstanceRequirement) -> Optional[DefaultPhase]:
        raise NotImplementedError


class RecoveryPlanOverriderFactory:
    def create(self, state_store, plans) -> RecoveryPlanOverrider:
        raise NotImplementedError


# -- the recovery plan manager -----------------------------------------------------------------

class DefaultRecoveryPlanManager(PlanManager):
    def __init__(self, state_store, config_store, recoverable_task_names: Set[str], failure_monitor: FailureMonitor,
                 namespace: Optional[str] = None, overriders: Optional[List[RecoveryPlanOverrider]] = None):
        self.state_store = state_store
        self.config_store = config_store
        self.recoverable_task_names = set(recoverable_task_names)
        self.failure_monitor = failure_monitor
        self.namespace = namespace
        self.overriders = list(overriders or [])
        self._plan = DefaultPlan(constants.RECOVERY_PLAN_NAME, [], ParallelStrategy())
        self._scan_memo: Dict[str, tuple] = {}   # task name -> (info bytes, status bytes, info, status, flags)
        self._lock = threading.RLock()
        self.logger = get_logger(__name__, namespace)

    # ``_plan`` is replaced wholesale (one atomic attribute store) and never mutated in place, so
    # readers and status updates take the current plan without the lock: a status arriving while
    # the offer loop regenerates the plan must not wait for that regeneration. The steps a new
    # plan carries over are the same objects, so an update applied to the outgoing plan lands.
    def get_plan(self):
        return self._plan

    def set_plan(self, plan) -> None:
        raise NotImplementedError("Setting plans on the RecoveryPlanManager is not allowed.")

    def _set_plan_internal(self, plan) -> None:
        with self._lock:
            self._plan = plan

    def get_candidates(self, dirty_assets):
        with self._lock:
            self.update_plan(dirty_assets)
            return self._plan.get_candidates(dirty_assets)

    def update(self, status) -> None:
        self._plan.update(status)

    def get_dirty_assets(self):
        return get_dirty_assets(self._plan)

    def update_plan(self, dirty_assets) -> None:
        with self._lock:
            try:
                new_reqs = self._new_recovery_requirements(dirty_assets)
            except TaskException:
                self.logger.exception("Failed to generate steps.")
                return
            default_reqs, phases = [], []
            for req in new_reqs:
                overridden = False
                for o in self.overriders:
                    ph = o.override(req)
                    if ph is not None:
                        overridden = True
                        phases.append(ph)
                if not overridden:
                    default_reqs.append(req)
            self._set_plan_internal(self._create_plan(default_reqs, phases))

    def _create_plan(self, default_reqs, override_phases):
        override_phases = list(override_phases) + self._create_phases(default_reqs)
        new_reqs = [s.get_pod_instance_requirement() for ph in override_phases for s in ph.get_children()
                    if s.get_pod_instance_requirement() is not None]
        in_progress = [ph for ph in self._plan.get_children()
                       if not any(asset_conflicts(s.get_pod_instance_requirement(), new_reqs)
                                  for s in ph.get_children() if s.get_pod_instance_requirement() is not None)]
        return DefaultPlan(constants.RECOVERY_PLAN_NAME, in_progress + override_phases, ParallelStrategy())

    def _create_phases(self, reqs):
        out = []
        for r in reqs:
            step = RecoveryStep(r.name, r, self.state_store, self.namespace)
            out.append(DefaultPhase(step.get_name(), [step], ParallelStrategy(), []))
        return out

    def _is_task_permanently_failed(self, t: P.TaskInfo) -> bool:
        return is_permanently_failed(t) or self.failure_monitor.has_failed(t)

    def _task_recovery_type(self, infos) -> RecoveryType:
        flags = [self._is_task_permanently_failed(t) for t in infos]
        if all(flags):
            return RecoveryType.PERMANENT
        if not any(flags):
            return RecoveryType.TRANSIENT
        return RecoveryType.NONE

    def _new_recovery_requirements(self, dirty_assets) -> List[PodInstanceRequirement]:
        out = []
        for failed in self._new_failed_pods(dirty_assets):
            pi = failed.pod_instance
            infos = [self.state_store.fetch_task_shared(f"{pi.name}-{t}") for t in failed.tasks_to_launch]
            infos = [i for i in infos if i is not None]
            rtype = self._task_recovery_type(infos)
            if rtype == RecoveryType.NONE:
                self.logger.error("Cannot recover tasks within pod: '%s' due to having recovery type: 'NONE'.",
                                  failed.name)
                continue
            req = failed.with_recovery_type(rtype)
            if not asset_conflicts(req, dirty_assets):
                out.append(req)
        return out

    def _scan(self):
        """Every task's TaskInfo and TaskStatus, plus which tasks need recovery and which were marked
        gone by the operator. The recovery plan is regenerated on every candidate query (each offer
        cycle and status pass, DefaultRecoveryPlanManager.java:164), which made every query parse and
        classify every task of the service; the classification depends only on the task's stored
        TaskInfo and TaskStatus (and the immutable config they point at), so it is kept per task and
        redone only for tasks whose stored bytes changed."""
        infos_b = self.state_store.fetch_tasks_bytes()
        statuses_b = self.state_store.fetch_statuses_bytes(list(infos_b))
        memo, fresh = self._scan_memo, {}
        infos, statuses, needing, gone = [], [], [], []
        for name, ib in infos_b.items():
            sb = statuses_b.get(name)
            hit = memo.get(name)
            if hit is None or hit[0] is not ib or hit[1] is not sb:
                if hit is not None and hit[0] == ib and hit[1] == sb:
                    hit = (ib, sb) + hit[2:]
                else:
                    info = self.state_store.shared_task(name, ib)     # read-only here
                    status = P.TaskStatus.FromString(sb) if sb is not None else None
                    need = (status is not None and
                            bool(task_utils.get_tasks_needing_recovery(self.config_store, [info], [status])))
                    is_gone = (status is not None and status.state == P.TASK_GONE_BY_OPERATOR
                               and status.task_id.value == info.task_id.value
                               and not task_utils.is_permanently_failed(info))
                    hit = (ib, sb, info, status, need, is_gone)
            fresh[name] = hit
            infos.append(hit[2])
            if hit[3] is not None:
                statuses.append(hit[3])
            if hit[4]:
                needing.append(hit[2])
            if hit[5]:
                gone.append(hit[2])
        self._scan_memo = fresh
        return infos, statuses, needing, gone

    def _new_failed_pods(self, dirty_assets) -> List[PodInstanceRequirement]:
        infos, statuses, needing, replace = self._scan()
        if replace:
            set_permanently_failed(self.state_store, replace)
            infos, statuses, needing, _ = self._scan()
        failed_tasks = [t for t in needing if t.name in self.recoverable_task_names]
        if not failed_tasks and not any(not s.is_complete() for ph in self._plan.get_children()
                                        for s in ph.get_children()):
            return []
        failed_pods = task_utils.get_pod_requirements(self.config_store, infos, statuses, failed_tasks,
                                                      backoff_mod.get_instance())
        failed_pods = [p for p in failed_pods if not asset_conflicts(p, dirty_assets)]
        incomplete = [s.get_pod_instance_requirement() for ph in self._plan.get_children()
                      for s in ph.get_children()
                      if not s.is_complete() and s.get_pod_instance_requirement() is not None]
        by_pod: Dict[str, list] = {}
        for r in incomplete:
            by_pod.setdefault(r.pod_instance.name, []).append(r)
        in_progress = []
        for name, reqs in by_pod.items():
            if not self._escalated(infos, reqs[0].pod_instance, reqs):
                in_progress.extend(reqs)
        return [p for p in failed_pods if not asset_conflicts(p, in_progress)]

    def _escalated(self, infos, pod_instance, reqs) -> bool:
        original = (RecoveryType.PERMANENT if any(r.recovery_type == RecoveryType.PERMANENT for r in reqs)
                    else RecoveryType.TRANSIENT)
        current = self._task_recovery_type(task_utils.get_pod_tasks(pod_instance, infos))
        return original == RecoveryType.TRANSIENT and current == RecoveryType.PERMANENT
