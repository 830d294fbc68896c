"""Pod decommissioning when ``count`` shrinks on a pod with ``allow-decommission``.

Reference: sdk/.../scheduler/decommission/{DecommissionPlanFactory,TriggerDecommissionStep,
EraseTaskStateStep}.java. One phase per pod instance to remove, highest index first (and pod
types in reverse spec order): mark DECOMMISSIONED + kill, unreserve each resource as it is
re-offered, then erase the task from the StateStore.
"""
from __future__ import annotations

import logging
from typing import Dict, List, Optional, Tuple

from dcos_commons_amd.framework import task_killer
from dcos_commons_amd.mesos import protos as P
from dcos_commons_amd.offer import constants
from dcos_commons_amd.offer.resources import get_all_resources_of, get_resource_ids
from dcos_commons_amd.offer.taskdata.labels import TaskException, TaskLabelReader
from dcos_commons_amd.scheduler.plan.elements import DefaultPhase, DefaultPlan
from dcos_commons_amd.scheduler.plan.status import Status
from dcos_commons_amd.scheduler.plan.strategy import SerialStrategy
from dcos_commons_amd.scheduler.uninstall import ResourceCleanupStep, UninstallStep
from dcos_commons_amd.state.goal_state_override import GoalStateOverride, OverrideProgress, OverrideStatus

LOGGER = logging.getLogger(__name__)
DECOMMISSIONING_STATUS = OverrideStatus(GoalStateOverride.DECOMMISSIONED, OverrideProgress.IN_PROGRESS)


class TriggerDecommissionStep(UninstallStep):
    def __init__(self, state_store, task_info: P.TaskInfo, namespace: Optional[str] = None):
        super().__init__("kill-" + task_info.name, namespace)
        self.state_store = state_store
        self.task_info = task_info

    def start(self) -> None:
        self._set_status(Status.IN_PROGRESS)
        self.state_store.store_goal_override_status(self.task_info.name, DECOMMISSIONING_STATUS)
        task_killer.kill_task(self.task_info.task_id)
        self._set_status(Status.COMPLETE)


class EraseTaskStateStep(UninstallStep):
    def __init__(self, state_store, task_name: str, namespace: Optional[str] = None):
        super().__init__("erase-" + task_name, namespace)
        self.state_store = state_store
        self.task_name = task_name

    def start(self) -> None:
        self.state_store.clear_task(self.task_name)
        self._set_status(Status.COMPLETE)


def get_pods_to_decommission(service_spec, tasks) -> List[Tuple[Tuple, List[P.TaskInfo]]]:
    ordered_types = [p.type for p in service_spec.pods]
    ordered_types.reverse()
    expected = {p.type: p.count for p in service_spec.pods}
    pods: Dict[Tuple, List[P.TaskInfo]] = {}
    for t in tasks:
        try:
            r = TaskLabelReader(t)
            ptype, idx = r.get_type(), r.get_index()
        except (TaskException, ValueError):
            LOGGER.error("Failed to retrieve task metadata. Omitting task from decommission: %s", t.name)
            continue
        exp = expected.get(ptype)
        if exp is not None and idx < exp:
            continue
        type_index = ordered_types.index(ptype) if ptype in ordered_types else -1
        pods.setdefault((type_index, ptype, idx), []).append(t)

    def sort_key(k):
        type_index, ptype, idx = k
        return (type_index, ptype if type_index == -1 else "", -idx)

    return [(k, pods[k]) for k in sorted(pods, key=sort_key)]


class DecommissionPlanFactory:
    def __init__(self, service_spec, state_store, namespace: Optional[str] = None):
        all_tasks = state_store.fetch_tasks_shared()
        self.pods_to_decommission = get_pods_to_decommission(service_spec, all_tasks)
        to_decom = {t.name for _, ts in self.pods_to_decommission for t in ts}
        for t in all_tasks:
            cur = state_store.fetch_goal_override_status(t.name)
            if t.name in to_decom:
                if cur.target != GoalStateOverride.DECOMMISSIONED:
                    state_store.store_goal_override_status(
                        t.name, OverrideStatus(GoalStateOverride.DECOMMISSIONED, OverrideProgress.PENDING))
            elif cur.target == GoalStateOverride.DECOMMISSIONED:
                state_store.store_goal_override_status(t.name, OverrideStatus.INACTIVE)
        self.resource_steps: List[ResourceCleanupStep] = []
        self.plan: Optional[DefaultPlan] = None
        if not self.pods_to_decommission:
            return
        phases = []
        for (_, ptype, idx), tasks in self.pods_to_decommission:
            steps = [TriggerDecommissionStep(state_store, t, namespace) for t in tasks]
            rsteps = [ResourceCleanupStep(rid, namespace) for rid in get_resource_ids(get_all_resources_of(tasks))]
            self.resource_steps.extend(rsteps)
            steps.extend(rsteps)
            steps.extend(EraseTaskStateStep(state_store, t.name, namespace) for t in tasks)
            phases.append(DefaultPhase(f"{ptype}-{idx}", steps, SerialStrategy(), []))
        self.plan = DefaultPlan(constants.DECOMMISSION_PLAN_NAME, phases)

    def get_plan(self) -> Optional[DefaultPlan]:
        return self.plan

    def get_resource_steps(self) -> List[ResourceCleanupStep]:
        return self.resource_steps

    def get_tasks_to_decommission(self) -> List[P.TaskInfo]:
        return [t for _, ts in self.pods_to_decommission for t in ts]
