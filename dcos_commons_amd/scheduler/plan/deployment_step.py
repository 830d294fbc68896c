"""The step that launches (a subset of) a pod instance's tasks and tracks them to goal state.

Reference: sdk/.../scheduler/plan/DeploymentStep.java:37-405. The ``update(TaskStatus)`` state
machine (:163) maps FAILED/ERROR -> DELAYED (+backoff), KILLED/LOST/GONE/... -> PENDING,
RUNNING with readiness passed -> COMPLETE (else STARTED), FINISHED -> COMPLETE for goal
FINISH/ONCE (PENDING for goal RUNNING). The step status is the minimum over its tasks (:344).
"""
from __future__ import annotations

from typing import Dict, List, Optional

from dcos_commons_amd.mesos import protos as P
from dcos_commons_amd.offer import common_id_utils
from dcos_commons_amd.offer.taskdata.labels import TaskException, TaskLabelReader
from dcos_commons_amd.scheduler.plan import backoff as backoff_mod
from dcos_commons_amd.specification.specs import GoalState
from dcos_commons_amd.state.goal_state_override import (
    GoalStateOverride,
    OverrideProgress,
    OverrideStatus,
)

from .elements import AbstractStep, bump_status_generation
from .pod_instance_requirement import PodInstanceRequirement
from .status import Status


def compute_status(statuses, has_errors: bool, is_prepared: bool) -> Optional[Status]:
    """DeploymentStep.getStatus(Set<Status>, hasErrors, isPrepared)."""
    if has_errors:
        return Status.ERROR
    if not statuses:
        return Status.PREPARED if is_prepared else Status.PENDING
    for s in (Status.ERROR, Status.DELAYED, Status.PENDING, Status.PREPARED, Status.STARTING, Status.STARTED):
        if s in statuses:
            return s
    if Status.COMPLETE in statuses and len(statuses) == 1:
        return Status.COMPLETE
    return None


class DeploymentStep(AbstractStep):
    def __init__(self, name: str, pod_instance_requirement: PodInstanceRequirement, state_store,
                 namespace: Optional[str] = None):
        super().__init__(name, namespace)
        self.state_store = state_store
        self.pod_instance_requirement = pod_instance_requirement
        pi = pod_instance_requirement.pod_instance
        self.goal_state_by_task_name: Dict[str, GoalState] = {
            f"{pi.name}-{t.name}": t.goal for t in pi.pod.tasks}
        self._errors: List[str] = []
        self._parameters: Dict[str, str] = {}
        # task_id value -> [TaskInfo, Status]
        self._tasks: Dict[str, list] = {}
        self._prepared = False
        self._update_status()

    def add_error(self, error: str) -> "DeploymentStep":
        self._errors.append(error)
        bump_status_generation()
        self._update_status()
        return self

    def update_initial_status(self, status: Status) -> "DeploymentStep":
        self._set_status(status)
        return self

    def update_parameters(self, parameters: Dict[str, str]) -> None:
        self._parameters = dict(parameters)

    def start(self) -> None:
        pass

    def get_pod_instance_requirement(self) -> Optional[PodInstanceRequirement]:
        return self.pod_instance_requirement.with_environment(self._parameters)

    def update_offer_status(self, recommendations) -> None:
        from dcos_commons_amd.offer.recommendations import LaunchOfferRecommendation

        with self._status_lock:
            self._tasks.clear()
            for r in recommendations:
                if isinstance(r, LaunchOfferRecommendation):
                    self._tasks[r.task_info.task_id.value] = [r.task_info, Status.PREPARED]
            if recommendations:
                for tid in list(self._tasks):
                    self._set_task_status(tid, Status.STARTING)
            self._prepared = True
            self._update_status()

    def get_errors(self) -> List[str]:
        return list(self._errors)

    def get_display_status(self) -> str:
        pi = self.pod_instance_requirement.pod_instance
        names = [f"{pi.name}-{t.name}" for t in pi.pod.tasks]
        return display_status(self.state_store, AbstractStep.get_status(self), names)

    def update(self, status: P.TaskStatus) -> None:
        tid = status.task_id.value
        if tid not in self._tasks:      # every step of every plan sees every status: skip lock-free
            return
        with self._status_lock:
            if tid not in self._tasks:
                return
            if self.is_complete():
                return
            state = status.state
            b = backoff_mod.get_instance()
            if state in (P.TASK_ERROR, P.TASK_FAILED):
                b.add_delay(status.task_id)
                self._set_task_status(tid, Status.DELAYED)
            elif state in (P.TASK_KILLED, P.TASK_KILLING, P.TASK_LOST, P.TASK_GONE, P.TASK_DROPPED,
                           P.TASK_UNREACHABLE):
                self._set_task_status(tid, Status.PENDING)
            elif state == P.TASK_GONE_BY_OPERATOR:
                b.clear_delay(status.task_id)
                self._set_task_status(tid, Status.PENDING)
            elif state in (P.TASK_STAGING, P.TASK_STARTING):
                self._set_task_status(tid, Status.STARTING)
            elif state == P.TASK_RUNNING:
                info = self._tasks[tid][0]
                if self._goal_state(status.task_id) == GoalState.RUNNING and \
                        TaskLabelReader(info).is_readiness_check_succeeded(status):
                    b.clear_delay(status.task_id)
                    self._set_task_status(tid, Status.COMPLETE)
                else:
                    self._set_task_status(tid, Status.STARTED)
            elif state == P.TASK_FINISHED:
                goal = self._goal_state(status.task_id)
                if goal in (GoalState.FINISH, GoalState.ONCE):
                    self._set_task_status(tid, Status.COMPLETE)
                elif goal == GoalState.RUNNING:
                    self._set_task_status(tid, Status.PENDING)
                else:
                    raise ValueError(f"Unsupported goal state {goal} for task {tid}")
            elif state == P.TASK_UNKNOWN:
                self.logger.warning("Discarding task status update for TASK_UNKNOWN")
            else:
                self.logger.error("Failed to process unexpected state: %s", state)
            self._update_status()

    def _goal_state(self, task_id) -> GoalState:
        try:
            name = common_id_utils.to_task_name(task_id)
        except TaskException:
            return GoalState.UNKNOWN
        return self.goal_state_by_task_name.get(name, GoalState.UNKNOWN)

    def _set_override_status(self, tid: str, status: Status) -> None:
        name = self._tasks[tid][0].name
        cur = self.state_store.fetch_goal_override_status(name)
        if cur.progress != OverrideProgress.COMPLETE:
            self.state_store.store_goal_override_status(name, cur.target.new_status(
                OverrideStatus.translate_status(status)))

    def _set_task_status(self, tid: str, status: Status) -> None:
        if tid in self._tasks:
            self._tasks[tid][1] = status
            self._set_override_status(tid, status)
        if status == Status.PENDING:
            self._prepared = True
        elif status == Status.DELAYED:
            self._prepared = False

    def _update_status(self) -> None:
        statuses = {v[1] for v in self._tasks.values()}
        st = compute_status(statuses, bool(self._errors), self._prepared)
        if st is not None:
            self._set_status(st)
        else:
            self.logger.warning("Unhandled task status set %s for step %s; leaving %s", statuses, self.get_name(),
                                self._status)

    def task_statuses(self) -> Dict[str, Status]:
        return {v[0].name: v[1] for v in self._tasks.values()}


def display_status(state_store, step_status: Status, task_names: List[str]) -> str:
    if task_names and all(state_store.fetch_goal_override_status(n).target == GoalStateOverride.PAUSED
                          for n in task_names):
        if step_status.is_running():
            return GoalStateOverride.PAUSED.transitioning_name
        if step_status in (Status.COMPLETE, Status.STARTED):
            return GoalStateOverride.PAUSED.serialized_name
    return str(step_status)
