"""Task predicates, spec diffing and recovery selection.

Reference: sdk/.../offer/TaskUtils.java (731 LoC): ``isTerminal`` :659, ``isRecoveryNeeded``
:615, ``getTasksNeedingRecovery`` :556, ``getTasksForReplacement`` :633 and the
``areDifferent`` spec comparison :154 that decides whether a running task must be relaunched
on a configuration update.
"""
from __future__ import annotations

import logging
from typing import Collection, Dict, Iterable, List, Optional

from dcos_commons_amd.mesos import protos as P
from dcos_commons_amd.offer.taskdata.labels import (
    ZONE_TASKENV,
    TaskException,
    TaskLabelReader,
)
from dcos_commons_amd.specification.specs import GoalState, PodInstance, PodSpec, ServiceSpec, TaskSpec

LOGGER = logging.getLogger(__name__)

_TERMINAL = frozenset([P.TASK_DROPPED, P.TASK_ERROR, P.TASK_FAILED, P.TASK_FINISHED, P.TASK_GONE,
                       P.TASK_KILLED])


def is_terminal(status) -> bool:
    state = status if isinstance(status, int) else status.state
    return state in _TERMINAL


def is_recovery_needed(status: P.TaskStatus) -> bool:
    return is_terminal(status) or status.state in (P.TASK_LOST, P.TASK_UNREACHABLE)


def get_task_instance_name(pod_instance: PodInstance, task) -> str:
    return f"{pod_instance.name}-{task if isinstance(task, str) else task.name}"


def get_task_names(pod_instance: PodInstance, tasks_to_launch: Optional[Collection[str]] = None) -> List[str]:
    return [get_task_instance_name(pod_instance, t) for t in pod_instance.pod.tasks
            if tasks_to_launch is None or t.name in tasks_to_launch]


def get_step_name(pod_instance: PodInstance, tasks_to_launch: Collection[str]) -> str:
    # Java List.toString(): "[a, b]"
    return f"{pod_instance.name}:[{', '.join(tasks_to_launch)}]"


def has_tasks_with_tls(service_spec: ServiceSpec) -> bool:
    return any(t.transport_encryption for p in service_spec.pods for t in p.tasks)


def are_equivalent(task_info: P.TaskInfo, pod_instance: PodInstance) -> bool:
    try:
        r = TaskLabelReader(task_info)
        return r.get_index() == pod_instance.index and r.get_type() == pod_instance.pod.type
    except (TaskException, ValueError):
        return False


def get_pod_tasks(pod_instance: PodInstance, tasks: Iterable[P.TaskInfo]) -> List[P.TaskInfo]:
    return [t for t in tasks if are_equivalent(t, pod_instance)]


def _resource_map(resources) -> Dict[str, object]:
    out = {}
    for r in resources:
        prev = out.get(r.name)
        out[r.name] = r
        if prev is not None and prev.name != "ports":
            raise ValueError(f"Non-port resources for a given task may not share the same name: {r.name}")
    return out


def _config_map(configs):
    out, paths = {}, set()
    for c in configs:
        if c.relative_path in paths:
            raise ValueError(f"Config templates for a given task may not share the same path: '{c.relative_path}'")
        paths.add(c.relative_path)
        if c.name in out:
            raise ValueError(f"Config templates for a given task may not share the same name: '{c.name}'")
        out[c.name] = c
    return out


def volumes_equal(first: TaskSpec, second: TaskSpec) -> bool:
    a = sorted(repr(v._eq_key()) for v in first.resource_set.volumes)
    b = sorted(repr(v._eq_key()) for v in second.resource_set.volumes)
    return a == b


def are_different(old: TaskSpec, new: TaskSpec) -> bool:
    """TaskUtils.areDifferent: True if the task must be relaunched to match ``new``."""
    if old.name != new.name or old.goal != new.goal:
        return True
    old_r = _resource_map(old.resource_set.resources)
    new_r = _resource_map(new.resource_set.resources)
    if len(old_r) != len(new_r):
        return True
    for name, nr in new_r.items():
        orr = old_r.get(name)
        if orr is None or orr != nr:
            return True
    if not volumes_equal(old, new):
        return True
    if old.labels != new.labels:
        return True
    if old.command != new.command:
        return True
    if old.health_check != new.health_check:
        return True
    if old.readiness_check != new.readiness_check:
        return True
    if _config_map(old.config_files) != _config_map(new.config_files):
        return True
    if old.discovery != new.discovery:
        return True
    if old.shared_memory != new.shared_memory or old.shared_memory_size != new.shared_memory_size:
        return True
    if old.kill_grace_period != new.kill_grace_period:
        return True
    return False


def get_pod_spec(service_spec: ServiceSpec, task_info: P.TaskInfo,
                 reader: Optional[TaskLabelReader] = None) -> Optional[PodSpec]:
    pod_type = (reader or TaskLabelReader(task_info)).get_type()
    return service_spec.pod(pod_type)


def get_task_spec(pod_instance: PodInstance, task_name: str) -> Optional[TaskSpec]:
    for t in pod_instance.pod.tasks:
        if get_task_instance_name(pod_instance, t) == task_name:
            return t
    return None


def get_task_spec_by_type(service_spec: ServiceSpec, pod_type: str, task_name: str) -> Optional[TaskSpec]:
    pod = service_spec.pod(pod_type)
    return pod.task(task_name) if pod else None


def get_goal_state(pod_instance: PodInstance, task_name: str) -> GoalState:
    spec = get_task_spec(pod_instance, task_name)
    if spec is None:
        raise TaskException("Failed to determine the goal state of Task: " + task_name)
    return spec.goal


def get_pod_instance(config_store, task_info: P.TaskInfo, reader: Optional[TaskLabelReader] = None) -> PodInstance:
    """Resolve a TaskInfo to its PodInstance using the config it was launched with (``reader``:
    the task's label reader, when the caller already has one)."""
    reader = reader or TaskLabelReader(task_info)
    config_id = reader.get_target_configuration()
    try:
        service_spec = config_store.fetch(config_id)
    except Exception as e:  # noqa: BLE001
        raise TaskException(
            f"Unable to retrieve ServiceSpecification ID {config_id} referenced by TaskInfo[{task_info.name}]") from e
    pod = get_pod_spec(service_spec, task_info, reader)
    if pod is None:
        raise TaskException(f"No TaskSpecification found for TaskInfo[{task_info.name}]")
    return PodInstance(pod, reader.get_index())


def get_task_spec_for_info(config_store, task_info: P.TaskInfo,
                           reader: Optional[TaskLabelReader] = None) -> Optional[TaskSpec]:
    return get_task_spec(get_pod_instance(config_store, task_info, reader), task_info.name)


def is_eligible_for_recovery(task_spec: TaskSpec) -> bool:
    if task_spec.goal == GoalState.RUNNING:
        return True
    if task_spec.goal in (GoalState.ONCE, GoalState.FINISH):
        return False
    raise ValueError(f"Unsupported goal state: {task_spec.goal}")


def is_permanently_failed(task_info: P.TaskInfo) -> bool:
    return TaskLabelReader(task_info).is_permanently_failed()


def get_tasks_needing_recovery(config_store, all_task_infos, all_statuses) -> List[P.TaskInfo]:
    status_map = {s.task_id.value: s for s in all_statuses}
    out = []
    for info in all_task_infos:
        status = status_map.get(info.task_id.value)
        if status is None:
            continue
        reader = TaskLabelReader(info)   # one label map per task for the spec lookup and the failed mark
        spec = get_task_spec_for_info(config_store, info, reader)
        if spec is None:
            raise TaskException(f"Failed to determine TaskSpec from TaskInfo: {info.name}")
        if is_eligible_for_recovery(spec) and (is_recovery_needed(status) or reader.is_permanently_failed()):
            out.append(info)
    return out


def get_tasks_for_replacement(all_statuses, all_task_infos) -> List[P.TaskInfo]:
    info_map = {t.task_id.value: t for t in all_task_infos}
    out = []
    for s in all_statuses:
        info = info_map.get(s.task_id.value)
        if s.state == P.TASK_GONE_BY_OPERATOR and info is not None and not is_permanently_failed(info):
            out.append(info)
    return out


def get_pod_requirements(config_store, all_task_infos, all_statuses, failed_tasks, backoff):
    """Group failed tasks into per-pod recovery requirements (TaskUtils.getPodRequirements)."""
    from dcos_commons_amd.scheduler.plan.pod_instance_requirement import PodInstanceRequirement

    pods: Dict[str, tuple] = {}
    for info in failed_tasks:
        try:
            pi = get_pod_instance(config_store, info)
        except TaskException:
            LOGGER.exception("Failed to get pod instance for task: %s", info.name)
            continue
        spec = get_task_spec(pi, info.name)
        if spec is None:
            LOGGER.error("No TaskSpec found for failed task: %s", info.name)
            continue
        pods.setdefault(pi.name, (pi, []))[1].append(spec)
    if not pods:
        return []
    launched_ids = {s.task_id.value for s in all_statuses}
    launched_names = {t.name for t in all_task_infos if t.task_id.value in launched_ids}
    reqs = []
    for name in sorted(pods):
        pi, failed_specs = pods[name]
        if any(t.essential for t in failed_specs):
            delayed = any(backoff.get_delay(get_task_instance_name(pi, t)) is not None for t in pi.pod.tasks)
            to_launch = [] if delayed else list(pi.pod.tasks)
        else:
            to_launch = [t for t in failed_specs if backoff.get_delay(get_task_instance_name(pi, t)) is None]
        to_launch = [t for t in to_launch
                     if is_eligible_for_recovery(t) and get_task_instance_name(pi, t.name) in launched_names]
        if not to_launch:
            continue
        reqs.append(PodInstanceRequirement(pi, [t.name for t in to_launch]))
    return reqs


def task_has_zone(task_info: P.TaskInfo) -> bool:
    return any(v.name == ZONE_TASKENV for v in task_info.command.environment.variables)


def get_task_zone(task_info: P.TaskInfo) -> str:
    for v in task_info.command.environment.variables:
        if v.name == ZONE_TASKENV:
            return v.value
    raise KeyError(ZONE_TASKENV)


def get_task_ip_address(status: P.TaskStatus) -> str:
    nis = status.container_status.network_infos
    if not nis:
        raise ValueError(f"No network info can be found for the task status: {status}")
    return nis[0].ip_addresses[0].ip_address
