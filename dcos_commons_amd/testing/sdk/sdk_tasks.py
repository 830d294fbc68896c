"""Task queries and relaunch checks against the local cluster.

Reference: testing/sdk_tasks.py (same names; a ``Task`` carries name, host, state, id,
framework/agent ids and scalar resources). Scheduler tasks are the Marathon tasks of the
scheduler processes and appear under the framework name ``marathon``, as on DC/OS.
"""
from __future__ import annotations

import logging
import time
from typing import Any, Dict, Iterable, List, Optional

LOG = logging.getLogger(__name__)
DEFAULT_TIMEOUT_SECONDS = 120
POLL_S = 0.1
COMPLETED_TASK_STATES = {"TASK_FINISHED", "TASK_KILLED", "TASK_FAILED", "TASK_LOST", "TASK_ERROR",
                         "TASK_GONE", "TASK_GONE_BY_OPERATOR", "TASK_DROPPED", "TASK_UNREACHABLE", "TASK_UNKNOWN"}
FATAL_TERMINAL_TASK_STATES = {"TASK_FAILED", "TASK_ERROR"}


def _cluster():
    from dcos_commons_amd.testing.cluster import current

    return current()


def _wait(fn, timeout_seconds: float, what: str):
    deadline = time.time() + timeout_seconds
    last: Optional[BaseException] = None
    while True:
        try:
            v = fn()
            if v:
                return v
        except AssertionError as e:
            last = e
        if time.time() >= deadline:
            raise AssertionError(f"Timed out after {timeout_seconds}s waiting for {what}" +
                                 (f": {last}" if last else ""))
        time.sleep(POLL_S)


class Task:
    """One task of ``get_summary()`` / ``get_service_tasks()``."""

    def __init__(self, name: str, host: str, state: str, task_id: str, executor_id: str, framework_id: str,
                 agent_id: str, resources: Dict[str, float]):
        self.name = name
        self.host = host
        self.state = state
        self.is_completed = state in COMPLETED_TASK_STATES
        self.id = task_id
        self.executor_id = executor_id
        self.framework_id = framework_id
        self.agent_id = agent_id
        self.resources = resources

    def __repr__(self) -> str:
        return (f'Task[name="{self.name}"\tstate={self.state}\tid={self.id}\thost={self.host}\t'
                f'framework_id={self.framework_id}\tagent_id={self.agent_id}]')


def _framework_name(service_name: str) -> str:
    return service_name


def _from_view(v) -> Task:
    eid = v.statuses[-1].executor_id.value if v.statuses else ""
    return Task(v.name, v.host, v.state, v.id, eid, v.framework_id, v.agent_id, dict(v.resources))


def _marathon_tasks(prefix: str, with_completed: bool) -> List[Task]:
    out = []
    for t in _cluster().marathon.tasks(prefix):
        if not with_completed and t.state != "TASK_RUNNING":
            continue
        out.append(Task(t.id.rsplit(".", 1)[0], t.host, t.state, t.id, "", "marathon", "local", {}))
    return out


def get_summary(with_completed: bool = False, task_name: Optional[str] = None) -> List[Task]:
    """All tasks of all frameworks (plus the schedulers under ``marathon``)."""
    out = [_from_view(v) for v in _cluster().tasks(include_terminal=with_completed)]
    out.extend(_marathon_tasks("", with_completed))
    if task_name is not None:
        out = [t for t in out if t.name == task_name]
    return out


def get_service_tasks(service_name: str, task_prefix: str = "", with_completed_tasks: bool = False) -> List[Task]:
    """Tasks of one service (framework name == service name) whose name starts with ``task_prefix``."""
    if service_name == "marathon":
        from dcos_commons_amd.testing.cluster import scheduler_task_prefix

        prefix = scheduler_task_prefix(task_prefix) if task_prefix.startswith("/") or "/" in task_prefix \
            else task_prefix
        return _marathon_tasks(prefix, with_completed_tasks)
    views = _cluster().tasks(_framework_name(service_name), include_terminal=with_completed_tasks)
    return [_from_view(v) for v in views if v.name.startswith(task_prefix)]


def get_task_ids(service_name: str, task_prefix: str = "") -> List[str]:
    return sorted(t.id for t in get_service_tasks(service_name, task_prefix))


def get_all_status_history(task_name: str, with_completed_tasks: bool = True) -> List[Dict[str, Any]]:
    """Every status of every instance of ``task_name``, oldest first, as the state-summary JSON
    shows them: ``{"state": "TASK_RUNNING", "timestamp": ..., "container_status": {"network_infos": [...]}}``."""
    statuses = []
    for v in _cluster().tasks(include_terminal=with_completed_tasks):
        if v.name == task_name:
            statuses.extend(v.statuses)
    statuses.sort(key=lambda s: s.timestamp)
    from google.protobuf import json_format

    from dcos_commons_amd.mesos import protos as P

    out = []
    for s in statuses:
        d = {"state": P.TaskState.Name(s.state), "timestamp": s.timestamp}
        if s.HasField("container_status"):
            d["container_status"] = json_format.MessageToDict(s.container_status, preserving_proto_field_name=True)
        out.append(d)
    return out


def get_failed_task_count(service_name: str, retry: bool = False) -> int:
    return len([t for t in get_service_tasks(service_name, with_completed_tasks=True)
                if t.state in FATAL_TERMINAL_TASK_STATES])


def check_running(service_name: str, expected_task_count: int, timeout_seconds: int = DEFAULT_TIMEOUT_SECONDS,
                  allow_more: bool = True) -> None:
    def fn():
        running = [t.name for t in get_service_tasks(service_name) if t.state == "TASK_RUNNING"]
        return len(running) >= expected_task_count if allow_more else len(running) == expected_task_count
    _wait(fn, timeout_seconds, f"{'at least' if allow_more else 'exactly'} {expected_task_count} running tasks "
                               f"in {service_name}")


def check_task_count(service_name: str, expected_task_count: int) -> List[Task]:
    tasks = get_service_tasks(service_name)
    assert len(tasks) == expected_task_count, f"expected {expected_task_count} tasks, got {tasks}"
    return tasks


def check_task_relaunched(task_name: str, old_task_id: str, ensure_new_task_not_completed: bool = True,
                          timeout_seconds: int = DEFAULT_TIMEOUT_SECONDS) -> None:
    def fn():
        tasks = get_summary(with_completed=True, task_name=task_name)
        assert tasks, f"No tasks were found with the given task name {task_name}"
        assert any(t.is_completed and t.id == old_task_id for t in tasks), \
            f"Unable to find any completed tasks with id {old_task_id}"
        assert any(t.id != old_task_id and (not t.is_completed or not ensure_new_task_not_completed)
                   for t in tasks), f"Unable to find any new tasks with name {task_name}"
        return True
    _wait(fn, timeout_seconds, f"{task_name} to relaunch (old id {old_task_id})")


def check_scheduler_relaunched(service_name: str, old_scheduler_task_id: str,
                               timeout_seconds: int = DEFAULT_TIMEOUT_SECONDS) -> None:
    def fn():
        ids = {t.id for t in get_service_tasks("marathon", task_prefix=service_name)}
        return len(ids) > 0 and (old_scheduler_task_id not in ids or len(ids) > 1)
    _wait(fn, timeout_seconds, f"scheduler of {service_name} to relaunch")


def check_task_not_relaunched(service_name: str, task_name: str, old_task_id: str,
                              multiservice_name: Optional[str] = None, with_completed: bool = False) -> None:
    from dcos_commons_amd.testing.sdk import sdk_plan

    sdk_plan.wait_for_completed_deployment(service_name, multiservice_name=multiservice_name)
    sdk_plan.wait_for_completed_recovery(service_name, multiservice_name=multiservice_name)
    ids = {t.id for t in get_summary(with_completed) if t.name == task_name}
    assert old_task_id in ids, f"Old task id {old_task_id} was not found in task_ids {ids}"
    assert len(ids) == 1, f"Length != 1. Expected task id {old_task_id} Task ids: {ids}"


def check_tasks_updated(service_name: str, prefix: str, old_task_ids: Iterable[str],
                        timeout_seconds: int = DEFAULT_TIMEOUT_SECONDS) -> None:
    """Every task of ``prefix`` has been replaced by a new one (and none of the old remain)."""
    old = set(old_task_ids)

    def fn():
        wait_for_active_framework(service_name)
        new = set(get_task_ids(service_name, prefix))
        return len(new - old) == len(new) and not (old & new) and len(new) >= len(old)
    _wait(fn, timeout_seconds, f"tasks of {service_name} starting with '{prefix}' to be updated from {sorted(old)}")


def check_tasks_not_updated(service_name: str, prefix: str, old_task_ids: Iterable[str]) -> None:
    from dcos_commons_amd.testing.sdk import sdk_plan

    sdk_plan.wait_for_completed_deployment(service_name)
    sdk_plan.wait_for_completed_recovery(service_name)
    ids = set(get_task_ids(service_name, prefix))
    missing = set(old_task_ids) - ids
    assert not missing, f"Tasks starting with '{prefix}' were updated: missing {sorted(missing)}, now {sorted(ids)}"


def wait_for_active_framework(service_name: str, timeout_seconds: int = DEFAULT_TIMEOUT_SECONDS) -> None:
    if service_name == "marathon":   # the stand-in's Marathon is not a Mesos framework: always up
        return
    _wait(lambda: any(f["name"] == service_name and f["active"] for f in _cluster().frameworks()),
          timeout_seconds, f"framework {service_name} to be active")


def get_tasks_avoiding_scheduler(service_name: str, task_name_pattern) -> List[Task]:
    """Tasks matching the regex that run on a different agent than the scheduler (on the stand-in
    every scheduler runs on the loopback host, so this is every matching task)."""
    import re

    rx = re.compile(task_name_pattern) if isinstance(task_name_pattern, str) else task_name_pattern
    return [t for t in get_service_tasks(service_name) if rx.match(t.name)]
