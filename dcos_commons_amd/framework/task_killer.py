"""Reliable task kill.

Reference: sdk/.../framework/TaskKiller.java:26-210. Every requested kill is remembered and
re-issued every 5 s until a terminal status for that TaskID arrives. The re-kill loop runs on a
daemon thread (disabled in simulation tests via ``reset(executor_enabled=False)``).
"""
from __future__ import annotations

import logging
import threading
from typing import Set

from dcos_commons_amd.mesos import protos as P
from dcos_commons_amd.utils.locks import new_lock

from . import driver

LOGGER = logging.getLogger(__name__)
KILL_INTERVAL_S = 5.0

_lock = new_lock("TaskKiller")
_tasks_to_kill: Set[str] = set()
# kills the plan scheduler issued to relaunch a pod in place: their terminal status frees
# reservations that come back in a new offer, so the status itself gives the offer loop nothing to do
_relaunch_kills: Set[str] = set()
_thread = None
_stop_event = threading.Event()
_executor_enabled = True

_ALIVE = frozenset([P.TASK_KILLING, P.TASK_RUNNING, P.TASK_STAGING, P.TASK_STARTING])


def reset(executor_enabled: bool = True) -> None:
    global _thread, _executor_enabled
    with _lock:
        if _thread is not None:
            _stop_event.set()
            t = _thread
        else:
            t = None
        _thread = None
        _tasks_to_kill.clear()
        _relaunch_kills.clear()
        _executor_enabled = executor_enabled
    if t is not None:
        t.join(timeout=KILL_INTERVAL_S)
    _stop_event.clear()


def _loop() -> None:
    while not _stop_event.wait(KILL_INTERVAL_S):
        kill_all_tasks()


def kill_task(task_id: P.TaskID, relaunch: bool = False) -> None:
    """``relaunch``: the kill frees the task's resources for a relaunch of its pod that the plan
    scheduler is already evaluating (PlanScheduler.killTasks)."""
    global _thread
    if not task_id.value:
        LOGGER.warning("Attempted to kill empty TaskID.")
        return
    with _lock:
        _tasks_to_kill.add(task_id.value)
        if relaunch:
            _relaunch_kills.add(task_id.value)
        if _thread is None and _executor_enabled:
            _thread = threading.Thread(target=_loop, name="TaskKiller", daemon=True)
            _thread.start()
    _kill_internal(task_id.value)


def update(status: P.TaskStatus) -> bool:
    """Returns True if the status is for a task we did NOT expect to die (kill-eligible)."""
    if status.state in _ALIVE:
        return True
    with _lock:
        _relaunch_kills.discard(status.task_id.value)
        if status.task_id.value in _tasks_to_kill:
            _tasks_to_kill.discard(status.task_id.value)
            return False
    return True


def ends_relaunch_kill(status: P.TaskStatus) -> bool:
    """Whether ``status`` is the terminal status of a relaunch kill (call before ``update``)."""
    if status.state in _ALIVE:
        return False
    with _lock:
        return status.task_id.value in _relaunch_kills


def pending_kills() -> Set[str]:
    with _lock:
        return set(_tasks_to_kill)


def kill_all_tasks() -> None:
    with _lock:
        copy = list(_tasks_to_kill)
    for tid in copy:
        _kill_internal(tid)


def _kill_internal(task_id: str) -> None:
    d = driver.get_instance()
    if d is None:
        LOGGER.warning("No driver set; cannot kill %s", task_id)
        return
    d.kill_task(P.TaskID(value=task_id))
