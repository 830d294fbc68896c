"""Explicit task reconciliation and new-work detection.

Reference: sdk/.../scheduler/ExplicitReconciler.java:36-251 (backoff 4 s -> x2 -> 30 s; offers are
refused until every non-terminal task has been reconciled) and WorkSetTracker.java:21-136.
``LaunchWatchdog`` has no reference counterpart (see its docstring).
"""
from __future__ import annotations

import logging
import time
from typing import Callable, Dict, Optional, Set

from dcos_commons_amd.framework import driver
from dcos_commons_amd.mesos import protos as P
from dcos_commons_amd.offer.task_utils import is_terminal
from dcos_commons_amd.utils.locks import new_rw_lock

MULTIPLIER = 2
BASE_BACKOFF_MS = 4000
MAX_BACKOFF_MS = 30000


class ExplicitReconciler:
    def __init__(self, state_store, namespace: Optional[str] = None,
                 clock_ms: Callable[[], float] = lambda: time.time() * 1000):
        self.state_store = state_store
        self.logger = logging.getLogger(__name__ + (f"({namespace})" if namespace else ""))
        rw = new_rw_lock("ExplicitReconciler")
        self._r, self._w = rw.read_lock, rw.write_lock
        self._unreconciled: Dict[str, P.TaskStatus] = {}
        self._complete = False
        self.clock_ms = clock_ms
        self._reset_timer()

    def _reset_timer(self) -> None:
        self._last_request_ms = 0.0
        self._backoff_ms = BASE_BACKOFF_MS

    def start(self) -> None:
        statuses = list(self.state_store.fetch_statuses())
        with self._w:
            for s in statuses:
                if not is_terminal(s):
                    self._unreconciled[s.task_id.value] = s
            if self._unreconciled:
                self._complete = False
            self._reset_timer()
        self.logger.info("Added %d unreconciled task(s) to reconciler", len(self._unreconciled))

    def reconcile(self) -> None:
        if self._complete:
            return
        to_reconcile = []
        with self._w:
            if self._unreconciled:
                now = self.clock_ms()
                if now >= self._last_request_ms + self._backoff_ms:
                    self._last_request_ms = now
                    self._backoff_ms = min(self._backoff_ms * MULTIPLIER, MAX_BACKOFF_MS)
                    to_reconcile = list(self._unreconciled.values())
                else:
                    return
        # Never hold the lock across the driver call (ExplicitReconciler.java:138-143).
        if not to_reconcile:
            self._complete = True
        else:
            d = driver.get_instance()
            if d is not None:
                d.reconcile_tasks(to_reconcile)

    def update(self, status: P.TaskStatus) -> None:
        with self._w:
            if not self._unreconciled:
                return
            self._unreconciled.pop(status.task_id.value, None)

    def is_reconciled(self) -> bool:
        with self._r:
            return not self._unreconciled

    def remaining(self) -> Set[str]:
        with self._r:
            return set(self._unreconciled)


class LaunchWatchdog:
    """Reconciles launches that never left TASK_STAGING.

    The launch is recorded (TaskInfo + a synthetic STAGING status) before the ACCEPT goes out
    (write-ahead, DefaultScheduler.java:455). If that ACCEPT is lost, the master never hears of
    the task and nothing ever updates it: the reference leaves the step STARTING until a
    scheduler restart re-runs explicit reconciliation. Here every recorded launch is watched;
    one still without a status after ``timeout_s`` is reconciled explicitly (the master answers
    TASK_UNKNOWN/TASK_LOST for a task it never saw, which sends the step back to PENDING), with
    the usual x2 backoff up to ``MAX_BACKOFF_MS``. ``timeout_s <= 0`` disables the watchdog
    (reference behaviour).
    """

    def __init__(self, timeout_s: float, namespace: Optional[str] = None,
                 clock: Callable[[], float] = time.monotonic):
        self.timeout_s = timeout_s
        self.clock = clock
        self.logger = logging.getLogger(__name__ + (f"({namespace})" if namespace else ""))
        self._lock = new_rw_lock("LaunchWatchdog").write_lock
        # task id -> (next deadline, current backoff, staging status)
        self._watched: Dict[str, tuple] = {}

    @property
    def enabled(self) -> bool:
        return self.timeout_s > 0

    def launched(self, status: P.TaskStatus) -> None:
        if not self.enabled or not status.task_id.value:
            return
        with self._lock:
            self._watched[status.task_id.value] = (self.clock() + self.timeout_s, self.timeout_s, status)

    def update(self, status: P.TaskStatus) -> None:
        if status.state == P.TASK_STAGING and status.source != P.TaskStatus.SOURCE_MASTER:
            return
        with self._lock:
            self._watched.pop(status.task_id.value, None)

    def watched(self) -> Set[str]:
        with self._lock:
            return set(self._watched)

    def poll(self) -> int:
        """Reconcile every overdue launch; returns how many were sent."""
        if not self._watched:
            return 0
        now = self.clock()
        due = []
        with self._lock:
            for tid, (deadline, backoff, st) in list(self._watched.items()):
                if now >= deadline:
                    nb = min(backoff * MULTIPLIER, MAX_BACKOFF_MS / 1000.0)
                    self._watched[tid] = (now + nb, nb, st)
                    due.append(st)
        if due:
            self.logger.warning("Reconciling %d launch(es) still STAGING after %.1fs: %s", len(due), self.timeout_s,
                                [s.task_id.value for s in due])
            d = driver.get_instance()
            if d is not None:
                d.reconcile_tasks(due)
        return len(due)


class WorkSetTracker:
    def __init__(self, namespace: Optional[str] = None):
        self._candidates: Set[tuple] = set()
        self._has_new_work = False
        self.logger = logging.getLogger(__name__ + (f"({namespace})" if namespace else ""))

    @staticmethod
    def _item(step) -> tuple:
        req = step.get_pod_instance_requirement()
        return (step.get_name(), req)

    def update_work_set(self, active_work_set) -> None:
        cur = {self._item(s) for s in active_work_set}
        new = cur - self._candidates
        if new:
            self.logger.info("New work: %s", sorted(n for n, _ in new))
            self._has_new_work = True
        self._candidates = cur

    def has_new_work(self) -> bool:
        ret = self._has_new_work
        self._has_new_work = False
        return ret
