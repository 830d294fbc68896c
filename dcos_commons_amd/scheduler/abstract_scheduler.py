"""Common service-scheduler logic.

Reference: sdk/.../scheduler/AbstractScheduler.java:36-262. ``get_client_status`` snapshots the
candidate steps and updates the WorkSetTracker; ``offers`` refuses to launch until explicit
reconciliation has finished; ``task_status`` stores the status and feeds the reconciler.
Additions: launches are watched until their first status (``LaunchWatchdog``), and a
reconciliation TASK_UNKNOWN is handled as TASK_LOST (``SDK_UNKNOWN_AS_LOST``).
"""
from __future__ import annotations

import logging
import threading
from typing import List, Optional

from dcos_commons_amd.framework.process_exit import ProcessExit
from dcos_commons_amd.mesos import protos as P
from dcos_commons_amd.scheduler.mesos_event_client import (
    MesosEventClient,
    OfferResponse,
    TaskStatusResponse,
)
from dcos_commons_amd.scheduler.plan.status import Status
from dcos_commons_amd.scheduler.reconciliation import ExplicitReconciler, LaunchWatchdog, WorkSetTracker
from dcos_commons_amd.state.state_store import StateStoreException
from dcos_commons_amd.storage.persister import Reason


def _cfg(scheduler_config, getter: str, default):
    fn = getattr(scheduler_config, getter, None)
    return fn() if callable(fn) else default


class AbstractScheduler(MesosEventClient):
    def __init__(self, service_spec, scheduler_config, state_store, plan_coordinator, plan_customizer=None,
                 namespace: Optional[str] = None):
        self.service_spec = service_spec
        self.scheduler_config = scheduler_config
        self.state_store = state_store
        self.plan_coordinator = plan_coordinator
        self.plan_customizer = plan_customizer
        self.namespace = namespace
        self.candidate_steps: List = []
        self.work_set_tracker: Optional[WorkSetTracker] = None
        self.reconciler: Optional[ExplicitReconciler] = None
        self.launch_watchdog = LaunchWatchdog(_cfg(scheduler_config, "launch_reconcile_s", 0.0), namespace)
        self.unknown_as_lost = _cfg(scheduler_config, "is_unknown_as_lost", False)
        self.logger = logging.getLogger(type(self).__module__ + (f"({namespace})" if namespace else ""))
        # set after every processed status: observers (benchmarks, tests) wait on it instead of
        # polling plan state
        self.status_processed = threading.Event()

    def customize_plans(self) -> None:
        if self.plan_customizer is None:
            return
        for pm in self.plan_coordinator.get_plan_managers():
            plan = pm.get_plan()
            if plan.is_recovery_plan():
                continue
            pm.set_plan(self.plan_customizer.update_plan(plan))

    def get_plans(self):
        return [pm.get_plan() for pm in self.plan_coordinator.get_plan_managers()]

    def get_plan(self, name: str):
        for p in self.get_plans():
            if p.get_name() == name:
                return p
        return None

    def registered(self, re_registered: bool) -> None:
        if not re_registered or self.reconciler is None:
            self.work_set_tracker = WorkSetTracker(self.namespace)
            self.reconciler = ExplicitReconciler(self.state_store, self.namespace)
            self.registered_with_mesos()
        self.reconciler.start()
        self.reconciler.reconcile()

    def _in_progress_steps(self):
        out = []
        for pm in self.plan_coordinator.get_plan_managers():
            for phase in pm.get_plan().get_children():
                for step in phase.get_children():
                    if step.is_running():
                        out.append(step)
        return out

    def offer_cycle_useful(self) -> bool:
        """After a RUNNING status (readiness passed, or no check): whether an offer cycle could
        find anything to do. False only while every incomplete step of every plan is launched and
        waiting (STARTING/STARTED): no step can become a candidate until one of them completes or
        fails (a failure is a terminal status, which always wakes the offer loop), and the
        scheduler is not idle, so there is nothing to suppress either. An 8-pod parallel deploy
        otherwise runs an empty cycle after each of the first seven readiness results, holding the
        interpreter the next result needs."""
        in_flight = False
        for pm in self.plan_coordinator.get_plan_managers():
            for phase in pm.get_plan().get_children():
                for step in phase.get_children():
                    st = step.get_status()
                    if st == Status.COMPLETE:
                        continue
                    if st in (Status.STARTING, Status.STARTED):
                        in_flight = True
                        continue
                    return True
        return not in_flight

    def get_client_status(self):
        self.candidate_steps = list(self.plan_coordinator.get_candidates())
        active = list(self.candidate_steps)
        seen = {id(s) for s in active}
        for s in self._in_progress_steps():
            if id(s) not in seen:
                active.append(s)
        if self.work_set_tracker is None:
            self.logger.error("WorkSetTracker is uninitialized (status requested before registration)")
            ProcessExit.exit(ProcessExit.ERROR, RuntimeError("WorkSetTracker uninitialized"))
        self.work_set_tracker.update_work_set(active)
        self.launch_watchdog.poll()
        return self.get_status()

    def offers(self, offers, launch_stream=None) -> OfferResponse:
        self.reconciler.reconcile()
        if not self.reconciler.is_reconciled():
            self.logger.info("Not ready for offers: waiting for task reconciliation to complete.")
            return OfferResponse.not_ready([])
        if launch_stream is not None and self.supports_launch_stream:
            return self.process_offers(offers, self.candidate_steps, launch_stream)
        return self.process_offers(offers, self.candidate_steps)

    def task_status(self, status) -> TaskStatusResponse:
        self.launch_watchdog.update(status)
        return self.task_status_processed(self._unknown_as_lost(status))

    def task_statuses(self, statuses) -> List[TaskStatusResponse]:
        """Statuses that arrived together (a status thread catching up after a slow write), in
        arrival order. A scheduler with ``process_status_updates`` stores them in one transaction
        (split where a status reads the stored history, ``status_reads_history``); the responses
        are what ``task_status`` returns."""
        batch_fn = getattr(self, "process_status_updates", None)
        if batch_fn is None or len(statuses) < 2:
            return [self.task_status(s) for s in statuses]
        out: List[TaskStatusResponse] = []
        run: List = []

        def flush():
            if not run:
                return
            try:
                errors = batch_fn(run)
            finally:
                self.status_processed.set()
            for st, err in zip(run, errors):
                if err is None and self.reconciler is not None:
                    try:
                        self.reconciler.update(st)
                    except Exception as e:  # noqa: BLE001
                        err = e
                out.append(TaskStatusResponse.processed() if err is None else self._status_failed(st, err))
            run.clear()

        for status in statuses:
            self.launch_watchdog.update(status)
            status = self._unknown_as_lost(status)
            if self.status_reads_history(status):
                # handled against the statuses before it already stored
                flush()
                out.append(self.task_status_processed(status))
                continue
            run.append(status)
        flush()
        return out

    def status_reads_history(self, status) -> bool:
        """Whether processing ``status`` reads the task's stored status (it is then processed
        alone, after the statuses before it are stored)."""
        return False

    def task_status_processed(self, status) -> TaskStatusResponse:
        """``task_status`` for a status that already went through the launch watchdog and the
        TASK_UNKNOWN mapping."""
        try:
            self.process_status_update(status)
            if self.reconciler is not None:
                self.reconciler.update(status)
        except Exception as e:  # noqa: BLE001
            return self._status_failed(status, e)
        finally:
            self.status_processed.set()
        return TaskStatusResponse.processed()

    def _unknown_as_lost(self, status):
        if (self.unknown_as_lost and status.state == P.TASK_UNKNOWN
                and status.reason == P.TaskStatus.REASON_RECONCILIATION):
            # The master has no record of the task (it never got the launch, or the agent was
            # wiped). The reference stores TASK_UNKNOWN and never recovers the task; treat it as
            # lost so the recovery plan relaunches it.
            lost = P.TaskStatus()
            lost.CopyFrom(status)
            lost.state = P.TASK_LOST
            lost.message = f"Unknown to the master on reconciliation: {status.message}"
            return lost
        return status

    def _status_failed(self, status, e: BaseException) -> TaskStatusResponse:
        if isinstance(e, StateStoreException):
            if e.reason == Reason.NOT_FOUND:
                self.logger.info("Status for unknown task %s: %s", status.task_id.value, e)
                return TaskStatusResponse.unknown_task()
        self.logger.warning("Failed to update TaskStatus received from Mesos: %s", e)
        return TaskStatusResponse.processed()

    def awaiting_reconciliation(self) -> bool:
        return self.reconciler is None or not self.reconciler.is_reconciled()

    # abstract
    def registered_with_mesos(self) -> None:
        raise NotImplementedError

    def get_status(self):
        raise NotImplementedError

    # process_offers(offers, steps, launch_stream) is implemented (see DefaultScheduler)
    supports_launch_stream = False

    def process_offers(self, offers, steps) -> OfferResponse:
        raise NotImplementedError

    def process_status_update(self, status) -> None:
        raise NotImplementedError

    def get_config_store(self):
        raise NotImplementedError

    def get_custom_endpoints(self):
        return {}
