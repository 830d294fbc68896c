"""Mesos callback sink for one framework.

Reference: sdk/.../framework/FrameworkScheduler.java:42-300. Stores the FrameworkID on first
registration, installs the driver and the master's domain, starts the offer processor and the
implicit reconciler, drops offers until the API server is up (short decline), strips resources
that belong to other frameworks/roles, routes status updates to the client and kills tasks it
does not know, and exits the process on disconnect/error.
"""
from __future__ import annotations

import logging
import threading
from typing import List

from dcos_commons_amd import metrics, trace
from dcos_commons_amd.mesos import protos as P
from dcos_commons_amd.offer import resources as ResourceUtils
from dcos_commons_amd.offer.evaluate.placement import IsLocalRegionRule
from dcos_commons_amd.scheduler.mesos_event_client import TaskStatusResult
from dcos_commons_amd.state.state_store import StateStoreException

from . import driver as driver_mod
from . import task_killer
from .offer_processing import ImplicitReconciler, OfferProcessor, TokenBucket, decline_short
from .process_exit import ProcessExit

LOGGER = logging.getLogger(__name__)

_NO_NEW_WORK_STATES = (P.TASK_STAGING, P.TASK_STARTING)
# terminal states whose agent has released the task's resources (an unreachable or lost agent
# releases nothing the master could offer again)
_RELEASING_STATES = frozenset([P.TASK_FINISHED, P.TASK_FAILED, P.TASK_KILLED, P.TASK_ERROR])


def can_create_work(status: P.TaskStatus) -> bool:
    """Whether a status can give the plans new work, i.e. whether it is worth waking the offer loop.

    A task moving through STAGING / STARTING, or RUNNING while its readiness check has not
    reported yet, only advances a step that is already launched (STARTING -> STARTED): no step
    becomes a candidate and nothing becomes idle, so an offer cycle run for it would find nothing
    to do while holding the interpreter that the pending check result needs. Everything else
    (readiness results, RUNNING without a check, terminal and unreachable states) wakes it."""
    if status.state in _NO_NEW_WORK_STATES:
        return False
    if status.state == P.TASK_RUNNING and status.HasField("check_status") and \
            status.check_status.HasField("command"):
        return status.check_status.command.HasField("exit_code")   # absent: the check is still pending
    return True


class FrameworkScheduler:
    def __init__(self, roles_whitelist, scheduler_config, persister, framework_store, client,
                 offer_processor: OfferProcessor = None, implicit_reconciler: ImplicitReconciler = None):
        self.roles_whitelist = set(roles_whitelist)
        # statuses wait for a running offer cycle only when the scheduler's state is local: with a
        # remote persister (ZooKeeper) both the cycle (its launch records) and the statuses wait on
        # round trips, and holding the statuses serializes writes that otherwise overlap (cluster
        # mode, 8 pods: deploy 106-131 ms without the gate, 148-155 ms with it, build container)
        self.status_cycle_wait_s = scheduler_config.status_cycle_wait_s() \
            if scheduler_config is not None and not getattr(persister, "remote", False) else 0.0
        self.framework_store = framework_store
        self.client = client
        self.offer_processor = offer_processor or OfferProcessor(
            client, persister, scheduler_config,
            token_bucket=TokenBucket(acquire_interval_s=scheduler_config.revive_interval_s(),
                                     burst_interval_s=scheduler_config.revive_burst_interval_s())
            if scheduler_config is not None else None,
            hold_s=scheduler_config.offer_hold_s() if scheduler_config is not None else 0.0,
            event_driven=scheduler_config.is_event_driven() if scheduler_config is not None else False,
            gc_all_offers=scheduler_config.is_reservation_gc_on_all_offers() if scheduler_config is not None else False,
            fast_unsuppress=scheduler_config.is_fast_unsuppress() if scheduler_config is not None else False,
            merge_agent_offers=scheduler_config.is_merge_agent_offers() if scheduler_config is not None else False,
            stream_launches=scheduler_config.is_stream_launches() if scheduler_config is not None else False,
            revive_only_unmatched=scheduler_config.is_revive_only_unmatched() if scheduler_config is not None else False)
        if implicit_reconciler is None:
            implicit_reconciler = ImplicitReconciler(
                scheduler_config.implicit_reconcile_delay_s() if scheduler_config is not None else 0.0,
                scheduler_config.implicit_reconcile_period_s() if scheduler_config is not None else 3600.0)
        self.implicit_reconciler = implicit_reconciler
        self._register_called = False
        self._api_server_started = threading.Event()
        self.api_server_wait_s = 0.0    # offers before the API server is up: declined (0) or held
        self._lock = threading.Lock()

    # -- configuration ---------------------------------------------------------------
    def set_api_server_started(self) -> "FrameworkScheduler":
        self._api_server_started.set()
        return self

    def disable_threading(self) -> "FrameworkScheduler":
        self.offer_processor.disable_threading()
        self.implicit_reconciler.disable_threading()
        return self

    def set_revive_token_bucket(self, bucket) -> "FrameworkScheduler":
        self.offer_processor.set_revive_token_bucket(bucket)
        return self

    @staticmethod
    def _exit(e: BaseException) -> None:
        LOGGER.error("Got exception when invoked by Mesos, shutting down.", exc_info=e)
        ProcessExit.exit(ProcessExit.ERROR, e)

    @staticmethod
    def _update_driver_and_domain(driver, master_info) -> None:
        driver_mod.set_driver(driver)
        if master_info is not None and master_info.HasField("domain"):
            IsLocalRegionRule.set_local_domain(master_info.domain)

    def _gate_statuses(self, driver) -> None:
        """Network drivers call the status callbacks from their own reader thread, which holds
        no lock of the scheduler's: there a status may wait for a running offer cycle
        (``OfferProcessor.wait_cycle_idle``). In-process masters deliver from their own threads
        and get no gate."""
        wait_s = self.status_cycle_wait_s
        set_gate = getattr(driver, "set_status_gate", None)
        if set_gate is not None and wait_s > 0:
            processor = self.offer_processor
            set_gate(lambda: processor.wait_cycle_idle(wait_s))

    # -- Mesos callbacks ---------------------------------------------------------------
    def prestart(self) -> None:
        """Create the offer-loop and reconciler threads before the driver subscribes (both wait
        for registration), so that the ``registered`` callback does not pay for thread start-up
        while the first offers queue behind it."""
        self.offer_processor.prestart()
        self.implicit_reconciler.prestart()

    def registered(self, driver, framework_id: P.FrameworkID, master_info) -> None:
        trace.instant("registered", "driver")
        try:
            with self._lock:
                again = self._register_called
                self._register_called = True
            if again:
                self.reregistered(driver, master_info)
                return
            try:
                self.framework_store.store_framework_id(framework_id)
            except StateStoreException as e:
                LOGGER.error("Unable to store registered framework ID '%s'", framework_id.value)
                ProcessExit.exit(ProcessExit.REGISTRATION_FAILURE, e)
            self._update_driver_and_domain(driver, master_info)
            self._gate_statuses(driver)
            self.client.registered(False)
            self.offer_processor.start()
            self.implicit_reconciler.start()
        except Exception as e:  # noqa: BLE001
            self._exit(e)

    def reregistered(self, driver, master_info) -> None:
        try:
            self._update_driver_and_domain(driver, master_info)
            self._gate_statuses(driver)
            self.client.registered(True)
        except Exception as e:  # noqa: BLE001
            self._exit(e)

    def resource_offers(self, driver, offers) -> None:
        trace.instant("offers_in", "driver", n=len(offers))
        try:
            metrics.increment_received_offers(len(offers))
            if not self._api_server_started.is_set() and not self._api_server_started.wait(self.api_server_wait_s):
                LOGGER.info("Declining %d offer%s: Waiting for API server to start.", len(offers),
                            "" if len(offers) == 1 else "s")
                decline_short(offers)
                return
            fid = self.framework_store.fetch_framework_id()
            fid = fid.value if fid is not None else None
            self.offer_processor.enqueue([self._filter_bad_resources(o, fid) for o in offers])
        except Exception as e:  # noqa: BLE001
            self._exit(e)

    def _filter_bad_resources(self, offer: P.Offer, framework_id) -> P.Offer:
        good = [r for r in offer.resources if ResourceUtils.is_processable(r, self.roles_whitelist, framework_id)]
        if len(good) == len(offer.resources):
            return offer
        LOGGER.info("Filtered %d resources from offer %s", len(offer.resources) - len(good), offer.id.value)
        out = P.Offer()
        out.CopyFrom(offer)
        del out.resources[:]
        out.resources.extend(good)
        return out

    def status_update(self, driver, status: P.TaskStatus) -> None:
        try:
            reconciling = self._received(status)
            with trace.span("status", "status", task=status.task_id.value, state=P.TaskState.Name(status.state)):
                resp = self.client.task_status(status)
            self._processed(status, resp, reconciling)
        except Exception as e:  # noqa: BLE001
            self._exit(e)

    def status_updates(self, driver, statuses: List[P.TaskStatus]) -> None:
        """Status updates that arrived together on the event stream (the driver calls this
        instead of ``status_update`` when it has read several at once, and acknowledges them
        after it returns): the client stores them in one transaction."""
        if len(statuses) == 1:
            self.status_update(driver, statuses[0])
            return
        try:
            flags = [self._received(s) for s in statuses]
            batch = getattr(self.client, "task_statuses", None)   # clients not built on MesosEventClient
            with trace.span("status_batch", "status", n=len(statuses)):
                resps = batch(statuses) if batch is not None else [self.client.task_status(s) for s in statuses]
            for status, resp, reconciling in zip(statuses, resps, flags):
                self._processed(status, resp, reconciling)
        except Exception as e:  # noqa: BLE001
            self._exit(e)

    def _received(self, status: P.TaskStatus) -> bool:
        LOGGER.info("Received status update for taskId=%s state=%s message='%s'", status.task_id.value,
                    P.TaskState.Name(status.state), status.message)
        metrics.record_status(status)
        # a status during explicit reconciliation may end it: wake the loop whatever the state
        awaiting = getattr(self.client, "awaiting_reconciliation", None)
        return awaiting is not None and awaiting()

    def _processed(self, status: P.TaskStatus, resp, reconciling: bool) -> None:
        relaunch_kill = task_killer.ends_relaunch_kill(status)
        eligible = task_killer.update(status)
        if resp.result == TaskStatusResult.UNKNOWN_TASK:
            if eligible:
                LOGGER.info("Received status update for unknown task, marking task to be killed: %s",
                            status.task_id.value)
                task_killer.kill_task(status.task_id)
            else:
                LOGGER.warning("Received status update for unknown task, but task should not be killed "
                               "again: %s", status.task_id.value)
        # A task that ended (finished, failed, killed: after a kill issued for a relaunch
        # too) released reservations the plans reuse: an in-place relaunch or recovery, or
        # the pod's next step. A revive has the master offer them now, and that offer wakes
        # the loop for the relaunch (after a relaunch kill no full cycle runs first: the
        # offers in hand cannot hold them). For a replacement placed elsewhere the offer
        # carries the stale reservations to release, which a scheduler that has gone idle
        # (suppressed) would otherwise never be offered.
        released = status.state in _RELEASING_STATES and resp.result != TaskStatusResult.UNKNOWN_TASK
        work = can_create_work(status) and not relaunch_kill
        if work and status.state == P.TASK_RUNNING:
            # a readiness result: does any plan have a step it could unblock, or is this the
            # end of the last launched step (the cycle then suppresses offers)?
            useful = getattr(self.client, "offer_cycle_useful", None)
            work = useful is None or useful()
        if resp.result == TaskStatusResult.UNKNOWN_TASK or reconciling or work:
            self.offer_processor.kick()
        if relaunch_kill or released:
            self.offer_processor.reoffer_released()

    def offer_rescinded(self, driver, offer_id: P.OfferID) -> None:
        try:
            self.offer_processor.dequeue(offer_id)
        except Exception as e:  # noqa: BLE001
            self._exit(e)

    def framework_message(self, driver, executor_id, agent_id, data: bytes) -> None:
        LOGGER.error("Received unsupported %d byte Framework Message from Executor %s on Agent %s", len(data),
                     executor_id.value, agent_id.value)

    def disconnected(self, driver) -> None:
        LOGGER.error("Disconnected from Master, shutting down.")
        ProcessExit.exit(ProcessExit.DISCONNECTED)

    def agent_lost(self, driver, agent_id) -> None:
        LOGGER.warning("Agent lost: %s", agent_id.value)

    def executor_lost(self, driver, executor_id, agent_id, status: int) -> None:
        LOGGER.warning("Lost Executor: %s on Agent: %s", executor_id.value, agent_id.value)

    def error(self, driver, message: str) -> None:
        LOGGER.error("SchedulerDriver returned an error, shutting down: %s", message)
        ProcessExit.exit(ProcessExit.ERROR)

    def stop(self) -> None:
        self.offer_processor.stop()
        self.implicit_reconciler.stop()
        close = getattr(self.client, "close", None)
        if callable(close):
            close()
