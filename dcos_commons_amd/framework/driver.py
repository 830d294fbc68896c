"""The scheduler-driver seam and its process-global instance.

Reference: sdk/.../framework/Driver.java (global ``SchedulerDriver`` singleton) and the
``org.apache.mesos.SchedulerDriver`` interface. Implementations:
* ``dcos_commons_amd.mesos.http_driver.V1HttpSchedulerDriver`` -- Mesos v1 HTTP scheduler API;
* ``dcos_commons_amd.mesos.local_master.LocalSchedulerDriver`` -- in-process Mesos master;
* ``dcos_commons_amd.testing.RecordingDriver`` -- records calls for simulation tests.
"""
from __future__ import annotations

import threading
from typing import Iterable, List, Optional

from dcos_commons_amd.mesos import protos as P


class SchedulerDriver:
    def accept_offers(self, offer_ids: Iterable[P.OfferID], operations: Iterable[P.Offer.Operation],
                      filters: P.Filters) -> None:
        raise NotImplementedError

    def decline_offer(self, offer_id: P.OfferID, filters: Optional[P.Filters] = None) -> None:
        raise NotImplementedError

    def decline_offers(self, offer_ids: Iterable[P.OfferID], filters: Optional[P.Filters] = None) -> None:
        for oid in offer_ids:
            self.decline_offer(oid, filters)

    def kill_task(self, task_id: P.TaskID) -> None:
        raise NotImplementedError

    def reconcile_tasks(self, statuses: List[P.TaskStatus]) -> None:
        raise NotImplementedError

    def revive_offers(self) -> None:
        raise NotImplementedError

    def suppress_offers(self) -> None:
        raise NotImplementedError

    def acknowledge_status_update(self, status: P.TaskStatus) -> None:
        pass

    def teardown(self) -> None:
        """Remove the framework from the master (uninstall complete)."""
        raise NotImplementedError

    def stop(self, failover: bool = True) -> None:
        pass


_driver: Optional[SchedulerDriver] = None
_lock = threading.Lock()


def get_instance() -> Optional[SchedulerDriver]:
    return _driver


def set_driver(driver: Optional[SchedulerDriver]) -> None:
    global _driver
    with _lock:
        _driver = driver
