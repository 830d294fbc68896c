"""The seam between the framework event pump and the service scheduler(s).

Reference: sdk/.../scheduler/MesosEventClient.java:14-490 (response types) and
sdk/.../scheduler/OfferResources.java.
"""
from __future__ import annotations

import enum
from typing import List

from dcos_commons_amd.mesos import protos as P


class ClientStatusResult(enum.Enum):
    WORKING = "WORKING"
    IDLE = "IDLE"


class WorkingState(enum.Enum):
    FOOTPRINT = "FOOTPRINT"
    LAUNCH = "LAUNCH"


class IdleRequest(enum.Enum):
    NONE = "NONE"
    START_UNINSTALL = "START_UNINSTALL"
    REMOVE_CLIENT = "REMOVE_CLIENT"


class ClientStatusResponse:
    __slots__ = ("result", "working_state", "has_new_work", "idle_request")

    def __init__(self, result, working_state=None, has_new_work=False, idle_request=None):
        self.result = result
        self.working_state = working_state
        self.has_new_work = has_new_work
        self.idle_request = idle_request

    @staticmethod
    def footprint(has_new_work: bool) -> "ClientStatusResponse":
        return ClientStatusResponse(ClientStatusResult.WORKING, WorkingState.FOOTPRINT, has_new_work)

    @staticmethod
    def launching(has_new_work: bool) -> "ClientStatusResponse":
        return ClientStatusResponse(ClientStatusResult.WORKING, WorkingState.LAUNCH, has_new_work)

    @staticmethod
    def idle() -> "ClientStatusResponse":
        return ClientStatusResponse(ClientStatusResult.IDLE, idle_request=IdleRequest.NONE)

    @staticmethod
    def ready_to_uninstall() -> "ClientStatusResponse":
        return ClientStatusResponse(ClientStatusResult.IDLE, idle_request=IdleRequest.START_UNINSTALL)

    @staticmethod
    def ready_to_remove() -> "ClientStatusResponse":
        return ClientStatusResponse(ClientStatusResult.IDLE, idle_request=IdleRequest.REMOVE_CLIENT)

    def _key(self):
        return (self.result, self.working_state, self.has_new_work, self.idle_request)

    def __eq__(self, other):
        return isinstance(other, ClientStatusResponse) and self._key() == other._key()

    def __hash__(self):
        return hash(self._key())

    def __repr__(self):
        if self.working_state is not None:
            ws = self.working_state.value + ("+newWork" if self.has_new_work else "")
            return f"{self.result.value}/{ws}"
        if self.idle_request is not None:
            return f"{self.result.value}/{self.idle_request.value}"
        return self.result.value


class OfferResult(enum.Enum):
    NOT_READY = "NOT_READY"
    PROCESSED = "PROCESSED"


class OfferResponse:
    """``streamed``: the recommendations were already sent to the master through the
    ``launch_stream`` callback; the caller must not ACCEPT them again."""

    __slots__ = ("result", "recommendations", "streamed")

    def __init__(self, result: OfferResult, recommendations, streamed: bool = False):
        self.result = result
        self.recommendations = list(recommendations)
        self.streamed = streamed

    @staticmethod
    def not_ready(recs=()) -> "OfferResponse":
        return OfferResponse(OfferResult.NOT_READY, recs)

    @staticmethod
    def processed(recs, streamed: bool = False) -> "OfferResponse":
        return OfferResponse(OfferResult.PROCESSED, recs, streamed)


class UnexpectedResult(enum.Enum):
    FAILED = "FAILED"
    PROCESSED = "PROCESSED"


class OfferResources:
    __slots__ = ("offer", "resources")

    def __init__(self, offer: P.Offer, resources=None):
        self.offer = offer
        self.resources: List[P.Resource] = list(resources or [])

    def add(self, r: P.Resource) -> "OfferResources":
        self.resources.append(r)
        return self

    def add_all(self, rs) -> "OfferResources":
        self.resources.extend(rs)
        return self


class UnexpectedResourcesResponse:
    __slots__ = ("result", "offer_resources")

    def __init__(self, result: UnexpectedResult, offer_resources):
        self.result = result
        self.offer_resources = list(offer_resources)

    @staticmethod
    def failed(r=()) -> "UnexpectedResourcesResponse":
        return UnexpectedResourcesResponse(UnexpectedResult.FAILED, r)

    @staticmethod
    def processed(r) -> "UnexpectedResourcesResponse":
        return UnexpectedResourcesResponse(UnexpectedResult.PROCESSED, r)


class TaskStatusResult(enum.Enum):
    UNKNOWN_TASK = "UNKNOWN_TASK"
    PROCESSED = "PROCESSED"


class TaskStatusResponse:
    __slots__ = ("result",)

    def __init__(self, result: TaskStatusResult):
        self.result = result

    @staticmethod
    def unknown_task() -> "TaskStatusResponse":
        return TaskStatusResponse(TaskStatusResult.UNKNOWN_TASK)

    @staticmethod
    def processed() -> "TaskStatusResponse":
        return TaskStatusResponse(TaskStatusResult.PROCESSED)


class MesosEventClient:
    def registered(self, re_registered: bool) -> None:
        raise NotImplementedError

    def unregistered(self) -> None:
        raise NotImplementedError

    def get_client_status(self) -> ClientStatusResponse:
        raise NotImplementedError

    def offers(self, offers, launch_stream=None) -> OfferResponse:
        """``launch_stream(recs)``, when the client supports it, sends one step's recorded
        recommendations to the master before the next step is evaluated; those recommendations
        are then returned with ``OfferResponse.streamed`` set on them."""
        raise NotImplementedError

    def get_unexpected_resources(self, unused_offers) -> UnexpectedResourcesResponse:
        raise NotImplementedError

    def task_status(self, status: P.TaskStatus) -> TaskStatusResponse:
        raise NotImplementedError

    def task_statuses(self, statuses: List[P.TaskStatus]) -> List[TaskStatusResponse]:
        """Several statuses delivered together, in arrival order (no reference counterpart: the
        reference handles one per driver callback). Clients that can store them in one
        transaction override this."""
        return [self.task_status(s) for s in statuses]

    def awaiting_reconciliation(self) -> bool:
        """True while explicit reconciliation has not finished. Offers are refused until then, so
        every status that arrives in that window may be the one that ends it, and the framework
        wakes the offer loop for each of them whatever its state (no reference counterpart: the
        reference's offer loop only polls)."""
        return False

    def get_http_endpoints(self):
        """Returns a list of ``dcos_commons_amd.http`` route providers."""
        return []
