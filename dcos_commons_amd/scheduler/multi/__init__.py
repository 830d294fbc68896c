"""Several services behind one Mesos framework.

Reference: sdk/.../scheduler/multi/{MultiServiceEventClient,MultiServiceManager,ServiceStore,
OfferDiscipline,AllDiscipline,ParallelFootprintDiscipline,DisciplineSelectionStore,
MultiServiceRunner,ServiceFactory}.java and http/endpoints/Multi*Resource.java.

* ``MultiServiceEventClient`` fans Mesos events out to the registered services: each WORKING
  service (allowed by the offer discipline) sees, in order, the offers the previous services left
  unused; unexpected reservations are routed to their owner by the reservation's ``namespace``
  label; task statuses by the service name embedded in the TaskID.
* ``ParallelFootprintDiscipline`` lets at most N services grow their footprint (reserve) at once
  (``RESERVE_DISCIPLINE``), persisting the selection in ``SelectedServices``.
* ``ServiceStore`` persists each dynamically added service's context under
  ``ServiceList/<name>/Context`` (<= 100 KiB) so the service list survives a restart.
* HTTP: ``/v1/service/<sanitized-name>/...`` is delegated to that service's own API, and
  ``/v1/health`` reports 200/202/417 across every service's deploy+recovery plans.
"""
from __future__ import annotations

import logging
from typing import Callable, Collection, Dict, List, Optional, Set

from dcos_commons_amd.http.api import Request, Response, Route, Router, json_ok, not_found
from dcos_commons_amd.offer import common_id_utils
from dcos_commons_amd.offer.resources import get_namespace, get_reservation
from dcos_commons_amd.scheduler.mesos_event_client import (
    ClientStatusResponse,
    ClientStatusResult,
    IdleRequest,
    MesosEventClient,
    OfferResources,
    OfferResponse,
    OfferResult,
    TaskStatusResponse,
    UnexpectedResourcesResponse,
    UnexpectedResult,
    WorkingState,
)
from dcos_commons_amd.storage.persister import Persister, PersisterException, Reason
from dcos_commons_amd.storage.persister_utils import join_paths, with_escaped_slashes
from dcos_commons_amd.utils.locks import new_rw_lock

LOGGER = logging.getLogger(__name__)


# ---------------------------------------------------------------------------------------
# offer disciplines


class OfferDiscipline:
    def update_services(self, service_names: Collection[str]) -> None:
        raise NotImplementedError

    def update_service_status(self, service_name: str, status: ClientStatusResponse) -> bool:
        raise NotImplementedError


class AllDiscipline(OfferDiscipline):
    def update_services(self, service_names) -> None:
        pass

    def update_service_status(self, service_name, status) -> bool:
        return True


class DisciplineSelectionStore:
    PATH = "SelectedServices"
    DELIM = "__"

    def __init__(self, persister: Persister):
        self.persister = persister
        self._cache: Optional[frozenset] = None

    def store_selected_services(self, names: Set[str]) -> bool:
        if self._cache is not None and set(names) == set(self._cache):
            return False
        self._cache = frozenset(names)
        self.persister.set(self.PATH, self.DELIM.join(sorted(names)).encode())
        return True

    def fetch_selected_services(self) -> frozenset:
        if self._cache is not None:
            return self._cache
        try:
            data = self.persister.get(self.PATH)
        except PersisterException as e:
            if e.reason != Reason.NOT_FOUND:
                raise
            data = b""
        self._cache = frozenset(x for x in (data or b"").decode().split(self.DELIM) if x)
        return self._cache


class ParallelFootprintDiscipline(OfferDiscipline):
    def __init__(self, reserve_limit: int, store: DisciplineSelectionStore):
        if reserve_limit <= 0:
            raise ValueError(f"Reservation limit must be 1 or greater, was: {reserve_limit}")
        self.max = reserve_limit
        self.store = store
        self.selected: Optional[Set[str]] = None

    def update_services(self, service_names) -> None:
        if self.selected is None:
            self.selected = set(self.store.fetch_selected_services())
            if self.selected:
                LOGGER.info("Recovered selected services for deployment: %s", sorted(self.selected))
        self.selected &= set(service_names)
        self.store.store_selected_services(self.selected)

    def update_service_status(self, service_name, status) -> bool:
        if self.selected is None:
            raise RuntimeError("update_service_status() called without any preceding call to update_services()")
        if status.result == ClientStatusResult.WORKING and status.working_state == WorkingState.FOOTPRINT:
            if len(self.selected) < self.max:
                self.selected.add(service_name)
            if service_name in self.selected:
                return True
            LOGGER.info("Service %s is waiting for a footprint slot (RESERVE_DISCIPLINE=%d)", service_name, self.max)
            return False
        self.selected.discard(service_name)
        return True


# ---------------------------------------------------------------------------------------
# service registry + store


class MultiServiceManager:
    def __init__(self):
        rw = new_rw_lock("MultiServiceManager")
        self._r, self._w = rw.read_lock, rw.write_lock
        self.services: Dict[str, object] = {}
        self.sanitized: Dict[str, str] = {}
        self.is_registered = False

    def get_service_names(self) -> List[str]:
        with self._r:
            return sorted(self.services)

    def get_service(self, name: str):
        with self._r:
            return self.services.get(name)

    def get_service_sanitized(self, sanitized: str):
        with self._r:
            orig = self.sanitized.get(sanitized)
            return self.services.get(orig) if orig is not None else None

    def put_service(self, service) -> "MultiServiceManager":
        name = service.service_spec.name
        sanitized = common_id_utils.to_sanitized_service_name(name)
        with self._w:
            prev = self.sanitized.get(sanitized)
            if prev is not None and prev != name:
                raise ValueError(f"Service named '{name}' conflicts with existing service '{prev}': matching "
                                 f"sanitized name '{sanitized}'")
            self.sanitized[sanitized] = name
            self.services[name] = service
            call_registered = self.is_registered
        if call_registered:
            service.registered(False)
        return self

    def get_matching_service(self, status):
        try:
            sanitized = common_id_utils.to_sanitized_service_name_from_id(status.task_id)
        except Exception:  # noqa: BLE001
            sanitized = None
        if not sanitized:
            LOGGER.error("Received task status with malformed id '%s', unable to route to service",
                         status.task_id.value)
            return None
        return self.get_service_sanitized(sanitized)

    def uninstall_services(self, names: Collection[str]) -> None:
        to_init = []
        with self._w:
            for name in names:
                cur = self.services.get(name)
                if cur is None:
                    LOGGER.warning("Service '%s' does not exist, cannot trigger uninstall", name)
                    continue
                if not hasattr(cur, "to_uninstall_scheduler"):
                    LOGGER.warning("Service '%s' is already uninstalling, leaving as-is", name)
                    continue
                u = cur.to_uninstall_scheduler()
                if self.is_registered:
                    to_init.append(u)
                self.services[name] = u
        for u in to_init:
            u.registered(False)

    def uninstall_service(self, name: str) -> None:
        self.uninstall_services([name])

    def remove_services(self, names: Collection[str]) -> None:
        with self._w:
            for name in names:
                self.services.pop(name, None)
                self.sanitized.pop(common_id_utils.to_sanitized_service_name(name), None)

    def all_services(self) -> list:
        with self._r:
            return list(self.services.values())

    def registered(self, re_registered: bool) -> None:
        with self._r:
            self.is_registered = True
            current = list(self.services.values())
        for s in current:
            s.registered(re_registered)


ServiceFactory = Callable[[bytes], object]


class ServiceStore:
    ROOT = "ServiceList"
    CONTEXT = "Context"
    CONTEXT_LIMIT = 100 * 1024

    def __init__(self, persister: Persister, service_factory: ServiceFactory):
        self.persister = persister
        self.factory = service_factory

    def _base(self, name: str) -> str:
        return join_paths(self.ROOT, with_escaped_slashes(name))

    def get(self, name: str) -> Optional[bytes]:
        try:
            return self.persister.get(join_paths(self._base(name), self.CONTEXT))
        except PersisterException as e:
            if e.reason == Reason.NOT_FOUND:
                return None
            raise

    def recover(self) -> list:
        try:
            children = self.persister.get_children(self.ROOT)
        except PersisterException as e:
            if e.reason == Reason.NOT_FOUND:
                return []
            raise
        out = []
        for child in children:
            try:
                out.append(self.factory(self.persister.get(join_paths(self.ROOT, child, self.CONTEXT))))
            except Exception:  # noqa: BLE001
                LOGGER.exception("Unable to reconstruct service %s during recovery, continuing without it", child)
        return out

    def put(self, context: bytes):
        service = self.factory(context)
        name = service.service_spec.name
        if context is not None and len(context) > self.CONTEXT_LIMIT:
            raise ValueError(f"Provided context for service='{name}' is {len(context)} bytes, but limit is "
                             f"{self.CONTEXT_LIMIT} bytes")
        self.persister.set(join_paths(self._base(name), self.CONTEXT), context or b"")
        return service

    def remove(self, name: str) -> None:
        try:
            self.persister.recursive_delete(self._base(name))
        except PersisterException as e:
            if e.reason != Reason.NOT_FOUND:
                raise

    def uninstall_callback(self) -> Callable[[str], None]:
        def cb(name: str) -> None:
            try:
                self.remove(name)
            except PersisterException:
                LOGGER.exception("Failed to clean up uninstalled service %s", name)
        return cb


# ---------------------------------------------------------------------------------------
# event client


def _filter_out_accepted(offers, recs):
    used = {r.offer_id.value for r in recs if r.get_operation() is not None}
    return [o for o in offers if o.id.value not in used]


class MultiServiceEventClient(MesosEventClient):
    def __init__(self, framework_name: str, scheduler_config, manager: MultiServiceManager, persister=None,
                 custom_endpoints=(), uninstall_callback: Optional[Callable[[str], None]] = None,
                 discipline: Optional[OfferDiscipline] = None, deregister_step=None):
        self.framework_name = framework_name
        self.scheduler_config = scheduler_config
        self.manager = manager
        self.custom_endpoints = list(custom_endpoints)
        self.uninstall_callback = uninstall_callback or (lambda name: None)
        if discipline is None:
            n = scheduler_config.multi_service_reserve_discipline() if scheduler_config is not None else 0
            discipline = (ParallelFootprintDiscipline(n, DisciplineSelectionStore(persister))
                          if n > 0 and persister is not None else AllDiscipline())
        self.discipline = discipline
        if deregister_step is None and scheduler_config is not None and scheduler_config.is_uninstall_enabled():
            from dcos_commons_amd.scheduler.uninstall import DeregisterStep

            deregister_step = DeregisterStep()
        self.deregister_step = deregister_step
        self.services_to_offer: List[str] = []

    def registered(self, re_registered: bool) -> None:
        self.manager.registered(re_registered)

    def unregistered(self) -> None:
        if self.deregister_step is None:
            raise RuntimeError("unregistered() called, but we are not uninstalling")
        self.deregister_step.set_complete()

    def get_client_status(self) -> ClientStatusResponse:
        self.services_to_offer = []
        to_uninstall, to_remove = [], []
        services = self.manager.all_services()
        if not services:
            return ClientStatusResponse.ready_to_remove() if self.deregister_step is not None \
                else ClientStatusResponse.idle()
        try:
            self.discipline.update_services({s.service_spec.name for s in services})
        except Exception:  # noqa: BLE001
            LOGGER.exception("Failed to update selected services in offer discipline, continuing anyway")
        all_idle, any_footprint, any_new = True, False, False
        for s in services:
            name = s.service_spec.name
            st = s.get_client_status()
            allowed = self.discipline.update_service_status(name, st)
            if st.result == ClientStatusResult.WORKING:
                all_idle = False
                if allowed:
                    self.services_to_offer.append(name)
                if st.working_state == WorkingState.FOOTPRINT:
                    any_footprint = True
                if st.has_new_work:
                    any_new = True
            elif st.idle_request == IdleRequest.REMOVE_CLIENT:
                to_remove.append(s)
            elif st.idle_request == IdleRequest.START_UNINSTALL:
                to_uninstall.append(name)
        if all_idle:
            resp = ClientStatusResponse.idle()
        elif any_footprint:
            resp = ClientStatusResponse.footprint(any_new)
        else:
            resp = ClientStatusResponse.launching(any_new)
        if to_uninstall:
            LOGGER.info("Starting uninstall for %d service(s): %s", len(to_uninstall), to_uninstall)
            self.manager.uninstall_services(to_uninstall)
        if to_remove:
            names = [s.service_spec.name for s in to_remove]
            LOGGER.info("Removing %d uninstalled service(s): %s", len(names), names)
            self.manager.remove_services(names)
            for s in to_remove:
                s.state_store.delete_all_data_if_namespaced()
                self.uninstall_callback(s.service_spec.name)
        return resp

    def offers(self, offers, launch_stream=None) -> OfferResponse:
        if not self.services_to_offer:
            return OfferResponse.processed([])
        recs, remaining, not_ready = [], list(offers), False
        for name in self.services_to_offer:
            s = self.manager.get_service(name)
            if s is None:
                LOGGER.warning("Service '%s' was scheduled to receive offers, then later removed", name)
                continue
            resp = s.offers(remaining)
            recs.extend(resp.recommendations)
            if remaining and resp.recommendations:
                remaining = _filter_out_accepted(remaining, resp.recommendations)
            if resp.result != OfferResult.PROCESSED:
                not_ready = True
        return OfferResponse.not_ready(recs) if not_ready else OfferResponse.processed(recs)

    def get_unexpected_resources(self, unused_offers) -> UnexpectedResourcesResponse:
        unexpected: Dict[str, OfferResources] = {}
        by_service: Dict[str, Dict[str, OfferResources]] = {}

        def entry(m, offer):
            return m.setdefault(offer.id.value, OfferResources(offer))

        default_service = self.manager.get_service_sanitized(self.framework_name)
        for offer in unused_offers:
            for r in offer.resources:
                ns = get_namespace(r)
                if ns:
                    entry(by_service.setdefault(ns, {}), offer).add(r)
                elif get_reservation(r) is not None:
                    if default_service is not None:
                        entry(by_service.setdefault(default_service.service_spec.name, {}), offer).add(r)
                    else:
                        LOGGER.error("Ignoring malformed resource in offer %s: neither namespace label nor default "
                                     "service found", offer.id.value)
        failed = False
        for name, offers_map in by_service.items():
            s = self.manager.get_service(name) or self.manager.get_service_sanitized(name)
            if s is None:
                # the owning service is gone: its reservations are garbage
                for orr in offers_map.values():
                    entry(unexpected, orr.offer).add_all(orr.resources)
                continue
            to_send = []
            from dcos_commons_amd.mesos import protos as P

            for orr in offers_map.values():
                o = P.Offer()
                o.CopyFrom(orr.offer)
                del o.resources[:]
                o.resources.extend(orr.resources)
                to_send.append(o)
            resp = s.get_unexpected_resources(to_send)
            if resp.result == UnexpectedResult.FAILED:
                failed = True
            for orr in resp.offer_resources:
                entry(unexpected, orr.offer).add_all(orr.resources)
        vals = list(unexpected.values())
        return UnexpectedResourcesResponse.failed(vals) if failed else UnexpectedResourcesResponse.processed(vals)

    def awaiting_reconciliation(self) -> bool:
        return any(s.awaiting_reconciliation() for s in self.manager.all_services())

    def offer_cycle_useful(self) -> bool:
        """After a readiness result: useful if any service could use a cycle (a service whose last
        launched step completed also frees the offer discipline for the others); no services:
        always (deregistration)."""
        services = self.manager.all_services()
        if not services:
            return True
        for s in services:
            useful = getattr(s, "offer_cycle_useful", None)
            if useful is None or useful():
                return True
        return False

    def task_status(self, status) -> TaskStatusResponse:
        s = self.manager.get_matching_service(status)
        if s is None:
            s = self.manager.get_service_sanitized(self.framework_name)
        if s is None:
            LOGGER.info("Received status for unknown task %s", status.task_id.value)
            return TaskStatusResponse.unknown_task()
        return s.task_status(status)

    def get_http_endpoints(self):
        from dcos_commons_amd.http.resources import PlansResource
        from dcos_commons_amd.scheduler.plan.elements import DefaultPhase, DefaultPlan
        from dcos_commons_amd.scheduler.plan.managers import DefaultPlanManager
        from dcos_commons_amd.scheduler.plan.strategy import SerialStrategy

        pms = []
        if self.deregister_step is not None:
            pms = [DefaultPlanManager.create_proceeding(DefaultPlan(
                "deploy", [DefaultPhase("deregister-framework", [self.deregister_step], SerialStrategy())],
                SerialStrategy()))]
        return [MultiHealthResource(self.manager, self.scheduler_config, pms), PlansResource(pms),
                MultiServiceResource(self.manager)] + self.custom_endpoints


# ---------------------------------------------------------------------------------------
# HTTP


class MultiServiceResource:
    """``/v1/service/<sanitized-name>/<rest>`` -> ``/v1/<rest>`` on that service's own API."""

    def __init__(self, manager: MultiServiceManager):
        self.manager = manager
        self._routers: Dict[int, Router] = {}

    def _router(self, service) -> Router:
        r = self._routers.get(id(service))
        if r is None:
            r = self._routers[id(service)] = Router(service.get_http_endpoints())
        return r

    def routes(self) -> List[Route]:
        return [Route(m, "/v1/service/{svc}/{rest:path}", self.handle) for m in ("GET", "POST", "PUT", "DELETE")] + \
            [Route("GET", "/v1/service", lambda r: json_ok(self.manager.get_service_names()))]

    def handle(self, req: Request) -> Response:
        svc = req.params["svc"]
        service = self.manager.get_service_sanitized(svc)
        if service is None:
            return not_found(f"Service {svc}")
        prefix = f"/v1/service/{svc}"
        sub = "/v1" + req.path[len(prefix):]
        import urllib.parse

        qs = urllib.parse.urlencode(req.query)
        return self._router(service).dispatch(req.method, sub + ("?" + qs if qs else ""), req.body, req.headers)


class MultiHealthResource:
    """``/v1/health`` for a multi-service scheduler: build info with 417 if any deploy/recovery
    plan has errors, 202 while any is incomplete, else 200 (MultiHealthResource.java)."""

    def __init__(self, manager: MultiServiceManager, scheduler_config, extra_plan_managers=()):
        self.manager = manager
        self.scheduler_config = scheduler_config
        self.extra = list(extra_plan_managers)

    def routes(self) -> List[Route]:
        return [Route("GET", "/v1/health", self.health)]

    def _plans(self):
        plans = [pm.get_plan() for pm in self.extra]
        for s in self.manager.all_services():
            for pm in s.plan_coordinator.get_plan_managers():
                p = pm.get_plan()
                if p.is_deploy_plan() or p.is_recovery_plan():
                    plans.append(p)
        return plans

    def health(self, req=None) -> Response:
        plans = self._plans()
        if any(p.get_errors() for p in plans):
            code = 417
        elif any(not p.is_complete() for p in plans):
            code = 202
        else:
            code = 200
        info = self.scheduler_config.build_info() if self.scheduler_config is not None else {}
        return json_ok(info, code)


class MultiServiceRunner:
    """Checks the multi-service schema, then registers and runs the framework
    (MultiServiceRunner.java)."""

    def __init__(self, scheduler_config, framework_config, persister, client, using_gpus: bool = False,
                 driver_factory=None):
        from dcos_commons_amd.state.schema_version_store import SchemaVersion, SchemaVersionStore

        SchemaVersionStore(persister).check(SchemaVersion.MULTI_SERVICE)
        self.scheduler_config = scheduler_config
        self.framework_config = framework_config
        self.persister = persister
        self.client = client
        self.using_gpus = using_gpus
        self.driver_factory = driver_factory
        self.framework_runner = None

    def run(self, block: bool = True):
        from dcos_commons_amd import metrics
        from dcos_commons_amd.framework.framework_runner import FrameworkRunner

        metrics.configure_statsd(self.scheduler_config)
        self.framework_runner = FrameworkRunner(self.scheduler_config, self.framework_config, self.using_gpus,
                                                self.scheduler_config.is_region_awareness_enabled(),
                                                driver_factory=self.driver_factory)
        if block:
            from dcos_commons_amd.framework.process_exit import install_signal_handlers

            install_signal_handlers()
        return self.framework_runner.start(self.persister, self.client, block=block)

    def stop(self) -> None:
        if self.framework_runner is not None:
            self.framework_runner.stop()
