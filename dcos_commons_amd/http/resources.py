"""The scheduler's v1 REST resources.

Reference: sdk/.../http/endpoints/*.java and http/queries/{Plans,Pod,Config,State,Endpoints,
Artifact}Queries.java. Paths, JSON shapes and status codes follow the reference:
``GET /v1/plans/<p>`` is 200 when COMPLETE, 202 while in progress, 417 with errors
(PlansQueries.java:54-68); plan commands answer 208 "already reported" when a no-op; pod
restart/replace clear launch backoff and kill (PodQueries.java:282); ``/v1/health`` maps the
plan states to the reference's service status codes (HealthResource.java:31-88).
"""
from __future__ import annotations

import io
import json
import logging
import re
import uuid
from typing import Dict, List, Optional, Tuple

from dcos_commons_amd import metrics, trace
from dcos_commons_amd.debug import PlansTracker, TaskReservationsTracker, TaskStatusesTracker, thread_dump
from dcos_commons_amd.framework import task_killer
from dcos_commons_amd.http import endpoint_utils
from dcos_commons_amd.http.api import (
    Request,
    Response,
    Route,
    already_reported,
    command_result,
    html,
    json_ok,
    not_found,
    plain,
    read_data,
    status_only,
)
from dcos_commons_amd.mesos import protos as P
from dcos_commons_amd.offer import constants
from dcos_commons_amd.offer.common_id_utils import to_task_name
from dcos_commons_amd.offer.taskdata.labels import TaskException, TaskLabelReader, get_vips_from_labels
from dcos_commons_amd.offer.task_utils import get_pod_instance, get_task_ip_address, get_task_zone, task_has_zone
from dcos_commons_amd.scheduler.plan import backoff
from dcos_commons_amd.scheduler.plan.pod_instance_requirement import RecoveryType
from dcos_commons_amd.state import state_store_utils
from dcos_commons_amd.state.config_store import ConfigStoreException
from dcos_commons_amd.state.goal_state_override import GoalStateOverride, OverrideProgress, OverrideStatus
from dcos_commons_amd.state.state_store import StateStoreException
from dcos_commons_amd.storage.persister import Reason
from dcos_commons_amd.storage.persister_cache import PersisterCache

LOGGER = logging.getLogger(__name__)
ENVVAR = re.compile(r"^[A-Za-z_][A-Za-z0-9_]*$")
UNKNOWN_POD_LABEL = "UNKNOWN_POD"
FILE_NAME_PREFIX = "file-"
FILE_SIZE_LIMIT = 1024


def _pod_name(pod_type: str, index: int) -> str:
    return f"{pod_type}-{index}"


# ---------------------------------------------------------------------------------------
# plans


def plan_info(plan) -> dict:
    # the plan's status is read before its phases' (PlanInfo.forPlan): a phase that completes
    # meanwhile shows COMPLETE under a plan still shown IN_PROGRESS, never the reverse
    status = str(plan.get_status())
    return {
        "phases": [{
            "id": str(ph.get_id()),
            "name": ph.get_name(),
            "steps": [{"id": str(s.get_id()), "status": s.get_display_status(), "name": s.get_name(),
                       "message": s.get_message()} for s in ph.get_children()],
            "strategy": ph.get_strategy().get_name(),
            "status": str(ph.get_status()),
        } for ph in plan.get_children()],
        "errors": list(plan.get_errors()),
        "strategy": plan.get_strategy().get_name(),
        "status": status,
    }


class PlansResource:
    def __init__(self, plan_managers):
        self._pms = plan_managers  # list or callable returning the current list

    def plan_managers(self):
        return self._pms() if callable(self._pms) else self._pms

    def _pm(self, name: str):
        return next((pm for pm in self.plan_managers() if pm.get_plan().get_name() == name), None)

    def routes(self) -> List[Route]:
        return [
            Route("GET", "/v1/plans", self.list),
            Route("GET", "/v1/plans/{plan}", lambda r: self.get(r.params["plan"])),
            Route("POST", "/v1/plans/{plan}/start", self.start),
            Route("POST", "/v1/plans/{plan}/stop", lambda r: self.stop(r.params["plan"])),
            Route("POST", "/v1/plans/{plan}/continue", lambda r: self.continue_plan(r.params["plan"], r.q("phase"))),
            Route("POST", "/v1/plans/{plan}/interrupt", lambda r: self.interrupt(r.params["plan"], r.q("phase"))),
            Route("POST", "/v1/plans/{plan}/forceComplete",
                  lambda r: self.force_complete(r.params["plan"], r.q("phase"), r.q("step"))),
            Route("POST", "/v1/plans/{plan}/restart",
                  lambda r: self.restart(r.params["plan"], r.q("phase"), r.q("step"))),
            # DeprecatedPlanResource: /v1/plan == deploy
            Route("GET", "/v1/plan", lambda r: self.get(constants.DEPLOY_PLAN_NAME)),
            Route("POST", "/v1/plan/continue", lambda r: self.continue_plan(constants.DEPLOY_PLAN_NAME, None)),
            Route("POST", "/v1/plan/interrupt", lambda r: self.interrupt(constants.DEPLOY_PLAN_NAME, None)),
            Route("POST", "/v1/plan/forceComplete",
                  lambda r: self.force_complete(constants.DEPLOY_PLAN_NAME, r.q("phase"), r.q("step"))),
            Route("POST", "/v1/plan/restart",
                  lambda r: self.restart(constants.DEPLOY_PLAN_NAME, r.q("phase"), r.q("step"))),
        ]

    def list(self, req: Request = None) -> Response:
        return json_ok([pm.get_plan().get_name() for pm in self.plan_managers()])

    def get(self, name: str) -> Response:
        pm = self._pm(name)
        if pm is None:
            return not_found(f"Plan {name}")
        plan = pm.get_plan()
        code = 417 if plan.has_errors() else (200 if plan.is_complete() else 202)
        return json_ok(plan_info(plan), code)

    def start(self, req: Request) -> Response:
        name = req.params["plan"]
        try:
            params = req.json() or {}
        except ValueError:
            return plain("Couldn't parse parameters: invalid JSON", 400)
        if not isinstance(params, dict):
            return plain("Couldn't parse parameters: expected a JSON object", 400)
        for k in params:
            if not ENVVAR.match(k):
                return plain(f"Couldn't parse parameters: {k} is not a valid environment variable name", 400)
        pm = self._pm(name)
        if pm is None:
            return not_found(f"Plan {name}")
        plan = pm.get_plan()
        params = {str(k): str(v) for k, v in params.items()}
        plan.update_parameters(params)
        if plan.is_complete():
            plan.restart()
        plan.proceed()
        shown = "{" + ", ".join(f"{k}={v}" for k, v in params.items()) + "}"
        return json_ok(command_result(f"start {name} with parameters: {shown}"))

    def stop(self, name: str) -> Response:
        pm = self._pm(name)
        if pm is None:
            return not_found(f"Plan {name}")
        plan = pm.get_plan()
        plan.interrupt()
        plan.restart()
        return json_ok(command_result("stop"))

    def _phases(self, pm, id_or_name: str):
        try:
            pid = uuid.UUID(id_or_name)
            return [p for p in pm.get_plan().get_children() if p.get_id() == pid]
        except ValueError:
            return [p for p in pm.get_plan().get_children() if p.get_name() == id_or_name]

    def continue_plan(self, name: str, phase: Optional[str]) -> Response:
        pm = self._pm(name)
        if pm is None:
            return not_found(f"Plan {name}")
        if phase is not None:
            phases = self._phases(pm, phase)
            if not phases:
                return not_found(f"Phase {phase}")
            if all(p.is_running() for p in phases) or all(p.is_complete() for p in phases):
                return already_reported()
            for p in phases:
                p.proceed()
        else:
            plan = pm.get_plan()
            if plan.is_running() or plan.is_complete():
                return already_reported()
            plan.proceed()
        return json_ok(command_result("continue"))

    def interrupt(self, name: str, phase: Optional[str]) -> Response:
        pm = self._pm(name)
        if pm is None:
            return not_found(f"Plan {name}")
        if phase is not None:
            phases = self._phases(pm, phase)
            if not phases:
                return not_found(f"Phase {phase}")
            if all(p.is_interrupted() for p in phases) or all(p.is_complete() for p in phases):
                return already_reported()
            for p in phases:
                p.get_strategy().interrupt()
        else:
            plan = pm.get_plan()
            if plan.is_interrupted() or plan.is_complete():
                return already_reported()
            plan.interrupt()
        return json_ok(command_result("interrupt"))

    def _element(self, plan_name, phase_name, step_name):
        pm = self._pm(plan_name)
        if pm is None:
            return None, not_found(f"Plan {plan_name}")
        if not phase_name and not step_name:
            return pm.get_plan(), None
        if not phase_name:
            return None, plain("Missing phase", 400)
        phases = self._phases(pm, phase_name)
        if not phases:
            return None, not_found(f"Phase {phase_name}")
        phase = phases[0]
        if not step_name:
            return phase, None
        try:
            sid = uuid.UUID(step_name)
            steps = [s for s in phase.get_children() if s.get_id() == sid]
        except ValueError:
            steps = [s for s in phase.get_children() if s.get_name() == step_name]
        if len(steps) != 1:
            return None, not_found(f"Step {step_name}")
        return steps[0], None

    def force_complete(self, plan, phase, step) -> Response:
        el, err = self._element(plan, phase, step)
        if err is not None:
            return err
        if el.is_complete():
            return already_reported()
        el.force_complete()
        return json_ok(command_result(f"forceComplete for Plan: {plan}, Phase: {phase}, Step: {step}"))

    def restart(self, plan, phase, step) -> Response:
        el, err = self._element(plan, phase, step)
        if err is not None:
            return err
        if el.is_pending():
            return already_reported()
        if hasattr(el, "proceed"):
            el.proceed()
        el.restart()
        return json_ok(command_result(f"restart for Plan: {plan}, Phase: {phase}, Step: {step}"))


# ---------------------------------------------------------------------------------------
# pods


class GroupedTasks:
    def __init__(self, state_store):
        statuses = {s.task_id.value: s for s in state_store.fetch_statuses()}
        self.by_type: Dict[str, Dict[int, list]] = {}
        self.unknown: list = []
        for info in state_store.fetch_tasks():
            entry = (info, statuses.get(info.task_id.value))
            try:
                r = TaskLabelReader(info)
                self.by_type.setdefault(r.get_type(), {}).setdefault(r.get_index(), []).append(entry)
            except (TaskException, ValueError):
                self.unknown.append(entry)
        for instances in self.by_type.values():
            for tasks in instances.values():
                tasks.sort(key=lambda e: e[0].name)

    def pod_instance_tasks(self, pod_instance_name: str):
        for t in sorted(self.by_type):
            for i in sorted(self.by_type[t]):
                if _pod_name(t, i) == pod_instance_name:
                    return self.by_type[t][i]
        return None


def set_pods_permanently_failed(config_store, state_store, task_infos) -> None:
    """Default ``replace`` failure setter (reference PodQueries.FailureSetter, PodQueries.java:438):
    stamps ``permanently-failed`` on every task of each pod instance the launched tasks belong to.
    Stub tasks that were never launched (empty TaskID) are skipped."""
    from dcos_commons_amd.scheduler.recovery import set_pod_permanently_failed

    pods = {}
    for info in task_infos:
        if not info.task_id.value:
            LOGGER.info("Not marking task %s as failed due to empty taskId", info.name)
            continue
        try:
            pi = get_pod_instance(config_store, info)
            pods[pi.name] = pi
        except (TaskException, ValueError, ConfigStoreException):
            LOGGER.exception("Failed to get pod for task %s", info.task_id.value)
    for pi in pods.values():
        set_pod_permanently_failed(state_store, pi)


class PodResource:
    def __init__(self, state_store, config_store, service_name: str, failure_setter=None):
        self.state_store = state_store
        self.config_store = config_store
        self.service_name = service_name
        self.failure_setter = failure_setter or set_pods_permanently_failed

    def routes(self) -> List[Route]:
        return [
            Route("GET", "/v1/pod", self.list),
            Route("GET", "/v1/pod/status", self.statuses),
            Route("GET", "/v1/pod/{name}/status", lambda r: self.status(r.params["name"])),
            Route("GET", "/v1/pod/{name}/info", lambda r: self.info(r.params["name"])),
            Route("POST", "/v1/pod/{name}/pause",
                  lambda r: self.override(r.params["name"], r.text(), GoalStateOverride.PAUSED)),
            Route("POST", "/v1/pod/{name}/resume",
                  lambda r: self.override(r.params["name"], r.text(), GoalStateOverride.NONE)),
            Route("POST", "/v1/pod/{name}/restart", lambda r: self.restart(r.params["name"], RecoveryType.TRANSIENT)),
            Route("POST", "/v1/pod/{name}/replace", lambda r: self.restart(r.params["name"], RecoveryType.PERMANENT)),
        ]

    def list(self, req=None) -> Response:
        names, unknown = set(), []
        for info in self.state_store.fetch_tasks():
            try:
                r = TaskLabelReader(info)
                names.add(_pod_name(r.get_type(), r.get_index()))
            except (TaskException, ValueError):
                unknown.append(info.name)
        return json_ok(sorted(names) + [f"{UNKNOWN_POD_LABEL}_{n}" for n in sorted(unknown)])

    def _state_string(self, task_name: str, status) -> Optional[str]:
        if status is None:
            return None
        ov = self.state_store.fetch_goal_override_status(task_name)
        if ov != OverrideStatus.INACTIVE:
            if ov.progress == OverrideProgress.COMPLETE:
                return ov.target.serialized_name
            if ov.progress in (OverrideProgress.IN_PROGRESS, OverrideProgress.PENDING):
                return ov.target.transitioning_name
            return None
        s = P.TaskState.Name(status.state)
        return s[len("TASK_"):] if s.startswith("TASK_") else s

    def _instance_json(self, pod_instance_name: str, tasks) -> dict:
        out = {"name": pod_instance_name, "tasks": []}
        for info, status in tasks:
            t = {"id": info.task_id.value, "name": info.name}
            s = self._state_string(info.name, status)
            if s is not None:
                t["status"] = s
            out["tasks"].append(t)
        return out

    def statuses(self, req=None) -> Response:
        g = GroupedTasks(self.state_store)
        resp = {"service": self.service_name}
        pods = []
        for t in sorted(g.by_type):
            pods.append({"name": t, "instances": [self._instance_json(_pod_name(t, i), g.by_type[t][i])
                                                  for i in sorted(g.by_type[t])]})
        if g.unknown:
            pods.append({"name": UNKNOWN_POD_LABEL,
                         "instances": [self._instance_json(_pod_name(UNKNOWN_POD_LABEL, 0), g.unknown)]})
        if pods:
            resp["pods"] = pods
        return json_ok(resp)

    def status(self, name: str) -> Response:
        tasks = GroupedTasks(self.state_store).pod_instance_tasks(name)
        if tasks is None:
            return not_found(f"Pod {name}")
        return json_ok(self._instance_json(name, tasks))

    def info(self, name: str) -> Response:
        tasks = GroupedTasks(self.state_store).pod_instance_tasks(name)
        if tasks is None:
            return not_found(f"Pod {name}")
        return json_ok([{"info": P.to_v0_json(i), "status": P.to_v0_json(s) if s is not None else None}
                        for i, s in tasks])

    def override(self, name: str, body: str, override: GoalStateOverride) -> Response:
        try:
            task_filter = set(str(x) for x in json.loads(body)) if body.strip() else set()
        except ValueError:
            return status_only(400)
        all_tasks = GroupedTasks(self.state_store).pod_instance_tasks(name)
        if all_tasks is None:
            return not_found(f"Pod {name}")
        if task_filter:
            prefixed = {f"{name}-{f}" for f in task_filter}
            tasks = [e for e in all_tasks if e[0].name in prefixed or e[0].name in task_filter]
        else:
            tasks = list(all_tasks)
        if not tasks or len(tasks) < len(task_filter):
            return not_found(f"Pod {name}")
        pending = override.new_status(OverrideProgress.PENDING)
        for info, _ in tasks:
            self.state_store.store_goal_override_status(info.name, pending)
        return self._kill(name, tasks)

    def restart(self, name: str, recovery_type: RecoveryType) -> Response:
        tasks = GroupedTasks(self.state_store).pod_instance_tasks(name)
        if not tasks:
            return not_found(f"Pod {name}")
        for info, _ in tasks:
            if info.task_id.value:
                try:
                    backoff.get_instance().clear_delay(to_task_name(info.task_id))
                except (TaskException, ValueError):
                    pass
        LOGGER.info("Performing %s of pod %s by killing %d tasks", "replace" if recovery_type == RecoveryType.PERMANENT
                    else "restart", name, len(tasks))
        if recovery_type == RecoveryType.PERMANENT:
            self.failure_setter(self.config_store, self.state_store, [info for info, _ in tasks])
        return self._kill(name, tasks)

    @staticmethod
    def _kill(name: str, tasks) -> Response:
        for info, _ in tasks:
            if info.task_id.value:  # a footprint placeholder was never launched: nothing to kill
                task_killer.kill_task(info.task_id)
        return json_ok({"pod": name, "tasks": [info.name for info, _ in tasks]})


# ---------------------------------------------------------------------------------------
# configurations / state / endpoints / artifacts


class ConfigResource:
    def __init__(self, config_store):
        self.config_store = config_store

    def routes(self) -> List[Route]:
        return [
            Route("GET", "/v1/configurations", lambda r: json_ok([str(u) for u in self.config_store.list()])),
            Route("GET", "/v1/configurations/targetId", self.target_id),
            Route("GET", "/v1/configurations/target", self.target),
            Route("GET", "/v1/configurations/{id}", lambda r: self.get(r.params["id"])),
        ]

    def get(self, cid: str) -> Response:
        try:
            u = uuid.UUID(cid)
        except ValueError:
            return status_only(400)
        try:
            return json_ok(self.config_store.fetch(u).to_dict())
        except ConfigStoreException as e:
            return status_only(404 if e.reason == Reason.NOT_FOUND else 500)

    def target_id(self, req=None) -> Response:
        try:
            return json_ok([str(self.config_store.get_target_config())])
        except ConfigStoreException as e:
            return status_only(404 if e.reason == Reason.NOT_FOUND else 500)

    def target(self, req=None) -> Response:
        try:
            tid = self.config_store.get_target_config()
        except ConfigStoreException as e:
            return status_only(404 if e.reason == Reason.NOT_FOUND else 500)
        try:
            return json_ok(self.config_store.fetch(tid).to_dict())
        except ConfigStoreException:
            return status_only(500)


def _parse_multipart_file(req: Request) -> Tuple[Optional[bytes], Optional[int]]:
    """(file bytes, size declared in its Content-Disposition) of the ``file`` form field, or of the
    raw body when the request is not multipart; (None, None) when there is no payload."""
    ctype = req.headers.get("Content-Type") or req.headers.get("content-type") or ""
    if "multipart/form-data" not in ctype:
        return (req.body or None), None
    m = re.search(r'boundary="?([^";]+)"?', ctype)
    if not m:
        return None, None
    boundary = ("--" + m.group(1)).encode()
    for part in (req.body or b"").split(boundary):
        if b'name="file"' not in part:
            continue
        head, _, data = part.partition(b"\r\n\r\n")
        size = re.search(rb";\s*size=(-?\d+)", head)
        return (data[:-2] if data.endswith(b"\r\n") else data), (int(size.group(1)) if size else None)
    return None, None


class StateResource:
    def __init__(self, framework_store, state_store, property_deserializer=None):
        self.framework_store = framework_store
        self.state_store = state_store
        from dcos_commons_amd.state.serializer import StringPropertyDeserializer

        self.deserialize = property_deserializer or StringPropertyDeserializer()

    def routes(self) -> List[Route]:
        return [
            Route("GET", "/v1/state/frameworkId", self.framework_id),
            Route("GET", "/v1/state/files", self.files),
            Route("GET", "/v1/state/files/{name}", lambda r: self.get_file(r.params["name"])),
            Route("PUT", "/v1/state/files/{name}", self.put_file),
            Route("GET", "/v1/state/zone/tasks", self.zones),
            Route("GET", "/v1/state/zone/tasks/{task}", lambda r: self.zone(r.params["task"])),
            Route("GET", "/v1/state/zone/{podType}/{ip}", lambda r: self.zone_by_ip(r.params["podType"], r.params["ip"])),
            Route("GET", "/v1/state/properties", lambda r: json_ok(self.state_store.fetch_property_keys())),
            Route("GET", "/v1/state/properties/{key}", lambda r: self.property(r.params["key"])),
            Route("PUT", "/v1/state/refresh", self.refresh),
        ]

    def framework_id(self, req=None) -> Response:
        fid = self.framework_store.fetch_framework_id()
        if fid is None:
            return status_only(404)
        return json_ok([fid.value])

    def _file_names(self):
        return sorted({k[len(FILE_NAME_PREFIX):] for k in self.state_store.fetch_property_keys()
                       if k.startswith(FILE_NAME_PREFIX)})

    def files(self, req=None) -> Response:
        return plain("[" + ", ".join(self._file_names()) + "]")

    def get_file(self, name: str) -> Response:
        try:
            return plain(self.state_store.fetch_property(FILE_NAME_PREFIX + name).decode("utf-8"))
        except StateStoreException:
            return plain("Failed to get the file", 404)

    def put_file(self, req: Request) -> Response:
        try:
            data, declared = _parse_multipart_file(req)
            data = read_data(io.BytesIO(data) if data is not None else None, declared, FILE_SIZE_LIMIT)
        except ValueError as e:
            return plain(str(e), 400)
        self.state_store.store_property(FILE_NAME_PREFIX + req.params["name"], data)
        return status_only(200)

    def _zones(self) -> Dict[str, str]:
        out = {}
        for name in self.state_store.fetch_task_names():
            info = self.state_store.fetch_task(name)
            if info is not None and task_has_zone(info):
                out[name] = get_task_zone(info)
        return out

    def zones(self, req=None) -> Response:
        return json_ok(self._zones())

    def zone(self, task: str) -> Response:
        z = self._zones()
        return plain(z[task]) if task in z else status_only(404)

    def zone_by_ip(self, pod_type: str, ip: str) -> Response:
        for name in self.state_store.fetch_task_names():
            if not name.startswith(pod_type):
                continue
            st, info = self.state_store.fetch_status(name), self.state_store.fetch_task(name)
            if st is None or info is None:
                return status_only(404)
            if task_has_zone(info) and get_task_ip_address(st) == ip:
                return plain(get_task_zone(info))
        return status_only(404)

    def property(self, key: str) -> Response:
        try:
            return json_ok(self.deserialize(key, self.state_store.fetch_property(key)))
        except StateStoreException as e:
            return status_only(404 if e.reason == Reason.NOT_FOUND else 500)

    def refresh(self, req=None) -> Response:
        p = self.state_store.persister
        if not isinstance(p, PersisterCache):
            return status_only(409)
        p.refresh()
        return json_ok(command_result("refresh"))


class EndpointsResource:
    def __init__(self, state_store, service_name: str, scheduler_config, custom_endpoints=None):
        self.state_store = state_store
        self.service_name = service_name
        self.scheduler_config = scheduler_config
        self.custom = dict(custom_endpoints or {})

    def routes(self) -> List[Route]:
        return [
            Route("GET", "/v1/endpoints", self.list),
            Route("GET", "/v1/endpoints/{name}", lambda r: self.get(r.params["name"])),
        ]

    @staticmethod
    def _ips(status) -> List[str]:
        if status is None or not status.HasField("container_status"):
            return []
        return [a.ip_address for n in status.container_status.network_infos for a in n.ip_addresses]

    def _discovery(self) -> Dict[str, dict]:
        out: Dict[str, dict] = {}
        for info in self.state_store.fetch_tasks():
            if not info.HasField("discovery"):
                continue
            d = info.discovery
            auto_name = d.name if d.HasField("name") else info.name
            host = TaskLabelReader(info).get_hostname()
            ips = self._ips(self.state_store.fetch_status(info.name)) or \
                self._ips(state_store_utils.get_task_status_from_property(self.state_store, info.name))
            for port in d.ports.ports:
                if port.visibility != constants.DISPLAYED_PORT_VISIBILITY or not port.name:
                    continue
                host_ip = host if not ips else (ips[0] if len(ips) == 1 else "[" + ", ".join(ips) + "]")
                autoip = endpoint_utils.to_auto_ip_endpoint(self.service_name, auto_name, port.number,
                                                            self.scheduler_config)
                addr = endpoint_utils.to_endpoint(host_ip, port.number)
                e = out.setdefault(port.name, {})
                e.setdefault("dns", []).append(autoip)
                e.setdefault("address", []).append(addr)
                for vip_name, vip_port in get_vips_from_labels(port):
                    e["vip"] = endpoint_utils.to_vip_endpoint(self.service_name, self.scheduler_config, vip_name,
                                                              vip_port)
        return dict(sorted(out.items()))

    def list(self, req=None) -> Response:
        return json_ok(sorted(set(self.custom) | set(self._discovery())))

    def get(self, name: str) -> Response:
        producer = self.custom.get(name)
        if producer is not None:
            return plain(producer() if callable(producer) else str(producer))
        e = self._discovery().get(name)
        return json_ok(e) if e is not None else status_only(404)


class ArtifactResource:
    def __init__(self, config_store):
        self.config_store = config_store

    def routes(self) -> List[Route]:
        return [Route("GET", "/v1/artifacts/template/{configId}/{podType}/{taskName}/{configName}", self.template)]

    def template(self, req: Request) -> Response:
        p = req.params
        try:
            u = uuid.UUID(p["configId"])
        except ValueError:
            return status_only(400)
        try:
            spec = self.config_store.fetch(u)
        except ConfigStoreException as e:
            return status_only(404 if e.reason == Reason.NOT_FOUND else 500)
        pod = spec.pod(p["podType"])
        task = next((t for t in pod.tasks if t.name == p["taskName"]), None) if pod is not None else None
        cfg = next((c for c in task.config_files if c.name == p["configName"]), None) if task is not None else None
        if cfg is None:
            return status_only(404)
        return plain(cfg.template_content)


# ---------------------------------------------------------------------------------------
# health / debug / metrics

SERVICE_STATUS = {  # name -> (http code, priority)
    "INITIALIZING": (318, 1), "RUNNING": (200, 1), "ERROR_CREATING_SERVICE": (500, 1),
    "DEPLOYING_PENDING": (204, 2), "DEPLOYING_STARTING": (202, 2), "DELAYED": (208, 1),
    "DEPLOYING_WAITING_USER": (207, 2), "DEGRADED": (206, 3), "RECOVERING_PENDING": (203, 4),
    "RECOVERING_STARTING": (205, 4), "BACKING_UP": (320, 5), "RESTORING": (321, 5),
    "UPGRADE_ROLLBACK_DOWNGRADE": (326, 6), "SERVICE_UNAVAILABLE": (503, -1),
}


class HealthResource:
    def __init__(self, plan_coordinator, framework_store=None):
        self.coordinator = plan_coordinator
        self.framework_store = framework_store

    def routes(self) -> List[Route]:
        return [Route("GET", "/v1/health", lambda r: self.health(r.q_bool("verbose")))]

    def _plans(self):
        return [pm.get_plan() for pm in self.coordinator.get_plan_managers()]

    @staticmethod
    def _pending_or_starting(plan, pending, starting, delayed):
        steps = [s for ph in plan.get_children() for s in ph.get_children()]
        counts = {k: len([s for s in steps if getattr(s, "is_" + k)()])
                  for k in ("pending", "delayed", "prepared", "starting", "started", "complete")}
        if counts["delayed"]:
            code = delayed
        elif counts["pending"] or counts["prepared"]:
            code = pending
        elif counts["starting"] or counts["started"]:
            code = starting
        else:
            code = None
        prio = SERVICE_STATUS[pending][1]
        head = (f"Status Code {SERVICE_STATUS[code][0]} is TRUE," if code else
                f"Status Code {SERVICE_STATUS[pending][0]} and {SERVICE_STATUS[starting][0]} are both FALSE")
        reason = (f"Priority {prio}. {head} Steps: Total({len(steps)}) Pending({counts['pending']}) "
                  f"Prepared({counts['prepared']}) Starting({counts['starting']}) Started({counts['started']}) "
                  f"Completed({counts['complete']}) Delayed({counts['delayed']})")
        return code, reason

    def evaluate(self, verbose: bool = False):
        plans = self._plans()
        deploy = next(p for p in plans if p.is_deploy_plan())
        recovery = next((p for p in plans if p.is_recovery_plan()), None)

        def fmt(name, truth, tail):
            c, pr = SERVICE_STATUS[name]
            return f"Priority {pr}. Status Code {c} is {'TRUE' if truth else 'FALSE'}. {tail}"

        fid = None
        if self.framework_store is not None:
            try:
                fid = self.framework_store.fetch_framework_id()
            except StateStoreException:
                fid = None
        initializing = None if fid is not None else "INITIALIZING"
        init_reason = fmt("INITIALIZING", fid is None, f"Registered with Framework ID {fid.value}." if fid is not None
                          else "Mesos registration pending, no Framework ID found.")
        errors = any(p.get_errors() for p in plans)
        err_code = "ERROR_CREATING_SERVICE" if errors else None
        err_reason = fmt("ERROR_CREATING_SERVICE", errors,
                         "Errors found in plans." if errors else "No errors found in plans.")
        if initializing:
            complete_code = None
            complete_reason = fmt("RUNNING", False, "Service still initializing.")
        elif deploy.is_complete():
            complete_code = "RUNNING"
            complete_reason = fmt("RUNNING", True, "Service deploy plan is complete.")
        else:
            complete_code = None
            complete_reason = fmt("RUNNING", False, "Service deploy plan is NOT complete.")
        deploying_code, deploying_reason = self._pending_or_starting(deploy, "DEPLOYING_PENDING", "DEPLOYING_STARTING",
                                                                     "DELAYED")
        waiting = deploy.is_interrupted() or any(s.is_interrupted() for ph in deploy.get_children()
                                                 for s in ph.get_children())
        waiting_code = "DEPLOYING_WAITING_USER" if waiting else None
        waiting_reason = fmt("DEPLOYING_WAITING_USER", waiting,
                             "Service deploy plan is awaiting user input to proceed." if waiting
                             else "Service deploy plan does NOT need user input.")
        degraded_reason = "Priority 3. Status Code 206 is FALSE, Not implemented yet."
        if recovery is None:
            rec_code = None
            rec_reason = ("Priority 4. Status Code 203 and 205 is FALSE. Recovery plan manager not found.(might be "
                          "uninstalling)")
        elif recovery.is_complete():
            rec_code = None
            rec_reason = "Priority 4. Status Code 203 and 205 is FALSE. Recovery plan is complete."
        else:
            rec_code, rec_reason = self._pending_or_starting(recovery, "RECOVERING_PENDING", "RECOVERING_STARTING",
                                                             "DELAYED")

        def matching(regex, name, what):
            ps = [p for p in plans if re.fullmatch(regex, p.get_name())]
            c, pr = SERVICE_STATUS[name]
            if not ps:
                return None, f"Priority {pr}. Status Code {c} is FALSE. No {what} plans detected."
            running = sorted(p.get_name() for p in ps if p.is_running())
            if not running:
                return None, (f"Priority {pr}. Status Code {c} is FALSE. Following {what} plans not running: "
                              + ", ".join(sorted(p.get_name() for p in ps)))
            return name, f"Priority {pr}. Status Code {c} is TRUE. Following {what} plans found running: " + \
                ", ".join(running)

        backup_code, backup_reason = matching(r".*back.*", "BACKING_UP", "backup")
        restore_code, restore_reason = matching(r".*restor.*", "RESTORING", "restore")
        upgrade_reason = "Priority 6. Status Code 326 is FALSE, Not implemented yet."

        code = err_code or initializing or deploying_code or waiting_code or rec_code or complete_code
        if code == "RUNNING":
            code = restore_code or backup_code or code
        if code is None:
            code = "SERVICE_UNAVAILABLE"
        body = {}
        if verbose:
            body["reasons"] = [err_reason, init_reason, waiting_reason, complete_reason, deploying_reason,
                               degraded_reason, rec_reason, backup_reason, restore_reason, upgrade_reason]
        body["value"] = SERVICE_STATUS[code][0]
        return code, body

    def health(self, verbose: bool = False) -> Response:
        code, body = self.evaluate(verbose)
        return json_ok(body, SERVICE_STATUS[code][0])


class DebugResource:
    """``/v1/debug/*`` and ``/v2/debug/offers`` (DebugResource, DebugOffersResource, PlansDebugResource,
    TaskStatusesResource, TaskReservationsResource)."""

    def __init__(self, scheduler):
        self.scheduler = scheduler
        self.plans_tracker = PlansTracker(scheduler.plan_coordinator, scheduler.state_store)
        self.statuses_tracker = TaskStatusesTracker(scheduler.plan_coordinator, scheduler.state_store)
        self.reservations_tracker = TaskReservationsTracker(scheduler.state_store)

    def routes(self) -> List[Route]:
        def f(r):
            return r.q("plan"), r.q("phase"), r.q("step")
        return [
            Route("GET", "/v1/debug/offers", self.offers),
            Route("GET", "/v1/debug/threads", lambda r: plain(thread_dump())),
            Route("GET", "/v2/debug/offers", self.offers_v2),
            Route("GET", "/v1/debug/plans", lambda r: json_ok(self.plans_tracker.get_json(*f(r)))),
            Route("GET", "/v1/debug/taskStatuses", lambda r: json_ok(self.statuses_tracker.get_json(*f(r)))),
            Route("GET", "/v1/debug/reservations", lambda r: json_ok(self.reservations_tracker.get_json(*f(r)))),
            Route("GET", "/v1/debug/trace", self.trace),
        ]

    @staticmethod
    def trace(req: Request) -> Response:
        """Chrome trace of the offer cycles, step evaluations, status updates and persister ops
        (``?enable=true`` / ``?enable=false`` toggles recording, ``?summary=true`` aggregates per
        span name, ``?clear=true`` empties the ring after reading)."""
        en = req.q("enable")
        if en is not None:
            trace.enable() if en.lower() in ("1", "true", "yes") else trace.disable()
        body = {"spans": trace.TRACER.summary(), "enabled": trace.enabled()} if req.q_bool("summary") \
            else trace.TRACER.to_json()
        if req.q_bool("clear"):
            trace.TRACER.clear()
        return json_ok(body)

    def offers(self, req: Request) -> Response:
        tracker = self.scheduler.offer_outcome_tracker
        if tracker is None:
            return status_only(404)
        return json_ok(tracker.to_json()) if req.q_bool("json") else html(tracker.to_html())

    def offers_v2(self, req: Request) -> Response:
        tracker = getattr(self.scheduler, "offer_outcome_tracker_v2", None)
        if tracker is None:
            return status_only(404)
        return json_ok(tracker.to_json())


class MetricsResource:
    """``/v1/metrics`` (Codahale JSON) and ``/v1/metrics/prometheus`` (ApiServer.java:63-66)."""

    def routes(self) -> List[Route]:
        return [
            Route("GET", "/v1/metrics", lambda r: json_ok(metrics.REGISTRY.to_json())),
            Route("GET", "/v1/metrics/prometheus",
                  lambda r: Response(200, metrics.REGISTRY.to_prometheus(), "text/plain; version=0.0.4")),
        ]
