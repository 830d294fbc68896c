"""Raw YAML ``ServiceSpec`` model with strict parsing.

Reference: sdk/.../specification/yaml/Raw*.java (21 files) and RawServiceSpec.java:31-112:
Jackson YAML with ``STRICT_DUPLICATE_DETECTION`` (duplicate keys are errors at every level,
``WriteOnceLinkedHashMap.java:18``). Unknown properties are rejected at every level except the pod:
``RawPod.java:18`` is the one Raw* class annotated ``@JsonIgnoreProperties(ignoreUnknown = true)``,
so pod-level keys such as helloworld ``gpu_resource.yml``'s ``container:`` block or
``graceful-shutdown.yml``'s ``user:`` are ignored (with a WARN naming them here). The other 20 Raw*
classes keep Jackson's default ``FAIL_ON_UNKNOWN_PROPERTIES``. Mapping order is preserved
(pods/tasks/phases keep YAML order, which drives plan order).
"""
from __future__ import annotations

import logging
import os
from typing import Any, Dict, List, Mapping, Optional

import yaml

from .template_utils import MissingValue, render_mustache, validate_missing_values


LOGGER = logging.getLogger(__name__)


class RawSpecError(ValueError):
    pass


# libyaml's scanner/parser when PyYAML was built with it (same YAML 1.1 grammar and safe
# constructors; ~4x faster on a 600-line svc.yml, which every scheduler start parses)
class _StrictLoader(getattr(yaml, "CSafeLoader", yaml.SafeLoader)):
    pass


def _construct_mapping(loader, node, deep=False):
    loader.flatten_mapping(node)
    out = {}
    for key_node, value_node in node.value:
        key = loader.construct_object(key_node, deep=deep)
        if not isinstance(key, str):
            key = str(key)
        if key in out:
            raise RawSpecError(f"Duplicate field '{key}' (line {key_node.start_mark.line + 1})")
        out[key] = loader.construct_object(value_node, deep=deep)
    return out


_StrictLoader.add_constructor(yaml.resolver.BaseResolver.DEFAULT_MAPPING_TAG, _construct_mapping)


_STR_TAG = "tag:yaml.org,2002:str"
_MAP_TAG = yaml.resolver.BaseResolver.DEFAULT_MAPPING_TAG
_SEQ_TAG = yaml.resolver.BaseResolver.DEFAULT_SEQUENCE_TAG
_MERGE_TAG = "tag:yaml.org,2002:merge"


def _to_python(loader, node) -> Any:
    """The safe constructor's result for ``node``, with the common cases -- string scalars,
    plain mappings and sequences -- converted directly. PyYAML's constructor spends most of a
    service spec's load in per-node bookkeeping (a generator per mapping, recursion state); a
    rendered svc.yml is almost all strings, maps and lists. Anything else (ints, bools, nulls,
    merge keys, explicit tags) goes through the loader's own constructors, so the results are
    the same, duplicate keys included."""
    tag = node.tag
    if tag == _STR_TAG and isinstance(node, yaml.ScalarNode):
        return node.value
    if tag == _MAP_TAG and isinstance(node, yaml.MappingNode):
        out = {}
        for key_node, value_node in node.value:
            if key_node.tag == _MERGE_TAG:
                return loader.construct_object(node, deep=True)   # `<<:` merges: the loader's flattening
            key = _to_python(loader, key_node)
            if not isinstance(key, str):
                key = str(key)
            if key in out:
                raise RawSpecError(f"Duplicate field '{key}' (line {key_node.start_mark.line + 1})")
            out[key] = _to_python(loader, value_node)
        return out
    if tag == _SEQ_TAG and isinstance(node, yaml.SequenceNode):
        return [_to_python(loader, n) for n in node.value]
    return loader.construct_object(node, deep=True)


def load_yaml_strict(text: str) -> Any:
    loader = _StrictLoader(text)
    try:
        node = loader.get_single_node()
        return None if node is None else _to_python(loader, node)
    except yaml.YAMLError as e:
        raise RawSpecError(f"Invalid YAML: {e}") from e
    finally:
        loader.dispose()


# Allowed keys per node type (Jackson FAIL_ON_UNKNOWN_PROPERTIES).
SERVICE_KEYS = {"name", "web-url", "scheduler", "pods", "plans"}
SCHEDULER_KEYS = {"principal", "zookeeper", "user"}
POD_KEYS = {"resource-sets", "placement", "count", "image", "rlimits", "uris", "tasks", "volume", "volumes",
            "pre-reserved-role", "secrets", "share-pid-namespace", "allow-decommission", "host-volumes",
            "seccomp-unconfined", "seccomp-profile-name", "ipc-mode", "shm-size", "networks"}
TASK_KEYS = {"goal", "essential", "cmd", "labels", "env", "configs", "cpus", "gpus", "memory", "ports",
             "health-check", "readiness-check", "volume", "volumes", "resource-set", "discovery",
             "kill-grace-period", "transport-encryption", "ipc-mode", "shm-size"}
RESOURCE_SET_KEYS = {"cpus", "gpus", "memory", "ports", "volume", "volumes"}
PORT_KEYS = {"port", "env-key", "advertise", "vip", "ranges"}
VIP_KEYS = {"port", "prefix"}
VOLUME_KEYS = {"path", "type", "profiles", "size"}
HEALTH_KEYS = {"cmd", "interval", "grace-period", "max-consecutive-failures", "delay", "timeout"}
READINESS_KEYS = {"cmd", "interval", "delay", "timeout"}
PLAN_KEYS = {"strategy", "phases"}
PHASE_KEYS = {"strategy", "steps", "pod"}
CONFIG_KEYS = {"template", "dest"}
DISCOVERY_KEYS = {"prefix", "visibility"}
SECRET_KEYS = {"secret", "env-key", "file"}
HOST_VOLUME_KEYS = {"host-path", "container-path", "mode"}
NETWORK_KEYS = {"host-ports", "container-ports", "labels"}
RLIMIT_KEYS = {"soft", "hard"}
TLS_KEYS = {"name", "type"}
RANGE_KEYS = {"begin", "end"}


# Raw* levels that ignore unknown keys instead of failing: only RawPod (RawPod.java:18).
LENIENT_LEVELS = frozenset({"pod"})


def _check(node: Any, allowed, where: str) -> Dict[str, Any]:
    if node is None:
        return {}
    if not isinstance(node, dict):
        raise RawSpecError(f"Expected a mapping for {where}, got {type(node).__name__}")
    unknown = set(node) - allowed
    if unknown:
        raise RawSpecError(f"Unrecognized field(s) {sorted(unknown)} in {where} (known: {sorted(allowed)})")
    return node


def _check_lenient(node: Any, allowed, where: str) -> Dict[str, Any]:
    """``@JsonIgnoreProperties(ignoreUnknown = true)``: unknown keys are dropped, not errors."""
    if node is None:
        return {}
    if not isinstance(node, dict):
        raise RawSpecError(f"Expected a mapping for {where}, got {type(node).__name__}")
    unknown = [k for k in node if k not in allowed]
    if not unknown:
        return node
    LOGGER.warning("Ignoring unrecognized field(s) %s in %s", unknown, where)
    return {k: v for k, v in node.items() if k in allowed}


def _map_of(node: Any, allowed, where: str) -> Dict[str, Dict[str, Any]]:
    if node is None:
        return {}
    if not isinstance(node, dict):
        raise RawSpecError(f"Expected a mapping for {where}")
    return {str(k): _check(v, allowed, f"{where}.{k}") for k, v in node.items()}


def _validate_port_map(ports, where):
    out = _map_of(ports, PORT_KEYS, where)
    for name, p in out.items():
        if p.get("vip") is not None:
            _check(p["vip"], VIP_KEYS, f"{where}.{name}.vip")
        for r in p.get("ranges") or []:
            _check(r, RANGE_KEYS, f"{where}.{name}.ranges")
    return out


class RawServiceSpec:
    """Validated raw YAML view; nested nodes stay plain (ordered) dicts."""

    def __init__(self, data: Dict[str, Any]):
        data = _check(data, SERVICE_KEYS, "service")
        self.name: Optional[str] = data.get("name")
        self.web_url: Optional[str] = data.get("web-url")
        self.scheduler: Dict[str, Any] = _check(data.get("scheduler"), SCHEDULER_KEYS, "scheduler")
        self.pods: Dict[str, Dict[str, Any]] = {}
        for pod_name, pod in (data.get("pods") or {}).items():
            pod = _check_lenient(pod, POD_KEYS, f"pods.{pod_name}")
            tasks = {}
            for tname, task in (pod.get("tasks") or {}).items():
                task = _check(task, TASK_KEYS, f"pods.{pod_name}.tasks.{tname}")
                w = f"pods.{pod_name}.tasks.{tname}"
                _validate_port_map(task.get("ports"), w + ".ports")
                _check(task.get("health-check"), HEALTH_KEYS, w + ".health-check")
                _check(task.get("readiness-check"), READINESS_KEYS, w + ".readiness-check")
                _check(task.get("volume"), VOLUME_KEYS, w + ".volume")
                _map_of(task.get("volumes"), VOLUME_KEYS, w + ".volumes")
                _map_of(task.get("configs"), CONFIG_KEYS, w + ".configs")
                _check(task.get("discovery"), DISCOVERY_KEYS, w + ".discovery")
                for te in task.get("transport-encryption") or []:
                    _check(te, TLS_KEYS, w + ".transport-encryption")
                if task.get("ipc-mode") == "SHARE_PARENT" and task.get("shm-size") is not None:
                    raise RawSpecError("shm size does not apply when IPC Mode is SHARE_PARENT")
                tasks[str(tname)] = task
            pod["tasks"] = tasks
            for rs_name, rs in _map_of(pod.get("resource-sets"), RESOURCE_SET_KEYS,
                                       f"pods.{pod_name}.resource-sets").items():
                _validate_port_map(rs.get("ports"), f"pods.{pod_name}.resource-sets.{rs_name}.ports")
                _check(rs.get("volume"), VOLUME_KEYS, f"pods.{pod_name}.resource-sets.{rs_name}.volume")
                _map_of(rs.get("volumes"), VOLUME_KEYS, f"pods.{pod_name}.resource-sets.{rs_name}.volumes")
            _map_of(pod.get("rlimits"), RLIMIT_KEYS, f"pods.{pod_name}.rlimits")
            _check(pod.get("volume"), VOLUME_KEYS, f"pods.{pod_name}.volume")
            _map_of(pod.get("volumes"), VOLUME_KEYS, f"pods.{pod_name}.volumes")
            _map_of(pod.get("secrets"), SECRET_KEYS, f"pods.{pod_name}.secrets")
            _map_of(pod.get("host-volumes"), HOST_VOLUME_KEYS, f"pods.{pod_name}.host-volumes")
            _map_of(pod.get("networks"), NETWORK_KEYS, f"pods.{pod_name}.networks")
            if pod.get("ipc-mode") == "SHARE_PARENT" and pod.get("shm-size") is not None:
                raise RawSpecError("shm size does not apply when IPC Mode is SHARE_PARENT")
            self.pods[str(pod_name)] = pod
        self.plans: Dict[str, Dict[str, Any]] = {}
        for plan_name, plan in (data.get("plans") or {}).items():
            plan = _check(plan, PLAN_KEYS, f"plans.{plan_name}")
            phases = {}
            for ph_name, ph in (plan.get("phases") or {}).items():
                ph = _check(ph, PHASE_KEYS, f"plans.{plan_name}.phases.{ph_name}")
                phases[str(ph_name)] = ph
            plan["phases"] = phases
            self.plans[str(plan_name)] = plan

    @staticmethod
    def from_bytes(data: bytes) -> "RawServiceSpec":
        return RawServiceSpec.from_string(data.decode("utf-8"))

    @staticmethod
    def from_string(text: str) -> "RawServiceSpec":
        parsed = load_yaml_strict(text)
        if not isinstance(parsed, dict):
            raise RawSpecError("Service spec YAML must be a mapping")
        return RawServiceSpec(parsed)

    @staticmethod
    def new_builder(path: str) -> "RawServiceSpecBuilder":
        return RawServiceSpecBuilder(path)


class RawServiceSpecBuilder:
    """RawServiceSpec.Builder: mustache-render the file against env, then parse."""

    def __init__(self, path: str):
        self.path = path
        self.env: Mapping[str, str] = dict(os.environ)
        self.strict = False

    def set_env(self, env: Mapping[str, str]) -> "RawServiceSpecBuilder":
        self.env = env
        return self

    def enable_strict_rendering(self) -> "RawServiceSpecBuilder":
        self.strict = True
        return self

    def build(self) -> RawServiceSpec:
        with open(self.path, "r", encoding="utf-8") as f:
            content = f.read()
        missing: List[MissingValue] = []
        name = os.path.basename(self.path)
        rendered = render_mustache(name, content, self.env, missing)
        if self.strict:
            validate_missing_values(name, self.env, missing)
        return RawServiceSpec.from_string(rendered)
