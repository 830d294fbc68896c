"""Service/pod/task specification model.

Mirrors the reference's ``specification`` package (sdk/.../specification/*.java): the
``ServiceSpec`` / ``PodSpec`` / ``TaskSpec`` / ``ResourceSet`` / ``ResourceSpec`` /
``VolumeSpec`` / ``PortSpec`` / ``NamedVIPSpec`` interfaces and their ``Default*``
implementations, collapsed into immutable dataclasses.

Persistence: :meth:`ServiceSpec.to_json_bytes` produces the JSON blob stored under
``Configurations/<uuid>``, using the reference's Jackson property names (``pod-specs``,
``task-specs``, ``resource-set``, ``resource-specifications`` ...) and its ``@type``
discriminator for the polymorphic ``ResourceSpec`` / ``VolumeSpec`` / ``PlacementRule``
hierarchies (``@JsonTypeInfo(use = NAME)``, e.g. ResourceSpec.java:11, VolumeSpec.java:12).
Protobuf ``Value`` fields are serialized with the protobuf JSON mapping.
"""
from __future__ import annotations

import enum
import functools
import json
import re
from dataclasses import dataclass, replace
from typing import Any, Dict, List, Optional, Tuple

from dcos_commons_amd.mesos import protos as P

ANY_ROLE = "*"
DISK_RESOURCE_TYPE = "disk"
PORTS_RESOURCE_TYPE = "ports"
CPUS_RESOURCE_TYPE = "cpus"
MEMORY_RESOURCE_TYPE = "mem"
GPUS_RESOURCE_TYPE = "gpus"
DEFAULT_SERVICE_USER = "root"
MESOS_MASTER_ZK_CONNECTION_STRING = "master.mesos:2181"
DEFAULT_IP_PROTOCOL = "tcp"
LONG_DECLINE_SECONDS = 3600


class SpecValidationError(ValueError):
    """Raised when a spec violates a structural constraint (reference ValidationUtils)."""


def _require(cond: bool, msg: str) -> None:
    if not cond:
        raise SpecValidationError(msg)


# ---------------------------------------------------------------------------------------
# enums


class GoalState(enum.Enum):
    """Reference: specification/GoalState.java:10-27."""

    UNKNOWN = "UNKNOWN"
    RUNNING = "RUNNING"
    FINISH = "FINISH"
    ONCE = "ONCE"

    @staticmethod
    def parse_persisted(value: Optional[str]) -> "GoalState":
        # DefaultServiceSpec.GoalStateDeserializer: FINISHED/ONCE -> ONCE
        if value in ("FINISHED", "ONCE"):
            return GoalState.ONCE
        if value == "FINISH":
            return GoalState.FINISH
        if value == "RUNNING":
            return GoalState.RUNNING
        return GoalState.UNKNOWN


class VolumeType(enum.Enum):
    ROOT = "ROOT"
    PATH = "PATH"
    MOUNT = "MOUNT"


class TransportEncryptionType(enum.Enum):
    TLS = "TLS"
    KEYSTORE = "KEYSTORE"


# ---------------------------------------------------------------------------------------
# protobuf Value helpers


def scalar_value(v: float) -> P.Value:
    val = P.Value(type=P.Value.SCALAR)
    val.scalar.value = float(v)
    return val


def ranges_value(ranges: List[Tuple[int, int]]) -> P.Value:
    val = P.Value(type=P.Value.RANGES)
    for b, e in ranges:
        r = val.ranges.range.add()
        r.begin, r.end = int(b), int(e)
    return val


_SCALAR, _RANGES = P.Value.SCALAR, P.Value.RANGES


def value_to_json(v: P.Value) -> dict:
    """``P.to_json(v)`` for the value shapes specs hold, without the generic reflection walk
    (this runs for every resource of every spec serialization): the same dict the protobuf JSON
    mapping produces, with 64-bit range bounds as strings. Other shapes take the generic path."""
    if v.HasField("type") and not (v.HasField("set") or v.HasField("text")):
        t = v.type
        if t == _SCALAR and v.HasField("scalar") and not v.HasField("ranges"):
            return {"type": "SCALAR", "scalar": {"value": v.scalar.value} if v.scalar.HasField("value") else {}}
        if t == _RANGES and v.HasField("ranges") and not v.HasField("scalar"):
            rs = []
            for r in v.ranges.range:
                d = {}
                if r.HasField("begin"):
                    d["begin"] = str(r.begin)
                if r.HasField("end"):
                    d["end"] = str(r.end)
                rs.append(d)
            return {"type": "RANGES", "ranges": {"range": rs} if rs else {}}
    return P.to_json(v)


def value_from_json(d: dict) -> P.Value:
    return P.from_json(P.Value, d)


def _value_key(v: P.Value) -> bytes:
    return v.SerializeToString(deterministic=True)


# ---------------------------------------------------------------------------------------
# resources


@dataclass(frozen=True, eq=False)
class ResourceSpec:
    """DefaultResourceSpec: a named scalar or range resource to reserve."""

    name: str
    value: P.Value
    role: str
    principal: str
    pre_reserved_role: str = ANY_ROLE

    TYPE_NAME = "DefaultResourceSpec"

    def validate(self) -> None:
        _require(bool(self.name), "ResourceSpec name must be non-empty")
        _require(bool(self.role), "ResourceSpec role must be non-empty")
        _require(bool(self.principal), "ResourceSpec principal must be non-empty")
        if self.value.HasField("scalar"):
            _require(self.value.scalar.value > 0,
                     f"Scalar resource value must be greater than zero: {self}")
        elif not self.value.HasField("ranges"):
            raise SpecValidationError(f"Expected resource value to be a scalar or range: {self}")

    def _base_dict(self) -> Dict[str, Any]:
        return {
            "@type": self.TYPE_NAME,
            "name": self.name,
            "value": value_to_json(self.value),
            "role": self.role,
            "pre-reserved-role": self.pre_reserved_role,
            "principal": self.principal,
        }

    def to_dict(self) -> Dict[str, Any]:
        return self._base_dict()

    def _eq_key(self):
        return (type(self).__name__, self.name, _value_key(self.value), self.role,
                self.principal, self.pre_reserved_role)

    def __eq__(self, other):
        return isinstance(other, ResourceSpec) and self._eq_key() == other._eq_key()

    def __hash__(self):
        return hash(self._eq_key())

    def __repr__(self):
        return (f"{type(self).__name__}(name={self.name}, value={P.to_text(self.value)}, "
                f"role={self.role}, pre-reserved-role={self.pre_reserved_role})")


@dataclass(frozen=True, eq=False, repr=False)
class VolumeSpec(ResourceSpec):
    """DefaultVolumeSpec: a disk resource + persistent volume at ``container_path``."""

    type: VolumeType = VolumeType.ROOT
    container_path: str = ""
    profiles: Tuple[str, ...] = ()

    TYPE_NAME = "DefaultVolumeSpec"
    _VALID_PATH = re.compile(r"[a-zA-Z0-9]+([a-zA-Z0-9_-]*)*")
    _VALID_PROFILE = re.compile(r"[a-zA-Z0-9_.-]{1,128}")

    @staticmethod
    def create_root_volume(size: float, container_path: str, role: str, pre_reserved_role: str,
                           principal: str) -> "VolumeSpec":
        v = VolumeSpec(name=DISK_RESOURCE_TYPE, value=scalar_value(size), role=role,
                       principal=principal, pre_reserved_role=pre_reserved_role or ANY_ROLE,
                       type=VolumeType.ROOT, container_path=container_path, profiles=())
        v.validate()
        return v

    @staticmethod
    def create_mount_volume(size: float, container_path: str, profiles, role: str,
                            pre_reserved_role: str, principal: str) -> "VolumeSpec":
        v = VolumeSpec(name=DISK_RESOURCE_TYPE, value=scalar_value(size), role=role,
                       principal=principal, pre_reserved_role=pre_reserved_role or ANY_ROLE,
                       type=VolumeType.MOUNT, container_path=container_path,
                       profiles=tuple(profiles or ()))
        v.validate()
        return v

    def validate(self) -> None:
        super().validate()
        _require(bool(self._VALID_PATH.fullmatch(self.container_path or "")),
                 f"Volume container-path '{self.container_path}' must match "
                 f"{self._VALID_PATH.pattern}")
        for p in self.profiles:
            _require(isinstance(p, str) and bool(self._VALID_PROFILE.fullmatch(p)), f"Invalid volume profile '{p}'")
        _require(len(set(self.profiles)) == len(self.profiles), f"Duplicate volume profiles: {list(self.profiles)}")
        if self.type == VolumeType.ROOT:
            _require(not self.profiles, f"ROOT volume '{self.container_path}' cannot have profiles")

    def with_disk_size(self, size: float) -> "VolumeSpec":
        return replace(self, value=scalar_value(size))

    def to_dict(self):
        d = self._base_dict()
        d.update({"type": self.type.value, "container-path": self.container_path,
                  "profiles": list(self.profiles)})
        return d

    def _eq_key(self):
        return super()._eq_key() + (self.type, self.container_path, self.profiles)

    def __repr__(self):
        return (f"VolumeSpec(type={self.type.value}, path={self.container_path}, "
                f"size={self.value.scalar.value}, profiles={list(self.profiles)})")


@dataclass(frozen=True)
class RangeSpec:
    begin: int
    end: int

    MIN_PORT = 0
    MAX_PORT = 65535

    def to_dict(self):
        return {"begin": self.begin, "end": self.end}


@dataclass(frozen=True, eq=False, repr=False)
class PortSpec(ResourceSpec):
    """PortSpec: a single named port (static, or dynamic when value is 0)."""

    env_key: Optional[str] = None
    port_name: str = ""
    visibility: int = P.DiscoveryInfo.EXTERNAL
    network_names: Tuple[str, ...] = ()
    ranges: Tuple[RangeSpec, ...] = ()

    TYPE_NAME = "PortSpec"

    def validate(self) -> None:
        super().validate()
        _require(bool(self.port_name), "portName must be non-empty")

    @property
    def port(self) -> int:
        return int(self.value.ranges.range[0].begin)

    def with_value(self, value: P.Value) -> "PortSpec":
        return replace(self, value=value)

    def to_dict(self):
        d = self._base_dict()
        d.update({
            "env-key": self.env_key,
            "port-name": self.port_name,
            "visibility": P.DiscoveryInfo.Visibility.Name(self.visibility),
            "network-names": list(self.network_names),
            "ranges": [r.to_dict() for r in self.ranges],
        })
        return d

    def _eq_key(self):
        return super()._eq_key() + (self.env_key, self.port_name, self.visibility,
                                    tuple(sorted(self.network_names)), self.ranges)

    def __repr__(self):
        return f"PortSpec(name={self.port_name}, port={self.port}, env-key={self.env_key})"


@dataclass(frozen=True, eq=False, repr=False)
class NamedVIPSpec(PortSpec):
    protocol: str = DEFAULT_IP_PROTOCOL
    vip_name: str = ""
    vip_port: int = 0

    TYPE_NAME = "NamedVIPSpec"

    def validate(self) -> None:
        super().validate()
        _require(bool(self.protocol), "protocol must be non-empty")
        _require(bool(self.vip_name), "vipName must be non-empty")

    def to_dict(self):
        d = super().to_dict()
        d.pop("ranges", None)
        d.update({"protocol": self.protocol, "vip-name": self.vip_name, "vip-port": self.vip_port})
        return d

    def _eq_key(self):
        return super()._eq_key() + (self.protocol, self.vip_name, self.vip_port)

    def __repr__(self):
        return (f"NamedVIPSpec(name={self.port_name}, port={self.port}, "
                f"vip={self.vip_name}:{self.vip_port})")


@dataclass(frozen=True)
class VipSpec:
    """DefaultVipSpec: an application port published under a VIP name and port (both ports
    non-negative, the name non-empty; reference specification/DefaultVipSpec.java)."""

    application_port: int
    vip_name: str
    vip_port: int

    def __post_init__(self):
        _require(self.application_port >= 0, "applicationPort must be non-negative")
        _require(bool(self.vip_name), "vipName must be non-empty")
        _require(self.vip_port >= 0, "vipPort must be non-negative")

    def to_dict(self):
        return {"application-port": self.application_port, "vip-name": self.vip_name, "vip-port": self.vip_port}

    @staticmethod
    def from_dict(d: Dict[str, Any]) -> "VipSpec":
        return VipSpec(int(d["application-port"]), d["vip-name"], int(d["vip-port"]))


def resource_spec_from_dict(d: Dict[str, Any]) -> ResourceSpec:
    t = d.get("@type", "DefaultResourceSpec")
    common = dict(
        name=d.get("name") or "",
        value=value_from_json(d.get("value") or {}),
        role=d.get("role") or "",
        principal=d.get("principal") or "",
        pre_reserved_role=d.get("pre-reserved-role") or ANY_ROLE,
    )
    if t == "DefaultVolumeSpec":
        return VolumeSpec(type=VolumeType(d.get("type", "ROOT")),
                          container_path=d.get("container-path") or "",
                          profiles=tuple(d.get("profiles") or ()), **common)
    if t in ("PortSpec", "NamedVIPSpec"):
        common["name"] = PORTS_RESOURCE_TYPE
        port = dict(
            env_key=d.get("env-key"),
            port_name=d.get("port-name") or "",
            visibility=P.DiscoveryInfo.Visibility.Value(d.get("visibility") or "EXTERNAL"),
            network_names=tuple(d.get("network-names") or ()),
        )
        if t == "NamedVIPSpec":
            return NamedVIPSpec(protocol=d.get("protocol") or DEFAULT_IP_PROTOCOL,
                                vip_name=d.get("vip-name") or "", vip_port=int(d.get("vip-port") or 0),
                                **port, **common)
        return PortSpec(ranges=tuple(RangeSpec(r["begin"], r["end"]) for r in d.get("ranges") or ()),
                        **port, **common)
    return ResourceSpec(**common)


@dataclass(frozen=True)
class ResourceSet:
    """DefaultResourceSet: the reservable unit shared by tasks naming the same set id."""

    id: str
    resources: Tuple[ResourceSpec, ...]
    volumes: Tuple[VolumeSpec, ...]
    role: str
    principal: str
    pre_reserved_role: Optional[str] = ANY_ROLE

    def validate(self) -> None:
        _require(bool(self.id), "ResourceSet id must be non-empty")
        _require(bool(self.resources), f"ResourceSet '{self.id}' must contain resources")
        _require(bool(self.role), "ResourceSet role must be non-empty")
        _require(bool(self.principal), "ResourceSet principal must be non-empty")

    def to_dict(self):
        d = {
            "id": self.id,
            "resource-specifications": [r.to_dict() for r in self.resources],
            "volume-specifications": [v.to_dict() for v in self.volumes],
            "role": self.role,
            "principal": self.principal,
        }
        if self.pre_reserved_role is not None:
            d["pre-reserved-role"] = self.pre_reserved_role
        return d

    @staticmethod
    def from_dict(d) -> "ResourceSet":
        return ResourceSet(
            id=d.get("id"),
            resources=tuple(resource_spec_from_dict(r) for r in d.get("resource-specifications") or ()),
            volumes=tuple(resource_spec_from_dict(v) for v in d.get("volume-specifications") or ()),
            role=d.get("role"),
            principal=d.get("principal"),
            pre_reserved_role=d.get("pre-reserved-role", ANY_ROLE),
        )

    def get_resource(self, name: str) -> Optional[ResourceSpec]:
        for r in self.resources:
            if r.name == name:
                return r
        return None

    def gpus(self) -> float:
        r = self.get_resource(GPUS_RESOURCE_TYPE)
        return r.value.scalar.value if r is not None else 0.0


class ResourceSetBuilder:
    """DefaultResourceSet.Builder semantics (cpus/gpus/memory/addVolume/addResource)."""

    def __init__(self, role: str, pre_reserved_role: Optional[str], principal: str):
        self.role = role
        self.pre_reserved_role = pre_reserved_role
        self.principal = principal
        self.id: Optional[str] = None
        self.resources: List[ResourceSpec] = []
        self.volumes: List[VolumeSpec] = []

    def _scalar(self, v: float, name: str) -> "ResourceSetBuilder":
        if any(r.name == name for r in self.resources):
            raise SpecValidationError(f"Cannot configure multiple {name} resources in a single ResourceSet")
        r = ResourceSpec(name=name, value=scalar_value(v), role=self.role, principal=self.principal,
                         pre_reserved_role=self.pre_reserved_role or ANY_ROLE)
        r.validate()
        self.resources.append(r)
        return self

    def cpus(self, v: float):
        return self._scalar(v, CPUS_RESOURCE_TYPE)

    def gpus(self, v: float):
        return self._scalar(v, GPUS_RESOURCE_TYPE)

    def memory(self, v: float):
        return self._scalar(v, MEMORY_RESOURCE_TYPE)

    def add_volume(self, vtype: str, size: float, container_path: str, profiles=None):
        try:
            t = VolumeType(vtype)
        except ValueError:
            raise SpecValidationError(
                f"Provided volume type '{vtype}' for path '{container_path}' is invalid. "
                f"Expected type to be one of: {[v.value for v in VolumeType]}")
        if any(v.container_path == container_path for v in self.volumes):
            raise SpecValidationError("Cannot configure multiple volumes with the same containerPath")
        profiles = list(profiles or [])
        if t == VolumeType.ROOT:
            if profiles:
                raise SpecValidationError(
                    f"Provided volume type '{vtype}' for path '{container_path}' cannot have profiles")
            self.volumes.append(VolumeSpec.create_root_volume(
                size, container_path, self.role, self.pre_reserved_role, self.principal))
        else:
            self.volumes.append(VolumeSpec.create_mount_volume(
                size, container_path, profiles, self.role, self.pre_reserved_role, self.principal))
        return self

    def add_resource(self, r: ResourceSpec):
        self.resources.append(r)
        return self

    def build(self) -> ResourceSet:
        rs = ResourceSet(id=self.id, resources=tuple(self.resources), volumes=tuple(self.volumes),
                         role=self.role, principal=self.principal,
                         pre_reserved_role=self.pre_reserved_role)
        rs.validate()
        return rs


# ---------------------------------------------------------------------------------------
# task-level specs


@dataclass(frozen=True)
class CommandSpec:
    value: str
    environment: Tuple[Tuple[str, str], ...] = ()

    @property
    def env(self) -> Dict[str, str]:
        return dict(self.environment)

    @staticmethod
    def build(value: str, environment: Optional[Dict[str, str]], env_override: Optional[Dict[str, str]]):
        """Builder semantics: task env first, then the router's overrides on top (sorted)."""
        combined: Dict[str, str] = {}
        combined.update({k: "" if v is None else str(v) for k, v in (environment or {}).items()})
        combined.update(env_override or {})
        _require(value is not None, "command value must be set")
        return CommandSpec(value=value, environment=tuple(sorted(combined.items())))

    def to_dict(self):
        return {"value": self.value, "environment": dict(self.environment)}

    @staticmethod
    def from_dict(d):
        return CommandSpec(d.get("value"), tuple(sorted((d.get("environment") or {}).items())))


@dataclass(frozen=True)
class ConfigFileSpec:
    name: str
    relative_path: str
    template_content: str

    def to_dict(self):
        return {"name": self.name, "relative-path": self.relative_path,
                "template-content": self.template_content}

    @staticmethod
    def from_dict(d):
        return ConfigFileSpec(d["name"], d["relative-path"], d["template-content"])


@dataclass(frozen=True)
class HealthCheckSpec:
    command: str
    max_consecutive_failures: int
    delay: int
    interval: int
    timeout: int
    grace_period: int

    def validate(self):
        _require(bool(self.command), "health check command must be non-empty")
        _require(self.max_consecutive_failures is not None and self.max_consecutive_failures >= 1,
                 "maxConsecutiveFailures must be >= 1")
        for n in ("delay", "interval", "timeout", "grace_period"):
            v = getattr(self, n)
            _require(v is not None and v >= 0, f"health check {n} must be >= 0")

    def to_dict(self):
        # "gracePeriod" is written too so that an older scheduler can still read the config
        # (DefaultHealthCheckSpec.getGracePeriodForDowngradeCompatibility)
        return {"command": self.command, "max-consecutive-failures": self.max_consecutive_failures,
                "delay": self.delay, "interval": self.interval, "timeout": self.timeout,
                "grace-period": self.grace_period, "gracePeriod": self.grace_period}

    @staticmethod
    def from_dict(d):
        gp = d.get("grace-period")
        if gp is None:
            gp = d.get("gracePeriod")
        return HealthCheckSpec(d.get("command"), d.get("max-consecutive-failures"), d.get("delay"),
                               d.get("interval"), d.get("timeout"), gp)


@dataclass(frozen=True)
class ReadinessCheckSpec:
    command: str
    interval: int
    timeout: int
    delay: int = 0

    def validate(self):
        _require(self.command is not None, "readiness check command must be set")
        for n in ("delay", "interval", "timeout"):
            v = getattr(self, n)
            _require(v is not None and v >= 0, f"readiness check {n} must be >= 0")

    def to_dict(self):
        return {"command": self.command, "delay": self.delay, "interval": self.interval,
                "timeout": self.timeout}

    @staticmethod
    def from_dict(d):
        return ReadinessCheckSpec(d.get("command"), d.get("interval"), d.get("timeout"), d.get("delay") or 0)


@dataclass(frozen=True)
class DiscoverySpec:
    prefix: Optional[str] = None
    visibility: Optional[int] = None

    def to_dict(self):
        return {"prefix": self.prefix,
                "visibility": None if self.visibility is None else P.DiscoveryInfo.Visibility.Name(self.visibility)}

    @staticmethod
    def from_dict(d):
        vis = d.get("visibility")
        return DiscoverySpec(d.get("prefix"), None if vis is None else P.DiscoveryInfo.Visibility.Value(vis))


@dataclass(frozen=True)
class TransportEncryptionSpec:
    name: str
    type: TransportEncryptionType

    def to_dict(self):
        return {"name": self.name, "type": self.type.value}

    @staticmethod
    def from_dict(d):
        return TransportEncryptionSpec(d["name"], TransportEncryptionType(d["type"]))


class IpcMode(enum.Enum):
    PRIVATE = "PRIVATE"
    SHARE_PARENT = "SHARE_PARENT"

    @staticmethod
    def parse(s: Optional[str]) -> Optional["IpcMode"]:
        if s is None:
            return None
        try:
            return IpcMode(s)
        except ValueError:
            raise SpecValidationError("Invalid IPC Mode")


@dataclass(frozen=True, eq=False)
class TaskSpec:
    """DefaultTaskSpec. Equality is *semantic* (``not TaskUtils.areDifferent``)."""

    name: str
    goal: GoalState
    resource_set: ResourceSet
    command: Optional[CommandSpec] = None
    essential: bool = True
    task_labels: Tuple[Tuple[str, str], ...] = ()
    health_check: Optional[HealthCheckSpec] = None
    readiness_check: Optional[ReadinessCheckSpec] = None
    config_files: Tuple[ConfigFileSpec, ...] = ()
    discovery: Optional[DiscoverySpec] = None
    kill_grace_period: int = 0
    transport_encryption: Tuple[TransportEncryptionSpec, ...] = ()
    shared_memory: Optional[IpcMode] = None
    shared_memory_size: Optional[int] = None

    @property
    def labels(self) -> Dict[str, str]:
        return dict(self.task_labels)

    def validate(self) -> None:
        _require(bool(self.name), "TaskSpec name must be non-empty")
        _require(self.goal is not None, "goalState must be set")
        _require(self.resource_set is not None, "resourceSet must be set")
        names = [c.name for c in self.config_files]
        _require(len(names) == len(set(names)), "configFiles.name must be unique")
        paths = [c.relative_path for c in self.config_files]
        _require(len(paths) == len(set(paths)), "configFiles.relativePath must be unique")
        _require(0 <= self.kill_grace_period <= LONG_DECLINE_SECONDS,
                 f"taskKillGracePeriodSeconds must be in [0, {LONG_DECLINE_SECONDS}]")
        if self.shared_memory == IpcMode.SHARE_PARENT and self.shared_memory_size is not None:
            raise SpecValidationError("shm size does not apply when IPC Mode is SHARE_PARENT")

    def __eq__(self, other):
        if not isinstance(other, TaskSpec):
            return False
        from dcos_commons_amd.offer.task_utils import are_different

        return not are_different(self, other)

    def __hash__(self):
        return hash((self.name, self.goal))

    def to_dict(self):
        return {
            "name": self.name,
            "goal": self.goal.value,
            "essential": self.essential,
            "resource-set": self.resource_set.to_dict(),
            "command-spec": self.command.to_dict() if self.command else None,
            "task-labels": dict(self.task_labels),
            "health-check-spec": self.health_check.to_dict() if self.health_check else None,
            "readiness-check-spec": self.readiness_check.to_dict() if self.readiness_check else None,
            "config-files": [c.to_dict() for c in self.config_files],
            "discovery-spec": self.discovery.to_dict() if self.discovery else None,
            "kill-grace-period": self.kill_grace_period,
            "transport-encryption": [t.to_dict() for t in self.transport_encryption],
            "ipc-mode": self.shared_memory.value if self.shared_memory else None,
            "shm-size": self.shared_memory_size,
        }

    @staticmethod
    def from_dict(d) -> "TaskSpec":
        return TaskSpec(
            name=d["name"],
            goal=GoalState.parse_persisted(d.get("goal")),
            essential=True if d.get("essential") is None else bool(d.get("essential")),
            resource_set=ResourceSet.from_dict(d["resource-set"]),
            command=CommandSpec.from_dict(d["command-spec"]) if d.get("command-spec") else None,
            task_labels=tuple(sorted((d.get("task-labels") or {}).items())),
            health_check=HealthCheckSpec.from_dict(d["health-check-spec"]) if d.get("health-check-spec") else None,
            readiness_check=(ReadinessCheckSpec.from_dict(d["readiness-check-spec"])
                             if d.get("readiness-check-spec") else None),
            config_files=tuple(ConfigFileSpec.from_dict(c) for c in d.get("config-files") or ()),
            discovery=DiscoverySpec.from_dict(d["discovery-spec"]) if d.get("discovery-spec") else None,
            kill_grace_period=int(d.get("kill-grace-period") or 0),
            transport_encryption=tuple(TransportEncryptionSpec.from_dict(t)
                                       for t in d.get("transport-encryption") or ()),
            shared_memory=IpcMode.parse(d.get("ipc-mode")),
            shared_memory_size=d.get("shm-size"),
        )


# ---------------------------------------------------------------------------------------
# pod-level specs


@dataclass(frozen=True)
class NetworkSpec:
    name: str
    port_mappings: Tuple[Tuple[int, int], ...] = ()
    labels: Tuple[Tuple[str, str], ...] = ()

    def to_dict(self):
        return {"network-name": self.name,
                "port-mappings": {str(k): v for k, v in self.port_mappings},
                "network-labels": dict(self.labels)}

    @staticmethod
    def from_dict(d):
        return NetworkSpec(d["network-name"],
                           tuple(sorted((int(k), int(v)) for k, v in (d.get("port-mappings") or {}).items())),
                           tuple(sorted((d.get("network-labels") or {}).items())))


_RLIMIT_NAMES = {
    name.replace("RLMT", "RLIMIT"): num
    for name, num in P.RLimitInfo.RLimit.Type.items() if name != "UNKNOWN"
}
RLIMIT_INFINITY = -1


@dataclass(frozen=True)
class RLimitSpec:
    name: str
    soft: Optional[int] = None
    hard: Optional[int] = None

    def validate(self):
        if self.name not in _RLIMIT_NAMES:
            raise SpecValidationError(
                f"{self.name} is not a valid rlimit, expected one of: {sorted(_RLIMIT_NAMES)}. See man setrlimit(2)")
        if (self.soft is None) != (self.hard is None):
            raise SpecValidationError("soft and hard rlimits must be either both set or both unset")
        if self.soft is not None and self.soft > self.hard:
            raise SpecValidationError("soft rlimit must be less than or equal to the hard rlimit")
        if (self.soft is not None and self.soft < RLIMIT_INFINITY) or (
                self.hard is not None and self.hard < RLIMIT_INFINITY):
            raise SpecValidationError("soft and hard rlimits must be positive with the exception of -1")
        if (self.soft == RLIMIT_INFINITY) ^ (self.hard == RLIMIT_INFINITY):
            raise SpecValidationError("both soft and hard limits must be set to -1 which represents unlimited.")

    @property
    def enum(self) -> int:
        return _RLIMIT_NAMES[self.name]

    def to_dict(self):
        return {"name": self.name, "soft": self.soft, "hard": self.hard}

    @staticmethod
    def from_dict(d):
        return RLimitSpec(d["name"], d.get("soft"), d.get("hard"))


@dataclass(frozen=True)
class SecretSpec:
    secret_path: str
    env_key: Optional[str] = None
    file_path: Optional[str] = None

    _VALID_FILE = re.compile(r"([.a-zA-Z0-9]+([.a-zA-Z0-9_-]*[/\\]*)*)?")

    def validate(self):
        _require(bool(self.secret_path), "secretPath must be non-empty")
        if self.file_path is not None:
            _require(bool(self._VALID_FILE.fullmatch(self.file_path)), f"invalid secret file path {self.file_path}")

    def to_dict(self):
        return {"@type": "DefaultSecretSpec", "secret": self.secret_path, "env-key": self.env_key,
                "file": self.file_path}

    @staticmethod
    def from_dict(d):
        return SecretSpec(d["secret"], d.get("env-key"), d.get("file"))


@dataclass(frozen=True)
class HostVolumeSpec:
    host_path: str
    container_path: str
    mode: Optional[str] = None  # "RW" | "RO"

    _VALID_CONTAINER = re.compile(r"([.a-zA-Z0-9]+([.a-zA-Z0-9_-]*[/\\]*)*)")
    _VALID_HOST = re.compile(r"(/[.a-zA-Z0-9]+([.a-zA-Z0-9_-]*[/\\]*)*)")

    def validate(self):
        _require(bool(self._VALID_HOST.fullmatch(self.host_path or "")), f"invalid host-path {self.host_path}")
        _require(bool(self._VALID_CONTAINER.fullmatch(self.container_path or "")),
                 f"invalid container-path {self.container_path}")
        if self.mode not in (None, "RW", "RO"):
            raise SpecValidationError("Unsupported host volume mode.")

    def to_dict(self):
        return {"@type": "DefaultHostVolumeSpec", "host-path": self.host_path,
                "container-path": self.container_path, "mode": self.mode}

    @staticmethod
    def from_dict(d):
        return HostVolumeSpec(d["host-path"], d["container-path"], d.get("mode"))


@dataclass(frozen=True)
class PodSpec:
    """DefaultPodSpec."""

    type: str
    count: int
    tasks: Tuple[TaskSpec, ...]
    user: Optional[str] = None
    allow_decommission: bool = False
    image: Optional[str] = None
    networks: Tuple[NetworkSpec, ...] = ()
    rlimits: Tuple[RLimitSpec, ...] = ()
    uris: Tuple[str, ...] = ()
    placement_rule: Any = None  # dcos_commons_amd.offer.evaluate.placement.PlacementRule
    volumes: Tuple[VolumeSpec, ...] = ()
    pre_reserved_role: str = ANY_ROLE
    secrets: Tuple[SecretSpec, ...] = ()
    share_pid_namespace: bool = False
    host_volumes: Tuple[HostVolumeSpec, ...] = ()
    seccomp_unconfined: bool = False
    seccomp_profile_name: Optional[str] = None
    shared_memory: Optional[IpcMode] = None
    shared_memory_size: Optional[int] = None

    def validate(self) -> None:
        _require(bool(self.type and self.type.strip()), "PodSpec type must be non-blank")
        _require(self.count is not None and self.count >= 0, "PodSpec count must be >= 0")
        _require(self.image is None or self.image != "", "PodSpec image must be non-empty if set")
        _require(bool(self.tasks), f"PodSpec '{self.type}' must have tasks")
        seen = set()
        for t in self.tasks:
            if not t.name:
                raise SpecValidationError(f"Empty name for TaskSpec in pod {self.type}")
            if t.name in seen:
                raise SpecValidationError(f"Duplicate task name in pod {self.type}: {t.name}")
            seen.add(t.name)
        if self.shared_memory == IpcMode.SHARE_PARENT and self.shared_memory_size is not None:
            raise SpecValidationError("shm size does not apply when IPC Mode is SHARE_PARENT")

    def task(self, name: str) -> Optional[TaskSpec]:
        for t in self.tasks:
            if t.name == name:
                return t
        return None

    def gpus_per_instance(self) -> float:
        seen = set()
        total = 0.0
        for t in self.tasks:
            if t.resource_set.id in seen:
                continue
            seen.add(t.resource_set.id)
            total += t.resource_set.gpus()
        return total

    def to_dict(self):
        return {
            "type": self.type,
            "user": self.user,
            "count": self.count,
            "allow-decommission": self.allow_decommission,
            "image": self.image,
            "networks": [n.to_dict() for n in self.networks],
            "rlimits": [r.to_dict() for r in self.rlimits],
            "uris": list(self.uris),
            "task-specs": [t.to_dict() for t in self.tasks],
            "placement-rule": self.placement_rule.to_dict() if self.placement_rule is not None else None,
            "volumes": [v.to_dict() for v in self.volumes],
            "pre-reserved-role": self.pre_reserved_role,
            "secrets": [s.to_dict() for s in self.secrets],
            "share-pid-namespace": self.share_pid_namespace,
            "host-volumes": [h.to_dict() for h in self.host_volumes],
            "seccomp-unconfined": self.seccomp_unconfined,
            "seccomp-profile-name": self.seccomp_profile_name,
            "ipc-mode": self.shared_memory.value if self.shared_memory else None,
            "shm-size": self.shared_memory_size,
        }

    @staticmethod
    def from_dict(d) -> "PodSpec":
        from dcos_commons_amd.offer.evaluate.placement import placement_rule_from_dict

        return PodSpec(
            type=d["type"],
            user=d.get("user"),
            count=int(d.get("count") or 0),
            allow_decommission=bool(d.get("allow-decommission")),
            image=d.get("image"),
            networks=tuple(NetworkSpec.from_dict(n) for n in d.get("networks") or ()),
            rlimits=tuple(RLimitSpec.from_dict(r) for r in d.get("rlimits") or ()),
            uris=tuple(d.get("uris") or ()),
            tasks=tuple(TaskSpec.from_dict(t) for t in d.get("task-specs") or ()),
            placement_rule=placement_rule_from_dict(d["placement-rule"]) if d.get("placement-rule") else None,
            volumes=tuple(resource_spec_from_dict(v) for v in d.get("volumes") or ()),
            pre_reserved_role=d.get("pre-reserved-role") or ANY_ROLE,
            secrets=tuple(SecretSpec.from_dict(s) for s in d.get("secrets") or ()),
            share_pid_namespace=bool(d.get("share-pid-namespace")),
            host_volumes=tuple(HostVolumeSpec.from_dict(h) for h in d.get("host-volumes") or ()),
            seccomp_unconfined=bool(d.get("seccomp-unconfined")),
            seccomp_profile_name=d.get("seccomp-profile-name"),
            shared_memory=IpcMode.parse(d.get("ipc-mode")),
            shared_memory_size=d.get("shm-size"),
        )


@dataclass(frozen=True)
class ReplacementFailurePolicy:
    permanent_failure_timeout_mins: int = 20
    min_replace_delay_mins: int = 10

    def validate(self) -> None:
        _require(self.permanent_failure_timeout_mins is not None and self.permanent_failure_timeout_mins >= 0,
                 "permanent-failure-timeout-mins must be >= 0")
        _require(self.min_replace_delay_mins is not None and self.min_replace_delay_mins >= 0,
                 "min-replace-delay-mins must be >= 0")

    def to_dict(self):
        return {"permanent-failure-timeout-mins": self.permanent_failure_timeout_mins,
                "min-replace-delay-mins": self.min_replace_delay_mins}

    @staticmethod
    def from_dict(d):
        return ReplacementFailurePolicy(d.get("permanent-failure-timeout-mins", 20),
                                        d.get("min-replace-delay-mins", 10))


@dataclass(frozen=True)
class ServiceSpec:
    """DefaultServiceSpec. Persisted as the ``Configurations/<uuid>`` JSON blob."""

    name: str
    pods: Tuple[PodSpec, ...]
    role: str = ""
    principal: str = ""
    user: str = DEFAULT_SERVICE_USER
    goal: GoalState = GoalState.RUNNING
    region: Optional[str] = None
    web_url: Optional[str] = None
    zookeeper_connection: str = MESOS_MASTER_ZK_CONNECTION_STRING
    replacement_failure_policy: Optional[ReplacementFailurePolicy] = None

    @staticmethod
    def create(name: str, pods, role: str = "", principal: str = "", user: Optional[str] = None,
               goal: GoalState = GoalState.RUNNING, region: Optional[str] = None,
               web_url: Optional[str] = None, zookeeper_connection: Optional[str] = None,
               replacement_failure_policy: Optional[ReplacementFailurePolicy] = None) -> "ServiceSpec":
        pods = tuple(pods)
        if not (user and user.strip()):
            user = next((p.user for p in pods if p.user), DEFAULT_SERVICE_USER)
        spec = ServiceSpec(
            name=name, pods=pods, role=role, principal=principal, user=user, goal=goal or GoalState.RUNNING,
            region=region, web_url=web_url,
            zookeeper_connection=(zookeeper_connection if zookeeper_connection and zookeeper_connection.strip()
                                  else MESOS_MASTER_ZK_CONNECTION_STRING),
            replacement_failure_policy=replacement_failure_policy)
        spec.validate()
        return spec

    def validate(self) -> None:
        _require(bool(self.name), "ServiceSpec name must be non-empty")
        _require(bool(self.pods), "ServiceSpec pods must be non-empty")
        types = [p.type for p in self.pods]
        _require(len(types) == len(set(types)), f"ServiceSpec pod types must be unique: {types}")

    def pod(self, pod_type: str) -> Optional[PodSpec]:
        for p in self.pods:
            if p.type == pod_type:
                return p
        return None

    def uses_gpus(self) -> bool:
        return any(p.gpus_per_instance() >= 1 for p in self.pods)

    def to_dict(self):
        return {
            "name": self.name,
            "role": self.role,
            "principal": self.principal,
            "user": self.user,
            "goal": self.goal.value,
            "region": self.region,
            "web-url": self.web_url,
            "zookeeper": self.zookeeper_connection,
            "replacement-failure-policy": (self.replacement_failure_policy.to_dict()
                                           if self.replacement_failure_policy else None),
            "pod-specs": [p.to_dict() for p in self.pods],
        }

    def to_json_string(self) -> str:
        return json.dumps(self.to_dict(), indent=2)

    def to_json_bytes(self) -> bytes:
        # the spec is immutable: serialize once (the loopback check and the config store both ask)
        data = self.__dict__.get("_json_bytes")
        if data is None:
            data = json.dumps(self.to_dict(), separators=(",", ":")).encode("utf-8")
            self.__dict__["_json_bytes"] = data
        return data

    get_bytes = to_json_bytes

    @staticmethod
    def from_dict(d) -> "ServiceSpec":
        return ServiceSpec(
            name=d["name"],
            role=d.get("role") or "",
            principal=d.get("principal") or "",
            user=d.get("user") or DEFAULT_SERVICE_USER,
            goal=GoalState.parse_persisted(d.get("goal") or "RUNNING"),
            region=d.get("region"),
            web_url=d.get("web-url"),
            zookeeper_connection=d.get("zookeeper") or MESOS_MASTER_ZK_CONNECTION_STRING,
            replacement_failure_policy=(ReplacementFailurePolicy.from_dict(d["replacement-failure-policy"])
                                        if d.get("replacement-failure-policy") else None),
            pods=tuple(PodSpec.from_dict(p) for p in d.get("pod-specs") or ()),
        )

    @staticmethod
    def from_json_bytes(data: bytes) -> "ServiceSpec":
        return ServiceSpec.from_dict(json.loads(data.decode("utf-8")))


@functools.lru_cache(maxsize=32)
def _parse_cached(data: bytes) -> "ServiceSpec":
    """JSON -> ServiceSpec, memoized by the exact bytes (specs are immutable, parsing is pure).
    ``lru_cache`` is thread-safe: services of a multi-service scheduler run their loopback checks
    concurrently."""
    return ServiceSpec.from_json_bytes(data)


class ServiceSpecFactory:
    """ConfigurationFactory<ServiceSpec>: parses persisted JSON configs."""

    def parse(self, data: bytes) -> ServiceSpec:
        return ServiceSpec.from_json_bytes(data)


def loopback_check(spec: ServiceSpec) -> ServiceSpecFactory:
    """DefaultServiceSpec.getConfigurationFactory: round-trip the spec through JSON and fail
    if the result differs (DefaultServiceSpec.java getConfigurationFactory)."""
    factory = ServiceSpecFactory()
    loop = _parse_cached(spec.to_json_bytes())
    if loop != spec:
        raise SpecValidationError(
            "Equality test failed: Loopback result is not equal to original:\n- Original:\n"
            + spec.to_json_string() + "\n- Result:\n" + loop.to_json_string())
    return factory


# ---------------------------------------------------------------------------------------
# pod instances


@dataclass(frozen=True, eq=False)
class PodInstance:
    """DefaultPodInstance: pod spec + index; name ``<type>-<index>``."""

    pod: PodSpec
    index: int

    @property
    def name(self) -> str:
        return f"{self.pod.type}-{self.index}"

    def conflicts_with(self, other: "PodInstance") -> bool:
        return self.pod.type == other.pod.type and self.index == other.index

    def __eq__(self, other):
        return isinstance(other, PodInstance) and self.name == other.name

    def __hash__(self):
        return hash(self.name)

    def __repr__(self):
        return f"PodInstance({self.name})"


def get_task_instance_name(pod_instance: PodInstance, task_name: str) -> str:
    """CommonIdUtils.getTaskInstanceName: ``<pod>-<index>-<task>``."""
    return f"{pod_instance.name}-{task_name}"
