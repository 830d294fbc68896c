"""Raw YAML -> internal ServiceSpec conversion.

Reference: sdk/.../specification/yaml/YAMLToInternalMappers.java:114-805 (``convertServiceSpec``
:114, ``convertPod`` :272, ``convertTask`` :407, ``convertResourceSet`` :516,
``convertPorts`` :718), plus ``DefaultServiceSpec.Generator``.
"""
from __future__ import annotations

import logging
import os
from typing import Dict, List, Optional

from dcos_commons_amd.config.task_env_router import TaskEnvRouter
from dcos_commons_amd.dcos import constants as dcos_constants
from dcos_commons_amd.framework.framework_config import FrameworkConfig
from dcos_commons_amd.mesos import protos as P
from dcos_commons_amd.offer.evaluate.placement import PassthroughRule, parse_marathon_constraints
from dcos_commons_amd.specification.specs import (
    ANY_ROLE,
    PORTS_RESOURCE_TYPE,
    CommandSpec,
    ConfigFileSpec,
    DiscoverySpec,
    GoalState,
    HealthCheckSpec,
    HostVolumeSpec,
    IpcMode,
    NamedVIPSpec,
    NetworkSpec,
    PodSpec,
    PortSpec,
    RangeSpec,
    ReadinessCheckSpec,
    ResourceSet,
    ResourceSetBuilder,
    RLimitSpec,
    SecretSpec,
    ServiceSpec,
    SpecValidationError,
    TaskSpec,
    TransportEncryptionSpec,
    TransportEncryptionType,
    VolumeSpec,
    VolumeType,
    ranges_value,
)

from .raw import RawServiceSpec

LOGGER = logging.getLogger(__name__)


class ConfigTemplateReader:
    def __init__(self, template_dir: Optional[str]):
        self.template_dir = template_dir or "."

    def read(self, name: str) -> str:
        with open(os.path.join(self.template_dir, name), "r", encoding="utf-8") as f:
            return f.read()


def _seccomp_unconfined(raw_pod) -> bool:
    unconfined = bool(raw_pod.get("seccomp-unconfined"))
    if unconfined and raw_pod.get("seccomp-profile-name"):
        raise ValueError("seccomp-unconfined and seccomp-profile-name cannot both be set for a pod")
    return unconfined


def _text(v):
    """Jackson coerces YAML scalars bound to String fields (``cmd: true`` -> "true")."""
    if v is None or isinstance(v, str):
        return v
    if isinstance(v, bool):
        return "true" if v else "false"
    return str(v)


def _labels(csv: str) -> Dict[str, str]:
    out = {}
    for kv in csv.split(","):
        parts = kv.split(":", 1)
        if len(parts) != 2:
            raise SpecValidationError(
                f"Illegal label string, got {csv}, should be comma-seperated key value pairs "
                "(seperated by colons). For example: k_0:v_0,k_1:v_1,...,k_n:v_n")
        out[parts[0]] = parts[1]
    return out


def _verify_distinct_discovery_prefixes(raw_pods) -> None:
    counts: Dict[str, int] = {}
    for pod in raw_pods.values():
        prefixes = set()
        for task in pod["tasks"].values():
            d = task.get("discovery")
            if d and d.get("prefix") is not None:
                prefixes.add(d["prefix"])
        for p in prefixes:
            counts[p] = counts.get(p, 0) + 1
    dups = [p for p, c in counts.items() if c > 1]
    if dups:
        raise SpecValidationError(f"Tasks in different pods cannot share DNS names: {dups}")


def _verify_distinct_endpoint_names(raw_pods) -> None:
    seen, dups = set(), set()

    def collect(ports):
        for name, p in (ports or {}).items():
            if not p.get("advertise"):
                continue
            if name in seen:
                dups.add(name)
            seen.add(name)

    for pod in raw_pods.values():
        for task in pod["tasks"].values():
            collect(task.get("ports"))
        for rs in (pod.get("resource-sets") or {}).values():
            collect(rs.get("ports"))
    if dups:
        raise SpecValidationError(f"Service has duplicate advertised ports across tasks: [{', '.join(sorted(dups))}]")


def _pod_role(pre_reserved_role: Optional[str], role: str) -> str:
    if pre_reserved_role is None or pre_reserved_role == ANY_ROLE:
        return role
    return f"{pre_reserved_role}/{role}"


def _convert_ports(role, pre_reserved_role, principal, raw_ports, network_names) -> List[PortSpec]:
    specs = []
    seen = set()
    for name, rp in raw_ports.items():
        port = int(rp.get("port") or 0)
        if port in seen and port > 0:
            raise SpecValidationError(f"Cannot have duplicate port values: Task has multiple ports with value {port}")
        seen.add(port)
        visibility = (P.DiscoveryInfo.EXTERNAL if rp.get("advertise") else P.DiscoveryInfo.CLUSTER)
        common = dict(name=PORTS_RESOURCE_TYPE, value=ranges_value([(port, port)]), role=role,
                      principal=principal, pre_reserved_role=pre_reserved_role or ANY_ROLE,
                      env_key=rp.get("env-key"), port_name=name, visibility=visibility,
                      network_names=tuple(network_names))
        # RangeSpec: a missing begin is MIN_PORT (0); a missing or zero end is MAX_PORT (65535)
        ranges = tuple(RangeSpec(int(r["begin"]) if r.get("begin") is not None else RangeSpec.MIN_PORT,
                                 int(r["end"]) if r.get("end") else RangeSpec.MAX_PORT)
                       for r in rp.get("ranges") or ())
        vip = rp.get("vip")
        if vip is None:
            spec = PortSpec(ranges=ranges, **common)
        else:
            vip_name = vip.get("prefix") or name
            matching = raw_ports.get(vip_name)
            if matching is not None and matching is not rp:
                raise SpecValidationError(
                    f"Provided VIP prefix '{vip_name}' in port '{name}' conflicts with other port also named "
                    f"'{vip_name}'. Expected VIP prefix to not collide with other ports' names.")
            spec = NamedVIPSpec(protocol=dcos_constants.DEFAULT_IP_PROTOCOL, vip_name=vip_name,
                                vip_port=int(vip.get("port") or 0), **common)
        spec.validate()
        specs.append(spec)
    return specs


def _convert_resource_set(rs_id, cpus, gpus, memory, raw_ports, raw_volume, raw_volumes, role,
                          pre_reserved_role, principal, network_names) -> ResourceSet:
    b = ResourceSetBuilder(role, pre_reserved_role, principal)
    if raw_volumes is not None:
        if raw_volume is not None:
            raise SpecValidationError(f"Both 'volume' and 'volumes' may not be specified at the same time: {rs_id}")
        for v in raw_volumes.values():
            b.add_volume(v.get("type"), float(v.get("size") or 0), v.get("path"), v.get("profiles") or [])
    if raw_volume is not None:
        b.add_volume(raw_volume.get("type"), float(raw_volume.get("size") or 0), raw_volume.get("path"),
                     raw_volume.get("profiles") or [])
    if cpus is not None:
        b.cpus(float(cpus))
    if gpus is not None:
        b.gpus(float(gpus))
    if memory is not None:
        b.memory(float(memory))
    if raw_ports is not None:
        for p in _convert_ports(role, pre_reserved_role, principal, raw_ports, network_names):
            b.add_resource(p)
    b.id = rs_id
    return b.build()


def _convert_volume(rv, role, pre_reserved_role, principal) -> VolumeSpec:
    try:
        t = VolumeType(rv.get("type"))
    except ValueError:
        raise SpecValidationError(
            f"Provided volume type '{rv.get('type')}' for path '{rv.get('path')}' is invalid. "
            f"Expected type to be one of: {[v.value for v in VolumeType]}")
    if t == VolumeType.ROOT:
        return VolumeSpec.create_root_volume(float(rv.get("size") or 0), rv.get("path"), role,
                                             pre_reserved_role, principal)
    return VolumeSpec.create_mount_volume(float(rv.get("size") or 0), rv.get("path"), rv.get("profiles") or [],
                                          role, pre_reserved_role, principal)


def _collate_ports(raw_pod) -> List[int]:
    ports = []
    for rs in (raw_pod.get("resource-sets") or {}).values():
        for p in (rs.get("ports") or {}).values():
            ports.append(int(p.get("port") or 0))
    for t in raw_pod["tasks"].values():
        for p in (t.get("ports") or {}).values():
            ports.append(int(p.get("port") or 0))
    return ports


def _convert_network(name, rn, ports) -> NetworkSpec:
    rn = rn or {}
    host_ports = rn.get("host-ports")
    container_ports = rn.get("container-ports")
    n = 0
    if host_ports is not None and container_ports is not None:
        if len(host_ports) != len(container_ports):
            raise SpecValidationError("You need to specify the same number of host ports and container ports")
        n = len(host_ports)
    supports = dcos_constants.network_supports_port_mapping(name)
    if not supports and n > 0:
        raise SpecValidationError(f"Virtual Network {name} doesn't support container->host port mapping")
    mappings = {}
    if supports:
        if n > 0:
            mappings = {int(h): int(c) for h, c in zip(host_ports, container_ports)}
        for p in ports:
            mappings.setdefault(p, p)
    labels = _labels(rn["labels"]) if rn.get("labels") else {}
    return NetworkSpec(name, tuple(sorted(mappings.items())), tuple(sorted(labels.items())))


def _convert_task(rt, reader: ConfigTemplateReader, task_name, additional_env, resource_sets, role,
                  pre_reserved_role, principal, network_names) -> TaskSpec:
    env = rt.get("env") or {}
    env = {str(k): ("" if v is None else (str(v).lower() if isinstance(v, bool) else str(v))) for k, v in env.items()}
    command = CommandSpec.build(_text(rt.get("cmd")), env, additional_env) if rt.get("cmd") is not None else None
    configs = []
    for cname, c in (rt.get("configs") or {}).items():
        configs.append(ConfigFileSpec(cname, c.get("dest"), reader.read(c.get("template"))))
    health = None
    if rt.get("health-check") is not None:
        h = rt["health-check"]
        health = HealthCheckSpec(_text(h.get("cmd")), h.get("max-consecutive-failures"), h.get("delay"),
                                 h.get("interval"), h.get("timeout"), h.get("grace-period"))
        health.validate()
    readiness = None
    if rt.get("readiness-check") is not None:
        r = rt["readiness-check"]
        readiness = ReadinessCheckSpec(_text(r.get("cmd")), r.get("interval"), r.get("timeout"),
                                       r.get("delay") if r.get("delay") is not None else 0)
        readiness.validate()
    discovery = None
    if rt.get("discovery") is not None:
        d = rt["discovery"]
        vis = P.DiscoveryInfo.CLUSTER
        if d.get("visibility") is not None:
            try:
                vis = P.DiscoveryInfo.Visibility.Value(d["visibility"])
            except ValueError:
                raise SpecValidationError(
                    f"Visibility must be one of: {list(P.DiscoveryInfo.Visibility.keys())}")
        discovery = DiscoverySpec(d.get("prefix"), vis)
    tls = tuple(TransportEncryptionSpec(t["name"], TransportEncryptionType(t["type"]))
                for t in rt.get("transport-encryption") or ())
    goal_str = (rt.get("goal") or "").upper()
    if goal_str == "FINISHED":
        raise SpecValidationError(
            f"Unsupported GoalState {goal_str} in task {task_name}, expected one of: [{', '.join(g.value for g in GoalState)}]")
    try:
        goal = GoalState(goal_str)
    except ValueError:
        raise SpecValidationError(f"Unsupported GoalState '{goal_str}' in task {task_name}")
    if rt.get("resource-set"):
        matches = [r for r in resource_sets if r.id == rt["resource-set"]]
        if not matches:
            raise SpecValidationError(f"Task {task_name} references unknown resource-set {rt['resource-set']}")
        rs = matches[0]
    else:
        rs = _convert_resource_set(task_name + "-resource-set", rt.get("cpus"), rt.get("gpus"), rt.get("memory"),
                                   rt.get("ports"), rt.get("volume"), rt.get("volumes"), role, pre_reserved_role,
                                   principal, network_names)
    labels = _labels(rt["labels"]) if rt.get("labels") else {}
    spec = TaskSpec(
        name=task_name, goal=goal, resource_set=rs, command=command,
        essential=True if rt.get("essential") is None else bool(rt.get("essential")),
        task_labels=tuple(sorted(labels.items())), health_check=health, readiness_check=readiness,
        config_files=tuple(configs), discovery=discovery,
        kill_grace_period=int(rt.get("kill-grace-period") or 0), transport_encryption=tls,
        shared_memory=IpcMode.parse(rt.get("ipc-mode")), shared_memory_size=rt.get("shm-size"))
    spec.validate()
    return spec


def convert_pod(raw_pod, reader: ConfigTemplateReader, pod_name: str, additional_env: Dict[str, str],
                role: str, principal: str, user: str) -> PodSpec:
    pre_reserved_role = raw_pod.get("pre-reserved-role") or ANY_ROLE
    rlimits = []
    for name, rl in (raw_pod.get("rlimits") or {}).items():
        spec = RLimitSpec(name, rl.get("soft"), rl.get("hard"))
        spec.validate()
        rlimits.append(spec)
    network_names: List[str] = []
    networks = []
    for net_name, rn in (raw_pod.get("networks") or {}).items():
        if not dcos_constants.is_supported_network(net_name):
            LOGGER.warning("Virtual network '%s' is not supported, unexpected behavior may result", net_name)
        network_names.append(net_name)
        networks.append(_convert_network(net_name, rn, _collate_ports(raw_pod)))
    resource_sets = []
    for rs_name, rs in (raw_pod.get("resource-sets") or {}).items():
        resource_sets.append(_convert_resource_set(
            rs_name, rs.get("cpus"), rs.get("gpus"), rs.get("memory"), rs.get("ports"), rs.get("volume"),
            rs.get("volumes"), role, pre_reserved_role, principal, network_names))
    secrets = []
    for s in (raw_pod.get("secrets") or {}).values():
        file_path = s.get("file")
        if file_path is None and s.get("env-key") is None:
            file_path = s.get("secret")
        spec = SecretSpec(s.get("secret"), s.get("env-key"), file_path)
        spec.validate()
        secrets.append(spec)
    host_volumes = []
    for hv in (raw_pod.get("host-volumes") or {}).values():
        mode = hv.get("mode") or None
        spec = HostVolumeSpec(hv.get("host-path"), hv.get("container-path"), mode)
        spec.validate()
        host_volumes.append(spec)
    volumes = []
    if raw_pod.get("volume") is not None:
        volumes.append(_convert_volume(raw_pod["volume"], role, pre_reserved_role, principal))
    for v in (raw_pod.get("volumes") or {}).values():
        volumes.append(_convert_volume(v, role, pre_reserved_role, principal))
    tasks = [
        _convert_task(rt, reader, tname, additional_env, resource_sets, role, pre_reserved_role, principal,
                      network_names)
        for tname, rt in raw_pod["tasks"].items()
    ]
    rule = parse_marathon_constraints(pod_name, raw_pod.get("placement"))
    count = raw_pod.get("count")
    if count is None:
        raise SpecValidationError(f"Pod '{pod_name}' is missing required 'count'")
    pod = PodSpec(
        type=pod_name, count=int(count), tasks=tuple(tasks), user=user,
        allow_decommission=bool(raw_pod.get("allow-decommission")), image=raw_pod.get("image"),
        networks=tuple(networks), rlimits=tuple(rlimits), uris=tuple(raw_pod.get("uris") or ()),
        placement_rule=None if isinstance(rule, PassthroughRule) else rule, volumes=tuple(volumes),
        pre_reserved_role=pre_reserved_role, secrets=tuple(secrets),
        share_pid_namespace=bool(raw_pod.get("share-pid-namespace")), host_volumes=tuple(host_volumes),
        seccomp_unconfined=_seccomp_unconfined(raw_pod),
        seccomp_profile_name=raw_pod.get("seccomp-profile-name"),
        shared_memory=IpcMode.parse(raw_pod.get("ipc-mode")), shared_memory_size=raw_pod.get("shm-size"))
    pod.validate()
    return pod


def convert_service_spec(raw: RawServiceSpec, framework_config: FrameworkConfig, router: TaskEnvRouter,
                         reader: ConfigTemplateReader) -> ServiceSpec:
    if not raw.name:
        raise SpecValidationError("Missing required 'name' in Service Spec")
    _verify_distinct_discovery_prefixes(raw.pods)
    _verify_distinct_endpoint_names(raw.pods)
    pods = []
    for pod_name, raw_pod in raw.pods.items():
        pods.append(convert_pod(raw_pod, reader, pod_name, router.get_config(pod_name),
                                _pod_role(raw_pod.get("pre-reserved-role"), framework_config.role),
                                framework_config.principal, framework_config.user))
    return ServiceSpec.create(
        name=raw.name, pods=pods, role=framework_config.role, principal=framework_config.principal,
        user=framework_config.user, web_url=framework_config.web_url,
        zookeeper_connection=framework_config.zookeeper_host_port)


class ServiceSpecGenerator:
    """DefaultServiceSpec.Generator."""

    def __init__(self, raw: RawServiceSpec, scheduler_config, config_template_dir: Optional[str] = None,
                 env: Optional[Dict[str, str]] = None):
        self.raw = raw
        self.scheduler_config = scheduler_config
        self.router = TaskEnvRouter(env)
        self.reader = ConfigTemplateReader(config_template_dir)
        self.multi_service_framework_config: Optional[FrameworkConfig] = None

    def set_all_pods_env(self, key: str, value: str) -> "ServiceSpecGenerator":
        self.router.set_all_pods_env(key, value)
        return self

    def set_pod_env(self, pod_type: str, key: str, value: str) -> "ServiceSpecGenerator":
        self.router.set_pod_env(pod_type, key, value)
        return self

    def set_multi_service_framework_config(self, fc: FrameworkConfig) -> "ServiceSpecGenerator":
        self.multi_service_framework_config = fc
        return self

    def set_config_template_reader(self, reader) -> "ServiceSpecGenerator":
        self.reader = reader
        return self

    def build(self) -> ServiceSpec:
        ns = self.scheduler_config.service_namespace() if self.scheduler_config is not None else None
        fc = self.multi_service_framework_config or FrameworkConfig.from_raw_service_spec(self.raw, ns)
        return convert_service_spec(self.raw, fc, self.router, self.reader)


def generate_service_spec(yaml_path: str, scheduler_config, env: Optional[Dict[str, str]] = None) -> ServiceSpec:
    """Convenience: render+parse ``yaml_path`` against ``env`` and convert it."""
    env = dict(os.environ if env is None else env)
    raw = RawServiceSpec.new_builder(yaml_path).set_env(env).build()
    return ServiceSpecGenerator(raw, scheduler_config, os.path.dirname(os.path.abspath(yaml_path)), env).build()
