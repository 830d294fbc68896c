"""Framework identity: name, role, principal, user, zk, pre-reserved roles.

Reference: sdk/.../framework/FrameworkConfig.java:29-233.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import List, Optional

from dcos_commons_amd.storage.persister_utils import with_escaped_slashes

SLASH_REPLACEMENT = "__"
_FROM_ENV = object()

DEFAULT_ROLE_SUFFIX = "-role"
DEFAULT_PRINCIPAL_SUFFIX = "-principal"
DEFAULT_SERVICE_USER = "root"
MESOS_MASTER_ZK_CONNECTION_STRING = "master.mesos:2181"


def _service_role(framework_name: str, namespace: Optional[str]) -> str:
    if namespace:
        return with_escaped_slashes(namespace)
    return with_escaped_slashes(framework_name) + DEFAULT_ROLE_SUFFIX


def _pre_reserved_roles(framework_role: str, pod_roles) -> List[str]:
    out = []
    for r in pod_roles:
        if r and r != "*":
            v = f"{r}/{framework_role}"
            if v not in out:
                out.append(v)
    return out


@dataclass(frozen=True)
class FrameworkConfig:
    framework_name: str
    role: str
    principal: str
    user: str = DEFAULT_SERVICE_USER
    zookeeper_host_port: str = MESOS_MASTER_ZK_CONNECTION_STRING
    pre_reserved_roles: List[str] = field(default_factory=list)
    web_url: Optional[str] = None

    @staticmethod
    def from_raw_service_spec(raw, namespace: Optional[str] = None) -> "FrameworkConfig":
        role = _service_role(raw.name, namespace)
        sched = raw.scheduler or {}
        return FrameworkConfig(
            framework_name=raw.name,
            role=role,
            principal=sched.get("principal") or raw.name + DEFAULT_PRINCIPAL_SUFFIX,
            user=sched.get("user") or DEFAULT_SERVICE_USER,
            zookeeper_host_port=sched.get("zookeeper") or MESOS_MASTER_ZK_CONNECTION_STRING,
            pre_reserved_roles=_pre_reserved_roles(role, [p.get("pre-reserved-role") or "*"
                                                          for p in raw.pods.values()]),
            web_url=raw.web_url,
        )

    @staticmethod
    def from_service_spec(spec, namespace: Optional[str] = None) -> "FrameworkConfig":
        role = _service_role(spec.name, namespace)
        return FrameworkConfig(
            framework_name=spec.name, role=role, principal=spec.principal, user=spec.user,
            zookeeper_host_port=spec.zookeeper_connection,
            pre_reserved_roles=_pre_reserved_roles(role, [p.pre_reserved_role for p in spec.pods]),
            web_url=spec.web_url)

    @staticmethod
    def from_env_store(env, namespace: Optional[str] = _FROM_ENV) -> "FrameworkConfig":
        """Multi-service mode: identity from the scheduler's environment. The service namespace
        (role) comes from ``MESOS_ALLOCATION_ROLE`` / ``MARATHON_APP_ENFORCE_GROUP_ROLE`` as
        SchedulerConfig.getServiceNamespace decides it, unless one is passed explicitly."""
        name = env.get_required("FRAMEWORK_NAME")
        if namespace is _FROM_ENV:
            from dcos_commons_amd.scheduler.scheduler_config import SchedulerConfig

            namespace = SchedulerConfig(env).service_namespace()
        return FrameworkConfig(
            framework_name=name,
            role=_service_role(name, namespace),
            principal=env.get_optional_non_empty("FRAMEWORK_PRINCIPAL", name + DEFAULT_PRINCIPAL_SUFFIX),
            user=env.get_optional_non_empty("FRAMEWORK_USER", DEFAULT_SERVICE_USER),
            zookeeper_host_port=env.get_optional_non_empty("FRAMEWORK_ZOOKEEPER", MESOS_MASTER_ZK_CONNECTION_STRING),
            pre_reserved_roles=list(dict.fromkeys(env.get_optional_string_list("FRAMEWORK_PRERESERVED_ROLES", []))),
            web_url=env.get_optional_non_empty("FRAMEWORK_WEB_URL", ""),
        )

    def all_resource_roles(self) -> List[str]:
        return sorted(set(self.pre_reserved_roles) | {self.role})

    def non_namespaced_role(self) -> str:
        return with_escaped_slashes(self.framework_name) + DEFAULT_ROLE_SUFFIX

    def namespaced_role(self) -> Optional[str]:
        """The top-level Marathon group of the service (``/path/to/svc`` -> ``path``), the quota role
        a group-role migration moves to; None outside a group (FrameworkConfig.getNamespacedRole)."""
        groups = self.non_namespaced_role().split(SLASH_REPLACEMENT)
        return groups[0] if len(groups) > 1 else None
