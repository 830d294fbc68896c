"""Cluster feature gates and the DC/OS version they derive from.

Reference: sdk/.../dcos/{Capabilities,DcosVersion}.java. ``Capabilities.for_version`` derives every
gate from the cluster version exactly as the reference does (named VIPs 1.8+, rlimits/GPUs/CNI
1.9+, secrets/refinement/partition awareness 1.10+, v1 API/domains 1.11+, profile mounts 1.12+,
seccomp 1.13+, shm 1.14+). Tests override single gates with ``with_overrides`` and install the
result with ``override_capabilities`` (Capabilities.overrideCapabilities). The default instance is
a current cluster where every gate is open: MI355X agents run on a modern Mesos, and the
scheduler must not refuse GPU pods because a version lookup was skipped.
"""
from __future__ import annotations

import enum
import json
import logging
import threading
from dataclasses import dataclass, replace
from typing import Mapping, Optional, Union

LOGGER = logging.getLogger(__name__)
DEV_VERSION_SUFFIX = "-dev"


class DcosVariant(enum.Enum):
    OPEN = "open"
    ENTERPRISE = "enterprise"
    UNKNOWN = "UNKNOWN"

    def __str__(self):
        return self.value


class DcosVersion:
    """``/dcos-metadata/dcos-version.json``: ``version`` plus the optional ``dcos-variant``."""

    VERSION_KEY = "version"
    VARIANT_KEY = "dcos-variant"

    def __init__(self, version: str, variant: DcosVariant = DcosVariant.UNKNOWN):
        self.version = version
        self.variant = variant

    @staticmethod
    def from_json(doc: Union[str, bytes, Mapping]) -> "DcosVersion":
        d = json.loads(doc) if isinstance(doc, (str, bytes)) else doc
        variant = DcosVariant.UNKNOWN
        raw = d.get(DcosVersion.VARIANT_KEY)
        if raw is not None:
            match = [v for v in (DcosVariant.OPEN, DcosVariant.ENTERPRISE) if v.value == raw]
            if match:
                variant = match[0]
            else:
                LOGGER.error("Unexpected dcos-variant : %s", raw)
        return DcosVersion(d[DcosVersion.VERSION_KEY], variant)

    def _element(self, index: int) -> str:
        elements = self.version.split(".")
        # Java's String.split drops trailing empty strings: "0." has one element
        while elements and elements[-1] == "":
            elements.pop()
        if len(elements) <= index:
            raise ValueError(f"Expected at least {index} dot-delimited element(s): {self.version}")
        return elements[index]

    def first_element(self) -> int:
        return int(self._element(0))

    def second_element(self) -> int:
        e = self._element(1)
        if e.endswith(DEV_VERSION_SUFFIX):
            e = e[:-len(DEV_VERSION_SUFFIX)]
        return int(e)

    def has_or_exceeds(self, major: int, minor: int) -> bool:
        try:
            first = self.first_element()
            if first != major:
                return first > major
            return self.second_element() >= minor
        except ValueError:
            LOGGER.error("Unable to parse DC/OS version string: %s", self.version)
            return False

    def __repr__(self):
        return f"DcosVersion({self.version}, {self.variant})"


# gate -> (major, minor) of the first DC/OS release that has it (Capabilities.java:60-135)
_GATES = {
    "supports_named_vips": (1, 8),
    "supports_env_based_secrets_directive_label": (1, 8),
    "supports_rlimits": (1, 9),
    "supports_gpu_resource": (1, 9),
    "supports_cni_networking": (1, 9),
    "supports_file_based_secrets": (1, 10),
    "supports_env_based_secrets": (1, 10),
    "supports_pre_reserved_resources": (1, 10),
    "supports_partition_awareness": (1, 10),
    "supports_v1_api_by_default": (1, 11),
    "supports_domains": (1, 11),
    "supports_region_awareness": (1, 11),
    "supports_profile_mount_volumes": (1, 12),
    "supports_seccomp": (1, 13),
    "supports_shm": (1, 14),
}


@dataclass(frozen=True)
class Capabilities:
    supports_named_vips: bool = True
    supports_env_based_secrets_directive_label: bool = True
    supports_rlimits: bool = True
    supports_gpu_resource: bool = True
    supports_cni_networking: bool = True
    supports_file_based_secrets: bool = True
    supports_env_based_secrets: bool = True
    supports_pre_reserved_resources: bool = True
    supports_partition_awareness: bool = True
    supports_v1_api_by_default: bool = True
    supports_domains: bool = True
    supports_region_awareness: bool = True
    supports_profile_mount_volumes: bool = True
    supports_seccomp: bool = True
    supports_shm: bool = True
    supports_default_executor: bool = True
    version: str = "1.14"

    @staticmethod
    def for_version(version: Union[str, DcosVersion]) -> "Capabilities":
        v = version if isinstance(version, DcosVersion) else DcosVersion(version)
        return Capabilities(version=v.version, **{k: v.has_or_exceeds(*mm) for k, mm in _GATES.items()})

    @property
    def dcos_version(self) -> DcosVersion:
        return DcosVersion(self.version)

    @property
    def supports_cni_port_mapping(self) -> bool:
        """CNI port mapping rides on CNI networking (same 1.9 gate)."""
        return self.supports_cni_networking

    def with_overrides(self, **kw) -> "Capabilities":
        if "supports_cni_port_mapping" in kw:
            kw["supports_cni_networking"] = kw.pop("supports_cni_port_mapping")
        return replace(self, **kw)


_instance: Optional[Capabilities] = None
_lock = threading.Lock()


def get_instance() -> Capabilities:
    global _instance
    if _instance is None:
        with _lock:
            if _instance is None:
                _instance = Capabilities()
    return _instance


def override_capabilities(c: Optional[Capabilities]) -> None:
    global _instance
    with _lock:
        _instance = c


def from_cluster(version_client) -> Capabilities:
    """Capabilities.getInstance's lookup: ask the cluster's version endpoint."""
    return Capabilities.for_version(version_client.get_dcos_version())
