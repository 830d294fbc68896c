"""Cluster feature gates (reference sdk/.../dcos/Capabilities.java:30-120).

The reference derives these from the DC/OS version; tests override them
(``Capabilities.overrideCapabilities``). The MI355X build defaults to a modern cluster
(reservation refinement, GPU resources, CNI port mapping, region awareness all available).
"""
from __future__ import annotations

import threading
from dataclasses import dataclass, replace
from typing import Optional


@dataclass(frozen=True)
class Capabilities:
    supports_pre_reserved_resources: bool = True
    supports_gpu_resource: bool = True
    supports_cni_port_mapping: bool = True
    supports_rlimits: bool = True
    supports_default_executor: bool = True
    supports_file_based_secrets: bool = True
    supports_env_based_secrets: bool = True
    supports_region_awareness: bool = True
    supports_seccomp: bool = True
    supports_shm: bool = True
    supports_domains: bool = True
    supports_v1_api_by_default: bool = True
    supports_partition_awareness: bool = True
    version: str = "1.13"

    def with_overrides(self, **kw) -> "Capabilities":
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
