"""Cluster DNS names (reference: testing/sdk_hosts.py).

Same rules as the scheduler's ``http.endpoint_utils``: autoip names
``<task>.<service>.autoip.dcos.thisdcos.directory`` and VIP names
``<vip>.<service>.l4lb.thisdcos.directory`` (foldered service names drop their slashes).
"""
from __future__ import annotations

SYSTEM_HOST_SUFFIX = "mesos"
AUTOIP_HOST_SUFFIX = "autoip.dcos.thisdcos.directory"
VIP_HOST_SUFFIX = "l4lb.thisdcos.directory"


def _safe_name(name: str) -> str:
    return name.replace("/", "")


def _safe_mesos_dns_taskname(task_name: str) -> str:
    """``/path/to/task`` -> ``task-to-path``."""
    return "-".join(reversed([p for p in task_name.split("/") if p]))


def _to_host(host_first: str, host_second: str, host_third: str, port: int = -1) -> str:
    host = f"{host_first}.{host_second}.{host_third}"
    return host if port == -1 else f"{host}:{port}"


def system_host(first: str, second: str, port: int = -1) -> str:
    return _to_host(first, second, SYSTEM_HOST_SUFFIX, port)


def autoip_host(service_name: str, task_name: str, port: int = -1) -> str:
    return _to_host(_safe_mesos_dns_taskname(task_name), _safe_name(service_name).replace(".", "-"),
                    AUTOIP_HOST_SUFFIX, port)


def custom_host(service_name: str, task_name: str, custom_domain: str, port: int = -1) -> str:
    return _to_host(_safe_mesos_dns_taskname(task_name), _safe_name(service_name), custom_domain, port)


def vip_host(service_name: str, vip_name: str, port: int = -1) -> str:
    return _to_host(_safe_name(vip_name), _safe_name(service_name), VIP_HOST_SUFFIX, port)


def scheduler_vip_host(service_name: str, vip_name: str, port: int = -1) -> str:
    return _to_host(_safe_name(vip_name), _safe_name(service_name), VIP_HOST_SUFFIX, port)


def get_foldered_dns_name(service_name: str) -> str:
    return service_name.lstrip("/").replace("/", "")


def get_crypto_id_domain() -> str:
    return "autoip.dcos.thisdcos.directory"
