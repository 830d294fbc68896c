"""Naming and cluster helpers for integration tests.

Reference: testing/sdk_utils.py (same function names and naming rules). The cluster is the local
DC/OS stand-in (``testing.cluster``): it is always "open" (no strict security mode) and reports the
DC/OS version it was created with.
"""
from __future__ import annotations

import copy
import functools
import logging
import os
import random
import string
from typing import Any, Dict

LOG = logging.getLogger(__name__)


class DCOS_SECURITY:
    disabled = 1
    permissive = 2
    strict = 3


def _cluster():
    from dcos_commons_amd.testing.cluster import current

    return current()


def get_package_name(default: str) -> str:
    return os.environ.get("INTEGRATION_TEST__PACKAGE_NAME") or default


def get_service_name(default: str) -> str:
    return os.environ.get("INTEGRATION_TEST__SERVICE_NAME") or default


def get_foldered_name(service_name: str) -> str:
    """Services under test live in the ``/test/integration`` Marathon folder."""
    return "/test/integration/" + service_name.lstrip("/")


def get_task_id_service_name(service_name: str) -> str:
    """``/test/integration/foo`` -> ``test.integration.foo`` (the prefix of its task ids)."""
    return service_name.lstrip("/").replace("/", ".")


def get_task_id_prefix(service_name: str, task_name: str) -> str:
    return f"{get_task_id_service_name(service_name)}__{task_name}"


def get_deslashed_service_name(service_name: str) -> str:
    return service_name.lstrip("/").replace("/", "__")


def get_role(service_name: str) -> str:
    return f"{get_deslashed_service_name(service_name)}-role"


def get_zk_path(service_name: str) -> str:
    return f"dcos-service-{get_deslashed_service_name(service_name)}"


def dcos_version() -> str:
    return _cluster().dcos_version


def _version_tuple(v: str):
    out = []
    for part in v.split("-")[0].split("."):
        try:
            out.append(int(part))
        except ValueError:
            out.append(0)
    return tuple(out)


def dcos_version_less_than(version: str) -> bool:
    return _version_tuple(dcos_version()) < _version_tuple(version)


def dcos_version_at_least(version: str) -> bool:
    return not dcos_version_less_than(version)


def is_open_dcos() -> bool:
    return True


def is_strict_mode() -> bool:
    return False


def get_security_mode() -> int:
    return DCOS_SECURITY.disabled


def get_cluster_zones() -> Dict[str, str]:
    """Agent hostname -> fault-domain zone."""
    return {a["hostname"]: a["zone"] for a in _cluster().agents() if a.get("zone")}


def pretty_duration(seconds: float) -> str:
    if seconds is None:
        return "--"
    ret = ""
    if seconds >= 86400:
        ret += f"{int(seconds // 86400)}d"
        seconds %= 86400
    if seconds >= 3600:
        ret += f"{int(seconds // 3600)}h"
        seconds %= 3600
    if seconds >= 60:
        ret += f"{int(seconds // 60)}m"
        seconds %= 60
    return ret + f"{seconds:.3f}s" if seconds or not ret else ret


def random_string(length: int = 8) -> str:
    return "".join(random.choice(string.ascii_lowercase + string.digits) for _ in range(length))


def merge_dictionaries(dict1: Dict[str, Any], dict2: Dict[str, Any]) -> Dict[str, Any]:
    """Deep merge; values of ``dict2`` win."""
    out = copy.deepcopy(dict1)
    for k, v in (dict2 or {}).items():
        if isinstance(v, dict) and isinstance(out.get(k), dict):
            out[k] = merge_dictionaries(out[k], v)
        else:
            out[k] = copy.deepcopy(v)
    return out


def get_service_roles(service_name: str) -> Dict[str, Any]:
    """The service's roles as the master sees them: ``framework-roles`` (MULTI_ROLE frameworks) or
    ``framework-role``, and ``task-roles`` (task name -> role of its resources)."""
    from dcos_commons_amd.testing.sdk import sdk_cmd

    state = sdk_cmd.cluster_request("GET", "/mesos/master/state").json()
    out: Dict[str, Any] = {}
    fw = next((f for f in state["frameworks"] if f["name"] == service_name and f["active"]), None)
    if fw is not None:
        out["framework-roles"] = fw.get("roles")
        out["framework-role"] = fw.get("role") if "roles" not in fw else None
        out["task-roles"] = {t["name"]: t["role"] for t in fw.get("tasks", [])}
    return out


def filter_role_from_config(config: Dict[str, Any]) -> Dict[str, Any]:
    out = copy.deepcopy(config)
    out.get("service", {}).pop("role", None)
    return out


def check_dcos_min_version_mark(item) -> None:
    """pytest hook helper: skip tests marked ``dcos_min_version(v)`` on older clusters."""
    import pytest

    for mark in item.iter_markers(name="dcos_min_version"):
        if mark.args and dcos_version_less_than(mark.args[0]):
            pytest.skip(f"requires DC/OS {mark.args[0]} or newer, cluster is {dcos_version()}")


def retry(timeout_s: float = 60.0, interval_s: float = 0.1, exceptions=(AssertionError, Exception)):
    """Decorator: retry the call until it returns without raising, for at most ``timeout_s``."""
    def deco(fn):
        @functools.wraps(fn)
        def wrapper(*a, **kw):
            import time

            deadline = time.time() + timeout_s
            while True:
                try:
                    return fn(*a, **kw)
                except exceptions:
                    if time.time() >= deadline:
                        raise
                    time.sleep(interval_s)
        return wrapper
    return deco
