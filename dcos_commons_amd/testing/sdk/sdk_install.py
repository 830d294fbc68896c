"""Package install / uninstall with verification.

Reference: testing/sdk_install.py. ``install`` renders and starts the package through Cosmos, waits
for the expected running tasks, the Marathon deployment and the deploy plan. ``uninstall`` runs the
SDK uninstall (scheduler with ``SDK_UNINSTALL``), then verifies that no reservation of the
service's role is left on any agent (except agents passed to ``ignore_dead_agent``) and that its
framework is gone from the master.
"""
from __future__ import annotations

import enum
import logging
import time
from typing import Any, Dict, List, Optional, Set, Union

from dcos_commons_amd.testing.sdk import sdk_marathon, sdk_plan, sdk_tasks, sdk_utils

LOG = logging.getLogger(__name__)
TIMEOUT_SECONDS = 120
_dead_agent_hosts: Set[str] = set()


class PackageVersion(enum.Enum):
    STUB_UNIVERSE = None        # the package built from this tree (latest registered version)
    LATEST_UNIVERSE = "latest"  # the newest released version


def _cluster():
    from dcos_commons_amd.testing.cluster import current

    return current()


def get_installed_service_names() -> List[str]:
    return ["/" + n for n in sorted(_cluster().cosmos.installed)]


def install(package_name: str, service_name: str, expected_running_tasks: int,
            additional_options: Optional[Dict[str, Any]] = None,
            package_version: Optional[Union[PackageVersion, str]] = PackageVersion.STUB_UNIVERSE,
            timeout_seconds: int = TIMEOUT_SECONDS, wait_for_deployment: bool = True,
            insert_strict_options: bool = True, wait_for_all_conditions: bool = True) -> None:
    start = time.time()
    if sdk_marathon.app_exists(service_name):
        raise Exception(f"Service is already installed: {service_name}")
    options = sdk_utils.merge_dictionaries({"service": {"name": service_name}}, additional_options or {})
    version = package_version.value if isinstance(package_version, PackageVersion) else package_version
    c = _cluster()
    if version == "latest":
        version = c.cosmos.versions(package_name)[-1]
    LOG.info("Installing package=%s service=%s options=%s version=%s", package_name, service_name, options, version)
    c.cosmos.install(package_name, None, options, version=version, wait=True)
    if expected_running_tasks > 0 and wait_for_all_conditions:
        sdk_tasks.check_running(service_name, expected_running_tasks, timeout_seconds)
    if wait_for_all_conditions:
        sdk_marathon.wait_for_deployment(service_name, timeout_seconds, None)
    if wait_for_deployment:
        sdk_plan.wait_for_completed_deployment(service_name, timeout_seconds)
    LOG.info("Installed package=%s service=%s after %s", package_name, service_name,
             sdk_utils.pretty_duration(time.time() - start))


def ignore_dead_agent(agent_host: str) -> None:
    """Orphaned reservations on this (dead) agent are tolerated by the next ``uninstall``."""
    _dead_agent_hosts.add(agent_host)


def _verify_completed_uninstall(service_name: str) -> None:
    c = _cluster()
    role = sdk_utils.get_role(service_name)
    orphans = [(h, r) for h, r in c.reserved_resources(role) if h not in _dead_agent_hosts]
    if orphans:
        raise Exception(f"Found {len(orphans)} orphaned resources after uninstall of {service_name}: "
                        + ", ".join(f"{h}:{r.name}" for h, r in orphans))
    frameworks = [f for f in c.frameworks() if f["name"] == service_name]
    if frameworks:
        raise Exception(f"Found {len(frameworks)} orphaned frameworks named {service_name}: {frameworks}")


def uninstall(package_name: str, service_name: str, timeout_seconds: int = TIMEOUT_SECONDS) -> None:
    start = time.time()
    c = _cluster()
    if not sdk_marathon.app_exists(service_name):
        LOG.info("Skipping uninstall of %s: app does not exist", service_name)
        return
    LOG.info("Uninstalling package=%s service=%s", package_name, service_name)
    c.cosmos.uninstall(service_name, timeout_s=timeout_seconds)
    try:
        _verify_completed_uninstall(service_name)
    except Exception:
        LOG.error("Scheduler logs of %s:\n%s", service_name, c.marathon.history_log_tails(service_name, 60))
        raise
    _dead_agent_hosts.clear()
    LOG.info("Uninstalled %s after %s", service_name, sdk_utils.pretty_duration(time.time() - start))
