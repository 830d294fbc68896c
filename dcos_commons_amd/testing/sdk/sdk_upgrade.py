"""Upgrade / downgrade / options-update flows (reference: testing/sdk_upgrade.py).

``test_upgrade`` installs the oldest registered version of the package (or the same one when only
one exists), upgrades to the newest and waits for every task to be relaunched on the new config;
``update_or_upgrade_or_downgrade`` is ``dcos <pkg> update start [--options] [--package-version]``.
"""
from __future__ import annotations

import json
import logging
import os
import tempfile
from typing import Any, Dict, Optional

from dcos_commons_amd.testing.sdk import sdk_cmd, sdk_install, sdk_plan, sdk_tasks

LOG = logging.getLogger(__name__)
TIMEOUT_SECONDS = 120


def _cosmos():
    from dcos_commons_amd.testing.cluster import current

    return current().cosmos


def get_config(package_name: str, service_name: str) -> Dict[str, Any]:
    return _cosmos().describe(service_name)["resolvedOptions"]


def _update(package_name: str, service_name: str, to_version: Optional[str], to_options: Optional[Dict[str, Any]]):
    cmd = "update start"
    path = None
    if to_options is not None:
        fd, path = tempfile.mkstemp(suffix=".json")
        with os.fdopen(fd, "w") as f:
            json.dump(to_options, f)
        cmd += f" --options={path}"
    if to_version:
        cmd += f" --package-version={to_version}"
    try:
        rc, out, err = sdk_cmd.svc_cli(package_name, service_name, cmd, check=True)
    finally:
        if path:
            os.unlink(path)
    return rc


def update_or_upgrade_or_downgrade(package_name: str, service_name: str, to_version: Optional[str],
                                   to_options: Dict[str, Any], expected_running_tasks: int,
                                   wait_for_deployment: bool = True, timeout_seconds: int = TIMEOUT_SECONDS) -> None:
    from dcos_commons_amd.testing.sdk import sdk_marathon

    task_ids = sdk_tasks.get_task_ids(service_name, "")
    if to_version is None and not to_options:
        return
    before = sdk_marathon.get_config(service_name).get("env", {})
    _update(package_name, service_name, to_version, to_options)
    after = sdk_marathon.get_config(service_name).get("env", {})
    # package coordinates alone do not touch tasks, nor do role changes (quota migration moves a
    # pod to the new role only when it is replaced: reference sdk_utils.filter_role_from_config);
    # anything else in the scheduler env may
    ignore = {"PACKAGE_VERSION", "PACKAGE_BUILD_TIME_EPOCH_MS", "PACKAGE_BUILD_TIME_STR",
              "ENABLE_ROLE_MIGRATION", "MESOS_ALLOCATION_ROLE"}
    changed = {k for k in set(before) | set(after) if k not in ignore and before.get(k) != after.get(k)}
    if wait_for_deployment:
        if changed:
            sdk_tasks.check_tasks_updated(service_name, "", task_ids, timeout_seconds)
        sdk_plan.wait_for_completed_deployment(service_name, timeout_seconds)
        sdk_tasks.check_running(service_name, expected_running_tasks, timeout_seconds)


def test_upgrade(package_name: str, service_name: str, expected_running_tasks: int,
                 from_options: Optional[Dict[str, Any]] = None, to_options: Optional[Dict[str, Any]] = None,
                 timeout_seconds: int = TIMEOUT_SECONDS, wait_for_deployment: bool = True) -> None:
    versions = _cosmos().versions(package_name)
    from_version, to_version = versions[0], versions[-1]
    sdk_install.install(package_name, service_name, expected_running_tasks, additional_options=from_options or {},
                        package_version=from_version, timeout_seconds=timeout_seconds,
                        wait_for_deployment=wait_for_deployment)
    if from_version == to_version and to_options is None:
        LOG.info("Only one version of %s is registered: skipping the upgrade half", package_name)
        return
    update_or_upgrade_or_downgrade(package_name, service_name, to_version, to_options or {},
                                   expected_running_tasks, wait_for_deployment, timeout_seconds)


def test_downgrade(package_name: str, service_name: str, expected_running_tasks: int,
                   timeout_seconds: int = TIMEOUT_SECONDS, to_options: Optional[Dict[str, Any]] = None) -> None:
    """To the oldest registered version (the reference's ``to_version``: its previous release),
    with ``to_options`` if given."""
    versions = _cosmos().versions(package_name)
    update_or_upgrade_or_downgrade(package_name, service_name, versions[0], to_options or {}, expected_running_tasks,
                                   True, timeout_seconds)
