"""Marathon app helpers (reference: testing/sdk_marathon.py)."""
from __future__ import annotations

import copy
import logging
from typing import Any, Dict, Optional

LOG = logging.getLogger(__name__)
TIMEOUT_SECONDS = 120


def _marathon():
    from dcos_commons_amd.testing.cluster import current

    return current().marathon


def app_exists(app_name: str) -> bool:
    return _marathon().app_exists(app_name)


def get_config(app_name: str) -> Dict[str, Any]:
    """The app definition without runtime-only fields, ready for ``update_app``. ``fetch`` stays (as in
    the reference's ``testing/sdk_marathon.py:40-52``): a package's scheduler is fetched on every
    restart."""
    app = copy.deepcopy(_marathon().get_app(app_name))
    for k in ("tasks", "tasksRunning", "deployments", "version", "uris", "lastTaskFailure"):
        app.pop(k, None)
    return app


def wait_for_deployment(app_name: str, timeout: int = TIMEOUT_SECONDS, expected_version: Optional[str] = None,
                        *_a) -> None:
    _marathon().wait_for_deployment(app_name, timeout)


def install_app(app_definition: Dict[str, Any], timeout: int = TIMEOUT_SECONDS) -> None:
    _marathon().install_app(app_definition, wait=True)


def update_app(config: Dict[str, Any], timeout: int = TIMEOUT_SECONDS, wait_for_completed_deployment: bool = True,
               force: bool = True) -> None:
    if "env" in config:
        LOG.info("Updating %s env:\n%s", config["id"], "\n".join(f"{k}={v}" for k, v in sorted(config["env"].items())))
    _marathon().update_app(config, wait=wait_for_completed_deployment)


def destroy_app(app_name: str, timeout: int = TIMEOUT_SECONDS) -> None:
    _marathon().destroy_app(app_name, timeout)


def restart_app(app_name: str) -> None:
    _marathon().restart_app(app_name, wait=True)


def get_scheduler_task_prefix(service_name: str) -> str:
    from dcos_commons_amd.testing.cluster import scheduler_task_prefix

    return scheduler_task_prefix(service_name)


def get_scheduler_host(service_name: str) -> str:
    from dcos_commons_amd.testing.sdk import sdk_tasks

    tasks = sdk_tasks.get_service_tasks("marathon", task_prefix=get_scheduler_task_prefix(service_name))
    if not tasks:
        raise Exception(f"No marathon tasks starting with '{get_scheduler_task_prefix(service_name)}'")
    return tasks[-1].host


def bump_cpu_count_config(service_name: str, key_name: str, delta: float = 0.1) -> float:
    config = get_config(service_name)
    updated = float(config["env"][key_name]) + delta
    config["env"][key_name] = str(round(updated, 6))
    update_app(config)
    return updated


def bump_task_count_config(service_name: str, key_name: str, delta: int = 1) -> int:
    config = get_config(service_name)
    updated = int(config["env"][key_name]) + delta
    config["env"][key_name] = str(updated)
    update_app(config)
    return updated


def create_group(group_id: str, options: Dict[str, Any]) -> None:
    """``POST /v2/groups``: e.g. ``options={"enforceRole": True}`` makes the group's name the role
    of every app under it (Marathon quota groups)."""
    from dcos_commons_amd.testing.sdk import sdk_cmd

    definition = dict(options)
    definition["id"] = "/" + group_id.strip("/")
    sdk_cmd.cluster_request("POST", "/marathon/v2/groups", json=definition, log_args=False, raise_on_error=False)


def update_group(group_id: str, options: Dict[str, Any]) -> None:
    from dcos_commons_amd.testing.sdk import sdk_cmd

    definition = dict(options)
    definition["id"] = "/" + group_id.strip("/")
    sdk_cmd.cluster_request("PUT", "/marathon/v2/groups", json=definition, log_args=False, raise_on_error=False)


def delete_group(group_id: str) -> None:
    from dcos_commons_amd.testing.sdk import sdk_cmd

    if group_id:   # an empty id would mean "/": every app of the cluster
        sdk_cmd.cluster_request("DELETE", f"/marathon/v2/groups/{group_id.strip('/')}", log_args=False,
                                raise_on_error=False)
