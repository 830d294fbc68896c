"""Endpoint and task-address helpers (reference: testing/sdk_networks.py)."""
from __future__ import annotations

from typing import Any, Dict, List

from dcos_commons_amd.testing.sdk import sdk_cmd, sdk_tasks


def get_endpoint_names(package_name: str, service_name: str) -> List[str]:
    return sdk_cmd.service_request("GET", service_name, "/v1/endpoints").json()


def get_endpoint(package_name: str, service_name: str, endpoint_name: str) -> Dict[str, Any]:
    return sdk_cmd.service_request("GET", service_name, f"/v1/endpoints/{endpoint_name}").json()


def get_endpoint_string(package_name: str, service_name: str, endpoint_name: str) -> str:
    return sdk_cmd.service_request("GET", service_name, f"/v1/endpoints/{endpoint_name}").text


def get_task_host(task_info: Dict[str, Any]) -> str:
    return task_info.get("offer_hostname") or task_info.get("host", "")


def get_task_ip(service_name: str, task_name: str) -> str:
    """Every task on the stand-in shares the loopback address (the agent's hostname is its id)."""
    tasks = [t for t in sdk_tasks.get_service_tasks(service_name) if t.name == task_name]
    assert tasks, f"no task {task_name} in {service_name}"
    return "127.0.0.1"


def check_task_network(task_name: str, expected_network_name: str = "dcos") -> None:
    """Overlay networks are not modelled: tasks always run on the host network here."""
    assert expected_network_name in (None, "", "dcos", "host"), expected_network_name
