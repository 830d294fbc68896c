"""Endpoint and task-network helpers (reference: testing/sdk_networks.py).

Task addresses come from the statuses the local master reports: host-network tasks (and
bridge-networked ones) carry the agent's address and no network name, virtual-network tasks carry
the network's name and an address from the agent's overlay subnet (``9.0.<agent>.0/24``).
"""
from __future__ import annotations

import json
from typing import Any, Dict, List, Optional

from dcos_commons_amd.testing.sdk import sdk_agents, sdk_cmd, sdk_tasks, sdk_utils

ENABLE_VIRTUAL_NETWORKS_OPTIONS = {"service": {"virtual_network_enabled": True}}


def _endpoint_info(service_name: str, endpoint_name: Optional[str], as_json: bool) -> Any:
    path = "/v1/endpoints" + (f"/{endpoint_name}" if endpoint_name else "")

    @sdk_utils.retry(timeout_s=5, interval_s=0.5)
    def fetch():
        r = sdk_cmd.service_request("GET", service_name, path)
        assert r.ok, f"Failed to get endpoint named {endpoint_name}: {r.status_code}"
        return r.json() if as_json else r.text
    return fetch()


def get_endpoint_names(package_name: str, service_name: str) -> List[str]:
    result = _endpoint_info(service_name, None, True)
    assert isinstance(result, list)
    return result


def get_endpoint(package_name: str, service_name: str, endpoint_name: str) -> Dict[str, Any]:
    assert endpoint_name, "Missing endpoint_name. To get list of endpoint names, use get_endpoint_names()."
    return _endpoint_info(service_name, endpoint_name, True)


def get_endpoint_string(package_name: str, service_name: str, endpoint_name: str) -> str:
    assert endpoint_name, "Missing endpoint_name. To get list of endpoint names, use get_endpoint_names()."
    return _endpoint_info(service_name, endpoint_name, False).strip()


def get_task_host(task_info: Dict[str, Any]) -> str:
    return task_info.get("offer_hostname") or task_info.get("host", "")


def _running_statuses(task_name: str) -> List[Dict[str, Any]]:
    statuses = [s for s in sdk_tasks.get_all_status_history(task_name, with_completed_tasks=False)
                if s["state"] == "TASK_RUNNING"]
    assert statuses, f"Unable to find any statuses for running task_name={task_name}"
    return statuses


def get_task_ip(service_name: str, task_name: str) -> str:
    """The address the newest TASK_RUNNING status of ``task_name`` reports."""
    tasks = [t for t in sdk_tasks.get_service_tasks(service_name) if t.name == task_name]
    assert tasks, f"no task {task_name} in {service_name}"
    for s in reversed(_running_statuses(task_name)):
        for n in s.get("container_status", {}).get("network_infos", []):
            for a in n.get("ip_addresses", []):
                return a["ip_address"]
    raise AssertionError(f"task {task_name} reports no address")


def check_task_network(task_name: str, expected_network_name: Optional[str] = "dcos") -> None:
    """Every RUNNING status of the task names ``expected_network_name`` (None: no name, i.e. the
    host network)."""
    for status in _running_statuses(task_name):
        for ni in status["container_status"]["network_infos"]:
            if expected_network_name is not None:
                assert ni.get("name") == expected_network_name, \
                    f"Expected network name:{expected_network_name} found:{ni.get('name')} ({status})"
            else:
                assert "name" not in ni, f"Task {task_name} has network name when it shouldn't, status:{status}"


def check_endpoint_on_overlay(package_name: str, service_name: str, endpoint_to_get: str,
                              expected_task_count: int) -> None:
    endpoint = get_endpoint(package_name, service_name, endpoint_to_get)
    assert "address" in endpoint, f"Missing 'address': {endpoint}"
    assert len(endpoint["address"]) == expected_task_count
    assert "dns" in endpoint, f"Missing 'dns': {endpoint}"
    assert len(endpoint["dns"]) == expected_task_count
    ips = {e.split(":")[0] for e in endpoint["address"]}
    agent_ips = {a["hostname"] for a in sdk_agents.get_agents()}
    assert not ips & agent_ips, "Overlay IPs should not match any agent IPs"
    for dns in endpoint["dns"]:
        assert "autoip.dcos.thisdcos.directory" in dns, "Expected 'autoip.dcos.thisdcos.directory' in DNS entry"


def get_srv_records(service_name: str) -> Dict[str, List[str]]:
    """task name -> Mesos-DNS record names of the service's running tasks (``/v1/enumerate``)."""
    rc, out, _ = sdk_cmd.master_ssh("curl localhost:8123/v1/enumerate", print_output=False)
    assert rc == 0
    fws = [f for f in json.loads(out)["frameworks"] if f["name"] == service_name and f["tasks"]]
    assert len(fws) == 1, f"Expected exactly one entry for service {service_name}: {fws}"
    out_map: Dict[str, List[str]] = {}
    for t in fws[0]["tasks"]:
        assert t["name"] not in out_map, f"Got multiple entries for task {t['name']}"
        out_map[t["name"]] = [r["name"] for r in t["records"]]
    return out_map
