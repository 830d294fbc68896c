"""Scheduler and task metrics (reference: testing/sdk_metrics.py).

The scheduler serves its Codahale-style registry at ``/v1/metrics`` (counters, gauges, timers), and
pushes it over StatsD to its container's metrics socket. Task metrics go through dcos-metrics: a
task writes StatsD to ``STATSD_UDP_HOST:STATSD_UDP_PORT`` and the agent's
``/system/v1/agent/<agent>/metrics/v0/containers/<container>/app`` serves it (the local cluster's
``testing.cluster.metrics``).
"""
from __future__ import annotations

import logging
import time
import json
from typing import Any, Callable, Dict, List, Optional, Union

from dcos_commons_amd.testing.sdk import sdk_cmd

LOG = logging.getLogger(__name__)


def get_scheduler_metrics(service_name: str, timeout_seconds: int = 60) -> Dict[str, Any]:
    return sdk_cmd.service_request("GET", service_name, "/v1/metrics", timeout_seconds=timeout_seconds).json()


def get_scheduler_counter(service_name: str, counter_name: str, timeout_seconds: int = 60) -> Optional[int]:
    counters = get_scheduler_metrics(service_name, timeout_seconds).get("counters", {})
    c = counters.get(counter_name)
    return None if c is None else int(c.get("count", c) if isinstance(c, dict) else c)


def get_scheduler_gauge(service_name: str, gauge_name: str, timeout_seconds: int = 60) -> Any:
    gauges = get_scheduler_metrics(service_name, timeout_seconds).get("gauges", {})
    g = gauges.get(gauge_name)
    return g.get("value") if isinstance(g, dict) else g


def _wait_value(getter, expected, timeout_seconds: int, what: str) -> Any:
    deadline = time.time() + timeout_seconds
    last = None
    while time.time() < deadline:
        try:
            last = getter()
            if last is not None and (expected(last) if callable(expected) else last >= expected):
                return last
        except Exception as e:  # noqa: BLE001 -- scheduler restarting
            LOG.info("metrics not available yet: %s", e)
        time.sleep(0.1)
    raise AssertionError(f"{what}: last value {last}")


def wait_for_scheduler_counter_value(service_name: str, counter_name: str, min_value: int,
                                     timeout_seconds: int = 60) -> int:
    return _wait_value(lambda: get_scheduler_counter(service_name, counter_name), min_value, timeout_seconds,
                       f"counter {counter_name} of {service_name} >= {min_value}")


def wait_for_scheduler_gauge_value(service_name: str, gauge_name: str, gauge_callback,
                                   timeout_seconds: int = 60) -> Any:
    return _wait_value(lambda: get_scheduler_gauge(service_name, gauge_name), gauge_callback, timeout_seconds,
                       f"gauge {gauge_name} of {service_name}")


def check_metrics_presence(emitted_metrics, expected_metrics) -> bool:
    """Whether every expected metric name was emitted (case-insensitive, as dcos-metrics may
    normalize names)."""
    names = {m.lower() for m in emitted_metrics}
    missing = [m for m in expected_metrics if m.lower() not in names]
    if missing:
        LOG.info("Missing metrics: %s", missing)
    return not missing


def get_metrics_from_cli(task_name: str) -> Union[Dict[str, Any], List[Dict[str, Any]]]:
    """``dcos task metrics details --json <task>``: the datapoints of the task's container."""
    rc, stdout, stderr = sdk_cmd.run_cli(f"task metrics details --json {task_name}")
    if rc:
        LOG.error("Error fetching metrics for %s: %s %s", task_name, stdout, stderr)
        return {}
    return list(json.loads(stdout))


def wait_for_metrics_from_cli(task_name: str, timeout_seconds: int) -> List[Dict[str, Any]]:
    deadline = time.time() + timeout_seconds
    while True:
        got = get_metrics_from_cli(task_name)
        if got:
            return list(got)
        if time.time() >= deadline:
            raise AssertionError(f"no metrics from task {task_name} within {timeout_seconds}s")
        time.sleep(0.5)


def get_metrics(package_name: str, service_name: str, pod_name: str, task_name: str) -> List[Dict[str, Any]]:
    """The task's dcos-metrics datapoints: its container ID from its pod's latest status, checked
    against the agent's container list, then the container's app metrics."""
    from dcos_commons_amd.testing.sdk import sdk_tasks

    task = next((t for t in sdk_tasks.get_service_tasks(service_name) if t.name == task_name), None)
    if task is None:
        raise Exception(f"Task named {task_name} not found in service {service_name}")
    rc, stdout, _ = sdk_cmd.svc_cli(package_name, service_name, f"pod info {pod_name}", print_output=False)
    assert rc == 0, "Pod info failed"
    cid = next((p["status"]["containerStatus"]["containerId"]["value"] for p in json.loads(stdout)
                if p["info"]["name"] == task_name and "status" in p), None)
    if cid is None:
        return []
    listed = sdk_cmd.cluster_request("GET", f"/system/v1/agent/{task.agent_id}/metrics/v0/containers").json()
    if cid not in listed:
        raise ValueError(f"container {cid} of {task_name} not among the agent's metrics containers {listed}")
    app = sdk_cmd.cluster_request("GET", f"/system/v1/agent/{task.agent_id}/metrics/v0/containers/{cid}/app").json()
    if app.get("dimensions", {}).get("task_name") != task_name:
        raise Exception(f"No metrics found for task {task_name} in service {service_name}")
    return list(app["datapoints"])


def wait_for_service_metrics(package_name: str, service_name: str, pod_name: str, task_name: str, timeout: int,
                             expected_metrics_callback: Callable[[List[str]], bool]) -> List[str]:
    deadline = time.time() + timeout
    while True:
        names = [m["name"] for m in get_metrics(package_name, service_name, pod_name, task_name)]
        if expected_metrics_callback(names):
            return names
        if time.time() >= deadline:
            raise AssertionError(f"metrics of {task_name} never matched: {names}")
        time.sleep(0.5)
