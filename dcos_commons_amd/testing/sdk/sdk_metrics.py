"""Scheduler metrics (reference: testing/sdk_metrics.py, scheduler half).

The scheduler serves its Codahale-style registry at ``/v1/metrics`` (counters, gauges, timers);
these helpers read and wait on it. Task metrics (dcos-metrics over StatsD) are not collected by the
local cluster.
"""
from __future__ import annotations

import logging
import time
from typing import Any, Dict, Optional

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
    names = set(emitted_metrics)
    missing = [m for m in expected_metrics if m not in names]
    if missing:
        LOG.info("Missing metrics: %s", missing)
    return not missing
