"""Plan queries and waits.

Reference: testing/sdk_plan.py (same names and status semantics: ``/v1/plans/<plan>`` answers 200
when COMPLETE, 202 while in progress and 417 when the plan has errors, and a wait gives up when the
service's tasks keep failing). The local cluster reacts in milliseconds, so waits poll every
``POLL_S`` and default to ``TIMEOUT_SECONDS`` = 120 s instead of the reference's 15 minutes.
"""
from __future__ import annotations

import logging
import time
from typing import Any, Callable, Dict, List, Optional, Union

from dcos_commons_amd.testing.sdk import sdk_cmd, sdk_tasks

LOG = logging.getLogger(__name__)
TIMEOUT_SECONDS = 120
SHORT_TIMEOUT_SECONDS = 30
MAX_NEW_TASK_FAILURES = 10
POLL_S = 0.1


class TaskFailuresExceededException(Exception):
    pass


def _plans_path(multiservice_name: Optional[str]) -> str:
    return "/v1/plans" if multiservice_name is None else f"/v1/service/{multiservice_name}/plans"


def get_deployment_plan(service_name: str, timeout_seconds: int = TIMEOUT_SECONDS) -> Dict[str, Any]:
    return get_plan(service_name, "deploy", timeout_seconds)


def get_recovery_plan(service_name: str, timeout_seconds: int = TIMEOUT_SECONDS) -> Dict[str, Any]:
    return get_plan(service_name, "recovery", timeout_seconds)


def get_decommission_plan(service_name: str, timeout_seconds: int = TIMEOUT_SECONDS) -> Dict[str, Any]:
    return get_plan(service_name, "decommission", timeout_seconds)


def list_plans(service_name: str, timeout_seconds: int = TIMEOUT_SECONDS,
               multiservice_name: Optional[str] = None) -> List:
    result = sdk_cmd.service_request("GET", service_name, _plans_path(multiservice_name),
                                     timeout_seconds=timeout_seconds).json()
    assert isinstance(result, list), result
    return result


def get_plan_once(service_name: str, plan: str, multiservice_name: Optional[str] = None) -> Dict[str, Any]:
    resp = sdk_cmd.service_request("GET", service_name, f"{_plans_path(multiservice_name)}/{plan}",
                                   retry=False, raise_on_error=False, log_args=False)
    if resp.status_code not in (200, 202, 417):   # 417: the plan has errors, still a plan
        resp.raise_for_status()
        raise sdk_cmd.HTTPError(resp)
    result = resp.json()
    assert isinstance(result, dict), result
    return result


def _poll(fn: Callable[[], Any], timeout_seconds: float, what: str, stop_on=()) -> Any:
    deadline = time.time() + timeout_seconds
    last_error: Optional[BaseException] = None
    while True:
        try:
            v = fn()
            if v:
                return v
        except stop_on:
            raise
        except Exception as e:  # noqa: BLE001 -- scheduler restarting, plan not there yet, ...
            last_error = e
        if time.time() >= deadline:
            raise TimeoutError(f"Timed out after {timeout_seconds}s waiting for {what}"
                               + (f" (last error: {last_error})" if last_error else ""))
        time.sleep(POLL_S)


def get_plan(service_name: str, plan: str, timeout_seconds: int = TIMEOUT_SECONDS,
             multiservice_name: Optional[str] = None) -> Dict[str, Any]:
    return _poll(lambda: get_plan_once(service_name, plan, multiservice_name), timeout_seconds,
                 f"plan {plan} of {service_name}")


def start_plan(service_name: str, plan: str, parameters: Optional[Dict[str, Any]] = None) -> None:
    sdk_cmd.service_request("POST", service_name, f"/v1/plans/{plan}/start",
                            json=parameters if parameters is not None else {})


def force_complete_step(service_name: str, plan: str, phase: str, step: str) -> None:
    sdk_cmd.service_request("POST", service_name, f"/v1/plans/{plan}/forceComplete?phase={phase}&step={step}")


def wait_for_completed_recovery(service_name: str, timeout_seconds: int = TIMEOUT_SECONDS,
                                multiservice_name: Optional[str] = None) -> Dict[str, Any]:
    return wait_for_completed_plan(service_name, "recovery", timeout_seconds, multiservice_name)


def wait_for_in_progress_recovery(service_name: str, timeout_seconds: int = TIMEOUT_SECONDS) -> Dict[str, Any]:
    return wait_for_in_progress_plan(service_name, "recovery", timeout_seconds)


def wait_for_kicked_off_deployment(service_name: str, timeout_seconds: int = TIMEOUT_SECONDS) -> Dict[str, Any]:
    return wait_for_kicked_off_plan(service_name, "deploy", timeout_seconds)


def wait_for_kicked_off_recovery(service_name: str, timeout_seconds: int = TIMEOUT_SECONDS) -> Dict[str, Any]:
    return wait_for_kicked_off_plan(service_name, "recovery", timeout_seconds)


def wait_for_completed_deployment(service_name: str, timeout_seconds: int = TIMEOUT_SECONDS,
                                  multiservice_name: Optional[str] = None) -> Dict[str, Any]:
    return wait_for_completed_plan(service_name, "deploy", timeout_seconds, multiservice_name)


def wait_for_completed_plan(service_name: str, plan_name: str, timeout_seconds: int = TIMEOUT_SECONDS,
                            multiservice_name: Optional[str] = None) -> Dict[str, Any]:
    return wait_for_plan_status(service_name, plan_name, "COMPLETE", timeout_seconds, multiservice_name)


def wait_for_completed_phase(service_name: str, plan_name: str, phase_name: str,
                             timeout_seconds: int = TIMEOUT_SECONDS) -> Dict[str, Any]:
    return wait_for_phase_status(service_name, plan_name, phase_name, "COMPLETE", timeout_seconds)


def wait_for_completed_step(service_name: str, plan_name: str, phase_name: str, step_name: str,
                            timeout_seconds: int = TIMEOUT_SECONDS) -> Dict[str, Any]:
    return wait_for_step_status(service_name, plan_name, phase_name, step_name, "COMPLETE", timeout_seconds)


def wait_for_kicked_off_plan(service_name: str, plan_name: str, timeout_seconds: int = TIMEOUT_SECONDS):
    return wait_for_plan_status(service_name, plan_name, ["PENDING", "STARTING", "IN_PROGRESS"], timeout_seconds)


def wait_for_in_progress_plan(service_name: str, plan_name: str, timeout_seconds: int = TIMEOUT_SECONDS):
    return wait_for_plan_status(service_name, plan_name, "IN_PROGRESS", timeout_seconds)


def wait_for_starting_plan(service_name: str, plan_name: str, timeout_seconds: int = TIMEOUT_SECONDS):
    return wait_for_plan_status(service_name, plan_name, "STARTING", timeout_seconds)


def wait_for_plan_status(service_name: str, plan_name: str, status: Union[List[str], str],
                         timeout_seconds: int = TIMEOUT_SECONDS,
                         multiservice_name: Optional[str] = None) -> Dict[str, Any]:
    """Waits for the plan to reach one of ``status``; aborts when more than
    ``MAX_NEW_TASK_FAILURES`` tasks of the service fail meanwhile (the service is crash-looping)."""
    statuses = [status] if isinstance(status, str) else list(status)
    initial_failures = sdk_tasks.get_failed_task_count(service_name)

    def fn():
        failures = sdk_tasks.get_failed_task_count(service_name)
        if failures - initial_failures > MAX_NEW_TASK_FAILURES:
            raise TaskFailuresExceededException(
                f"Service not recoverable: {service_name} ({failures - initial_failures} new task failures "
                f"while waiting for {plan_name} to reach {statuses})")
        plan = get_plan_once(service_name, plan_name, multiservice_name)
        return plan if plan and plan["status"] in statuses else False
    return _poll(fn, timeout_seconds, f"{plan_name} plan of {service_name} to reach {statuses}",
                 stop_on=(TaskFailuresExceededException,))


def wait_for_phase_status(service_name: str, plan_name: str, phase_name: str, status: str,
                          timeout_seconds: int = TIMEOUT_SECONDS) -> Dict[str, Any]:
    def fn():
        plan = get_plan_once(service_name, plan_name)
        phase = get_phase(plan, phase_name)
        return plan if phase and phase["status"] == status else False
    return _poll(fn, timeout_seconds, f"phase {plan_name}.{phase_name} of {service_name} to reach {status}")


def wait_for_step_status(service_name: str, plan_name: str, phase_name: str, step_name: str, status: str,
                         timeout_seconds: int = TIMEOUT_SECONDS) -> Dict[str, Any]:
    def fn():
        plan = get_plan_once(service_name, plan_name)
        step = get_step(get_phase(plan, phase_name), step_name)
        return plan if step and step["status"] == status else False
    return _poll(fn, timeout_seconds,
                 f"step {plan_name}.{phase_name}.{step_name} of {service_name} to reach {status}")


def recovery_plan_is_empty(service_name: str) -> bool:
    plan = get_recovery_plan(service_name)
    return len(plan["phases"]) == 0 and len(plan["errors"]) == 0 and plan["status"] == "COMPLETE"


def get_child(parent: Optional[Dict[str, Any]], children_field: str, name: str) -> Any:
    if parent is None:
        return None
    for child in parent.get(children_field, []):
        if child["name"] == name:
            return child
    return None


def get_phase(plan: Dict[str, Any], name: str) -> Any:
    return get_child(plan, "phases", name)


def get_step(phase: Dict[str, Any], name: str) -> Any:
    return get_child(phase, "steps", name)


def get_all_step_names(plan: Dict[str, Any]) -> List[str]:
    return [step["name"] for phase in plan["phases"] for step in phase["steps"]]


def plan_string(plan_name: str, plan: Dict[str, Any]) -> str:
    """Tree rendering like ``dcos <svc> plan status <plan>``."""
    if not plan:
        return f"{plan_name}=NULL!"
    lines = [f"{plan_name} ({plan.get('strategy', '?')} strategy) ({plan.get('status', '?')})"]
    phases = plan.get("phases", [])
    for i, ph in enumerate(phases):
        last = i + 1 == len(phases)
        lines.append(f"{'└─' if last else '├─'} {ph['name']} ({ph.get('strategy', '?')} strategy) ({ph['status']})")
        steps = ph.get("steps", [])
        for k, st in enumerate(steps):
            lines.append(f"{'   ' if last else '│  '}{'└─' if k + 1 == len(steps) else '├─'} "
                         f"{st['name']} ({st['status']})")
    if plan.get("errors"):
        lines.append("errors: " + ", ".join(plan["errors"]))
    return "\n".join(lines)
