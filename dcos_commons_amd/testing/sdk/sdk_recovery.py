"""Permanent-recovery check (reference: testing/sdk_recovery.py).

``check_permanent_recovery`` replaces ``pod_name`` and verifies that exactly the tasks of that pod
(plus ``pods_with_updated_tasks``, e.g. the rolling restart a Cassandra seed replacement causes)
were relaunched and every other pod kept its tasks.
"""
from __future__ import annotations

import json
import logging
from typing import List, Optional

from dcos_commons_amd.testing.sdk import sdk_cmd, sdk_plan, sdk_tasks

LOG = logging.getLogger(__name__)


def check_permanent_recovery(package_name: str, service_name: str, pod_name: str, recovery_timeout_s: int,
                             pods_with_updated_tasks: Optional[List[str]] = None) -> None:
    sdk_plan.wait_for_completed_deployment(service_name)
    sdk_plan.wait_for_completed_recovery(service_name)
    rc, stdout, _ = sdk_cmd.svc_cli(package_name, service_name, "pod list")
    assert rc == 0, "Pod list failed"
    pods = set(json.loads(stdout))
    to_update = set((pods_with_updated_tasks or []) + [pod_name])
    replaced = {pod: set(sdk_tasks.get_task_ids(service_name, f"{pod}-")) for pod in to_update}
    others = {pod: set(sdk_tasks.get_task_ids(service_name, f"{pod}-")) for pod in pods - to_update}
    LOG.info("Replacing %s: tasks to replace %s, tasks to keep %s", pod_name, replaced, others)
    sdk_cmd.svc_cli(package_name, service_name, f"pod replace {pod_name}", check=True)
    # (no wait for a kicked-off recovery: on the local cluster it can start and complete between
    # two polls; the relaunched tasks are the evidence)
    for pod, ids in replaced.items():
        sdk_tasks.check_tasks_updated(service_name, f"{pod}-", ids, recovery_timeout_s)
    sdk_plan.wait_for_completed_recovery(service_name, recovery_timeout_s)
    for pod, ids in others.items():
        sdk_tasks.check_tasks_not_updated(service_name, f"{pod}-", ids)
