"""Diagnostics on test failure (reference: testing/sdk_diag.py).

``dump_service`` writes, for one service, every plan (rendered trees and JSON), the scheduler's
state views, the scheduler log tail and each task's status history and sandbox ``stdout``/``stderr``
into ``<artifact dir>/<service>/``. ``handle_test_report`` is the pytest hook helper.
"""
from __future__ import annotations

import json
import logging
import os
from typing import List, Optional

LOG = logging.getLogger(__name__)


def _cluster():
    from dcos_commons_amd.testing.cluster import current

    return current()


def dump_service(service_name: str, out_dir: str) -> str:
    from dcos_commons_amd.testing.sdk import sdk_cmd, sdk_plan

    c = _cluster()
    d = os.path.join(out_dir, service_name.strip("/").replace("/", "_"))
    os.makedirs(d, exist_ok=True)

    def write(name: str, text: str) -> None:
        with open(os.path.join(d, name), "w", encoding="utf-8") as f:
            f.write(text)
    try:
        for plan in sdk_plan.list_plans(service_name, timeout_seconds=5):
            p = sdk_plan.get_plan_once(service_name, plan)
            write(f"plan-{plan}.txt", sdk_plan.plan_string(plan, p) + "\n")
            write(f"plan-{plan}.json", json.dumps(p, indent=2))
        for path in ("/v1/state/properties", "/v1/configurations/target", "/v1/pod/status"):
            r = sdk_cmd.service_request("GET", service_name, path, retry=False, raise_on_error=False)
            write(path.strip("/").replace("/", "-") + ".json", r.text)
    except Exception as e:  # noqa: BLE001 -- best effort
        write("scheduler-unreachable.txt", f"{e}\n")
    try:
        write("scheduler-log-tail.txt", c.marathon.log_tail(service_name, 200))
    except KeyError:
        pass
    from dcos_commons_amd.mesos import protos as P

    for t in c.tasks(service_name, include_terminal=True):
        lines = [f"{P.TaskState.Name(s.state)} {s.message}" for s in t.statuses]
        write(f"task-{t.name}-{t.id[-8:]}-statuses.txt", "\n".join(lines) + "\n")
        if c.executor == "process":
            sandbox = c.behavior.sandbox_of(t.id)
            for stream in ("stdout", "stderr"):
                try:
                    with open(os.path.join(sandbox, stream), "r", encoding="utf-8", errors="replace") as f:
                        write(f"task-{t.name}-{t.id[-8:]}-{stream}.txt", f.read()[-20000:])
                except (OSError, TypeError):
                    pass
    return d


def handle_test_report(item, report, out_dir: Optional[str] = None, services: Optional[List[str]] = None) -> None:
    """Call from ``pytest_runtest_makereport``: on a failed test phase dump every installed
    service (or ``services``) under ``out_dir`` (default ``gpurun_out/diag`` or ``$SDK_DIAG_DIR``)."""
    if report.passed or report.skipped:
        return
    from dcos_commons_amd.testing import cluster

    if cluster.cluster._current is None:
        return
    out_dir = out_dir or os.environ.get("SDK_DIAG_DIR") or os.path.join("gpurun_out", "diag", item.name)
    from dcos_commons_amd.testing.sdk import sdk_install

    for svc in services or sdk_install.get_installed_service_names():
        try:
            LOG.info("Diagnostics for %s written to %s", svc, dump_service(svc, out_dir))
        except Exception:  # noqa: BLE001
            LOG.exception("diagnostics for %s failed", svc)
