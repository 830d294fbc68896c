"""Debug trackers served under ``/v1/debug``.

Reference: sdk/.../debug/{PlansTracker,TaskStatusesTracker,TaskReservationsTracker}.java. JSON
field names follow the reference's Jackson bean names (``schedulerState``, ``activePlans``,
``serviceTopology``, ``totalSteps``, ``taskStatus`` ...).
"""
from __future__ import annotations

import sys
import threading
import traceback
from typing import List, Optional

from dcos_commons_amd.offer import constants
from dcos_commons_amd.offer.task_utils import get_task_instance_name
from dcos_commons_amd.state import state_store_utils


def _eq(a: str, b: Optional[str]) -> bool:
    return b is None or a.lower() == b.lower()


class PlansTracker:
    def __init__(self, plan_coordinator, state_store):
        self.coordinator = plan_coordinator
        self.state_store = state_store

    def _validate(self, plan, phase, step) -> Optional[str]:
        if step is not None and (plan is None or phase is None):
            return "Step specified without parent Phase and Plan values."
        if phase is not None and plan is None:
            return "Phase specified without parent Plan."
        pms = []
        if plan is not None:
            pms = [pm for pm in self.coordinator.get_plan_managers() if pm.get_plan().get_name().lower() == plan.lower()]
            if len(pms) != 1:
                return "Supplied plan not found in list of all available plans!"
        phases = []
        if phase is not None:
            phases = [p for p in pms[0].get_plan().get_children() if p.get_name().lower() == phase.lower()]
            if len(phases) != 1:
                return "Supplied phase not found in set of possible phases with supplied plan!"
        if step is not None:
            if len([s for s in phases[0].get_children() if s.get_name().lower() == step.lower()]) != 1:
                return "Supplied step not found in set of possible steps with supplied plan and phase!"
        return None

    def get_json(self, plan=None, phase=None, step=None) -> dict:
        if plan is not None or phase is not None or step is not None:
            err = self._validate(plan, phase, step)
            if err:
                return {"invalid-input": err}
        topology, plans, active, by_name = [], [], [], {}
        for pm in self.coordinator.get_plan_managers():
            p = pm.get_plan()
            by_name[p.get_name()] = p
            if p.is_running():
                active.append(p.get_name())
            topology.append({"name": p.get_name(), "type": "plan", "children": [
                {"name": ph.get_name(), "type": "phase", "children": [
                    {"name": s.get_name(), "type": "step", "children": None} for s in ph.get_children()]}
                for ph in p.get_children()]})
            if not _eq(p.get_name(), plan):
                continue
            phases = []
            for ph in p.get_children():
                if not _eq(ph.get_name(), phase):
                    continue
                phases.append({"name": ph.get_name(), "status": str(ph.get_status()),
                               "strategy": ph.get_strategy().get_name(),
                               "steps": [{"name": s.get_name(), "status": str(s.get_status()),
                                          "errors": list(s.get_errors())}
                                         for s in ph.get_children() if _eq(s.get_name(), step)]})
            steps = [s for ph in p.get_children() for s in ph.get_children()]
            plans.append({"name": p.get_name(), "status": str(p.get_status()), "strategy": p.get_strategy().get_name(),
                          "phases": phases, "totalSteps": len(steps),
                          "completedSteps": len([s for s in steps if s.is_complete()])})
        state = "RUNNING"
        deploy = by_name.get(constants.DEPLOY_PLAN_NAME)
        if deploy is not None and deploy.is_running():
            state = "DEPLOYING"
        if state_store_utils.get_deployment_was_completed(self.state_store) or \
                (deploy is not None and deploy.is_complete()):
            state = "DEPLOYED"
        rec = by_name.get(constants.RECOVERY_PLAN_NAME)
        if rec is not None and rec.is_running():
            state = "RECOVERING"
        dec = by_name.get(constants.DECOMMISSION_PLAN_NAME)
        if dec is not None and dec.is_running():
            state = "DECOMMISSIONING"
        return {"schedulerState": state, "activePlans": active, "plans": plans, "serviceTopology": topology}


class TaskStatusesTracker:
    def __init__(self, plan_coordinator, state_store):
        self.coordinator = plan_coordinator
        self.state_store = state_store

    def get_json(self, plan=None, phase=None, step=None) -> List[dict]:
        out = []
        for pm in self.coordinator.get_plan_managers():
            p = pm.get_plan()
            if not _eq(p.get_name(), plan):
                continue
            phases = []
            for ph in p.get_children():
                if not _eq(ph.get_name(), phase):
                    continue
                steps = []
                for s in ph.get_children():
                    if not _eq(s.get_name(), step):
                        continue
                    req = s.get_pod_instance_requirement()
                    if req is None:
                        continue
                    pi = req.pod_instance
                    spec = next((t for t in pi.pod.tasks if t.name in s.get_name()), None)
                    if spec is None:
                        continue
                    name = get_task_instance_name(pi, spec.name)
                    entry = {"name": name, "taskStatus": "TASK_UNKNOWN", "taskId": ""}
                    st = self.state_store.fetch_status(name)
                    if st is not None:
                        from dcos_commons_amd.mesos import protos as P

                        entry["taskId"] = st.task_id.value
                        entry["taskStatus"] = P.TaskState.Name(st.state)
                    steps.append({"name": s.get_name(), "taskStatus": [entry]})
                phases.append({"name": ph.get_name(), "steps": steps})
            out.append({"name": p.get_name(), "phases": phases})
        return out


class TaskReservationsTracker:
    def __init__(self, state_store):
        self.state_store = state_store

    def get_json(self, plan=None, phase=None, step=None) -> dict:
        from dcos_commons_amd.scheduler.uninstall import get_resource_ids_by_agent_host

        return {k: sorted(v) for k, v in get_resource_ids_by_agent_host(self.state_store).items()}


def thread_dump() -> str:
    """``/v1/debug/threads`` (reference uses the JMX ThreadMXBean dump)."""
    frames = sys._current_frames()
    lines = []
    for t in threading.enumerate():
        lines.append(f'"{t.name}" daemon={t.daemon} ident={t.ident}')
        f = frames.get(t.ident)
        if f is not None:
            lines.extend("    " + l.rstrip() for l in traceback.format_stack(f))
        lines.append("")
    return "\n".join(lines)
