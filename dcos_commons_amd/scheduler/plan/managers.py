"""Plan managers and the cross-plan coordinator.

Reference: sdk/.../scheduler/plan/{DefaultPlanManager,DecommissionPlanManager,
DefaultPlanCoordinator,PlanCustomizer}.java. The coordinator pre-computes *dirty assets*
(pod instances being worked on) so two plans never operate on the same pod at once.
"""
from __future__ import annotations

import logging
import threading
from typing import Collection, List, Optional, Set

from .elements import get_dirty_assets
from .pod_instance_requirement import PodInstanceRequirement

LOGGER = logging.getLogger(__name__)


class PlanManager:
    def get_plan(self):
        raise NotImplementedError

    def set_plan(self, plan) -> None:
        raise NotImplementedError

    def get_candidates(self, dirty_assets) -> list:
        raise NotImplementedError

    def update(self, status) -> None:
        raise NotImplementedError

    def get_dirty_assets(self) -> Set[PodInstanceRequirement]:
        raise NotImplementedError


class DefaultPlanManager(PlanManager):
    def __init__(self, plan):
        self._plan = plan
        self._lock = threading.Lock()

    @staticmethod
    def create_proceeding(plan) -> "DefaultPlanManager":
        return DefaultPlanManager(plan)

    @staticmethod
    def create_interrupted(plan) -> "DefaultPlanManager":
        plan.interrupt()
        return DefaultPlanManager(plan)

    def get_plan(self):
        with self._lock:
            return self._plan

    def set_plan(self, plan) -> None:
        with self._lock:
            self._plan = plan

    def get_candidates(self, dirty_assets):
        return self.get_plan().get_candidates(dirty_assets)

    def update(self, status) -> None:
        self.get_plan().update(status)

    def get_dirty_assets(self):
        return get_dirty_assets(self.get_plan())


class DecommissionPlanManager(DefaultPlanManager):
    def __init__(self, plan, resource_steps, tasks_to_decommission):
        super().__init__(plan)
        self.resource_steps = list(resource_steps)
        self.tasks_to_decommission = list(tasks_to_decommission)


class PlanCustomizer:
    """Hook to rewrite plans (including the uninstall plan) at build time."""

    def update_plan(self, plan):
        return plan

    def update_uninstall_plan(self, plan):
        return plan


class DefaultPlanCoordinator:
    def __init__(self, plan_managers: Collection[PlanManager], namespace: Optional[str] = None):
        if not plan_managers:
            raise ValueError("At least one plan manager is required")
        self.plan_managers: List[PlanManager] = list(plan_managers)
        self.logger = logging.getLogger(__name__ + (f"({namespace})" if namespace else ""))

    def get_plan_managers(self) -> List[PlanManager]:
        return self.plan_managers

    @staticmethod
    def _relevant(pm: PlanManager, dirty: Set[PodInstanceRequirement]) -> List[PodInstanceRequirement]:
        running_reqs = []
        for phase in pm.get_plan().get_children():
            for step in phase.get_children():
                if step.is_running():
                    req = step.get_pod_instance_requirement()
                    if req is not None:
                        running_reqs.append(req)
        return [d for d in dirty if not any(r.conflicts_with(d) for r in running_reqs)]

    def get_candidates(self) -> list:
        dirtied: Set[PodInstanceRequirement] = set()
        for pm in self.plan_managers:
            if not pm.get_plan().is_interrupted():
                dirtied |= pm.get_dirty_assets()
        candidates = []
        for pm in self.plan_managers:
            plan = pm.get_plan()
            if plan.is_interrupted():
                continue
            try:
                steps = list(pm.get_candidates(self._relevant(pm, dirtied)))
                candidates.extend(steps)
                for s in steps:
                    req = s.get_pod_instance_requirement()
                    if req is not None:
                        dirtied.add(req)
            except Exception:  # noqa: BLE001
                self.logger.exception("Error with %s plan manager", plan.get_name())
        return candidates
