"""Hook that rewrites plans at scheduler build time (reference: scheduler/plan/PlanCustomizer.java:6).

``SchedulerBuilder.set_plan_customizer`` installs one; ``AbstractScheduler.customize_plans`` passes
every non-recovery plan through ``update_plan`` and ``UninstallScheduler`` passes its plan through
``update_uninstall_plan``. Both default to returning the plan unchanged.
"""
from __future__ import annotations


class PlanCustomizer:
    def update_plan(self, plan):
        return plan

    def update_uninstall_plan(self, plan):
        return plan
