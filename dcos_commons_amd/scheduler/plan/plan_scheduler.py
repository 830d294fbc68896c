"""Matches candidate steps against offers.

Reference: sdk/.../scheduler/plan/PlanScheduler.java:27-166. For each candidate step, in order:
``step.start()``, kill the live tasks sharing the resource sets about to be relaunched, run the
``OfferEvaluator``, hand the recommendations to the step, and remove consumed offers before the
next step (greedy).

Difference from the reference: the reference evaluates every step of a cycle against the task set
stored before the cycle, so placement rules that count tasks (``MAX_PER`` zone/region/attribute,
``GROUP_BY``, task-type avoid/colocate) cannot see pods matched earlier in the same cycle and a
parallel phase can over-place. Here each matched step's TaskInfos join the snapshot before the next
step is evaluated (with or without launch streaming).
"""
from __future__ import annotations

import logging
from typing import Optional

from dcos_commons_amd.framework import task_killer
from dcos_commons_amd.offer.recommendations import StoreTaskInfoRecommendation
from dcos_commons_amd.offer.task_utils import is_terminal
from dcos_commons_amd.utils.logging_utils import get_logger

LOGGER = logging.getLogger(__name__)


class PlanScheduler:
    def __init__(self, offer_evaluator, state_store, namespace: Optional[str] = None):
        self.offer_evaluator = offer_evaluator
        self.state_store = state_store
        self.logger = get_logger(__name__, namespace)

    def resource_offers(self, offers, steps, on_step=None) -> list:
        """``on_step(recs)``, when given, receives each step's recommendations as soon as that
        step is matched (launch streaming); its return value replaces them in the result."""
        all_recs = []
        available = list(offers)
        # Read the stored task set once per cycle; the TaskInfos of each matched step are merged
        # into it, so later steps see the pods placed earlier in this cycle.
        all_tasks = {t.name: t for t in self.state_store.fetch_tasks_shared()} if steps else {}
        for step in steps:
            recs = self._step_offers(available, step, all_tasks)
            if recs:
                used = {r.offer_id.value for r in recs}
                if on_step is not None:
                    recs = on_step(recs)
                for r in recs:
                    if isinstance(r, StoreTaskInfoRecommendation) and r.task_info.task_id.value:
                        all_tasks[r.task_info.name] = r.state_store_task_info()
                all_recs.extend(recs)
                available = [o for o in available if o.id.value not in used]
        return all_recs

    def _step_offers(self, offers, step, all_tasks) -> list:
        if not (step.is_pending() or step.is_prepared()):
            return []
        step.start()
        req = step.get_pod_instance_requirement()
        if req is None:
            step.update_offer_status([])
            return []
        self._kill_tasks(req)
        try:
            recs = self.offer_evaluator.evaluate(req, offers, all_tasks)
        except Exception:  # noqa: BLE001
            self.logger.exception("Failed generate OfferRecommendations.")
            return []
        if not recs:
            self.logger.info("Unable to find any offers which fulfill requirement provided by step %s",
                             step.get_name())
            step.update_offer_status([])
            return []
        step.update_offer_status([r for r in recs if r.get_operation() is not None])
        return recs

    def _kill_tasks(self, req) -> None:
        """Kills the live tasks on the resource sets ``req`` relaunches (as relaunch kills: their
        end asks the master to offer the freed reservations again)."""
        pi = req.pod_instance
        sets = {t.resource_set.id for t in pi.pod.tasks if t.name in req.tasks_to_launch}
        for t in pi.pod.tasks:
            if t.resource_set.id not in sets:
                continue
            name = f"{pi.name}-{t.name}"
            info = self.state_store.fetch_task_shared(name)
            if info is None or not info.task_id.value:
                continue  # never launched (a footprint placeholder): nothing runs to kill
            status = self.state_store.fetch_status(name)
            if status is None or not is_terminal(status):
                task_killer.kill_task(info.task_id, relaunch=True)
