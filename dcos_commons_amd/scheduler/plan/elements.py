"""Plan / Phase / Step composite tree and the aggregate-status rules.

Reference: sdk/.../scheduler/plan/{Element,ParentElement,Plan,Phase,Step,AbstractStep,
DefaultPhase,DefaultPlan,PlanUtils}.java. A parent's status is *derived* from its children
via :func:`get_aggregate_status` (PlanUtils.java:105-170, rule order is significant).
"""
from __future__ import annotations

import logging
import threading
import uuid
from typing import Dict, Iterable, List, Optional, Set

from dcos_commons_amd.offer import constants
from dcos_commons_amd.scheduler.plan import backoff as backoff_mod
from dcos_commons_amd.utils import ids

from .pod_instance_requirement import PodInstanceRequirement
from .status import Status

LOGGER = logging.getLogger(__name__)

# ---------------------------------------------------------------------------------------
# Status generation: bumped (under a lock, so it only ever grows) after every change that can
# alter an aggregate status -- a step's status, its interrupted flag or its errors, a strategy's
# interrupted flag. A phase/plan caches its aggregate together with the generation it read
# *before* computing it, so a change that lands during the computation invalidates the entry.
# Plan status is read far more often than it changes: every offer cycle's candidate walk, every
# status update, every /v1/plans request and the plan-status metric.

_status_gen = 0
_status_gen_lock = threading.Lock()


def bump_status_generation() -> None:
    global _status_gen
    with _status_gen_lock:
        _status_gen += 1


def status_generation() -> int:
    return _status_gen


# ---------------------------------------------------------------------------------------
# PlanUtils


def asset_conflicts(asset: PodInstanceRequirement, dirty_assets: Iterable[PodInstanceRequirement]) -> bool:
    return any(asset.conflicts_with(d) for d in dirty_assets)


def is_eligible(element: "Element", dirty_assets) -> bool:
    # one status read: a parent's status is a full aggregate over its children
    if element.get_status() in (Status.COMPLETE, Status.ERROR):
        return False
    if element.is_interrupted():
        return False
    if isinstance(element, Step):
        req = element.get_pod_instance_requirement()
        return req is None or not asset_conflicts(req, dirty_assets)
    return True


def get_dirty_assets(plan: Optional["Plan"]) -> Set[PodInstanceRequirement]:
    if plan is None:
        return set()
    out = set()
    for phase in plan.get_children():
        for step in phase.get_children():
            st = step.get_status()
            if st in (Status.PREPARED, Status.STARTING):
                req = step.get_pod_instance_requirement()
                if req is not None:
                    out.add(req)
    return out


def get_launchable_tasks(plans: Iterable["Plan"]) -> Set[str]:
    out = set()
    for plan in plans:
        for phase in plan.get_children():
            for step in phase.get_children():
                req = step.get_pod_instance_requirement()
                if req is None:
                    continue
                for t in req.tasks_to_launch:
                    out.add(f"{req.pod_instance.name}-{t}")
    return out


def _all(status: Status, statuses) -> bool:
    return all(s == status for s in statuses)


def _any(status: Status, statuses) -> bool:
    return any(s == status for s in statuses)


def get_aggregate_status(parent_name: str, child_statuses: List[Status], candidate_statuses: List[Status],
                         errors: List[str], is_interrupted: bool, log_unexpected: bool = True) -> Status:
    if errors or _any(Status.ERROR, child_statuses):
        return Status.ERROR
    if _all(Status.COMPLETE, child_statuses):
        return Status.COMPLETE
    if is_interrupted:
        return Status.WAITING
    if _all(Status.DELAYED, candidate_statuses) and _all(Status.DELAYED, child_statuses):
        return Status.DELAYED
    if _any(Status.PREPARED, child_statuses):
        return Status.IN_PROGRESS
    if _any(Status.WAITING, candidate_statuses):
        return Status.WAITING
    if _any(Status.IN_PROGRESS, candidate_statuses):
        return Status.IN_PROGRESS
    if _any(Status.COMPLETE, child_statuses) and _any(Status.PENDING, candidate_statuses):
        return Status.IN_PROGRESS
    if _any(Status.COMPLETE, child_statuses) and _any(Status.STARTING, candidate_statuses):
        return Status.IN_PROGRESS
    if _any(Status.COMPLETE, child_statuses) and _any(Status.STARTED, candidate_statuses):
        return Status.IN_PROGRESS
    if _any(Status.PENDING, candidate_statuses):
        return Status.PENDING
    if _any(Status.WAITING, child_statuses):
        return Status.WAITING
    if _any(Status.STARTING, candidate_statuses):
        return Status.STARTING
    if _any(Status.STARTED, candidate_statuses):
        return Status.STARTED
    if log_unexpected:
        LOGGER.warning("(%s status=ERROR) Unexpected state. Children: %s Candidates: %s",
                       parent_name, child_statuses, candidate_statuses)
    return Status.ERROR


# ---------------------------------------------------------------------------------------
# Element


class Element:
    def get_id(self) -> uuid.UUID:
        raise NotImplementedError

    def get_name(self) -> str:
        raise NotImplementedError

    def get_status(self) -> Status:
        raise NotImplementedError

    def update(self, status) -> None:
        raise NotImplementedError

    def restart(self) -> None:
        raise NotImplementedError

    def force_complete(self) -> None:
        raise NotImplementedError

    def get_errors(self) -> List[str]:
        raise NotImplementedError

    def interrupt(self) -> None:
        raise NotImplementedError

    def proceed(self) -> None:
        raise NotImplementedError

    def is_interrupted(self) -> bool:
        raise NotImplementedError

    def update_parameters(self, parameters: Dict[str, str]) -> None:
        pass

    # convenience predicates
    def has_errors(self) -> bool:
        return self.get_status() == Status.ERROR

    def is_pending(self) -> bool:
        return self.get_status() == Status.PENDING

    def is_prepared(self) -> bool:
        return self.get_status() == Status.PREPARED

    def is_starting(self) -> bool:
        return self.get_status() == Status.STARTING

    def is_started(self) -> bool:
        return self.get_status() == Status.STARTED

    def is_complete(self) -> bool:
        return self.get_status() == Status.COMPLETE

    def is_delayed(self) -> bool:
        return self.get_status() == Status.DELAYED

    def is_running(self) -> bool:
        return self.get_status().is_running()

    @property
    def name(self) -> str:
        return self.get_name()

    def get_message(self) -> str:
        return f"{type(self).__name__}: {self.get_name()} [{self.get_id()}] with status: {self.get_status()}"


class ParentElement(Element):
    def get_children(self) -> List[Element]:
        raise NotImplementedError

    def get_strategy(self):
        raise NotImplementedError

    def interrupt(self) -> None:
        self.get_strategy().interrupt()

    def proceed(self) -> None:
        self.get_strategy().proceed()

    def is_interrupted(self) -> bool:
        return self.get_strategy().is_interrupted()

    def update_parameters(self, parameters: Dict[str, str]) -> None:
        for c in self.get_children():
            c.update_parameters(parameters)

    def update(self, status) -> None:
        for c in self.get_children():
            c.update(status)

    def restart(self) -> None:
        for c in self.get_children():
            c.restart()

    def force_complete(self) -> None:
        for c in self.get_children():
            c.force_complete()

    def _child_errors(self, parent_errors: List[str]) -> List[str]:
        out = list(parent_errors)
        for c in self.get_children():
            out.extend(c.get_errors())
        return out

    # Children change status on other threads (status updates, the offer loop) while the
    # aggregate is computed: the child statuses, the strategy's candidates and the candidates'
    # statuses are three separate reads, and a step completing between them yields a combination
    # no rule covers (e.g. children [STARTED], candidates [COMPLETE]). Such a torn read is retried
    # instead of being reported as ERROR; a persistent one still is.
    _TORN_READ_RETRIES = 3

    # (generation, status) of the last aggregate, when it may be reused (see _status_gen)
    _status_cache = None
    # whether the last computed aggregate was cacheable (read by the parent plan)
    _last_cacheable = False

    def _cacheable(self, children, child_statuses) -> bool:
        """An aggregate may be reused until the generation moves when everything it read reports
        its changes through the generation: AbstractStep children that are not DELAYED (a DELAYED
        step turns PENDING by itself once its backoff expires), cacheable child phases, and a
        deterministic strategy (RandomStrategy picks a different candidate on every call)."""
        if not getattr(self.get_strategy(), "deterministic", False):
            return False
        for c, s in zip(children, child_statuses):
            if isinstance(c, AbstractStep):
                if s is Status.DELAYED or c._status is Status.DELAYED:
                    return False
            elif not (isinstance(c, ParentElement) and c._last_cacheable):
                return False
        return True

    def get_status(self) -> Status:
        gen = _status_gen
        cached = self._status_cache
        if cached is not None and cached[0] == gen:
            return cached[1]
        children = self.get_children()
        errors = self.get_errors()
        for attempt in range(self._TORN_READ_RETRIES + 1):
            child_statuses = [c.get_status() for c in children]
            candidate_statuses = [c.get_status() for c in self.get_strategy().get_candidates(children, [])]
            last = attempt == self._TORN_READ_RETRIES
            st = get_aggregate_status(self.get_name(), child_statuses, candidate_statuses, errors,
                                      self.is_interrupted(), log_unexpected=last)
            if st != Status.ERROR or errors or Status.ERROR in child_statuses or last:
                break
        cacheable = self._cacheable(children, child_statuses)
        self._last_cacheable = cacheable
        self._status_cache = (gen, st) if cacheable else None
        return st


class Step(Element):
    def start(self) -> None:
        raise NotImplementedError

    def get_pod_instance_requirement(self) -> Optional[PodInstanceRequirement]:
        raise NotImplementedError

    def update_offer_status(self, recommendations) -> None:
        raise NotImplementedError

    def get_display_status(self) -> str:
        return str(self.get_status())

    def get_message(self) -> str:
        msg = super().get_message()
        display = self.get_display_status()
        if display != str(self.get_status()):
            msg += f" (display:{display})"
        return msg


class AbstractStep(Step):
    def __init__(self, name: str, namespace: Optional[str] = None):
        self._id = ids.uuid4()
        self._name = name
        self._status = Status.PENDING
        self._interrupted = False
        self._status_lock = threading.RLock()
        self.namespace = namespace
        self.logger = logging.getLogger(type(self).__module__ + (f"({namespace})" if namespace else ""))

    def get_id(self):
        return self._id

    def get_name(self):
        return self._name

    def get_status(self) -> Status:
        # Hot path (strategies and aggregate statuses read every step, every cycle): a plain
        # attribute read is atomic, so only the states with side conditions take the lock.
        st = self._status
        if st is not Status.DELAYED and not self._interrupted:
            return st
        with self._status_lock:
            if self._interrupted and self._status in (Status.PENDING, Status.PREPARED):
                return Status.WAITING
            if self._status == Status.DELAYED:
                req = self.get_pod_instance_requirement()
                if req is not None:
                    b = backoff_mod.get_instance()
                    if all(b.get_delay(f"{req.pod_instance.name}-{t}") is None for t in req.tasks_to_launch):
                        self._set_status(Status.PENDING)
            return self._status

    def _set_status(self, new_status: Status) -> None:
        with self._status_lock:
            old = self._status
            self._status = new_status
        if old != new_status:
            bump_status_generation()
            self.logger.info("%s: changed status from: %s to: %s (interrupted=%s)", self._name, old, new_status,
                             self._interrupted)

    set_status = _set_status

    def interrupt(self) -> None:
        with self._status_lock:
            self._interrupted = True
        bump_status_generation()

    def proceed(self) -> None:
        with self._status_lock:
            self._interrupted = False
        bump_status_generation()

    def is_interrupted(self) -> bool:
        return self._interrupted        # a plain attribute read is atomic

    def restart(self) -> None:
        self.logger.warning("Restarting step: '%s [%s]'", self._name, self._id)
        req = self.get_pod_instance_requirement()
        if req is not None:
            b = backoff_mod.get_instance()
            for t in req.tasks_to_launch:
                b.clear_delay(f"{req.pod_instance.name}-{t}")
        self._set_status(Status.PENDING)

    def force_complete(self) -> None:
        self.logger.warning("Forcing completion of step: '%s [%s]'", self._name, self._id)
        self._set_status(Status.COMPLETE)

    def get_errors(self) -> List[str]:
        return []

    def start(self) -> None:
        pass

    def update(self, status) -> None:
        pass

    def update_offer_status(self, recommendations) -> None:
        pass

    def get_pod_instance_requirement(self) -> Optional[PodInstanceRequirement]:
        return None

    def __repr__(self):
        return f"{type(self).__name__}({self._name}: {self._status})"


class DefaultPhase(ParentElement):
    def __init__(self, name: str, steps: List[Step], strategy, errors: Optional[List[str]] = None):
        self._id = ids.uuid4()
        self._name = name
        self._steps = list(steps)
        self._strategy = strategy
        self._errors = list(errors or [])

    def get_id(self):
        return self._id

    def get_name(self):
        return self._name

    def get_children(self):
        return self._steps

    def get_strategy(self):
        return self._strategy

    def get_errors(self):
        return self._child_errors(self._errors)

    def __repr__(self):
        return f"DefaultPhase({self._name})"


Phase = DefaultPhase


class DefaultPlan(ParentElement):
    def __init__(self, name: str, phases: List[DefaultPhase], strategy=None, errors: Optional[List[str]] = None):
        from .strategy import SerialStrategy

        self._id = ids.uuid4()
        self._name = name
        self._phases = list(phases)
        self._strategy = strategy if strategy is not None else SerialStrategy()
        self._errors = list(errors or [])

    def get_id(self):
        return self._id

    def get_name(self):
        return self._name

    def get_children(self):
        return self._phases

    def get_strategy(self):
        return self._strategy

    def get_errors(self):
        return self._child_errors(self._errors)

    def get_candidates(self, dirty_assets) -> List[Step]:
        out: List[Step] = []
        for phase in self._strategy.get_candidates(self._phases, dirty_assets):
            for step in phase.get_strategy().get_candidates(phase.get_children(), dirty_assets):
                if not step.is_delayed():
                    out.append(step)
        return out

    def is_deploy_plan(self) -> bool:
        return self._name == constants.DEPLOY_PLAN_NAME

    def is_recovery_plan(self) -> bool:
        return self._name == constants.RECOVERY_PLAN_NAME

    def is_decommission_plan(self) -> bool:
        return self._name == constants.DECOMMISSION_PLAN_NAME

    def __str__(self):
        rows = [f"Plan: {self._name} ({self.get_status()})"]
        for phase in self._phases:
            rows.append(f"  Phase: {phase.get_name()} ({phase.get_status()})")
            for step in phase.get_children():
                rows.append(f"    Step: {step.get_name()} ({step.get_status()})")
        errs = self.get_errors()
        if errs:
            rows.append("Errors:")
            rows.extend(f"  {e}" for e in errs)
        return "\n".join(rows)


Plan = DefaultPlan
