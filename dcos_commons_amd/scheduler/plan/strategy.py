"""Plan/phase strategies: serial, parallel, random, dependency (DAG) and canary.

Reference: sdk/.../scheduler/plan/strategy/*.java. ``CanaryStrategy`` interrupts the first N
pending steps and needs N ``proceed()`` calls (default 2) before handing over to the wrapped
strategy.
"""
from __future__ import annotations

import random
import threading
from typing import Callable, Dict, Iterable, List, Optional

from .elements import bump_status_generation, is_eligible

DEFAULT_CANARY_PROCEED_COUNT = 2


class Strategy:
    # the same elements in the same states always give the same candidates (aggregate statuses
    # computed through this strategy may be cached, see elements._status_gen)
    deterministic = False

    def get_candidates(self, elements, dirty_assets) -> list:
        raise NotImplementedError

    def get_name(self) -> str:
        raise NotImplementedError

    def interrupt(self) -> None:
        raise NotImplementedError

    def proceed(self) -> None:
        raise NotImplementedError

    def is_interrupted(self) -> bool:
        raise NotImplementedError

    @property
    def name(self) -> str:
        return self.get_name()


class InterruptibleStrategy(Strategy):
    def __init__(self):
        self._interrupted = False
        self._lock = threading.Lock()

    def interrupt(self) -> None:
        with self._lock:
            self._interrupted = True
        bump_status_generation()

    def proceed(self) -> None:
        with self._lock:
            self._interrupted = False
        bump_status_generation()

    def is_interrupted(self) -> bool:
        return self._interrupted


class DependencyStrategyHelper:
    """Element -> set(parents) DAG; candidates are eligible elements whose parents completed."""

    def __init__(self, elements: Iterable = ()):
        # dict keyed by id() preserves insertion order and avoids requiring hashable elements
        self._deps: Dict[int, tuple] = {}
        for e in elements:
            self.add_element(e)

    def add_element(self, e) -> None:
        if id(e) not in self._deps:
            self._deps[id(e)] = (e, [])

    def add_dependency(self, child, parent) -> None:
        self.add_element(parent)
        self.add_element(child)
        parents = self._deps[id(child)][1]
        if all(p is not parent for p in parents):
            parents.append(parent)

    def get_candidates(self, is_interrupted: bool, dirty_assets) -> list:
        if is_interrupted:
            return []
        out = []
        for e, parents in self._deps.values():
            if is_eligible(e, dirty_assets) and all(p.is_complete() for p in parents):
                out.append(e)
        return out


class SerialStrategy(InterruptibleStrategy):
    deterministic = True

    def __init__(self):
        super().__init__()
        self._helper: Optional[DependencyStrategyHelper] = None

    def _get_helper(self, elements) -> DependencyStrategyHelper:
        if self._helper is None:
            helper = DependencyStrategyHelper(elements)
            incomplete = [e for e in elements if not e.is_complete()]
            incomplete.reverse()
            for i in range(1, len(incomplete)):
                previous = incomplete[i - 1]
                for cur in incomplete[i:]:
                    helper.add_dependency(previous, cur)
            self._helper = helper
        return self._helper

    def get_candidates(self, elements, dirty_assets):
        return self._get_helper(elements).get_candidates(self.is_interrupted(), dirty_assets)

    def get_name(self):
        return "serial"


class ParallelStrategy(InterruptibleStrategy):
    deterministic = True

    def get_candidates(self, elements, dirty_assets):
        # a dependency helper with no edges: every eligible element, in order
        if self._interrupted:
            return []
        return [e for e in elements if is_eligible(e, dirty_assets)]

    def get_name(self):
        return "parallel"


class RandomStrategy(InterruptibleStrategy):
    def get_candidates(self, elements, dirty_assets):
        cands = DependencyStrategyHelper(elements).get_candidates(self.is_interrupted(), dirty_assets)
        if not cands:
            return []
        return [random.choice(cands)]

    def get_name(self):
        return "random"


class DependencyStrategy(InterruptibleStrategy):
    deterministic = True

    def __init__(self, helper: DependencyStrategyHelper):
        super().__init__()
        self.helper = helper

    def get_candidates(self, elements, dirty_assets):
        return self.helper.get_candidates(self.is_interrupted(), dirty_assets)

    def get_name(self):
        return "dependency"


class CanaryStrategy(Strategy):
    def __init__(self, post_canary: Strategy, steps: List, required_proceeds: int = DEFAULT_CANARY_PROCEED_COUNT):
        self.required_proceeds = required_proceeds
        self.strategy = post_canary
        canary = [s for s in steps if s.is_pending() or s.is_interrupted()][:required_proceeds]
        for s in canary:
            s.interrupt()
        self.canary_steps = canary

    def _next_canary_step(self):
        for s in self.canary_steps:
            if s.is_interrupted():
                return s
        return None

    def _next_proceed_step(self):
        for s in self.canary_steps:
            if not s.is_interrupted() and not s.is_complete():
                return s
        return None

    def get_candidates(self, elements, dirty_assets):
        if self._next_canary_step() is not None:
            return [s for s in self.canary_steps if is_eligible(s, dirty_assets)]
        return self.strategy.get_candidates(elements, dirty_assets)

    def get_name(self):
        return self.strategy.get_name() + "-canary"

    @property
    def deterministic(self) -> bool:
        return getattr(self.strategy, "deterministic", False)

    def interrupt(self) -> None:
        if self._next_canary_step() is not None:
            return
        self.strategy.interrupt()

    def proceed(self) -> None:
        s = self._next_canary_step()
        if s is not None:
            s.proceed()
            return
        self.strategy.proceed()

    def is_interrupted(self) -> bool:
        if self._next_canary_step() is not None and self._next_proceed_step() is None:
            return True
        return self.strategy.is_interrupted()


# -- generators (StrategyGenerator) -------------------------------------------------------

StrategyGenerator = Callable[[List], Strategy]


def serial_generator(elements=None) -> Strategy:
    return SerialStrategy()


def parallel_generator(elements=None) -> Strategy:
    return ParallelStrategy()


def random_generator(elements=None) -> Strategy:
    return RandomStrategy()


def canary_generator(post: StrategyGenerator, required_proceeds: int = DEFAULT_CANARY_PROCEED_COUNT):
    def gen(steps):
        return CanaryStrategy(post(steps), steps, required_proceeds)
    return gen


# PlanGenerator registry (PlanGenerator.java:55-66)
PHASE_STRATEGIES = {
    "serial": serial_generator,
    "parallel": parallel_generator,
    "serial-canary": canary_generator(serial_generator),
    "canary": canary_generator(serial_generator),
    "parallel-canary": canary_generator(parallel_generator),
}
PLAN_STRATEGIES = {
    "serial": serial_generator,
    "parallel": parallel_generator,
}


def phase_strategy_generator(name: Optional[str]) -> StrategyGenerator:
    if not name:
        return serial_generator
    gen = PHASE_STRATEGIES.get(name)
    if gen is None:
        raise ValueError(f"Unsupported phase strategy '{name}', expected one of {sorted(PHASE_STRATEGIES)}")
    return gen


def plan_strategy_generator(name: Optional[str]) -> StrategyGenerator:
    if not name:
        return serial_generator
    gen = PLAN_STRATEGIES.get(name)
    if gen is None:
        raise ValueError(f"Unsupported plan strategy '{name}', expected one of {sorted(PLAN_STRATEGIES)}")
    return gen
