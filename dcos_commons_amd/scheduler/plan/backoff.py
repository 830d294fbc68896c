"""Task launch backoff (opt-in via ``ENABLE_BACKOFF``).

Reference: sdk/.../scheduler/plan/backoff/{Backoff,ExponentialBackoff,DisabledBackoff}.java:
factor 1.15, initial 60 s, max 300 s. A process-wide singleton, as in the reference.
"""
from __future__ import annotations

import os
import threading
import time
from typing import Callable, Dict, Optional

from dcos_commons_amd.offer import common_id_utils


class Backoff:
    def add_delay(self, task) -> None:
        raise NotImplementedError

    def get_delay(self, task_instance_name: str) -> Optional[float]:
        """Remaining delay in seconds, or None if the task may launch now."""
        raise NotImplementedError

    def clear_delay(self, task) -> bool:
        raise NotImplementedError


def _name(task) -> Optional[str]:
    if isinstance(task, str):
        return task
    try:
        return common_id_utils.to_task_name(task)
    except Exception:  # noqa: BLE001
        return None


class DisabledBackoff(Backoff):
    def add_delay(self, task) -> None:
        pass

    def get_delay(self, task_instance_name: str) -> Optional[float]:
        return None

    def clear_delay(self, task) -> bool:
        return False


class ExponentialBackoff(Backoff):
    def __init__(self, factor: float = 1.15, initial_s: float = 60, max_s: float = 300,
                 clock: Callable[[], float] = time.monotonic):
        self.factor = factor
        self.initial = float(initial_s)
        self.max = float(max_s)
        self.clock = clock
        self._delays: Dict[str, list] = {}  # name -> [reference_ts, current_delay]
        self._lock = threading.Lock()

    def add_delay(self, task) -> None:
        name = _name(task)
        if name is None:
            return
        with self._lock:
            d = self._delays.get(name)
            if d is None:
                self._delays[name] = [self.clock(), self.initial]
            else:
                d[1] = min(d[1] * self.factor, self.max)
                d[0] = self.clock()

    def get_delay(self, task_instance_name: str) -> Optional[float]:
        with self._lock:
            d = self._delays.get(task_instance_name)
        if d is None:
            return None
        pending = d[0] + d[1] - self.clock()
        return pending if pending > 0 else None

    def clear_delay(self, task) -> bool:
        name = _name(task)
        if name is None:
            return False
        with self._lock:
            return self._delays.pop(name, None) is not None


_instance: Optional[Backoff] = None
_lock = threading.Lock()


def get_instance() -> Backoff:
    global _instance
    if _instance is None:
        with _lock:
            if _instance is None:
                env = os.environ
                if env.get("ENABLE_BACKOFF", "").lower() in ("true", "1", "yes"):
                    _instance = ExponentialBackoff(float(env.get("FRAMEWORK_BACKOFF_FACTOR", 1.15)),
                                                   float(env.get("FRAMEWORK_INITIAL_BACKOFF", 60)),
                                                   float(env.get("FRAMEWORK_MAX_LAUNCH_DELAY", 300)))
                else:
                    _instance = DisabledBackoff()
    return _instance


def set_instance(b: Optional[Backoff]) -> None:
    """Override the singleton (tests; SchedulerBuilder with an explicit config)."""
    global _instance
    with _lock:
        _instance = b
