"""Run one job per item on its own thread and collect failures (reference:
frameworks/helloworld/tests/scale/threading_utils.py)."""
from __future__ import annotations

import logging
import threading
import time
from typing import Any, Callable, Iterable, List, Optional

LOG = logging.getLogger(__name__)


class ResultThread(threading.Thread):
    """A thread that remembers whether its target raised, and what it returned."""

    def __init__(self, target: Callable[..., Any], name: str, args=(), kwargs=None):
        super().__init__(name=name, daemon=True)
        self._target_fn, self._args, self._kwargs = target, args, dict(kwargs or {})
        self.result: Any = None
        self.error: Optional[BaseException] = None
        self.duration_s: Optional[float] = None

    def run(self) -> None:
        start = time.time()
        try:
            self.result = self._target_fn(*self._args, **self._kwargs)
        except BaseException as e:  # noqa: BLE001 -- reported by wait_and_get_failures
            LOG.exception("%s failed", self.name)
            self.error = e
        finally:
            self.duration_s = time.time() - start


def spawn_threads(names: Iterable[str], target: Callable[..., Any], daemon: bool = True,
                  **kwargs: Any) -> List[ResultThread]:
    """Starts ``target(name, **kwargs)`` on one thread per name."""
    threads = []
    for name in names:
        t = ResultThread(target, name=name, args=(name,), kwargs=kwargs)
        t.daemon = daemon
        t.start()
        threads.append(t)
    return threads


def wait_and_get_failures(threads: List[ResultThread], timeout: float = 600.0) -> List[ResultThread]:
    """Joins every thread within ``timeout`` overall; returns those that raised or did not finish."""
    deadline = time.time() + timeout
    for t in threads:
        t.join(max(0.0, deadline - time.time()))
    failed = [t for t in threads if t.is_alive() or t.error is not None]
    for t in failed:
        LOG.error("%s: %s", t.name, "timed out" if t.is_alive() else repr(t.error))
    return failed
