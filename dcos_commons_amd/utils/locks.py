"""Lock-order (deadlock) detection: the Python counterpart of the reference's
``CycleDetectingLockUtils`` (reference sdk/.../state/CycleDetectingLockUtils.java:13-46), which
wraps Guava's ``CycleDetectingLockFactory`` and exits the process with
``DEADLOCK_ENCOUNTERED`` when two locks are ever taken in inconsistent order.

Every lock produced by :func:`new_lock` / :func:`new_rw_lock` records, per thread, which locks
are held when it is acquired. Those "held-before" edges form a global graph; if acquiring lock
``B`` while holding ``A`` would close a cycle (``B`` was previously held while acquiring ``A``)
the policy callback fires. By default that is :func:`ProcessExit.exit` with code 7, unless
``DISABLE_DEADLOCK_EXIT`` is set, in which case :class:`PotentialDeadlockError` is raised.
"""
from __future__ import annotations

import itertools
import os
import threading
from typing import Callable, Dict, List, Optional, Set


class PotentialDeadlockError(RuntimeError):
    pass


_graph_lock = threading.Lock()
_edges: Dict[int, Set[int]] = {}
_names: Dict[int, str] = {}
_ids = itertools.count(1)
_held = threading.local()


def _held_stack() -> List[int]:
    st = getattr(_held, "stack", None)
    if st is None:
        st = []
        _held.stack = st
    return st


def _reachable(src: int, dst: int) -> Optional[List[int]]:
    """Return a path src -> ... -> dst in the order graph, or None."""
    stack = [(src, [src])]
    seen = {src}
    while stack:
        node, path = stack.pop()
        if node == dst:
            return path
        for nxt in _edges.get(node, ()):
            if nxt not in seen:
                seen.add(nxt)
                stack.append((nxt, path + [nxt]))
    return None


def _default_policy(message: str) -> None:
    if os.environ.get("DISABLE_DEADLOCK_EXIT", "").lower() in ("1", "true", "yes"):
        raise PotentialDeadlockError(message)
    from dcos_commons_amd.framework.process_exit import ProcessExit

    ProcessExit.exit(ProcessExit.DEADLOCK_ENCOUNTERED, PotentialDeadlockError(message))


_policy: Callable[[str], None] = _default_policy


def set_policy(policy: Optional[Callable[[str], None]]) -> None:
    """Override what happens on a detected cycle (tests use a raising policy)."""
    global _policy
    _policy = policy or _default_policy


def raising_policy(message: str) -> None:
    raise PotentialDeadlockError(message)


class _OrderTracker:
    def __init__(self, name: str, check: bool):
        self.lock_id = next(_ids)
        self.check = check
        _names[self.lock_id] = name

    def before_acquire(self) -> None:
        if not self.check:
            return
        stack = _held_stack()
        if not stack or self.lock_id in stack:
            return
        # Fast path: every held -> this edge is already known (and was cycle-checked when it was
        # added). Set membership reads are atomic under the GIL, so no graph lock is needed.
        lid = self.lock_id
        if all(lid in _edges.get(held, ()) for held in stack):
            return
        with _graph_lock:
            for held in stack:
                if self.lock_id in _edges.get(held, ()):
                    continue
                path = _reachable(self.lock_id, held)
                if path is not None:
                    names = " -> ".join(_names[i] for i in path + [self.lock_id])
                    msg = f"Lock-order cycle detected acquiring {_names[self.lock_id]}: {names}"
                    break
                _edges.setdefault(held, set()).add(self.lock_id)
            else:
                msg = None
        if msg:
            _policy(msg)

    def acquired(self) -> None:
        _held_stack().append(self.lock_id)

    def released(self) -> None:
        stack = _held_stack()
        for i in range(len(stack) - 1, -1, -1):
            if stack[i] == self.lock_id:
                del stack[i]
                break


class CycleDetectingLock:
    """Re-entrant lock with lock-order cycle detection."""

    def __init__(self, name: str, check: bool = True):
        self._lock = threading.RLock()
        self._tracker = _OrderTracker(name, check)

    def acquire(self, blocking: bool = True, timeout: float = -1) -> bool:
        self._tracker.before_acquire()
        ok = self._lock.acquire(blocking, timeout)
        if ok:
            self._tracker.acquired()
        return ok

    def release(self) -> None:
        self._tracker.released()
        self._lock.release()

    def __enter__(self):
        self.acquire()
        return self

    def __exit__(self, *exc):
        self.release()


class _RWView:
    def __init__(self, owner: "CycleDetectingRWLock", write: bool):
        self._owner = owner
        self._write = write

    def acquire(self) -> None:
        if self._write:
            self._owner.acquire_write()
        else:
            self._owner.acquire_read()

    def release(self) -> None:
        if self._write:
            self._owner.release_write()
        else:
            self._owner.release_read()

    def __enter__(self):
        self.acquire()
        return self

    def __exit__(self, *exc):
        self.release()


class CycleDetectingRWLock:
    """Readers-writer lock (writer re-entrant, writer may take read) with cycle detection."""

    def __init__(self, name: str, check: bool = True):
        self._cond = threading.Condition(threading.Lock())
        self._readers: Dict[int, int] = {}
        self._writer: Optional[int] = None
        self._write_depth = 0
        self._tracker = _OrderTracker(name, check)
        self._waiting = 0  # threads blocked in _cond.wait(): release only notifies when > 0
        self.read_lock = _RWView(self, False)
        self.write_lock = _RWView(self, True)

    def acquire_read(self) -> None:
        self._tracker.before_acquire()
        me = threading.get_ident()
        with self._cond:
            while self._writer is not None and self._writer != me:
                self._waiting += 1
                try:
                    self._cond.wait()
                finally:
                    self._waiting -= 1
            self._readers[me] = self._readers.get(me, 0) + 1
        self._tracker.acquired()

    def release_read(self) -> None:
        me = threading.get_ident()
        self._tracker.released()
        with self._cond:
            n = self._readers.get(me, 0) - 1
            if n <= 0:
                self._readers.pop(me, None)
            else:
                self._readers[me] = n
            if self._waiting:
                self._cond.notify_all()

    def acquire_write(self) -> None:
        self._tracker.before_acquire()
        me = threading.get_ident()
        with self._cond:
            if self._writer == me:
                self._write_depth += 1
            else:
                while self._writer is not None or any(t != me for t in self._readers):
                    self._waiting += 1
                    try:
                        self._cond.wait()
                    finally:
                        self._waiting -= 1
                self._writer = me
                self._write_depth = 1
        self._tracker.acquired()

    def release_write(self) -> None:
        self._tracker.released()
        with self._cond:
            self._write_depth -= 1
            if self._write_depth == 0:
                self._writer = None
            if self._waiting:
                self._cond.notify_all()


def deadlock_checks_enabled() -> bool:
    return True


def new_lock(name: str, check: bool = True) -> CycleDetectingLock:
    return CycleDetectingLock(name, check)


def new_rw_lock(name: str, check: bool = True) -> CycleDetectingRWLock:
    return CycleDetectingRWLock(name, check)


def reset_graph_for_tests() -> None:
    with _graph_lock:
        _edges.clear()
