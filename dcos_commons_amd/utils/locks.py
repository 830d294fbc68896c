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
    try:
        return _held.stack
    except AttributeError:
        st = _held.stack = []
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


def _check_order(lock_id: int, stack: List[int]) -> None:
    """Acquiring ``lock_id`` while holding ``stack`` (non-empty, without ``lock_id``): record the
    held -> acquired edges, and run the policy if one would close a cycle."""
    # Fast path: every held -> this edge is already known (and was cycle-checked when it was
    # added). Set membership reads are atomic under the GIL, so no graph lock is needed.
    for held in stack:
        known = _edges.get(held)
        if known is None or lock_id not in known:
            break
    else:
        return
    msg = None
    with _graph_lock:
        for held in stack:
            if lock_id in _edges.get(held, ()):
                continue
            path = _reachable(lock_id, held)
            if path is not None:
                names = " -> ".join(_names[i] for i in path + [lock_id])
                msg = f"Lock-order cycle detected acquiring {_names[lock_id]}: {names}"
                break
            _edges.setdefault(held, set()).add(lock_id)
    if msg:
        _policy(msg)


def _release_id(stack: List[int], lock_id: int) -> None:
    if stack and stack[-1] == lock_id:
        stack.pop()
        return
    for i in range(len(stack) - 1, -1, -1):
        if stack[i] == lock_id:
            del stack[i]
            return


def _new_id(name: str) -> int:
    lock_id = next(_ids)
    _names[lock_id] = name
    return lock_id


class CycleDetectingLock:
    """Re-entrant lock with lock-order cycle detection."""

    __slots__ = ("_lock", "_id", "_check")

    def __init__(self, name: str, check: bool = True):
        self._lock = threading.RLock()
        self._id = _new_id(name)
        self._check = check

    def acquire(self, blocking: bool = True, timeout: float = -1) -> bool:
        stack = _held_stack()
        if self._check and stack and self._id not in stack:
            _check_order(self._id, stack)
        ok = self._lock.acquire(blocking, timeout)
        if ok:
            stack.append(self._id)
        return ok

    def release(self) -> None:
        _release_id(_held_stack(), self._id)
        self._lock.release()

    def __enter__(self):
        self.acquire()
        return self

    def __exit__(self, *exc):
        self.release()


class _RWView:
    __slots__ = ("acquire", "release")

    def __init__(self, owner: "CycleDetectingRWLock", write: bool):
        self.acquire = owner.acquire_write if write else owner.acquire_read
        self.release = owner.release_write if write else owner.release_read

    def __enter__(self):
        self.acquire()
        return self

    def __exit__(self, *exc):
        self.release()


_get_ident = threading.get_ident


class CycleDetectingRWLock:
    """Readers-writer lock (writer re-entrant, writer may take read) with cycle detection.

    The uncontended paths (no writer in the way, nobody waiting) take the internal mutex once
    through its C-level context manager; only a blocked acquire goes through the condition."""

    def __init__(self, name: str, check: bool = True):
        self._mutex = threading.Lock()
        self._cond = threading.Condition(self._mutex)
        self._readers: Dict[int, int] = {}
        self._writer: Optional[int] = None
        self._write_depth = 0
        self._id = _new_id(name)
        self._check = check
        self._waiting = 0  # threads blocked in _cond.wait(): release only notifies when > 0
        self.read_lock = _RWView(self, False)
        self.write_lock = _RWView(self, True)

    def acquire_read(self) -> None:
        stack = _held_stack()
        if self._check and stack and self._id not in stack:
            _check_order(self._id, stack)
        me = _get_ident()
        with self._mutex:
            while self._writer is not None and self._writer != me:
                self._waiting += 1
                try:
                    self._cond.wait()
                finally:
                    self._waiting -= 1
            readers = self._readers
            readers[me] = readers.get(me, 0) + 1
        stack.append(self._id)

    def release_read(self) -> None:
        me = _get_ident()
        _release_id(_held_stack(), self._id)
        with self._mutex:
            readers = self._readers
            n = readers.get(me, 0) - 1
            if n <= 0:
                readers.pop(me, None)
            else:
                readers[me] = n
            if self._waiting:
                self._cond.notify_all()

    def acquire_write(self) -> None:
        stack = _held_stack()
        if self._check and stack and self._id not in stack:
            _check_order(self._id, stack)
        me = _get_ident()
        with self._mutex:
            if self._writer == me:
                self._write_depth += 1
            else:
                while self._writer is not None or (self._readers and any(t != me for t in self._readers)):
                    self._waiting += 1
                    try:
                        self._cond.wait()
                    finally:
                        self._waiting -= 1
                self._writer = me
                self._write_depth = 1
        stack.append(self._id)

    def release_write(self) -> None:
        _release_id(_held_stack(), self._id)
        with self._mutex:
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
