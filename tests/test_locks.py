"""Lock-order cycle detection and the readers-writer lock (reference:
sdk/.../state/CycleDetectingLockUtils.java:13-46 on Guava's CycleDetectingLockFactory; the
reference has no dedicated test, the behaviour is exercised through MemPersister/PersisterCache).
Also the plan aggregate-status retry for torn reads of concurrently changing steps."""
import threading
import time

import pytest

from dcos_commons_amd.scheduler.plan.status import Status
from dcos_commons_amd.utils import locks


@pytest.fixture(autouse=True)
def raising():
    locks.set_policy(locks.raising_policy)
    yield
    locks.set_policy(None)


def test_inconsistent_order_is_detected():
    a, b = locks.new_lock("A"), locks.new_lock("B")
    with a:
        with b:
            pass
    with b:
        with pytest.raises(locks.PotentialDeadlockError) as e:
            a.acquire()
    assert "A" in str(e.value) and "B" in str(e.value)


def test_transitive_cycle_is_detected():
    a, b, c = locks.new_lock("A1"), locks.new_lock("B1"), locks.new_lock("C1")
    with a, b:
        pass
    with b, c:
        pass
    with c:
        with pytest.raises(locks.PotentialDeadlockError):
            a.acquire()


def test_consistent_order_and_reentrancy_are_fine():
    a, b = locks.new_lock("A2"), locks.new_lock("B2")
    for _ in range(3):
        with a:
            with a:          # re-entrant
                with b:
                    pass
    unchecked = locks.new_lock("U", check=False)
    with b:
        with unchecked:
            pass
    with unchecked:
        with b:
            pass


def test_known_edge_fast_path_still_checks_new_edges():
    a, b, c = locks.new_lock("A3"), locks.new_lock("B3"), locks.new_lock("C3")
    with a, b:
        pass
    with a, b:               # known edge: fast path
        pass
    with b, c:
        pass
    with c:
        with pytest.raises(locks.PotentialDeadlockError):
            with a:
                pass


def test_rw_lock_order_participates():
    rw, m = locks.new_rw_lock("RW"), locks.new_lock("M")
    with rw.read_lock:
        with m:
            pass
    with m:
        with pytest.raises(locks.PotentialDeadlockError):
            rw.write_lock.acquire()


def test_rw_readers_share_writer_excludes():
    rw = locks.new_rw_lock("RW2")
    inside = []
    gate = threading.Event()

    def reader(i):
        with rw.read_lock:
            inside.append(i)
            gate.wait(5)
    ts = [threading.Thread(target=reader, args=(i,)) for i in range(3)]
    for t in ts:
        t.start()
    deadline = time.time() + 5
    while len(inside) < 3 and time.time() < deadline:
        time.sleep(0.001)
    assert len(inside) == 3          # all readers are in at once
    got_write = threading.Event()

    def writer():
        with rw.write_lock:
            got_write.set()
    w = threading.Thread(target=writer)
    w.start()
    time.sleep(0.05)
    assert not got_write.is_set()    # the writer waits for the readers
    gate.set()
    assert got_write.wait(5)         # and is woken when the last reader leaves
    for t in ts + [w]:
        t.join(5)


def test_writer_is_reentrant_and_may_read():
    rw = locks.new_rw_lock("RW3")
    with rw.write_lock:
        with rw.write_lock:
            with rw.read_lock:
                pass
    blocked = threading.Event()
    done = threading.Event()

    def reader():
        blocked.set()
        with rw.read_lock:
            done.set()
    with rw.write_lock:
        t = threading.Thread(target=reader)
        t.start()
        blocked.wait(5)
        time.sleep(0.05)
        assert not done.is_set()
    assert done.wait(5)
    t.join(5)


# ---------------------------------------------------------------------------------------
# aggregate status under concurrent step changes


class _FlipStep:
    """A step whose status changes between the parent's separate reads."""

    def __init__(self, seq):
        self.seq = list(seq)
        self.i = 0

    def get_status(self):
        s = self.seq[min(self.i, len(self.seq) - 1)]
        self.i += 1
        return s


def test_torn_aggregate_read_is_retried(monkeypatch):
    from dcos_commons_amd.scheduler.plan import elements

    calls = []
    real = elements.get_aggregate_status

    def spy(name, children, candidates, errors, interrupted, log_unexpected=True):
        calls.append((list(children), list(candidates)))
        return real(name, children, candidates, errors, interrupted, log_unexpected)
    monkeypatch.setattr(elements, "get_aggregate_status", spy)

    class Parent(elements.ParentElement):
        def __init__(self, child):
            self.child = child

        def get_children(self):
            return [self.child]

        def get_errors(self):
            return []

        def is_interrupted(self):
            return False

        def get_name(self):
            return "p"

        def get_strategy(self):
            parent = self

            class S:
                def get_candidates(self, children, dirty):
                    return [c for c in children if c is parent.child]
            return S()
    # first pass reads STARTED (child), then COMPLETE (candidate): a torn read; second pass is
    # consistent COMPLETE/COMPLETE
    step = _FlipStep([Status.STARTED, Status.COMPLETE, Status.COMPLETE, Status.COMPLETE])
    assert Parent(step).get_status() == Status.COMPLETE
    assert len(calls) == 2
