"""Framework-layer units: the offer queue, the revive token bucket, the revive manager and the
task killer.

Mirrors the reference's suites under sdk/scheduler/src/test/java/com/mesosphere/sdk/framework/
({OfferQueueTest,TokenBucketTest,ReviveManagerTest,TaskKillerTest}.java). The offer-processor,
framework-scheduler and implicit-reconciler suites live in ``test_framework_layer``.
"""
import uuid

import pytest

import testutils as U
from dcos_commons_amd.framework import driver, task_killer
from dcos_commons_amd.framework.offer_processing import OfferQueue, ReviveManager, TokenBucket
from dcos_commons_amd.mesos import protos as P
from dcos_commons_amd.testing.harness import RecordingDriver

CAPACITY = 10
DAY = 86400.0


@pytest.fixture
def drv():
    d = RecordingDriver()
    driver.set_driver(d)
    task_killer.reset(executor_enabled=False)
    yield d
    task_killer.reset(executor_enabled=False)
    driver.set_driver(None)


def _offer(oid=None):
    return U.get_offer(offer_id=P.OfferID(value=oid or U.OFFER_ID.value))


# ---------------------------------------------------------------------------------------
# OfferQueue


def test_queue_starts_empty():
    assert OfferQueue().is_empty()


def test_enqueue():
    q = OfferQueue(CAPACITY)
    q.offer(_offer())
    assert q.size() == 1
    assert q.remaining_capacity() == CAPACITY - 1


def test_exceed_capacity():
    q = OfferQueue()
    n = q.remaining_capacity()
    assert n == 100
    for _ in range(n):
        assert q.offer(_offer())
    assert q.remaining_capacity() == 0
    assert not q.offer(_offer())


@pytest.mark.parametrize("count", [1, CAPACITY // 2, CAPACITY])
def test_take_all(count):
    q = OfferQueue(CAPACITY)
    for _ in range(count):
        q.offer(_offer())
    assert len(q.take_all(0)) == count
    assert q.remaining_capacity() == CAPACITY


def test_unbounded_queue():
    q = OfferQueue(0)
    for _ in range(500):
        assert q.offer(_offer())
    assert q.remaining_capacity() == -1 and q.size() == 500


def test_remove_from_empty_queue():
    q = OfferQueue()
    q.remove(U.OFFER_ID)
    assert q.is_empty()


def test_remove_single_offer():
    q = OfferQueue()
    q.offer(_offer())
    assert q.size() == 1
    assert q.remove(U.OFFER_ID)
    assert q.is_empty()


def test_remove_unknown_offer():
    q = OfferQueue()
    q.offer(_offer(str(uuid.uuid4())))
    assert not q.remove(U.OFFER_ID)
    assert q.size() == 1


def test_remove_one_leaves_others():
    q = OfferQueue()
    for _ in range(q.remaining_capacity() // 2):
        q.offer(_offer(str(uuid.uuid4())))
    q.offer(_offer())
    before = q.remaining_capacity()
    q.remove(U.OFFER_ID)
    assert q.remaining_capacity() == before + 1


# ---------------------------------------------------------------------------------------
# TokenBucket


class Clock:
    def __init__(self):
        self.t = 1000.0

    def __call__(self):
        return self.t


def _bucket(**kw):
    kw.setdefault("acquire_interval_s", 5.0)
    return TokenBucket(**kw)


def test_acquire_fails_on_empty_bucket():
    assert not _bucket(initial=0).try_acquire()


def test_acquire_succeeds_with_one_token():
    assert _bucket(initial=1).try_acquire()


def test_acquire_too_fast_fails():
    b = _bucket(initial=2)
    assert b.try_acquire()
    assert not b.try_acquire()


def test_zero_acquire_interval_allows_back_to_back():
    b = _bucket(initial=2, acquire_interval_s=0)
    assert b.try_acquire() and b.try_acquire()


def test_exhaust_tokens():
    b = _bucket(initial=1, acquire_interval_s=0)
    assert b.try_acquire()
    assert not b.try_acquire()


def test_replenish_tokens():
    b = _bucket(initial=1, acquire_interval_s=0, increment_interval_s=0.1)
    assert b.try_acquire()
    assert not b.try_acquire()
    b.increment()
    assert b.try_acquire()


def test_refill_follows_the_increment_interval_and_caps():
    clock = Clock()
    b = _bucket(initial=0, capacity=3, acquire_interval_s=0, increment_interval_s=256, clock=clock)
    assert not b.try_acquire()
    clock.t += 256
    assert b.try_acquire()
    assert not b.try_acquire()
    clock.t += 256 * 10  # refills stop at the capacity
    assert [b.try_acquire() for _ in range(4)] == [True, True, True, False]


def test_acquire_interval_enforced():
    clock = Clock()
    b = _bucket(initial=2, acquire_interval_s=0.1, clock=clock)
    assert b.try_acquire()
    assert not b.try_acquire()
    clock.t += 0.1
    assert b.try_acquire()


def test_seconds_until_available():
    clock = Clock()
    b = _bucket(initial=1, acquire_interval_s=5, increment_interval_s=256, clock=clock)
    assert b.seconds_until_available() == 0
    b.try_acquire()
    clock.t += 2
    assert b.seconds_until_available() == pytest.approx(254)  # empty: wait for the next token


@pytest.mark.parametrize("kw", [
    {"capacity": 0}, {"initial": -1}, {"increment_interval_s": 0}, {"increment_interval_s": -1},
    {"acquire_interval_s": -1},
])
def test_invalid_configuration(kw):
    with pytest.raises(ValueError):
        _bucket(**kw)


def test_reference_defaults():
    b = TokenBucket()
    assert (b.count, b.capacity, b.increment_interval_s, b.acquire_interval_s) == (256, 256, 256.0, 5.0)


# ---------------------------------------------------------------------------------------
# ReviveManager


def _manager(suppress=True, bucket=None):
    return ReviveManager(bucket or TokenBucket(acquire_interval_s=DAY), suppress_enabled=suppress)


def test_no_revive_unless_requested(drv):
    _manager().revive_if_requested()
    assert drv.revives == 0


def test_revives_are_throttled(drv):
    m = _manager()
    m.request_revive()
    m.revive_if_requested()
    m.request_revive()
    m.revive_if_requested()
    assert drv.revives == 1


def test_managers_share_one_bucket(drv):
    bucket = TokenBucket(acquire_interval_s=DAY)
    a, b = _manager(bucket=bucket), _manager(bucket=bucket)
    a.request_revive()
    b.request_revive()
    a.revive_if_requested()
    b.revive_if_requested()  # throttled
    assert drv.revives == 1


def test_suppress_then_revive(drv):
    m = _manager(bucket=TokenBucket(acquire_interval_s=0))
    m.suppress_if_active()
    assert drv.suppresses == 1
    m.request_revive_if_suppressed()
    m.revive_if_requested()
    assert drv.revives == 1
    # the revive did not seem to work (no offers yet): still treated as suppressed
    m.is_suppressed = True
    m.request_revive_if_suppressed()
    m.revive_if_requested()
    assert drv.revives == 2
    m.notify_offers_received()
    # not suppressed any more: needing offers alone does not revive ...
    m.request_revive_if_suppressed()
    m.revive_if_requested()
    assert drv.revives == 2
    # ... but new work does
    m.request_revive()
    m.revive_if_requested()
    assert drv.revives == 3


def test_no_double_suppress(drv):
    m = _manager()
    m.suppress_if_active()
    m.suppress_if_active()
    assert drv.suppresses == 1


def test_suppress_again_after_offers_arrive(drv):
    m = _manager()
    m.suppress_if_active()
    m.notify_offers_received()
    m.suppress_if_active()
    assert drv.suppresses == 2


def test_suppress_disabled(drv):
    m = _manager(suppress=False)
    m.suppress_if_active()
    assert drv.suppresses == 0


# ---------------------------------------------------------------------------------------
# TaskKiller


def _status(state, reason=None):
    s = U.generate_status(U.TASK_ID, state)
    if reason is not None:
        s.reason = reason
    return s


def _complete_killing(drv, count):
    task_killer.update(_status(P.TASK_KILLED))
    task_killer.kill_all_tasks()
    assert drv.kills == [U.TASK_ID.value] * count


def test_empty_task_id_is_ignored(drv):
    task_killer.kill_task(P.TaskID(value=""))
    task_killer.kill_all_tasks()
    assert drv.kills == []


def test_kill_without_a_driver_is_logged_not_raised():
    """The reference throws (Driver.getInstance: IllegalStateException); here the kill is kept
    and reissued once a driver is set."""
    driver.set_driver(None)
    task_killer.reset(executor_enabled=False)
    task_killer.kill_task(U.TASK_ID)
    assert task_killer.pending_kills() == {U.TASK_ID.value}
    d = RecordingDriver()
    driver.set_driver(d)
    task_killer.kill_all_tasks()
    assert d.kills == [U.TASK_ID.value]
    task_killer.reset(executor_enabled=False)
    driver.set_driver(None)


def test_kill_is_issued_immediately(drv):
    task_killer.kill_task(U.TASK_ID)
    assert drv.kills == [U.TASK_ID.value]
    _complete_killing(drv, 1)


def test_kill_is_reissued_until_terminal(drv):
    task_killer.kill_task(U.TASK_ID)
    task_killer.kill_all_tasks()
    assert len(drv.kills) == 2
    _complete_killing(drv, 2)


def test_non_terminal_status_keeps_killing(drv):
    task_killer.kill_task(U.TASK_ID)
    task_killer.kill_all_tasks()
    task_killer.update(_status(P.TASK_RUNNING))
    task_killer.kill_all_tasks()
    assert len(drv.kills) == 3
    _complete_killing(drv, 3)


def test_kill_loop_is_broken(drv):
    task_killer.kill_task(U.TASK_ID)
    lost = _status(P.TASK_LOST, P.TaskStatus.REASON_RECONCILIATION)
    # already queued for killing: not eligible for another kill
    assert not task_killer.update(lost)
    # no longer queued: a later status makes it eligible again
    assert task_killer.update(lost)
