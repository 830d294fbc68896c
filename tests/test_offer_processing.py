"""Revive rate limiting and the framework benchmarks (reference: sdk/scheduler/src/test/java/.../
framework/TokenBucketTest.java, ReviveManagerTest.java; BASELINE.json configs 3 and 4)."""
import pytest

from dcos_commons_amd.framework.offer_processing import ReviveManager, TokenBucket


class Clock:
    def __init__(self):
        self.t = 1000.0

    def __call__(self):
        return self.t


def test_token_bucket_reference_defaults():
    c = Clock()
    b = TokenBucket(clock=c)  # capacity 256, +1 / 256 s, 5 s between acquires
    assert b.try_acquire()
    assert not b.try_acquire()
    c.t += 4.9
    assert not b.try_acquire() and b.seconds_until_available() == pytest.approx(0.1)
    c.t += 0.1
    assert b.try_acquire()


def test_token_bucket_exhausts_and_refills():
    c = Clock()
    b = TokenBucket(initial=2, capacity=2, increment_interval_s=10, acquire_interval_s=0, clock=c)
    assert b.try_acquire() and b.try_acquire() and not b.try_acquire()
    c.t += 9.9
    assert not b.try_acquire()
    c.t += 0.1
    assert b.try_acquire() and not b.try_acquire()
    c.t += 100  # refill never exceeds capacity
    assert b.try_acquire() and b.try_acquire() and not b.try_acquire()


def test_token_bucket_burst_regime_falls_back_when_drained():
    c = Clock()
    b = TokenBucket(initial=8, capacity=8, acquire_interval_s=1.0, burst_interval_s=0.0625, clock=c)
    # more than burst_floor (4) tokens left: 62.5 ms spacing
    for _ in range(4):
        assert b.try_acquire()
        assert not b.try_acquire()
        c.t += 0.0625
    assert b.count == 4
    # at the floor: the slow spacing applies again
    assert not b.try_acquire()
    c.t += 0.9375
    assert b.try_acquire()


@pytest.mark.parametrize("kw", [dict(initial=-1), dict(capacity=0), dict(increment_interval_s=0),
                                dict(acquire_interval_s=-1), dict(acquire_interval_s=1, burst_interval_s=2)])
def test_token_bucket_rejects_bad_config(kw):
    with pytest.raises(ValueError):
        TokenBucket(**kw)


def test_revive_manager_fast_unsuppress_skips_spacing_once():
    c = Clock()
    calls = []

    class D:
        def revive_offers(self):
            calls.append("revive")

        def suppress_offers(self):
            calls.append("suppress")

    from dcos_commons_amd.framework import driver

    driver.set_driver(D())
    try:
        rm = ReviveManager(TokenBucket(clock=c), fast_unsuppress=True)
        rm.request_revive()
        rm.revive_if_requested()
        rm.suppress_if_active()
        rm.request_revive_if_suppressed()  # straight after the first revive: bypasses the 5 s spacing
        rm.revive_if_requested()
        rm.request_revive()  # not suppressed any more: spacing applies
        rm.revive_if_requested()
        assert calls == ["revive", "suppress", "revive"] and rm.revive_requested
    finally:
        driver.set_driver(None)


@pytest.mark.parametrize("framework", ["cassandra", "hdfs"])
def test_framework_bench_cycle(framework):
    from dcos_commons_amd.benchmarks.framework_bench import FrameworkBench

    cyc = FrameworkBench(framework, timeout_s=60).run_cycle()
    # scheduler cost only (synthetic payloads); the reference cadence needs 11-54 s here
    assert cyc.deploy_s < 5 and cyc.second_s < 5
    assert cyc.tasks == (3 if framework == "cassandra" else 10)


def _offer(oid, agent, cpus, reserved_cpus=0.0, executors=()):
    from dcos_commons_amd.mesos import protos as P

    o = P.Offer(hostname=agent)
    o.id.value, o.agent_id.value, o.framework_id.value = oid, agent, "fw"
    r = o.resources.add(name="cpus", type=P.Value.SCALAR)
    r.scalar.value = cpus
    r.allocation_info.role = "svc-role"
    if reserved_cpus:
        rr = o.resources.add(name="cpus", type=P.Value.SCALAR)
        rr.scalar.value = reserved_cpus
        res = rr.reservations.add(type=P.Resource.ReservationInfo.DYNAMIC, role="svc-role", principal="p")
        res.labels.labels.add(key="resource_id", value="rid-1")
        rr.allocation_info.role = "svc-role"
    for e in executors:
        o.executor_ids.add(value=e)
    return o


def test_merge_agent_offers_combines_per_agent():
    from dcos_commons_amd.framework.offer_processing import merge_agent_offers

    a1 = _offer("o1", "agent-a", 2.0, executors=["e1"])
    a2 = _offer("o2", "agent-a", 1.0, reserved_cpus=0.5, executors=["e1", "e2"])
    b1 = _offer("o3", "agent-b", 4.0)
    merged, members = merge_agent_offers([a1, b1, a2])
    assert [o.id.value for o in merged] == ["o1", "o3"]
    assert [o.id.value for o in members["o1"]] == ["o1", "o2"] and "o3" not in members
    m = merged[0]
    unreserved = [r.scalar.value for r in m.resources if not len(r.reservations)]
    reserved = [r.scalar.value for r in m.resources if len(r.reservations)]
    assert unreserved == [3.0] and reserved == [0.5]  # identical resources merged like the master does
    assert all(r.allocation_info.role == "svc-role" for r in m.resources)
    assert [e.value for e in m.executor_ids] == ["e1", "e2"]
    assert merged[1] is b1


def test_accepter_names_every_member_offer():
    from dcos_commons_amd.framework import driver
    from dcos_commons_amd.framework.offer_processing import OfferAccepter, merge_agent_offers
    from dcos_commons_amd.mesos import protos as P
    from dcos_commons_amd.offer.recommendations import LaunchOfferRecommendation

    calls = []

    class D:
        def accept_offers(self, offer_ids, ops, filters):
            calls.append(sorted(o.value for o in offer_ids))

    merged, members = merge_agent_offers([_offer("o1", "agent-a", 2.0), _offer("o2", "agent-a", 1.0)])
    task = P.TaskInfo(name="t")
    task.task_id.value = "t__1"
    task.agent_id.value = "agent-a"
    rec = LaunchOfferRecommendation(merged[0], task, P.ExecutorInfo())
    driver.set_driver(D())
    try:
        OfferAccepter().accept([rec], members)
    finally:
        driver.set_driver(None)
    assert calls == [["o1", "o2"]]



def test_cluster_bench_cycle():
    """The cluster-mode bench: scheduler process + v1 HTTP API + ZooKeeper, real task processes."""
    from dcos_commons_amd.benchmarks.cluster_bench import ClusterBench

    b = ClusterBench(agents=2, timeout_s=60.0)
    try:
        r = b.run_cycle()
    finally:
        b.close()
    assert 0 < r["deploy_s"] < 30 and 0 < r["mttr_restart_s"] < 30 and 0 < r["mttr_replace_s"] < 30
