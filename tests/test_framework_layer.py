"""Framework layer: OfferQueue, OfferProcessor cycles, TaskKiller, ImplicitReconciler,
FrameworkScheduler callbacks.

Pinned against the reference's framework suite
(sdk/scheduler/src/test/java/com/mesosphere/sdk/framework/OfferQueueTest.java, OfferProcessorTest
.java incl. the 50-thread enqueue test, TaskKillerTest.java, ImplicitReconcilerTest.java,
FrameworkSchedulerTest.java): a recording driver stands in for the mocked SchedulerDriver.
"""
import threading
import time
import uuid

import pytest

from dcos_commons_amd.framework import driver, task_killer
from dcos_commons_amd.framework.offer_processing import (
    ImplicitReconciler,
    OfferProcessor,
    OfferQueue,
)
from dcos_commons_amd.mesos import protos as P
from dcos_commons_amd.offer.recommendations import (
    ReserveOfferRecommendation,
)
from dcos_commons_amd.scheduler.mesos_event_client import (
    ClientStatusResponse,
    OfferResources,
    OfferResponse,
    UnexpectedResourcesResponse,
)
from dcos_commons_amd.storage.mem_persister import MemPersister


class RecordingDriver:
    def __init__(self):
        self.lock = threading.Lock()
        self.accepts, self.declines, self.kills, self.reconciles = [], [], [], []
        self.revives = self.suppresses = 0

    def accept_offers(self, offer_ids, operations, filters=None):
        with self.lock:
            self.accepts.append(([o.value for o in offer_ids], [op.type for op in operations]))

    def decline_offer(self, offer_id, filters=None):
        self.decline_offers([offer_id], filters)

    def decline_offers(self, offer_ids, filters=None):
        with self.lock:
            self.declines.append(([o.value for o in offer_ids], filters.refuse_seconds if filters else None))

    def kill_task(self, task_id):
        with self.lock:
            self.kills.append(task_id.value)

    def reconcile_tasks(self, statuses):
        with self.lock:
            self.reconciles.append([s.task_id.value for s in statuses])

    def revive_offers(self):
        self.revives += 1

    def suppress_offers(self):
        self.suppresses += 1

    def declined_ids(self):
        return {i for ids, _ in self.declines for i in ids}


@pytest.fixture
def drv():
    d = RecordingDriver()
    driver.set_driver(d)
    task_killer.reset(executor_enabled=False)
    yield d
    task_killer.reset(executor_enabled=False)
    driver.set_driver(None)


def offer(oid=None, cpus=1.0, agent="agent-1", reserved_id=None):
    o = P.Offer(hostname="host")
    o.id.value = oid or str(uuid.uuid4())
    o.agent_id.value, o.framework_id.value = agent, "fw"
    r = o.resources.add(name="cpus", type=P.Value.SCALAR)
    r.scalar.value = cpus
    if reserved_id:
        res = r.reservations.add(type=P.Resource.ReservationInfo.DYNAMIC, role="svc-role", principal="p")
        res.labels.labels.add(key="resource_id", value=reserved_id)
    return o


class Client:
    """A scripted MesosEventClient."""

    def __init__(self, status=None, offers_fn=None, unexpected_fn=None):
        self.status = status or ClientStatusResponse.launching(False)
        self.offers_fn = offers_fn or (lambda offers: OfferResponse.processed([]))
        self.unexpected_fn = unexpected_fn or (lambda offers: UnexpectedResourcesResponse.processed([]))
        self.received = []
        self.lock = threading.Lock()

    def get_client_status(self):
        return self.status

    def offers(self, offers, launch_stream=None):
        with self.lock:
            self.received.extend(o.id.value for o in offers)
        return self.offers_fn(offers)

    def get_unexpected_resources(self, offers):
        return self.unexpected_fn(offers)

    def unregistered(self):
        pass


def processor(client, **kw):
    p = OfferProcessor(client, MemPersister(), **kw)
    return p


# ---------------------------------------------------------------------------------------
# OfferQueue


def test_offer_queue_basics():
    q = OfferQueue(capacity=3)
    assert q.is_empty() and q.take_all(0) == []
    os_ = [offer(f"o{i}") for i in range(4)]
    assert [q.offer(o) for o in os_] == [True, True, True, False]   # capacity
    assert q.size() == 3
    assert not q.remove(P.OfferID(value="unknown"))
    assert q.remove(P.OfferID(value="o1"))
    assert [o.id.value for o in q.take_all(0)] == ["o0", "o2"]
    assert q.is_empty()
    assert not q.remove(P.OfferID(value="o0"))          # remove from an empty queue


def test_offer_queue_take_waits_and_wakes():
    q = OfferQueue()
    t0 = time.monotonic()
    assert q.take_all(0.05) == []
    assert time.monotonic() - t0 >= 0.045
    threading.Timer(0.02, lambda: q.offer(offer("late"))).start()
    got = q.take_all(2.0)
    assert [o.id.value for o in got] == ["late"]
    wake = threading.Event()
    threading.Timer(0.02, wake.set).start()
    t0 = time.monotonic()
    assert q.take_all(2.0, wake) == [] and time.monotonic() - t0 < 1.0


# ---------------------------------------------------------------------------------------
# OfferProcessor cycles (synchronous)


def test_unused_offers_declined_long_when_idle(drv):
    p = processor(Client(status=ClientStatusResponse.idle())).disable_threading()
    p.start()
    p.enqueue([offer("a"), offer("b")])
    assert drv.declined_ids() == {"a", "b"}
    assert all(refuse == 3600 for _, refuse in drv.declines)
    assert drv.suppresses == 1


def test_not_ready_offers_declined_short(drv):
    c = Client(offers_fn=lambda offers: OfferResponse.not_ready([]))
    p = processor(c).disable_threading()
    p.start()
    p.enqueue([offer("a")])
    assert drv.declines == [(["a"], 5)]


def test_unused_offers_declined_long_while_working_without_holding(drv):
    p = processor(Client()).disable_threading()
    p.start()
    p.enqueue([offer("a")])
    assert drv.declines == [(["a"], 3600)]


def test_held_offers_are_reevaluated_then_declined(drv):
    c = Client()
    p = processor(c, hold_s=0.05).disable_threading()
    p.start()
    p.enqueue([offer("a")])
    assert drv.declines == [] and c.received == ["a"]
    p.process_queued_offers(0)                       # the held offer is evaluated again
    assert c.received == ["a", "a"]
    time.sleep(0.06)
    p.process_queued_offers(0)
    assert drv.declines == [(["a"], 5)]              # expired holds go back short


def test_accepted_and_unexpected_resources(drv):
    """Recommendations are accepted; unused offers' unexpected reservations are released in one
    ACCEPT with DESTROY before UNRESERVE (OfferProcessor.java:300-330)."""
    def offers_fn(offers):
        o = offers[0]
        return OfferResponse.processed([ReserveOfferRecommendation(o, o.resources[0])])

    def unexpected_fn(offers):
        out = []
        for o in offers:
            if o.id.value == "stale":
                vol = P.Resource()
                vol.CopyFrom(o.resources[0])
                vol.disk.persistence.id = "pid"
                out.append(OfferResources(o, [o.resources[0], vol]))
        return UnexpectedResourcesResponse.processed(out)
    p = processor(Client(offers_fn=offers_fn, unexpected_fn=unexpected_fn)).disable_threading()
    p.start()
    p.enqueue([offer("used", agent="agent-1"), offer("stale", agent="agent-2", reserved_id="old")])
    by_offer = {ids[0]: ops for ids, ops in drv.accepts}
    assert by_offer["used"] == [P.Offer.Operation.RESERVE]
    ops = by_offer["stale"]
    assert ops.index(P.Offer.Operation.DESTROY) < ops.index(P.Offer.Operation.UNRESERVE)
    assert "stale" not in drv.declined_ids()


def test_uninstalled_client_tears_down(drv):
    torn = []

    class D(RecordingDriver):
        def teardown(self):
            torn.append(True)

        def stop(self, failover=True):
            torn.append(failover)
    d = D()
    driver.set_driver(d)
    from dcos_commons_amd.scheduler.mesos_event_client import IdleRequest

    st = ClientStatusResponse.idle()
    st.idle_request = IdleRequest.REMOVE_CLIENT
    p = processor(Client(status=st)).disable_threading()
    p.start()
    p.enqueue([offer("a")])
    assert torn == [True, False]


@pytest.mark.parametrize("capacity,expect_declines", [(0, False), (10, True)])
def test_fifty_threads_enqueue(drv, capacity, expect_declines):
    """OfferProcessorTest.testAsyncOffers{Unlimited,Limited}QueueSize: 50 threads x 3 offers."""
    gate = threading.Event()
    if not expect_declines:
        gate.set()

    def offers_fn(offers):
        gate.wait(10)            # bounded case: the processor stalls while the threads pile offers up
        return OfferResponse.processed([ReserveOfferRecommendation(o, o.resources[0]) for o in offers])
    c = Client(offers_fn=offers_fn)
    p = processor(c, queue_capacity=capacity, offer_wait_s=0.01)
    p.start()
    sent = []
    lock = threading.Lock()

    def send():
        os_ = [offer() for _ in range(3)]
        with lock:
            sent.extend(o.id.value for o in os_)
        p.enqueue(os_)
    ts = [threading.Thread(target=send) for _ in range(50)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    gate.set()
    p.await_offers_processed(10)
    p.stop()
    declined = drv.declined_ids()
    assert set(c.received) | declined == set(sent)
    assert set(c.received) & declined == set()
    if expect_declines:
        assert declined                       # the bounded queue sheds load by declining
    else:
        assert not declined and len(c.received) == 150


def test_stream_callback_accepts_before_the_cycle_ends(drv):
    """Launch streaming: a client that streams gets its recs ACCEPTed from inside offers()."""
    seen_during = []

    class Streaming(Client):
        def offers(self, offers, launch_stream=None):
            o = offers[0]
            recs = [ReserveOfferRecommendation(o, o.resources[0])]
            launch_stream(recs)
            seen_during.append(len(drv.accepts))
            return OfferResponse.processed(recs, streamed=True)
    p = processor(Streaming(), stream_launches=True).disable_threading()
    p.start()
    p.enqueue([offer("a")])
    assert seen_during == [1]
    assert drv.accepts == [(["a"], [P.Offer.Operation.RESERVE])]     # not accepted twice


# ---------------------------------------------------------------------------------------
# TaskKiller


def test_task_killer_breaks_the_kill_loop(drv):
    tid = P.TaskID(value="svc__pod-0-task__1")
    task_killer.kill_task(tid)
    assert drv.kills == [tid.value] and task_killer.pending_kills() == {tid.value}
    lost = P.TaskStatus(state=P.TASK_LOST)
    lost.task_id.CopyFrom(tid)
    # the expected death completes the kill and is NOT eligible for another kill
    assert task_killer.update(lost) is False
    assert task_killer.pending_kills() == set()
    # an unexpected death is eligible (it was not scheduled for killing)
    assert task_killer.update(lost) is True
    running = P.TaskStatus(state=P.TASK_RUNNING)
    running.task_id.CopyFrom(tid)
    assert task_killer.update(running) is True


def test_task_killer_ignores_empty_ids_and_rekills(drv):
    task_killer.kill_task(P.TaskID(value=""))
    assert drv.kills == []
    task_killer.kill_task(P.TaskID(value="a"))
    task_killer.kill_task(P.TaskID(value="b"))
    task_killer.kill_all_tasks()
    assert sorted(drv.kills) == ["a", "a", "b", "b"]


# ---------------------------------------------------------------------------------------
# ImplicitReconciler


def test_implicit_reconciler(drv):
    r = ImplicitReconciler(0.0, 3600.0).disable_threading()
    r.start()
    assert drv.reconciles == [[]]           # single-threaded: reconciles once, immediately
    with pytest.raises(RuntimeError):
        r.start()
    threaded = ImplicitReconciler(0.0, 0.02)
    threaded.start()
    time.sleep(0.15)
    threaded.stop()
    assert len(drv.reconciles) >= 3


def test_implicit_reconciler_prestart_waits_for_start(drv):
    """A thread created ahead of registration reconciles nothing until ``start``; ``stop`` ends a
    thread that was never started."""
    r = ImplicitReconciler(0.0, 3600.0)
    r.prestart()
    time.sleep(0.05)
    assert drv.reconciles == [] and r._thread.is_alive()
    r.start()
    deadline = time.monotonic() + 2
    while not drv.reconciles and time.monotonic() < deadline:
        time.sleep(0.005)
    assert drv.reconciles == [[]]
    r.stop()
    idle = ImplicitReconciler(0.0, 3600.0)
    idle.prestart()
    idle.stop()
    idle._thread.join(1)
    assert not idle._thread.is_alive() and drv.reconciles == [[]]


def test_offer_processor_prestart_runs_no_cycle_before_start(drv):
    """The loop thread exists before registration, but an offer-less cycle does nothing until the
    processor is started; ``start`` after ``prestart`` keeps the one thread."""
    c = Client()
    p = processor(c, offer_wait_s=0.01)
    p.prestart()
    thread = p._thread
    time.sleep(0.05)
    assert c.received == [] and thread.is_alive()
    p.start()
    assert p._thread is thread
    p.enqueue([offer("o1")])
    deadline = time.monotonic() + 2
    while not c.received and time.monotonic() < deadline:
        time.sleep(0.005)
    assert c.received == ["o1"]
    p.stop()


# ---------------------------------------------------------------------------------------
# FrameworkScheduler callbacks


class _StatusClient(Client):
    def __init__(self, known=()):
        super().__init__()
        self.known = set(known)
        self.statuses = []
        self.registrations = []

    def registered(self, re_registered):
        self.registrations.append(re_registered)

    def task_status(self, status):
        from dcos_commons_amd.scheduler.mesos_event_client import TaskStatusResponse

        self.statuses.append(status.task_id.value)
        return TaskStatusResponse.processed() if status.task_id.value in self.known else \
            TaskStatusResponse.unknown_task()


def _fs(client, persister=None):
    from dcos_commons_amd.framework.framework_scheduler import FrameworkScheduler
    from dcos_commons_amd.state.framework_store import FrameworkStore

    persister = persister or MemPersister()
    fs = FrameworkScheduler({"svc-role"}, None, persister, FrameworkStore(persister), client)
    return fs.disable_threading(), FrameworkStore(persister)


def test_register_stores_framework_id_and_reregister(drv):
    c = _StatusClient()
    fs, store = _fs(c)
    fs.registered(drv, P.FrameworkID(value="fw-1"), None)
    assert store.fetch_framework_id().value == "fw-1"
    fs.registered(drv, P.FrameworkID(value="fw-1"), None)     # a second registration is a re-registration
    assert c.registrations == [False, True]


def test_offers_declined_until_api_server_started(drv):
    c = _StatusClient()
    fs, _ = _fs(c)
    fs.registered(drv, P.FrameworkID(value="fw-1"), None)
    fs.resource_offers(drv, [offer("early")])
    assert drv.declines == [(["early"], 5)] and c.received == []
    fs.set_api_server_started()
    fs.resource_offers(drv, [offer("later")])
    assert c.received == ["later"]


def test_offer_rescinded_is_dequeued(drv):
    c = _StatusClient()
    fs, _ = _fs(c)
    fs.offer_processor.multithreaded = True          # keep offers queued (no synchronous processing)
    fs.set_api_server_started()
    fs.offer_processor.enqueue([offer("x"), offer("y")])
    fs.offer_rescinded(drv, P.OfferID(value="x"))
    assert [o.id.value for o in fs.offer_processor.queue.take_all(0)] == ["y"]


def test_foreign_reservations_are_filtered(drv):
    c = _StatusClient()
    fs, _ = _fs(c)
    fs.registered(drv, P.FrameworkID(value="fw-1"), None)
    fs.set_api_server_started()
    got = []
    fs.offer_processor.enqueue = lambda offers: got.extend(offers)
    o = offer("o")
    foreign = o.resources.add(name="mem", type=P.Value.SCALAR)
    foreign.scalar.value = 64
    res = foreign.reservations.add(type=P.Resource.ReservationInfo.DYNAMIC, role="other-role", principal="x")
    res.labels.labels.add(key="resource_id", value="theirs")
    fs.resource_offers(drv, [o])
    assert [r.name for r in got[0].resources] == ["cpus"]


class _ReconcilingClient(_StatusClient):
    """Explicit reconciliation is pending until the first status arrives."""

    def __init__(self):
        super().__init__(known={"t"})
        self.reconciled = False

    def awaiting_reconciliation(self):
        return not self.reconciled

    def task_status(self, status):
        resp = super().task_status(status)
        self.reconciled = True
        return resp


def test_status_that_ends_reconciliation_wakes_the_offer_loop(drv):
    """A TASK_STARTING cannot create work on its own (can_create_work is False), but when it is the
    status that ends explicit reconciliation the offer loop must run now: offers were refused until
    then, and without the kick they would wait for the next offer or the 5 s poll."""
    c = _ReconcilingClient()
    fs, _ = _fs(c)
    kicks = []
    fs.offer_processor.kick = lambda: kicks.append(1)
    starting = P.TaskStatus(task_id=P.TaskID(value="t"), state=P.TASK_STARTING)
    fs.status_update(drv, starting)
    assert kicks == [1]
    fs.status_update(drv, starting)          # reconciled: a STARTING no longer wakes the loop
    assert kicks == [1]


def test_abstract_scheduler_reports_reconciliation_progress():
    from dcos_commons_amd.scheduler.abstract_scheduler import AbstractScheduler

    class _Reconciler:
        done = False

        def is_reconciled(self):
            return self.done

    s = AbstractScheduler.__new__(AbstractScheduler)
    s.reconciler = None
    assert s.awaiting_reconciliation()                    # not registered yet
    s.reconciler = _Reconciler()
    assert s.awaiting_reconciliation()
    s.reconciler.done = True
    assert not s.awaiting_reconciliation()


def test_unknown_task_status_kills_once(drv):
    c = _StatusClient(known={"known"})
    fs, _ = _fs(c)
    st = P.TaskStatus(state=P.TASK_RUNNING)
    st.task_id.value = "stray"
    fs.status_update(drv, st)
    assert drv.kills == ["stray"]
    # the master answers the kill of an unknown task with LOST: no kill loop
    lost = P.TaskStatus(state=P.TASK_LOST, reason=P.TaskStatus.REASON_RECONCILIATION)
    lost.task_id.value = "stray"
    fs.status_update(drv, lost)
    assert drv.kills == ["stray"]
    ok = P.TaskStatus(state=P.TASK_RUNNING)
    ok.task_id.value = "known"
    fs.status_update(drv, ok)
    assert drv.kills == ["stray"] and c.statuses == ["stray", "stray", "known"]


def test_offer_rescinded_during_its_cycle_is_neither_held_nor_declined(drv):
    """A rescind (driver thread) that lands while the offer thread evaluates the offer: the cycle
    must not hold the dead offer again (it would be re-evaluated and ACCEPTed after the master
    dropped it) nor decline it."""
    c = Client()
    p = processor(c, hold_s=10.0).disable_threading()
    p.start()

    def rescinding(offers):
        for o in offers:
            if o.id.value == "a":
                p.dequeue(o.id)
        return OfferResponse.processed([])
    c.offers_fn = rescinding
    p.enqueue([offer("a"), offer("b")])
    assert p.held_offer_ids() == ["b"]
    assert drv.declines == []


def test_held_offers_survive_concurrent_rescinds(drv):
    """Rescinds hammering the processor from another thread while cycles run over held offers
    (the held map used to be iterated unguarded: 'dictionary changed size during iteration')."""
    import threading as _t

    c = Client()
    p = processor(c, hold_s=60.0).disable_threading()
    p.start()
    stop = _t.Event()
    errors = []

    def rescinder():
        i = 0
        while not stop.is_set():
            p.dequeue(P.OfferID(value=f"o{i % 200}"))
            i += 1

    t = _t.Thread(target=rescinder, daemon=True)
    t.start()
    try:
        for n in range(60):
            try:
                p.enqueue([offer(f"o{(n * 7 + k) % 200}") for k in range(20)])
            except RuntimeError as e:  # pragma: no cover - the regression
                errors.append(e)
    finally:
        stop.set()
        t.join()
    assert errors == []


# ---------------------------------------------------------------------------------------
# MI355X offer-loop latency knobs: status wake-ups and revives that cannot bring new work


def _st(state, check_exit=None, check=False):
    s = P.TaskStatus(state=state)
    s.task_id.value = "svc__task__1"
    if check or check_exit is not None:
        cs = s.check_status
        cs.type = P.CheckInfo.COMMAND if hasattr(P, "CheckInfo") else 1
        cs.command.SetInParent()
        if check_exit is not None:
            cs.command.exit_code = check_exit
    return s


@pytest.mark.parametrize("status,wakes", [
    (_st(P.TASK_STAGING), False),
    (_st(P.TASK_STARTING), False),
    (_st(P.TASK_RUNNING, check=True), False),          # readiness check still pending
    (_st(P.TASK_RUNNING, check_exit=0), True),         # readiness passed: the step completes
    (_st(P.TASK_RUNNING, check_exit=1), True),         # readiness failed
    (_st(P.TASK_RUNNING), True),                       # no readiness check: RUNNING completes
    (_st(P.TASK_FAILED), True),
    (_st(P.TASK_LOST), True),
    (_st(P.TASK_FINISHED), True),
    (_st(P.TASK_KILLED), True),
])
def test_only_statuses_that_can_create_work_wake_the_offer_loop(status, wakes):
    from dcos_commons_amd.framework.framework_scheduler import can_create_work

    assert can_create_work(status) is wakes


class _Step:
    def __init__(self, pending):
        self.pending = pending

    def is_pending(self):
        return self.pending

    def is_prepared(self):
        return False


@pytest.mark.parametrize("flag,pending,hold_s,revives", [
    (True, False, 10.0, 0),    # the new work launched from offers in hand: no revive
    (True, True, 10.0, 1),     # a candidate is still unmatched: revive for more offers
    (False, False, 10.0, 1),   # reference: every new work set revives
    # no held offers: leftovers were long-declined, and this revive is what clears their filters
    (True, False, 0.0, 1),
])
def test_revive_only_for_unmatched_new_work(drv, flag, pending, hold_s, revives):
    client = Client(status=ClientStatusResponse.launching(True))
    client.candidate_steps = [_Step(pending)]
    p = processor(client, revive_only_unmatched=flag, hold_s=hold_s).disable_threading()
    p.start()
    p.enqueue([offer("a")])
    assert drv.revives == revives


def test_scheduler_process_switch_interval_flag():
    import sys

    from dcos_commons_amd.scheduler.scheduler_config import SchedulerConfig

    assert SchedulerConfig.for_testing().gil_switch_interval_s() == 0.0      # the interpreter's 5 ms
    assert SchedulerConfig.for_testing(SDK_GIL_SWITCH_INTERVAL_MS=20).gil_switch_interval_s() == 0.02
    assert sys.getswitchinterval() > 0


def test_cpu_set_flag():
    from dcos_commons_amd.scheduler.scheduler_config import SchedulerConfig, parse_cpu_list

    assert parse_cpu_list("0-3,8,10-11") == [0, 1, 2, 3, 8, 10, 11]
    assert parse_cpu_list(" 5 ") == [5]
    for bad in ("", "3-1", "-1", "a"):
        with pytest.raises(ValueError):
            parse_cpu_list(bad)
    assert SchedulerConfig.for_testing().cpu_set() is None
    assert SchedulerConfig.for_testing(SDK_CPU_SET="2,3").cpu_set() == [2, 3]


# ---------------------------------------------------------------------------------------
# relaunch kills: their end asks for a revive, not an offer cycle


def _status(tid, state):
    s = P.TaskStatus(state=state)
    s.task_id.value = tid
    return s


def test_task_killer_tracks_relaunch_kills(drv):
    task_killer.kill_task(P.TaskID(value="relaunched"), relaunch=True)
    task_killer.kill_task(P.TaskID(value="plain"))
    assert drv.kills == ["relaunched", "plain"]
    assert not task_killer.ends_relaunch_kill(_status("relaunched", P.TASK_KILLING))   # not terminal yet
    assert task_killer.ends_relaunch_kill(_status("relaunched", P.TASK_KILLED))
    assert not task_killer.ends_relaunch_kill(_status("plain", P.TASK_KILLED))
    assert task_killer.update(_status("relaunched", P.TASK_KILLED)) is False          # expected death
    assert not task_killer.ends_relaunch_kill(_status("relaunched", P.TASK_KILLED))   # consumed


class CountingClient(Client):
    def __init__(self, **kw):
        super().__init__(**kw)
        self.status_calls = 0

    def get_client_status(self):
        self.status_calls += 1
        return super().get_client_status()


def test_reoffer_wakes_for_a_revive_only(drv):
    c = CountingClient()
    from dcos_commons_amd.framework.offer_processing import TokenBucket

    p = processor(c, hold_s=10.0, event_driven=True,
                  token_bucket=TokenBucket(acquire_interval_s=5.0, burst_interval_s=1.0)).disable_threading()
    p.start()   # no thread: the cycles are driven below
    p.revive_manager.bucket.try_acquire()     # a revive just happened: the burst spacing is running
    p.reoffer_released()
    p.process_queued_offers(0.5)
    # one revive, despite the spacing (it spends a token), and no client status / evaluation pass
    assert drv.revives == 1 and c.status_calls == 0 and not p.revive_manager.revive_requested
    # a kick in the same wake-up asks for a full cycle as well
    p.reoffer_released()
    p.kick()
    p.process_queued_offers(0.5)
    assert c.status_calls == 1 and drv.revives == 2
    # without event-driven wake-ups (the reference cadence) nothing is requested
    q = processor(CountingClient())
    q.reoffer_released()
    assert q._reoffer_requests == 0


def test_relaunch_kill_status_revives_instead_of_kicking(drv):
    from dcos_commons_amd.framework.framework_scheduler import FrameworkScheduler
    from dcos_commons_amd.scheduler.mesos_event_client import TaskStatusResponse

    calls = []

    class OP:
        def kick(self):
            calls.append("kick")

        def reoffer_released(self):
            calls.append("revive")

    class C:
        def task_status(self, status):
            return TaskStatusResponse.processed()

    class Unknown:
        def task_status(self, status):
            return TaskStatusResponse.unknown_task()

    fs = FrameworkScheduler.__new__(FrameworkScheduler)
    fs.client, fs.offer_processor = C(), OP()
    task_killer.kill_task(P.TaskID(value="t1"), relaunch=True)
    fs.status_update(drv, _status("t1", P.TASK_KILLED))
    task_killer.kill_task(P.TaskID(value="t2"))
    fs.status_update(drv, _status("t2", P.TASK_KILLED))
    # any other end that releases resources: a cycle for the work it creates, and a re-offer
    assert calls == ["revive", "kick", "revive"]
    calls.clear()
    fs.status_update(drv, _status("t5", P.TASK_LOST))   # an unreachable agent releases nothing
    assert calls == ["kick"]
    # a replaced task's end arrives after its successor was stored (unknown task): a full cycle,
    # and a revive so the master offers the stale reservations for release even if we are idle
    # a FINISH/ONCE task that finished released reservations its pod's next step may reuse
    calls.clear()
    fs.status_update(drv, _status("t4", P.TASK_FINISHED))
    assert calls == ["kick", "revive"]
    calls.clear()
    fs.client = Unknown()
    task_killer.kill_task(P.TaskID(value="t3"), relaunch=True)
    fs.status_update(drv, _status("t3", P.TASK_KILLED))
    assert calls == ["kick", "revive"]


def test_reoffer_bypasses_spacing_only_above_the_bucket_floor(drv):
    """A crash loop that keeps releasing reservations drains the bucket to its floor; from there
    the re-offer revives keep the slow spacing like any other revive."""
    from dcos_commons_amd.framework.offer_processing import ReviveManager, TokenBucket

    class Clock:
        t = 1000.0

        def __call__(self):
            return self.t

    c = Clock()
    rm = ReviveManager(TokenBucket(initial=4, capacity=4, acquire_interval_s=5.0, burst_interval_s=1.0, clock=c))
    revived = 0
    for _ in range(4):
        rm.request_revive(bypass_spacing=True)
        revived += rm.revive_if_requested()
    # tokens 4 -> 2: the first two revives bypass the 1 s spacing; at the floor (2) they do not
    assert revived == 2 and rm.revive_requested and drv.revives == 2
    c.t += 5.0
    assert rm.revive_if_requested() and drv.revives == 3


def test_revive_only_wakeup_schedules_a_fallback_cycle(drv):
    """After a revive-only wake-up the loop runs a full cycle REOFFER_FALLBACK_CYCLE_S later
    unless an offer comes first (a kill the master answered with LOST frees nothing)."""
    from dcos_commons_amd.framework import offer_processing as OP

    c = CountingClient()
    p = processor(c, hold_s=10.0, event_driven=True).disable_threading()
    p.start()
    p.reoffer_released()
    t0 = time.monotonic()
    p.process_queued_offers(0.5)
    assert c.status_calls == 0 and p._fallback_cycle_at is not None
    assert p._fallback_cycle_at - t0 <= OP.REOFFER_FALLBACK_CYCLE_S + 0.05
    p.process_queued_offers(0)          # what the loop runs when the fallback time comes
    assert c.status_calls == 1 and p._fallback_cycle_at is None


def test_readiness_result_kicks_only_when_a_cycle_can_do_something(drv):
    """A RUNNING status with its readiness result asks the client whether an offer cycle could
    find work; other states keep their routing (a terminal status always wakes the loop)."""
    from dcos_commons_amd.framework.framework_scheduler import FrameworkScheduler
    from dcos_commons_amd.scheduler.mesos_event_client import TaskStatusResponse

    calls = []

    class OP:
        def kick(self):
            calls.append("kick")

        def reoffer_released(self):
            calls.append("revive")

    class C:
        useful = False

        def task_status(self, status):
            return TaskStatusResponse.processed()

        def offer_cycle_useful(self):
            return self.useful

    def ready(tid):
        s = _status(tid, P.TASK_RUNNING)
        s.check_status.type = P.CheckInfo.COMMAND
        s.check_status.command.exit_code = 0
        return s

    fs = FrameworkScheduler.__new__(FrameworkScheduler)
    fs.client, fs.offer_processor = C(), OP()
    fs.status_update(drv, ready("a"))
    assert calls == []                                  # other launched steps still pending
    fs.client.useful = True
    fs.status_update(drv, ready("b"))
    assert calls == ["kick"]
    calls.clear()
    fs.client.useful = False
    fs.status_update(drv, _status("c", P.TASK_FAILED))   # a failure always wakes the loop
    assert calls == ["kick", "revive"]


def test_offer_cycle_useful_follows_the_plans():
    """False only while every incomplete step is launched and waiting for its task."""
    from dcos_commons_amd.scheduler.abstract_scheduler import AbstractScheduler
    from dcos_commons_amd.scheduler.plan.status import Status

    class Step:
        def __init__(self, st):
            self.st = st

        def get_status(self):
            return self.st

    class Node:
        def __init__(self, children):
            self.children = children

        def get_children(self):
            return self.children

    class PM:
        def __init__(self, *statuses):
            self.plan = Node([Node([Step(s) for s in statuses])])

        def get_plan(self):
            return self.plan

    class Coord:
        def __init__(self, *pms):
            self.pms = pms

        def get_plan_managers(self):
            return list(self.pms)

    def useful(*pms):
        s = AbstractScheduler.__new__(AbstractScheduler)
        s.plan_coordinator = Coord(*pms)
        return s.offer_cycle_useful()

    assert not useful(PM(Status.COMPLETE, Status.STARTED, Status.STARTING), PM())
    assert useful(PM(Status.COMPLETE, Status.STARTED, Status.PENDING))        # a step to launch
    assert useful(PM(Status.STARTED), PM(Status.WAITING))                     # e.g. held back by a conflict
    assert useful(PM(Status.COMPLETE, Status.COMPLETE), PM())                 # all done: time to suppress
    assert useful(PM(Status.STARTED, Status.DELAYED))


def test_multi_service_offer_cycle_useful_is_any_service():
    from dcos_commons_amd.scheduler.multi import MultiServiceEventClient

    class S:
        def __init__(self, useful):
            self.useful = useful

        def offer_cycle_useful(self):
            return self.useful

    class M:
        def __init__(self, services):
            self.services = services

        def all_services(self):
            return self.services

    c = MultiServiceEventClient.__new__(MultiServiceEventClient)
    c.manager = M([])
    assert c.offer_cycle_useful()                     # nothing left: deregistration may proceed
    c.manager = M([S(False), S(False)])
    assert not c.offer_cycle_useful()
    c.manager = M([S(False), S(True)])                # e.g. a service waiting on the offer discipline
    assert c.offer_cycle_useful()
    c.manager = M([S(False), object()])               # a service without the predicate: always
    assert c.offer_cycle_useful()


@pytest.mark.parametrize("hold_s", [0.0, 10.0])
def test_early_reoffer_revive_keeps_the_work_set_revive_after_a_long_decline(drv, hold_s):
    """a cycle that starts with the re-offer REVIVE (released reservations) and finds
    new work asks for a revive of its own. With held offers (hold_s > 0) that second revive would
    only repeat the first. With hold_s == 0 the cycle declines its leftovers for an hour, and only
    a REVIVE issued after that decline clears those filters, so it must not be cancelled."""
    c = Client(status=ClientStatusResponse.launching(True))
    p = processor(c, hold_s=hold_s, event_driven=True).disable_threading()
    p.start()
    p.reoffer_released()
    p.enqueue([offer("a")])
    if hold_s == 0:
        assert drv.declines == [(["a"], 3600)]
        # the work-set revive survives the cycle: sent now or, when the spacing holds it, pending
        assert drv.revives == 2 or (drv.revives == 1 and p.revive_manager.revive_requested)
    else:
        assert drv.declines == [] and drv.revives == 1 and not p.revive_manager.revive_requested
