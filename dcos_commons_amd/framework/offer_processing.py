"""The offer-processing loop and its helpers.

Reference: sdk/.../framework/{OfferProcessor,OfferQueue,ReviveManager,TokenBucket,OfferAccepter,
ImplicitReconciler}.java. Per cycle: take queued offers -> client status (revive / suppress /
remove) -> client.offers -> unexpected-resource cleanup (DESTROY before UNRESERVE) -> decline ->
ACCEPT (one call per agent, RESERVE/CREATE/.../LAUNCH_GROUP in order) -> revive if requested.

MI355X-build changes (all opt-in knobs, reference behaviour is the default of each knob):
* **event-driven wake-up** -- ``kick()`` (called on every status update) wakes the loop
  immediately instead of waiting out the 5 s offer poll (OfferProcessor.java:46);
* **bounded offer holding** -- while the service is WORKING, unused offers can be held for up to
  ``hold_s`` and re-evaluated as plans advance instead of being declined for an hour and
  re-obtained through a (rate-limited) REVIVE. ``hold_s=0`` is the reference behaviour;
* **launch streaming** -- each matched step is recorded and ACCEPTed before the next step is
  evaluated (``stream_launches``), so a large parallel deploy starts its first pods while the
  rest are still being matched. The reference sends every ACCEPT after the whole cycle.
"""
from __future__ import annotations

import collections
import logging
import threading
import time
from typing import Callable, Dict, List, Optional, Tuple

from dcos_commons_amd import metrics, trace
from dcos_commons_amd.mesos import protos as P
from dcos_commons_amd.offer import constants
from dcos_commons_amd.offer.recommendations import DestroyOfferRecommendation, UnreserveOfferRecommendation
from dcos_commons_amd.scheduler.mesos_event_client import (
    ClientStatusResult,
    IdleRequest,
    OfferResult,
    UnexpectedResult,
)
from dcos_commons_amd.storage.persister_utils import clear_all_data

from . import driver
from .process_exit import ProcessExit

LOGGER = logging.getLogger(__name__)
DEFAULT_OFFER_WAIT_S = 5.0
DEFAULT_QUEUE_CAPACITY = 100
ACCEPT_FILTERS = P.Filters(refuse_seconds=1)


# after a revive-only wake-up (a relaunch kill ended), the longest wait for the re-offer before a
# full cycle re-evaluates the offers in hand
REOFFER_FALLBACK_CYCLE_S = 0.05


class OfferQueue:
    def __init__(self, capacity: int = DEFAULT_QUEUE_CAPACITY):
        self.capacity = capacity
        self._q: collections.deque = collections.deque()
        self._cond = threading.Condition()

    def offer(self, o: P.Offer) -> bool:
        with self._cond:
            if self.capacity and len(self._q) >= self.capacity:
                return False
            self._q.append(o)
            self._cond.notify_all()
            return True

    def take_all(self, wait_s: float, wake: Optional[threading.Event] = None) -> List[P.Offer]:
        with self._cond:
            if wake is not None and wake.is_set():
                wake.clear()  # a kick that arrived while the last cycle ran is consumed here
                wait_s = 0
            if not self._q and wait_s > 0:
                deadline = time.monotonic() + wait_s
                while not self._q:
                    if wake is not None and wake.is_set():
                        wake.clear()
                        break
                    remaining = deadline - time.monotonic()
                    if remaining <= 0:
                        break
                    self._cond.wait(min(remaining, 0.05) if wake is not None else remaining)
            out = list(self._q)
            self._q.clear()
            return out

    def notify(self) -> None:
        with self._cond:
            self._cond.notify_all()

    def remove(self, offer_id: P.OfferID) -> bool:
        with self._cond:
            before = len(self._q)
            self._q = collections.deque(o for o in self._q if o.id.value != offer_id.value)
            return len(self._q) != before

    def is_empty(self) -> bool:
        with self._cond:
            return not self._q

    def size(self) -> int:
        with self._cond:
            return len(self._q)

    def remaining_capacity(self) -> int:
        """Free slots (OfferQueue.getRemainingCapacity); unbounded queues report -1."""
        with self._cond:
            return self.capacity - len(self._q) if self.capacity else -1


class TokenBucket:
    """Revive rate limiter: capacity 256, +1 token every 256 s, >= 5 s between acquires
    (TokenBucket.java:17-24,81).

    ``burst_interval_s`` (default: same as ``acquire_interval_s``, i.e. the reference's flat
    spacing) applies instead of ``acquire_interval_s`` while more than ``burst_floor`` tokens
    (default half the capacity) remain: a healthy bucket lets a burst of new work revive promptly,
    a bucket drained by a crash loop falls back to the slow spacing. The capacity and refill rate
    bound the sustained rate either way.
    """

    def __init__(self, initial: int = 256, capacity: int = 256, increment_interval_s: float = 256.0,
                 acquire_interval_s: float = 5.0, clock: Callable[[], float] = time.monotonic,
                 burst_interval_s: Optional[float] = None, burst_floor: Optional[int] = None):
        if initial < 0 or capacity < 1 or increment_interval_s <= 0 or acquire_interval_s < 0:
            raise ValueError("TokenBucket construction failed with invalid configuration")
        if burst_interval_s is not None and not 0 <= burst_interval_s <= acquire_interval_s:
            raise ValueError("TokenBucket burst interval must be within [0, acquire interval]")
        self.burst_interval_s = acquire_interval_s if burst_interval_s is None else burst_interval_s
        self.burst_floor = capacity // 2 if burst_floor is None else burst_floor
        self.initial = initial
        self.count = initial
        self.capacity = capacity
        self.increment_interval_s = increment_interval_s
        self.acquire_interval_s = acquire_interval_s
        self.clock = clock
        self._last_acquire: Optional[float] = None
        self._last_increment = clock()
        self._lock = threading.Lock()

    def _refill(self) -> None:
        now = self.clock()
        n = int((now - self._last_increment) // self.increment_interval_s)
        if n > 0:
            self.count = min(self.capacity, self.count + n)
            self._last_increment += n * self.increment_interval_s

    def _spacing(self) -> float:
        return self.burst_interval_s if self.count > self.burst_floor else self.acquire_interval_s

    def try_acquire(self, ignore_spacing: bool = False) -> bool:
        with self._lock:
            self._refill()
            now = self.clock()
            if self.count > 0 and (ignore_spacing or self._last_acquire is None or
                                   now - self._last_acquire >= self._spacing()):
                self.count -= 1
                self._last_acquire = now
                return True
            return False

    def seconds_until_available(self) -> float:
        """How long until ``try_acquire`` can next succeed (0 if it can now)."""
        with self._lock:
            self._refill()
            now = self.clock()
            wait = 0.0
            if self._last_acquire is not None:
                wait = max(0.0, self._spacing() - (now - self._last_acquire))
            if self.count <= 0:
                wait = max(wait, self.increment_interval_s - (now - self._last_increment))
            return wait

    def increment(self) -> None:
        """Adds one token now, up to the capacity (the reference's refill-thread tick)."""
        with self._lock:
            self.count = min(self.capacity, self.count + 1)

    def reset(self) -> None:
        with self._lock:
            self.count = self.initial
            self._last_acquire = None


class ReviveManager:
    """Revive/suppress bookkeeping (ReviveManager.java:40-150).

    ``fast_unsuppress``: the first REVIVE after a SUPPRESS is not held to the burst spacing (it
    still spends a token, so the 256-token budget bounds crash loops); spacing applies between
    revives of one working period, where revive storms happen. The reference always waits for
    the spacing, which puts up to 5 s on the MTTR of a failure that follows a recent revive.
    """

    def __init__(self, token_bucket: TokenBucket, suppress_enabled: bool = True, fast_unsuppress: bool = False):
        self.bucket = token_bucket
        self.suppress_enabled = suppress_enabled
        self.fast_unsuppress = fast_unsuppress
        self.revive_requested = False
        self.is_suppressed = False
        self._revive_bypass = False

    def notify_offers_received(self) -> None:
        self.is_suppressed = False
        metrics.not_suppressed()

    def suppress_if_active(self) -> None:
        if self.is_suppressed:
            return
        if self.suppress_enabled:
            d = driver.get_instance()
            if d is not None:
                d.suppress_offers()
            metrics.increment_suppresses()
        self.is_suppressed = True

    def request_revive_if_suppressed(self) -> None:
        if self.is_suppressed:
            self.request_revive()

    def request_revive(self, bypass_spacing: bool = False) -> None:
        """``bypass_spacing``: a one-off revive for a known event (reservations released for a
        relaunch) that is not held to the burst spacing while the bucket is above its burst floor;
        it still spends a token, and a drained bucket (a crash loop) keeps the slow spacing."""
        if bypass_spacing and self.bucket.count > self.bucket.burst_floor:
            self._revive_bypass = True
        if self.is_suppressed and self.fast_unsuppress:
            self._revive_bypass = True
        self.revive_requested = True

    def cancel_request(self) -> None:
        """The work that asked for a revive was matched with offers already in hand."""
        self.revive_requested = False
        self._revive_bypass = False

    def revive_if_requested(self) -> bool:
        """Revives if a revive is requested and the bucket allows it; True if it did."""
        if not self.revive_requested:
            return False
        if not self.bucket.try_acquire(ignore_spacing=self._revive_bypass):
            metrics.increment_revive_throttles()
            return False
        d = driver.get_instance()
        if d is not None:
            d.revive_offers()
        self.revive_requested = False
        self._revive_bypass = False
        self.is_suppressed = False
        metrics.increment_revives()
        return True


class OfferAccepter:
    """Groups operations per agent (keeping op order) and issues one ACCEPT per agent."""

    @staticmethod
    def group_by_agent(recs) -> Dict[str, list]:
        out: Dict[str, list] = {}
        for r in recs:
            out.setdefault(r.agent_id.value, []).append(r)
        return dict(sorted(out.items()))

    def accept(self, recs, members: Optional[Dict[str, List[P.Offer]]] = None) -> None:
        """``members``: merged offer id -> the real offers it stands for (``merge_agent_offers``);
        an ACCEPT on a merged offer names every member (Mesos accepts several offers of one agent
        in one call)."""
        if not recs:
            return
        with trace.span("accept", "offers", recs=len(recs)):
            self._accept(recs, members)

    def _accept(self, recs, members) -> None:
        d = driver.get_instance()
        for agent, agent_recs in self.group_by_agent(recs).items():
            ops, offer_ids, seen = [], [], set()
            for r in agent_recs:
                op = r.get_operation()
                if op is None:
                    continue
                ops.append(op)
                group = members.get(r.offer_id.value) if members else None
                for oid in ([o.id for o in group] if group else [r.offer_id]):
                    if oid.value not in seen:
                        seen.add(oid.value)
                        offer_ids.append(oid)
            if not ops:
                continue
            LOGGER.info("Sending %d operation(s) for agent %s: %s", len(ops), agent,
                        [P.Offer.Operation.Type.Name(o.type) for o in ops])
            d.accept_offers(offer_ids, ops, ACCEPT_FILTERS)


def filter_out_accepted(offers, recs) -> List[P.Offer]:
    used = {r.offer_id.value for r in recs if r.get_operation() is not None}
    return [o for o in offers if o.id.value not in used]


def to_cleanup_recommendations(offer_resources_list) -> list:
    destroys, unreserves = [], []
    for orr in offer_resources_list:
        for r in orr.resources:
            if r.HasField("disk") and r.disk.HasField("persistence"):
                destroys.append(DestroyOfferRecommendation(orr.offer, r))
            unreserves.append(UnreserveOfferRecommendation(orr.offer, r))
    return destroys + unreserves


def recycled_offers(offers, offer_resources_list):
    """Copies of ``offers`` in which every stale reservation is shown as what its UNRESERVE
    (after DESTROY) yields: the resource with its last reservation popped and no volume."""
    from dcos_commons_amd.mesos.resource_math import ResourceBag, pop_reservation, strip_volume

    stale = {}
    for orr in offer_resources_list:
        stale.setdefault(orr.offer.id.value, []).extend(orr.resources)
    out = []
    for o in offers:
        rs = stale.get(o.id.value)
        if not rs:
            out.append(o)
            continue
        c = P.Offer()
        c.CopyFrom(o)
        del c.resources[:]
        remaining = list(rs)
        alloc = None
        bag = ResourceBag()
        for r in o.resources:
            if r.HasField("allocation_info") and alloc is None:
                alloc = r.allocation_info
            match = next((i for i, x in enumerate(remaining) if x == r), None)
            bag.add(r if match is None else strip_volume(pop_reservation(r)))
            if match is not None:
                remaining.pop(match)
        # Mesos merges identical resources (e.g. the freed cpus and the offer's unreserved cpus)
        for r in bag.to_resources():
            if alloc is not None:
                r.allocation_info.CopyFrom(alloc)
            c.resources.add().CopyFrom(r)
        out.append(c)
    return out


def merge_agent_offers(offers) -> Tuple[List[P.Offer], Dict[str, List[P.Offer]]]:
    """One evaluation unit per agent: offers of the same agent are combined into a copy of the
    first (resources merged the way the master would, executor ids unioned). Returns the offers to
    evaluate and ``{merged id: [member offers]}`` for every agent that had more than one.

    Why: an agent's resources can be split across outstanding offers (a held offer plus the
    resources a finished task released, offered separately). A step that needs both (e.g. a pod's
    own reservation plus new unreserved resources for its next resource set) passes on neither
    offer alone, and would wait until the held one is declined and re-offered whole. The
    reference evaluates offers one at a time (OfferEvaluator.java:113-248) but does not hold them.
    """
    from dcos_commons_amd.mesos.resource_math import ResourceBag

    by_agent: Dict[str, List[P.Offer]] = {}
    for o in offers:
        by_agent.setdefault(o.agent_id.value, []).append(o)
    out: List[P.Offer] = []
    members: Dict[str, List[P.Offer]] = {}
    for group in by_agent.values():
        if len(group) == 1:
            out.append(group[0])
            continue
        m = P.Offer()
        m.CopyFrom(group[0])
        del m.resources[:]
        del m.executor_ids[:]
        bag, alloc, execs = ResourceBag(), None, []
        for o in group:
            for r in o.resources:
                if alloc is None and r.HasField("allocation_info"):
                    alloc = r.allocation_info
                bag.add(r)
            for e in o.executor_ids:
                if e.value not in execs:
                    execs.append(e.value)
        for r in bag.to_resources():
            if alloc is not None:
                r.allocation_info.CopyFrom(alloc)
            m.resources.add().CopyFrom(r)
        for e in execs:
            m.executor_ids.add(value=e)
        members[m.id.value] = list(group)
        out.append(m)
    return out, members


def _targeted_resource_ids(recs) -> set:
    from dcos_commons_amd.offer.resources import get_resource_id

    out = set()
    for r in recs:
        if isinstance(r, (DestroyOfferRecommendation, UnreserveOfferRecommendation)):
            rid = get_resource_id(r.resource)
            if rid is not None:
                out.add(rid)
    return out


def _drop_targeted(offer_resources_list, targeted: set):
    from dcos_commons_amd.offer.resources import get_resource_id
    from dcos_commons_amd.scheduler.mesos_event_client import OfferResources

    out = []
    for orr in offer_resources_list:
        keep = [r for r in orr.resources if get_resource_id(r) not in targeted]
        if keep:
            out.append(OfferResources(orr.offer, keep))
    return out


def decline(offers, refuse_seconds: float) -> None:
    d = driver.get_instance()
    f = P.Filters(refuse_seconds=refuse_seconds)
    for o in offers:
        d.decline_offer(o.id, f)


def decline_short(offers) -> None:
    if offers:
        decline(offers, constants.SHORT_DECLINE_SECONDS)
        metrics.increment_declines_short(len(offers))


def decline_long(offers) -> None:
    if offers:
        decline(offers, constants.LONG_DECLINE_SECONDS)
        metrics.increment_declines_long(len(offers))


class OfferProcessor:
    def __init__(self, client, persister, scheduler_config=None, token_bucket: Optional[TokenBucket] = None,
                 queue_capacity: int = DEFAULT_QUEUE_CAPACITY, offer_wait_s: Optional[float] = None,
                 hold_s: float = 0.0, event_driven: bool = False, gc_all_offers: bool = False,
                 fast_unsuppress: bool = False, merge_agent_offers: bool = False, stream_launches: bool = False,
                 revive_only_unmatched: bool = False):
        self.client = client
        self.persister = persister
        self.offer_wait_s = offer_wait_s if offer_wait_s is not None else (
            scheduler_config.offer_wait_s() if scheduler_config is not None else DEFAULT_OFFER_WAIT_S)
        suppress = scheduler_config.is_suppress_enabled() if scheduler_config is not None else True
        self.revive_manager = ReviveManager(token_bucket or TokenBucket(), suppress, fast_unsuppress)
        self.queue = OfferQueue(queue_capacity)
        self.accepter = OfferAccepter()
        self.multithreaded = True
        self.hold_s = hold_s
        self._declined_long_in_cycle = False  # some offer of the running cycle was declined for an hour
        self.event_driven = event_driven
        # reference: stale reservations are only collected from offers nothing was launched on,
        # and only while the service is WORKING (OfferProcessor.java:300-330), so a pod replaced
        # onto the same agent, or a scheduler that goes idle, leaks them until the next work.
        # gc_all_offers collects them from every offer, idle or not.
        self.gc_all_offers = gc_all_offers
        self.merge_agent_offers = merge_agent_offers
        # ACCEPT each step's launch as soon as it is matched instead of after the whole cycle
        self.stream_launches = stream_launches
        # drop a revive requested for new work when that work was matched in the same cycle. Only
        # with held offers: with hold_s == 0 the cycle's leftovers were long-declined, and that
        # revive is what clears their filters for a later relaunch of the same step (which adds no
        # new work and so asks for no revive of its own)
        self.revive_only_unmatched = revive_only_unmatched and hold_s > 0
        # (real) offer id -> (offer, hold deadline). Rescinds arrive on the driver's thread while
        # the offer thread evaluates, so the map is only touched under _held_lock, and an offer
        # rescinded mid-cycle is remembered so that the cycle does not hold it again.
        self._held: Dict[str, tuple] = {}
        self._held_lock = threading.Lock()
        self._rescinded: set = set()
        self._initialized = False
        self._prestart_lock = threading.Lock()
        self._deregistered = False
        self._in_progress = set()
        self._in_progress_lock = threading.Lock()
        self._wake = threading.Event()
        # why the loop was woken: ``kick`` asks for a full cycle, ``reoffer_released`` for a revive.
        # Requests bump a counter; the offer thread compares it with the value it last acted on,
        # so a request made while it reads is seen on the next cycle instead of being reset away.
        self._eval_requests = 0
        self._reoffer_requests = 0
        self._eval_seen = 0
        self._reoffer_seen = 0
        # after a revive-only wake-up, a full cycle runs at this time unless an offer or a kick
        # brings one sooner (a kill of a task the master did not know frees nothing to re-offer)
        self._fallback_cycle_at: Optional[float] = None
        self._stop = threading.Event()
        self._thread: Optional[threading.Thread] = None
        self.cycles = 0
        # set while a cycle evaluates offers; status callbacks of a network driver wait for it to
        # clear (``wait_cycle_idle``) rather than take the interpreter lock from the cycle
        self._cycle_cv = threading.Condition()
        self._cycle_active = False

    def disable_threading(self) -> "OfferProcessor":
        self.multithreaded = False
        return self

    def set_revive_token_bucket(self, bucket: TokenBucket) -> "OfferProcessor":
        self.revive_manager.bucket = bucket
        return self

    def prestart(self) -> None:
        """Create the loop thread before SUBSCRIBE goes out, so that thread start-up overlaps the
        registration round trip instead of delaying the event thread's reading of the first offers
        (it ran inside the ``registered`` callback: ~0.3 ms of the 1.1 ms from registration to the
        first offers on the build container). Until ``start`` the loop only waits: no offers can
        arrive before registration, and an empty cycle returns at once while not initialized."""
        with self._prestart_lock:
            if self.multithreaded and self._thread is None:
                self._thread = threading.Thread(target=self._loop, name="OfferProcessor", daemon=True)
                self._thread.start()

    def start(self) -> None:
        self.prestart()
        self._initialized = True

    def stop(self) -> None:
        self._stop.set()
        self._wake.set()
        self.queue.notify()
        if self._thread is not None:
            self._thread.join(timeout=5)

    def _loop(self) -> None:
        prewarm = getattr(self.client, "prewarm", None)
        if prewarm is not None:
            # registration to the first offers is a master round trip: build what the first
            # evaluation would otherwise build meanwhile, in steps that give the interpreter to the
            # event thread and stop once offers are queued (never fatal: the evaluation builds
            # whatever is missing)
            def stop() -> bool:
                time.sleep(0)
                return self._stop.is_set() or not self.queue.is_empty()
            try:
                prewarm(stop)
            except Exception:  # noqa: BLE001
                LOGGER.debug("offer-evaluation prewarm failed", exc_info=True)
        while not self._stop.is_set():
            try:
                wait = self.offer_wait_s
                if self.event_driven and self.revive_manager.revive_requested:
                    # a throttled revive is retried the moment the bucket allows it, not at the
                    # next offer poll
                    wait = min(wait, max(0.001, self.revive_manager.bucket.seconds_until_available()))
                fallback = self._fallback_cycle_at
                if fallback is not None:
                    wait = min(wait, max(0.0, fallback - time.monotonic()))
                self.process_queued_offers(wait)
            except Exception as e:  # noqa: BLE001
                LOGGER.exception("Error encountered when processing offers, exiting to avoid zombie state")
                ProcessExit.exit(ProcessExit.ERROR, e)
                return

    def kick(self) -> None:
        """Wake the loop now (status update / plan change) instead of at the next offer poll."""
        if self.event_driven:
            self._eval_requests += 1
            self._wake.set()
            self.queue.notify()

    def reoffer_released(self) -> None:
        """A task ended (finished, failed, killed; a kill issued for a relaunch included) and
        released reservations the plans reuse in place. The master offers released resources
        again at its next allocation; wake the loop for a REVIVE (an allocation now) that is not
        held to the burst spacing while the bucket is above its floor. The offer that carries them
        wakes the loop for the relaunch. The revive is taken on the offer thread, like every
        revive (OfferProcessor.java:300-309)."""
        if self.event_driven:
            self._reoffer_requests += 1
            self._wake.set()
            self.queue.notify()

    def enqueue(self, offers) -> None:
        with self._in_progress_lock:
            self._in_progress.update(o.id.value for o in offers)
        for o in offers:
            if not self.queue.offer(o):
                LOGGER.warning("Offer queue is full: Declining offer and removing from in progress: '%s'", o.id.value)
                decline_short([o])
                with self._in_progress_lock:
                    self._in_progress.discard(o.id.value)
        if not self.multithreaded:
            self.process_queued_offers(0)

    def dequeue(self, offer_id: P.OfferID) -> None:
        """The master rescinded ``offer_id``: drop it from the queue and from the held set."""
        self.queue.remove(offer_id)
        with self._held_lock:
            self._held.pop(offer_id.value, None)
            self._rescinded.add(offer_id.value)

    def held_offer_ids(self) -> List[str]:
        with self._held_lock:
            return list(self._held)

    def await_offers_processed(self, timeout_s: float = 5.0) -> None:
        deadline = time.monotonic() + timeout_s
        while time.monotonic() < deadline:
            with self._in_progress_lock:
                if not self._in_progress:
                    return
            time.sleep(0.01)
        raise TimeoutError("Timed out waiting for offers to be processed")

    def process_queued_offers(self, wait_s: float) -> None:
        with self._held_lock:
            # rescinds from earlier cycles concern offers that are gone by now; from here on, a
            # rescind of an offer this cycle takes is recorded and honoured when the cycle ends
            self._rescinded.clear()
        new_offers = self.queue.take_all(wait_s, self._wake if self.event_driven else None)
        if self._stop.is_set():
            return
        seen, self._reoffer_seen = self._reoffer_seen, self._reoffer_requests
        reoffer = seen != self._reoffer_seen
        seen, self._eval_seen = self._eval_seen, self._eval_requests
        eval_wake = seen != self._eval_seen
        if reoffer and not new_offers and not eval_wake:
            self._reoffer_revive()
            self._fallback_cycle_at = time.monotonic() + REOFFER_FALLBACK_CYCLE_S
            return
        self._fallback_cycle_at = None
        # released reservations: the REVIVE goes out before the cycle, so the master allocates them
        # while the cycle runs instead of after it
        revived_early = reoffer and self._reoffer_revive()
        self._declined_long_in_cycle = False
        now = time.monotonic()
        with self._held_lock:
            held = [o for o, _ in self._held.values()]
        offers = held + new_offers
        self.cycles += 1
        try:
            if new_offers:
                self.revive_manager.notify_offers_received()
            if not offers and not self._initialized:
                return
            if self._deregistered:
                return
            with metrics.process_offers_timer(), trace.span("offer_cycle", "offers", new=len(new_offers),
                                                               held=len(held)) as sp:
                if self._check_status():
                    with self._cycle_cv:
                        self._cycle_active = True
                    try:
                        self._evaluate(offers, now)
                    finally:
                        with self._cycle_cv:
                            self._cycle_active = False
                            self._cycle_cv.notify_all()
                    sp.set(working=True)
                    if self.revive_only_unmatched and self.revive_manager.revive_requested and \
                            self._candidates_all_launched():
                        # the new work was matched in this very cycle: asking the master for more
                        # offers would only bring back this cycle's leftovers for another pass
                        self.revive_manager.cancel_request()
                    if getattr(self.client, "consume_recheck_request", None) is not None and \
                            self.client.consume_recheck_request():
                        # the client started work that changes its status (e.g. uninstall's
                        # deregister step): re-check now rather than at the next offer poll
                        self._eval_requests += 1
                        self._wake.set()
                elif self._deregistered:
                    # the framework was just torn down: its offers went with it
                    with self._held_lock:
                        self._held.clear()
                    return
                elif offers:
                    with self._held_lock:
                        self._held.clear()
                    if self.gc_all_offers:
                        offers = self._collect_garbage(offers)
                    decline_long(offers)
                    self._declined_long_in_cycle = True
            if revived_early and (self.hold_s > 0 or not self._declined_long_in_cycle):
                # the master has allocated everything available since that REVIVE: a revive this
                # cycle asked for (new work) would only repeat it. Not when this cycle declined
                # offers for an hour (hold_s == 0): only a REVIVE issued after that decline clears
                # its filters, so the cycle's own work-set revive must still go out
                self.revive_manager.cancel_request()
            elif reoffer:
                # throttled before the cycle: requested again after the cycle's own revive
                # bookkeeping, so neither a suppress nor a cancelled work-set revive drops it
                self.revive_manager.request_revive(bypass_spacing=True)
            self.revive_manager.revive_if_requested()
        finally:
            metrics.increment_processed_offers(len(new_offers))
            with self._in_progress_lock:
                for o in new_offers:
                    self._in_progress.discard(o.id.value)

    def wait_cycle_idle(self, timeout_s: float) -> bool:
        """Blocks while an offer cycle is evaluating, for at most ``timeout_s``; True if it waited.

        The scheduler's threads share one interpreter lock. A status batch handled while a cycle
        runs takes that lock whenever the cycle releases it (every ACCEPT written to the master
        socket releases it), and the cycle then waits for the whole batch: on the MI355X box an
        8-pod cycle ran 7.2 ms of wall time for 4.9 ms of its own CPU, the rest spent behind the
        first pods' STARTING/RUNNING updates (profiles/split_timeline_n8_r06_box.txt). Nothing in
        a cycle waits for a status, so the statuses that queue up meanwhile are handled in one
        batch when it ends, and the last pod's launch leaves that much earlier."""
        with self._cycle_cv:
            if not self._cycle_active:
                return False
            self._cycle_cv.wait_for(lambda: not self._cycle_active, timeout_s)
            return True

    def _reoffer_revive(self) -> bool:
        self.revive_manager.request_revive(bypass_spacing=True)
        return self.revive_manager.revive_if_requested()

    def _candidates_all_launched(self) -> bool:
        steps = getattr(self.client, "candidate_steps", None)
        if not steps:
            return False
        return not any(s.is_pending() or s.is_prepared() for s in steps)

    def _check_status(self) -> bool:
        resp = self.client.get_client_status()
        if resp.result == ClientStatusResult.WORKING:
            if resp.has_new_work:
                self.revive_manager.request_revive()
            else:
                self.revive_manager.request_revive_if_suppressed()
            return True
        if resp.idle_request == IdleRequest.NONE:
            self.revive_manager.suppress_if_active()
        elif resp.idle_request == IdleRequest.REMOVE_CLIENT:
            self._deregistered = True
            self._destroy_framework()
        elif resp.idle_request == IdleRequest.START_UNINSTALL:
            raise RuntimeError("Got unsupported START_UNINSTALL response. This should have been handled by a "
                               "MultiServiceEventClient")
        return False

    def _collect_garbage(self, offers):
        """Idle path: release unexpected reservations, return the offers still unused."""
        un = self.client.get_unexpected_resources(offers)
        if un.result != UnexpectedResult.PROCESSED:
            return offers
        recs = to_cleanup_recommendations(un.offer_resources)
        metrics.increment_recommendations(recs)
        self.accepter.accept(recs)
        return filter_out_accepted(offers, recs)

    def _evaluate(self, offers, now: float) -> None:
        members: Dict[str, List[P.Offer]] = {}
        if self.merge_agent_offers:
            offers, members = merge_agent_offers(offers)

        def real(os_):
            return [m for o in os_ for m in members.get(o.id.value, (o,))]

        pre_cleanup = []
        cleanup_result = UnexpectedResult.PROCESSED
        eval_offers = offers
        if self.gc_all_offers and offers:
            # Reservation recycling: stale reservations are released at the head of the same
            # ACCEPT that may re-reserve them (Mesos applies an ACCEPT's operations in order), so
            # a replaced pod can land on the resources of its predecessor without waiting for
            # another offer round (reference: UNRESERVE in one cycle, re-offer after the 1 s
            # accept filter and the next allocation, OfferProcessor.java:300-330).
            un = self.client.get_unexpected_resources(offers)
            cleanup_result = un.result
            if un.result == UnexpectedResult.PROCESSED and un.offer_resources:
                pre_cleanup = to_cleanup_recommendations(un.offer_resources)
                eval_offers = recycled_offers(offers, un.offer_resources)
        streamed_pre = set()
        stream = None
        if self.stream_launches:
            pre_by_offer: Dict[str, list] = {}
            for r in pre_cleanup:
                pre_by_offer.setdefault(r.offer_id.value, []).append(r)

            def stream(recs):
                # the agent's stale-reservation cleanup goes at the head of the same ACCEPT
                head = []
                for oid in {r.offer_id.value for r in recs}:
                    for r in pre_by_offer.pop(oid, ()):
                        streamed_pre.add(id(r))
                        head.append(r)
                metrics.increment_recommendations(head + list(recs))
                self.accepter.accept(head + list(recs), members)
        resp = self.client.offers(eval_offers, launch_stream=stream) if stream is not None else \
            self.client.offers(eval_offers)
        cleanup_recs = []
        unused = filter_out_accepted(offers, list(resp.recommendations) + pre_cleanup)
        if not self.gc_all_offers and unused:
            un = self.client.get_unexpected_resources(unused)
            cleanup_result = un.result
            cleanup_recs = to_cleanup_recommendations(un.offer_resources)
            unused = filter_out_accepted(unused, cleanup_recs)
        used = {o.id.value for o in real(offers)} - {o.id.value for o in real(unused)}
        unused = real(unused)
        to_decline_short, to_decline_long = [], []
        with self._held_lock:
            for oid in used:
                self._held.pop(oid, None)
            # a rescinded offer is gone from the master: neither held nor declined
            unused = [o for o in unused if o.id.value not in self._rescinded]
            if unused:
                if resp.result == OfferResult.PROCESSED and cleanup_result == UnexpectedResult.PROCESSED:
                    if self.hold_s > 0:
                        for o in unused:
                            prev = self._held.get(o.id.value)
                            deadline = prev[1] if prev is not None else now + self.hold_s
                            if deadline <= now:
                                self._held.pop(o.id.value, None)
                                to_decline_short.append(o)
                            else:
                                self._held[o.id.value] = (o, deadline)
                    else:
                        to_decline_long = unused
                else:
                    for o in unused:
                        self._held.pop(o.id.value, None)
                    to_decline_short = unused
        decline_short(to_decline_short)
        decline_long(to_decline_long)
        self._declined_long_in_cycle = self._declined_long_in_cycle or bool(to_decline_long)
        if resp.streamed:
            all_recs = [r for r in pre_cleanup if id(r) not in streamed_pre] + cleanup_recs
        else:
            all_recs = pre_cleanup + list(resp.recommendations) + cleanup_recs
        metrics.increment_recommendations(all_recs)
        self.accepter.accept(all_recs, members)

    def release_held(self) -> None:
        """Decline every held offer (e.g. when the scheduler goes idle or stops)."""
        with self._held_lock:
            held = [o for o, _ in self._held.values()]
            self._held.clear()
        decline_short(held)

    def _destroy_framework(self) -> None:
        try:
            clear_all_data(self.persister)
        except Exception as e:  # noqa: BLE001
            raise RuntimeError("Failed to delete all persister data") from e
        d = driver.get_instance()
        if d is not None:
            d.teardown()
            d.stop(False)
        self.client.unregistered()


class ImplicitReconciler:
    """Periodic ``reconcileTasks([])`` (delay 0, period 1 h by default)."""

    def __init__(self, delay_s: float = 0.0, period_s: float = 3600.0):
        self.delay_s = delay_s
        self.period_s = period_s
        self.multithreaded = True
        self.started = False
        self._stop = threading.Event()
        self._go = threading.Event()
        self._prestart_lock = threading.Lock()
        self._thread = None

    def disable_threading(self) -> "ImplicitReconciler":
        self.multithreaded = False
        return self

    @staticmethod
    def _reconcile() -> None:
        try:
            d = driver.get_instance()
            if d is not None:
                d.reconcile_tasks([])
        except Exception:  # noqa: BLE001
            LOGGER.exception("Failed to trigger implicit reconciliation")

    def prestart(self) -> None:
        """Create the thread ahead of registration (see ``OfferProcessor.prestart``); it waits for
        ``start`` before its first delay."""
        with self._prestart_lock:
            if self.multithreaded and self._thread is None:
                self._thread = threading.Thread(target=self._loop, name="ImplicitReconciler", daemon=True)
                self._thread.start()

    def _loop(self) -> None:
        self._go.wait()
        if self._stop.wait(self.delay_s):
            return
        while True:
            self._reconcile()
            if self._stop.wait(self.period_s):
                return

    def start(self) -> None:
        if self.started:
            raise RuntimeError("Start was already called")
        self.started = True
        if not self.multithreaded:
            self._reconcile()
            return
        self._go.set()
        self.prestart()

    def stop(self) -> None:
        self._stop.set()
        self._go.set()
        self.started = False
