"""Status callbacks of a network driver wait for a running offer cycle (``OfferProcessor.
wait_cycle_idle``, ``SDK_STATUS_CYCLE_WAIT_MS``): bounded, skipped when no cycle runs, and wired by
``FrameworkScheduler`` only into drivers that offer the gate (in-process masters deliver from their
own threads and get none)."""
import threading
import time

from dcos_commons_amd.framework.framework_scheduler import FrameworkScheduler
from dcos_commons_amd.framework.offer_processing import OfferProcessor
from dcos_commons_amd.mesos import protos as P
from dcos_commons_amd.mesos.http_driver import V1HttpSchedulerDriver
from dcos_commons_amd.scheduler.scheduler_config import SchedulerConfig


def _processor():
    return OfferProcessor(client=None, persister=None)


def test_wait_returns_at_once_without_a_cycle():
    p = _processor()
    t0 = time.monotonic()
    p.wait_cycle_idle(5.0)
    assert time.monotonic() - t0 < 0.5


def test_wait_blocks_until_the_cycle_ends_and_is_bounded():
    p = _processor()
    with p._cycle_cv:
        p._cycle_active = True
    done = threading.Event()

    def waiter():
        p.wait_cycle_idle(5.0)
        done.set()
    threading.Thread(target=waiter, daemon=True).start()
    assert not done.wait(0.2)
    with p._cycle_cv:
        p._cycle_active = False
        p._cycle_cv.notify_all()
    assert done.wait(2.0)
    # a cycle that does not end: the wait gives up after its bound
    with p._cycle_cv:
        p._cycle_active = True
    t0 = time.monotonic()
    p.wait_cycle_idle(0.1)
    assert 0.09 <= time.monotonic() - t0 < 1.0


class _Sched:
    def __init__(self):
        self.got = []

    def status_updates(self, driver, statuses):
        self.got.append(("batch", len(statuses)))

    def status_update(self, driver, status):
        self.got.append(("one", status.task_id.value))


def test_driver_runs_the_gate_before_every_status_callback():
    sched = _Sched()
    d = V1HttpSchedulerDriver("http://127.0.0.1:1", sched, P.FrameworkInfo(name="x"))
    d.implicit_acknowledgements = False
    order = []
    d.set_status_gate(lambda: order.append(len(sched.got)))
    st = P.TaskStatus(state=P.TASK_RUNNING)
    st.task_id.value = "t1"
    d._on_updates([st])
    d._on_updates([st, st])
    ev = P.Event(type=P.Event.UPDATE)
    ev.update.status.CopyFrom(st)
    d._on_event(ev)
    assert sched.got == [("one", "t1"), ("batch", 2), ("one", "t1")]
    assert order == [0, 1, 2]      # each gate ran before its callback


def test_framework_scheduler_wires_the_gate_only_when_enabled():
    class Drv:
        gate = None

        def set_status_gate(self, g):
            self.gate = g
    for wait_ms, wired in (("100", True), ("0", False)):
        cfg = SchedulerConfig.for_testing(SDK_STATUS_CYCLE_WAIT_MS=wait_ms)
        fs = FrameworkScheduler([], cfg, None, None, None, offer_processor=_processor())
        drv = Drv()
        fs._gate_statuses(drv)
        assert (drv.gate is not None) == wired
        if wired:
            drv.gate()          # no cycle running: returns at once
    # a driver without the hook (the in-process LocalMaster's) is left alone
    FrameworkScheduler([], SchedulerConfig.for_testing(), None, None, None,
                       offer_processor=_processor())._gate_statuses(object())


def test_no_gate_with_a_remote_persister():
    """With ZooKeeper state the cycle and the statuses both wait on round trips: no gate."""
    class Remote:
        remote = True

    class Drv:
        gate = None

        def set_status_gate(self, g):
            self.gate = g
    fs = FrameworkScheduler([], SchedulerConfig.for_testing(), Remote(), None, None, offer_processor=_processor())
    drv = Drv()
    fs._gate_statuses(drv)
    assert drv.gate is None
