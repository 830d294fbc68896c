"""Scheduler metrics (Dropwizard-style registry) with JSON, Prometheus and StatsD export.

Reference: sdk/.../metrics/Metrics.java:26-209 and PlanReporter.java:19-21. Metric names are the
reference's: ``offers.received``, ``offers.processed``, ``offers.process`` (timer), ``revives``,
``revives.throttles``, ``declines.short``, ``declines.long``, ``suppresses``, ``is_suppressed``,
``operation.<type>``, ``task_status.<state>``, ``plan_status.<plan>`` (-1/0/1/2).
MI355X additions: ``deploy.plan_complete_seconds`` and ``recovery.mttr_seconds`` histograms fed
by the benchmark harness and the plan reporter.
"""
from __future__ import annotations

import socket
import threading
import time
from typing import Dict, List, Optional

from dcos_commons_amd.mesos import protos as P

RECEIVED_OFFERS = "offers.received"
PROCESSED_OFFERS = "offers.processed"
PROCESS_OFFERS = "offers.process"
REVIVES = "revives"
REVIVE_THROTTLES = "revives.throttles"
DECLINE_SHORT = "declines.short"
DECLINE_LONG = "declines.long"
SUPPRESSES = "suppresses"
IS_SUPPRESSED = "is_suppressed"


class Timer:
    def __init__(self):
        self.count = 0
        self.total = 0.0
        self.min = None
        self.max = None
        self.samples: List[float] = []

    def update(self, seconds: float) -> None:
        self.count += 1
        self.total += seconds
        self.min = seconds if self.min is None else min(self.min, seconds)
        self.max = seconds if self.max is None else max(self.max, seconds)
        self.samples.append(seconds)
        if len(self.samples) > 1028:
            del self.samples[:len(self.samples) - 1028]

    def snapshot(self) -> dict:
        s = sorted(self.samples)

        def q(p):
            if not s:
                return 0.0
            return s[min(len(s) - 1, int(p * len(s)))]
        return {"count": self.count, "max": self.max or 0.0, "mean": (self.total / self.count) if self.count else 0.0,
                "min": self.min or 0.0, "p50": q(0.5), "p75": q(0.75), "p95": q(0.95), "p99": q(0.99),
                "duration_units": "seconds"}

    class _Ctx:
        def __init__(self, t):
            self.t = t
            self.start = time.perf_counter()

        def stop(self):
            self.t.update(time.perf_counter() - self.start)

        def __enter__(self):
            return self

        def __exit__(self, *exc):
            self.stop()

    def time(self):
        return Timer._Ctx(self)


PLAN_STATUS_VALUES = {"ERROR": -1, "COMPLETE": 0, "WAITING": 1, "PENDING": 1, "IN_PROGRESS": 2, "PREPARED": 2,
                      "STARTED": 2, "STARTING": 2}


class MetricRegistry:
    def __init__(self):
        self._lock = threading.Lock()
        self.counters: Dict[str, int] = {}
        self.gauges: Dict[str, object] = {}
        self.timers: Dict[str, Timer] = {}

    def inc(self, name: str, amount: int = 1) -> None:
        with self._lock:
            self.counters[name] = self.counters.get(name, 0) + amount

    def counter(self, name: str) -> int:
        return self.counters.get(name, 0)

    def gauge(self, name: str, value) -> None:
        with self._lock:
            self.gauges[name] = value

    def timer(self, name: str) -> Timer:
        with self._lock:
            t = self.timers.get(name)
            if t is None:
                t = self.timers[name] = Timer()
            return t

    def to_json(self) -> dict:
        with self._lock:
            gauges = {}
            for k, v in self.gauges.items():
                gauges[k] = {"value": v() if callable(v) else v}
            return {
                "version": "4.0.0",
                "gauges": gauges,
                "counters": {k: {"count": v} for k, v in self.counters.items()},
                "histograms": {},
                "meters": {},
                "timers": {k: t.snapshot() for k, t in self.timers.items()},
            }

    def to_prometheus(self) -> str:
        lines = []

        def pname(n):
            return n.replace(".", "_").replace("-", "_")
        snap = self.to_json()
        for k, v in sorted(snap["counters"].items()):
            lines.append(f"# TYPE {pname(k)} counter")
            lines.append(f"{pname(k)} {v['count']}")
        for k, v in sorted(snap["gauges"].items()):
            val = v["value"]
            if isinstance(val, bool):
                val = 1 if val else 0
            lines.append(f"# TYPE {pname(k)} gauge")
            lines.append(f"{pname(k)} {val}")
        for k, v in sorted(snap["timers"].items()):
            n = pname(k)
            lines.append(f"# TYPE {n} summary")
            for q in ("p50", "p75", "p95", "p99"):
                lines.append(f'{n}{{quantile="0.{q[1:]}"}} {v[q]}')
            lines.append(f"{n}_count {v['count']}")
            lines.append(f"{n}_sum {v['mean'] * v['count']}")
        return "\n".join(lines) + "\n"

    def reset(self) -> None:
        with self._lock:
            self.counters.clear()
            self.gauges.clear()
            self.timers.clear()


REGISTRY = MetricRegistry()
_is_suppressed = False
REGISTRY.gauge(IS_SUPPRESSED, lambda: _is_suppressed)


def increment_received_offers(n: int) -> None:
    REGISTRY.inc(RECEIVED_OFFERS, n)


def increment_processed_offers(n: int) -> None:
    REGISTRY.inc(PROCESSED_OFFERS, n)


def process_offers_timer():
    return REGISTRY.timer(PROCESS_OFFERS).time()


def not_suppressed() -> None:
    global _is_suppressed
    _is_suppressed = False


def increment_suppresses() -> None:
    global _is_suppressed
    REGISTRY.inc(SUPPRESSES)
    _is_suppressed = True


def increment_revives() -> None:
    REGISTRY.inc(REVIVES)


def increment_revive_throttles() -> None:
    REGISTRY.inc(REVIVE_THROTTLES)


def increment_declines_short(n: int) -> None:
    REGISTRY.inc(DECLINE_SHORT, n)


def increment_declines_long(n: int) -> None:
    REGISTRY.inc(DECLINE_LONG, n)


def increment_recommendations(recs) -> None:
    for r in recs:
        op = r.get_operation()
        if op is not None:
            REGISTRY.inc("operation." + P.Offer.Operation.Type.Name(op.type).lower())


def record_status(status: P.TaskStatus) -> None:
    REGISTRY.inc("task_status." + P.TaskState.Name(status.state).lower())


def update_plan_status(namespace: Optional[str], plan_name: str, status) -> None:
    name = f"plan_status.{namespace}.{plan_name}" if namespace else f"plan_status.{plan_name}"
    REGISTRY.gauge(name, PLAN_STATUS_VALUES.get(str(status), 1))


class PlanReporter:
    """Scrapes plan statuses into ``plan_status.*`` gauges every 5 s (PlanReporter.java:21)."""

    def __init__(self, namespace: Optional[str], managers, period_s: float = 5.0, start_thread: bool = True):
        self.namespace = namespace
        self.managers = list(managers)
        self.has_scraped = False
        self._stop = threading.Event()
        if start_thread:
            self._thread = threading.Thread(target=self._loop, args=(period_s,), daemon=True, name="PlanReporter")
            self._thread.start()

    def scrape(self) -> None:
        for m in self.managers:
            p = m.get_plan()
            update_plan_status(self.namespace, p.get_name(), p.get_status())
        self.has_scraped = True

    def _loop(self, period: float) -> None:
        while not self._stop.is_set():
            try:
                self.scrape()
            except Exception:  # noqa: BLE001
                pass
            self._stop.wait(period)

    def stop(self) -> None:
        self._stop.set()


class StatsDReporter:
    """Pushes counters/gauges as StatsD UDP datagrams every ``interval_s`` (Metrics.configureStatsd)."""

    def __init__(self, host: str, port: int, interval_s: float = 10.0, prefix: str = ""):
        self.addr = (host, int(port))
        self.interval = interval_s
        self.prefix = prefix
        self._sock = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
        self._stop = threading.Event()
        self._last: Dict[str, int] = {}
        self._thread = threading.Thread(target=self._loop, daemon=True, name="StatsD")
        self._thread.start()

    def report(self) -> None:
        snap = REGISTRY.to_json()
        out = []
        for k, v in snap["counters"].items():
            delta = v["count"] - self._last.get(k, 0)
            self._last[k] = v["count"]
            out.append(f"{self.prefix}{k}:{delta}|c")
        for k, v in snap["gauges"].items():
            val = v["value"]
            if isinstance(val, bool):
                val = int(val)
            out.append(f"{self.prefix}{k}:{val}|g")
        for k, v in snap["timers"].items():
            out.append(f"{self.prefix}{k}:{v['mean'] * 1000:.3f}|ms")
        for line in out:
            try:
                self._sock.sendto(line.encode(), self.addr)
            except OSError:
                pass

    def _loop(self) -> None:
        while not self._stop.wait(self.interval):
            self.report()

    def stop(self) -> None:
        self._stop.set()


def configure_statsd(scheduler_config) -> Optional[StatsDReporter]:
    host, port = scheduler_config.statsd_host(), scheduler_config.statsd_port()
    if not host or not port:
        return None
    return StatsDReporter(host, port, scheduler_config.statsd_poll_interval_s())
