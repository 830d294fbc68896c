"""Chrome-trace spans for the scheduler's hot paths.

The reference has no tracer: its only timing is the ``offers.process`` timer around each offer
cycle (sdk/scheduler/src/main/java/com/mesosphere/sdk/framework/OfferProcessor.java:327-337,
metrics/Metrics.java:114), and everything else is log lines plus the debug trackers
(SURVEY.md §5.1). Deploy-to-COMPLETE time is spent in the offer cycle, in step evaluation and in
persister writes, so this module records one span for each of those:

* ``offer_cycle``   one ``OfferProcessor.process_queued_offers`` pass (offers in, recs out)
* ``evaluate``      one ``OfferEvaluator.evaluate`` call (one step against the cycle's offers)
* ``persister.*``   every Persister operation (wrapped by :class:`TracingPersister`)
* ``status``        one TaskStatus through ``FrameworkScheduler.status_update``
* ``accept``        the ACCEPT calls of one cycle

Events use the Chrome trace-event format (``ph: "X"`` complete events, microsecond clock), so a
dump opens directly in Perfetto or ``chrome://tracing``. Recording is off unless
``SDK_TRACE=1`` or ``SDK_TRACE_FILE=<path>`` is set, and a disabled :func:`span` costs one
attribute read plus a shared no-op context manager. The buffer is a bounded ring
(``SDK_TRACE_MAX_EVENTS``, default 200,000) so a long-running scheduler cannot grow without bound.
``GET /v1/debug/trace`` serves the buffer; ``SDK_TRACE_FILE`` is also written at exit.
"""
from __future__ import annotations

import atexit
import collections
import json
import os
import threading
import time
from typing import Any, Dict, List, Mapping, Optional

from dcos_commons_amd.storage.persister import Persister

_PID = os.getpid()


class _NullSpan:
    __slots__ = ()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        return False

    def set(self, **args) -> None:
        pass


_NULL = _NullSpan()


class _Span:
    __slots__ = ("tracer", "name", "cat", "args", "t0", "c0")

    def __init__(self, tracer: "Tracer", name: str, cat: str, args: Dict[str, Any]):
        self.tracer = tracer
        self.name = name
        self.cat = cat
        self.args = args

    def __enter__(self):
        self.c0 = time.thread_time_ns()
        self.t0 = time.perf_counter_ns()
        return self

    def __exit__(self, exc_type, exc, tb):
        t1 = time.perf_counter_ns()
        # the thread's own CPU time inside the span: wall minus this is time spent waiting (I/O,
        # locks, the interpreter lock held by another thread)
        self.args["cpu_us"] = (time.thread_time_ns() - self.c0) // 1000
        if exc_type is not None:
            self.args["error"] = exc_type.__name__
        self.tracer._record(self.name, self.cat, self.t0, t1 - self.t0, self.args)
        return False

    def set(self, **args) -> None:
        """Attach result attributes (e.g. recommendation counts) before the span closes."""
        self.args.update(args)


class Tracer:
    def __init__(self, enabled: bool = False, max_events: int = 200_000, path: Optional[str] = None):
        self.enabled = enabled
        self.path = path
        self._events: collections.deque = collections.deque(maxlen=max_events)
        self._lock = threading.Lock()
        self._epoch_ns = time.perf_counter_ns()
        self.dropped = 0

    def span(self, name: str, cat: str = "sdk", **args):
        if not self.enabled:
            return _NULL
        return _Span(self, name, cat, args)

    def instant(self, name: str, cat: str = "sdk", **args) -> None:
        if not self.enabled:
            return
        ev = {"name": name, "cat": cat, "ph": "i", "s": "t", "ts": (time.perf_counter_ns() - self._epoch_ns) / 1e3,
              "pid": _PID, "tid": threading.get_ident(), "args": args}
        with self._lock:
            self._append(ev)

    def _append(self, ev) -> None:
        if len(self._events) == self._events.maxlen:
            self.dropped += 1
        self._events.append(ev)

    def _record(self, name: str, cat: str, t0_ns: int, dur_ns: int, args: Dict[str, Any]) -> None:
        ev = {"name": name, "cat": cat, "ph": "X", "ts": (t0_ns - self._epoch_ns) / 1e3, "dur": dur_ns / 1e3,
              "pid": _PID, "tid": threading.get_ident()}
        if args:
            ev["args"] = args
        with self._lock:
            self._append(ev)

    def events(self) -> List[dict]:
        with self._lock:
            return list(self._events)

    def clear(self) -> None:
        with self._lock:
            self._events.clear()
            self.dropped = 0

    def to_json(self) -> dict:
        evs = self.events()
        names = {ev["tid"] for ev in evs}
        meta = [{"name": "thread_name", "ph": "M", "pid": _PID, "tid": t, "args": {"name": _thread_name(t)}}
                for t in sorted(names)]
        return {"traceEvents": meta + evs, "displayTimeUnit": "ms",
                "otherData": {"enabled": self.enabled, "dropped": self.dropped,
                              # ts 0 on the host's monotonic clock: aligns traces of several processes
                              "epoch_monotonic_ns": self._epoch_ns}}

    def summary(self) -> Dict[str, dict]:
        """Per-span-name count / total / mean / max in milliseconds (for benches and logs)."""
        out: Dict[str, dict] = {}
        for ev in self.events():
            if ev.get("ph") != "X":
                continue
            s = out.setdefault(ev["name"], {"count": 0, "total_ms": 0.0, "max_ms": 0.0})
            d = ev["dur"] / 1e3
            s["count"] += 1
            s["total_ms"] += d
            s["max_ms"] = max(s["max_ms"], d)
        for s in out.values():
            s["mean_ms"] = s["total_ms"] / s["count"]
        return out

    def dump(self, path: Optional[str] = None) -> Optional[str]:
        path = path or self.path
        if not path:
            return None
        tmp = path + ".tmp"
        with open(tmp, "w") as f:
            json.dump(self.to_json(), f)
        os.replace(tmp, path)
        return path


def _thread_name(ident: int) -> str:
    for t in threading.enumerate():
        if t.ident == ident:
            return t.name
    return str(ident)


def _from_env() -> Tracer:
    path = os.environ.get("SDK_TRACE_FILE") or None
    enabled = bool(path) or os.environ.get("SDK_TRACE", "").lower() in ("1", "true", "yes")
    max_events = int(os.environ.get("SDK_TRACE_MAX_EVENTS", "200000"))
    t = Tracer(enabled, max_events, path)
    if path:
        atexit.register(t.dump)
    return t


TRACER = _from_env()


def span(name: str, cat: str = "sdk", **args):
    """``with trace.span("offer_cycle", offers=n) as s: ...; s.set(recs=k)``"""
    t = TRACER
    if not t.enabled:
        return _NULL
    return _Span(t, name, cat, args)


def instant(name: str, cat: str = "sdk", **args) -> None:
    TRACER.instant(name, cat, **args)


def enable(max_events: Optional[int] = None) -> Tracer:
    """Turn recording on at run time (tests, benches, ``/v1/debug/trace?enable=true``)."""
    TRACER.enabled = True
    if max_events is not None and max_events != TRACER._events.maxlen:
        with TRACER._lock:
            TRACER._events = collections.deque(TRACER._events, maxlen=max_events)
    return TRACER


def disable() -> None:
    TRACER.enabled = False


def enabled() -> bool:
    return TRACER.enabled


class TracingPersister(Persister):
    """Wraps a Persister so every operation is a ``persister.<op>`` span. Installed by the persister
    factory when tracing is on at startup; it forwards everything else to the wrapped backend."""

    def __init__(self, inner: Persister):
        self.inner = inner

    def __getattr__(self, item):  # PersisterCache.refresh(), backend-specific helpers
        return getattr(self.inner, item)

    @property
    def remote(self) -> bool:
        return self.inner.remote

    def get(self, path: str) -> Optional[bytes]:
        with span("persister.get", "persister", path=path):
            return self.inner.get(path)

    def get_children(self, path: str):
        with span("persister.get_children", "persister", path=path):
            return self.inner.get_children(path)

    def set(self, path: str, data: bytes) -> None:
        with span("persister.set", "persister", path=path, bytes=len(data) if data else 0):
            self.inner.set(path, data)

    def get_many(self, paths):
        with span("persister.get_many", "persister", n=len(paths)):
            return self.inner.get_many(paths)

    def set_many(self, path_bytes: Mapping[str, bytes]) -> None:
        with span("persister.set_many", "persister", n=len(path_bytes),
                  bytes=sum(len(v) for v in path_bytes.values() if v)):
            self.inner.set_many(path_bytes)

    def recursive_copy(self, src: str, dst: str) -> None:
        with span("persister.recursive_copy", "persister", src=src, dst=dst):
            self.inner.recursive_copy(src, dst)

    def recursive_delete_many(self, paths) -> None:
        with span("persister.recursive_delete_many", "persister", n=len(paths)):
            self.inner.recursive_delete_many(paths)

    def recursive_delete(self, path: str) -> None:
        with span("persister.recursive_delete", "persister", path=path):
            self.inner.recursive_delete(path)

    def close(self) -> None:
        self.inner.close()
