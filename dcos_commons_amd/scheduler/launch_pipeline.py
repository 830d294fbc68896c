"""Overlaps the write-ahead records of streamed launches with the evaluation of later steps.

With launch streaming (``SDK_STREAM_LAUNCHES``) every matched step is recorded (its TaskInfos and
STAGING statuses written to the state store) and ACCEPTed before the next step is evaluated. On a
ZooKeeper-backed scheduler the record is a network round trip, and in an 8-pod parallel deploy the
offer cycle spends most of its time waiting for eight of them one after another. Here the step's
recommendations go to a writer thread instead and the cycle evaluates the next step at once; the
writer records everything that has queued up in ONE ``PersistentLaunchRecorder.record`` call (one
ZooKeeper multi) and then sends the ACCEPTs in step order. The write-ahead contract is unchanged:
nothing reaches the master before its record is durable, and a record that fails drops its
operations (as ``DefaultScheduler._record`` does). The cycle drains the pipeline before it returns,
so the next cycle sees every write of this one.

No reference counterpart: the reference evaluates the whole cycle, records all of it in one write,
then sends every ACCEPT (DefaultScheduler.java:431-470, OfferProcessor.java:300-330).
"""
from __future__ import annotations

import logging
import threading
from typing import Callable, List, Optional, Tuple

LOGGER = logging.getLogger(__name__)


class LaunchPipeline:
    """One writer thread per scheduler, started at the first submit and parked on the condition
    variable between offer cycles (a thread per cycle would also give the v1 driver, in sync-call
    mode, one new keep-alive master connection per cycle: ADVICE r5)."""

    def __init__(self, record: Callable[[list], bool], name: str = "launch-writer"):
        self._record = record          # -> False when the write failed (its operations are dropped)
        self._name = name
        self._cv = threading.Condition()
        self._queue: List[Tuple[list, Callable[[list], None]]] = []
        self._busy = False
        self._closed = False
        self._failed: List[list] = []
        self._thread: Optional[threading.Thread] = None
        self.writes = 0                # records written (for tests and traces)
        self.threads_started = 0       # writer threads started over the pipeline's life (tests)

    def submit(self, recs: list, send: Callable[[list], None]) -> None:
        """Queue one step's recommendations; ``send(recs)`` ACCEPTs them once recorded."""
        with self._cv:
            if self._closed:
                raise RuntimeError("launch pipeline is closed")
            self._queue.append((recs, send))
            if self._thread is None:
                self._thread = threading.Thread(target=self._run, name=self._name, daemon=True)
                self.threads_started += 1
                self._thread.start()
            self._cv.notify_all()

    def _run(self) -> None:
        while True:
            with self._cv:
                while not self._queue and not self._closed:
                    self._cv.wait()
                if not self._queue:
                    self._thread = None
                    self._cv.notify_all()
                    return
                items, self._queue = self._queue, []
                self._busy = True
            try:
                ok = self._record([r for recs, _ in items for r in recs])
                self.writes += 1
                for recs, send in items:
                    if not ok:
                        self._failed.append(recs)
                        continue
                    try:
                        send(recs)
                    except Exception:  # noqa: BLE001
                        LOGGER.exception("Failed to send %d recorded operation(s)", len(recs))
            except Exception:  # noqa: BLE001
                LOGGER.exception("Launch writer failed; dropping %d step(s)", len(items))
                self._failed.extend(recs for recs, _ in items)
            finally:
                with self._cv:
                    self._busy = False
                    self._cv.notify_all()

    def drain(self) -> List[list]:
        """Waits until every submitted step is recorded and sent (the writer then parks until the
        next cycle submits); returns the recommendation lists whose record failed."""
        with self._cv:
            while self._queue or self._busy:
                self._cv.wait()
            failed, self._failed = self._failed, []
        return failed

    def close(self, timeout: float = 5.0) -> None:
        """Finishes what is queued, then ends the writer thread."""
        with self._cv:
            self._closed = True
            self._cv.notify_all()
            thread = self._thread
        if thread is not None and thread is not threading.current_thread():
            thread.join(timeout)
