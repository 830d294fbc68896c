"""An agent's side of a task's lifecycle, run where the agent runs (its own process or rank).

``LocalMaster`` drives a task's synthetic lifecycle (STARTING, RUNNING, readiness check, exit)
itself, on its dispatcher thread, for every agent. On a Mesos cluster that work belongs to the
agents: the master applies ACCEPTs, keeps the offer and reservation books, and forwards the status
updates agents send. An agent registered with a *runtime* works that way here: the master sends
it ``launch`` / ``kill`` / ``fail`` / ``drop`` / ``reset``, and this class (in the agent's own
process: a ``torchrun`` rank owning its GPU, or a helper process) runs the task and reports
``starting``, ``running``, ``ready`` / ``check_failed`` and ``exited`` back, each report batched
with whatever else became due at the same moment. The master turns the reports into the same
``TaskStatus`` updates its own lifecycle would have produced (``LocalMaster.runtime_reports``).

The readiness check runs here, on the agent's GPU (``check(devices) -> bool``, e.g. the fused HIP
probe), honouring the check's ``delay_seconds`` and ``interval_seconds``.

Messages (master -> agent): ``launch`` {task, name, devices, check: {delay, interval} | null,
health, timing: {starting, running, check_exec, finish_after, exit_state}}, ``kill`` {task},
``fail`` {task, state, message}, ``drop`` {task}, ``reset``. Reports (agent -> master, in one
``status`` message): {task, event, [state, message, reason]}.
"""
from __future__ import annotations

import heapq
import itertools
import logging
import os
import threading
import time
from typing import Callable, Dict, List, Optional

LOGGER = logging.getLogger(__name__)

# TaskState numbers of the reports (mesos.proto), so this module needs no protobuf import
TASK_FINISHED, TASK_FAILED, TASK_KILLED = 2, 3, 4
REASON_COMMAND_EXECUTOR_FAILED = 1


class _Task:
    __slots__ = ("id", "name", "devices", "check", "timing", "epoch", "done")

    def __init__(self, msg: dict):
        self.id = msg["task"]
        self.name = msg.get("name", "")
        self.devices = list(msg.get("devices") or [])
        self.check = msg.get("check")
        self.timing = msg.get("timing") or {}
        self.epoch = 0
        self.done = False


class AgentRuntime:
    def __init__(self, report: Callable[[List[dict]], None], check: Optional[Callable[[List[int]], bool]] = None,
                 name: str = "agent-runtime"):
        self._report = report
        self._check = check
        self._tasks: Dict[str, _Task] = {}
        self._heap: list = []
        self._seq = itertools.count()
        self._cond = threading.Condition()
        self._running = True
        self._out: List[dict] = []       # reports produced by the current action, sent together
        self._act = threading.Lock()     # one action at a time: the caller's inline ones, the timer thread's
        self.checks = 0
        # STARTING / RUNNING go out before a check runs, unless this agent's checks have been
        # finishing within this window: then they leave with the check's result in one report
        # (one master hop and one status batch at the scheduler instead of two). Default 0 =
        # always first: on the box the merged report put the scheduler's handling of STARTING /
        # RUNNING behind the check instead of beside it, 1 pod +0.25 ms in the traced deploy
        # (profiles/prewarm_window_ab_r06_box.txt)
        self.report_window_s = float(os.environ.get("SDK_AGENT_REPORT_WINDOW_MS", "0") or 0) / 1000.0
        self._last_check_s: Optional[float] = None
        self._thread = threading.Thread(target=self._run, name=name, daemon=True)
        self._thread.start()

    # -- master messages (any thread) -----------------------------------------------------
    def handle(self, msg: dict) -> None:
        """Runs the message's action on the calling thread (the agent link's reader: a launch's
        STARTING, RUNNING and a due check need no hop to another thread), serialized with the
        timer thread's actions; the reports it produced go out in one message."""
        op = msg.get("op")
        fn = {"launch": self._launch, "kill": self._kill, "fail": self._fail, "drop": self._drop,
              "reset": self._reset}.get(op)
        if fn is None:
            LOGGER.warning("agent runtime: unknown op %r", op)
            return
        self._run_actions([(fn, (msg,))])

    def shutdown(self) -> None:
        with self._cond:
            self._running = False
            self._cond.notify_all()

    # -- actor plumbing --------------------------------------------------------------------
    def _at(self, delay: float, fn, *args) -> None:
        with self._cond:
            heapq.heappush(self._heap, (time.monotonic() + max(0.0, delay), next(self._seq), fn, args))
            self._cond.notify()

    def _run(self) -> None:
        while True:
            with self._cond:
                while self._running and (not self._heap or self._heap[0][0] > time.monotonic()):
                    wait = None if not self._heap else self._heap[0][0] - time.monotonic()
                    self._cond.wait(wait if wait is None else max(0.0, min(wait, 0.5)))
                if not self._running:
                    return
                due = []
                now = time.monotonic()
                # everything due now runs before the reports go out, so they leave in one message
                while self._heap and self._heap[0][0] <= now:
                    due.append(heapq.heappop(self._heap))
            self._run_actions([(fn, args) for _, _, fn, args in due])

    def _run_actions(self, actions) -> None:
        with self._act:
            for fn, args in actions:
                try:
                    fn(*args)
                except Exception:  # noqa: BLE001
                    LOGGER.exception("agent runtime action %s failed", getattr(fn, "__name__", fn))
            out, self._out = self._out, []
        if out:
            try:
                self._report(out)
            except Exception:  # noqa: BLE001
                LOGGER.exception("agent runtime: report failed")

    def _emit(self, task: _Task, event: str, **fields) -> None:
        self._out.append(dict(fields, task=task.id, event=event))

    def _then(self, delay: float, fn, task: _Task) -> None:
        """The task's next step: due now, it runs in this same action (its report joins the
        current message); later, it is scheduled."""
        if delay <= 0:
            fn(task, task.epoch)
        else:
            self._at(delay, fn, task, task.epoch)

    # -- lifecycle --------------------------------------------------------------------------
    def _launch(self, msg: dict) -> None:
        task = _Task(msg)
        old = self._tasks.get(task.id)
        if old is not None:
            old.done = True
        self._tasks[task.id] = task
        self._then(float(task.timing.get("starting", 0.0)), self._starting, task)

    def _live(self, task: _Task, epoch: int) -> bool:
        return not task.done and task.epoch == epoch and self._tasks.get(task.id) is task

    def _starting(self, task: _Task, epoch: int) -> None:
        if not self._live(task, epoch):
            return
        self._emit(task, "starting")
        self._then(float(task.timing.get("running", 0.0)), self._running_step, task)

    def _running_step(self, task: _Task, epoch: int) -> None:
        if not self._live(task, epoch):
            return
        self._emit(task, "running")
        if task.check is not None:
            delay = float(task.check.get("delay", 0.0)) + float(task.timing.get("check_exec", 0.0))
            self._then(delay, self._run_check, task)
        finish = task.timing.get("finish_after")
        if finish is not None:
            self._at(float(finish), self._finish, task, task.epoch)

    def _run_check(self, task: _Task, epoch: int) -> None:
        if not self._live(task, epoch):
            return
        ok = True
        if self._check is not None:
            # STARTING / RUNNING are reported before the check runs, as an executor reports them,
            # unless the last check took less than the report window (a resident GPU probe takes
            # ~0.1 ms): an executor's status updates are batched the same way by the agent
            last = self._last_check_s
            if last is None or last > self.report_window_s:
                out, self._out = self._out, []
                if out:
                    self._report(out)
            self.checks += 1
            t0 = time.monotonic()
            try:
                ok = bool(self._check(task.devices))
            except Exception:  # noqa: BLE001
                LOGGER.exception("check of %s raised", task.name)
                ok = False
            self._last_check_s = time.monotonic() - t0
        if ok:
            self._emit(task, "ready")
            return
        self._emit(task, "check_failed")
        self._at(float(task.check.get("interval", 1.0)), self._run_check, task, task.epoch)

    def _finish(self, task: _Task, epoch: int) -> None:
        if not self._live(task, epoch):
            return
        self._end(task, "exited", state=int(task.timing.get("exit_state", TASK_FINISHED)), message="task exited")

    def _end(self, task: _Task, event: str, **fields) -> None:
        task.done = True
        self._tasks.pop(task.id, None)
        self._emit(task, event, **fields)

    def _kill(self, msg: dict) -> None:
        task = self._tasks.get(msg["task"])
        if task is not None:
            self._end(task, "exited", state=TASK_KILLED, message="Task killed by scheduler")

    def _fail(self, msg: dict) -> None:
        task = self._tasks.get(msg["task"])
        if task is not None:
            self._end(task, "exited", state=int(msg.get("state", TASK_FAILED)),
                      message=msg.get("message", "task failed"),
                      reason=int(msg.get("reason", REASON_COMMAND_EXECUTOR_FAILED)))

    def _drop(self, msg: dict) -> None:
        """The master ended the task itself (teardown, agent removed): forget it silently."""
        task = self._tasks.pop(msg["task"], None)
        if task is not None:
            task.done = True

    def _reset(self, msg: dict) -> None:
        for t in self._tasks.values():
            t.done = True
        self._tasks.clear()
        with self._cond:
            self._heap = [e for e in self._heap if e[2] not in (self._starting, self._running_step, self._run_check,
                                                                self._finish)]
            heapq.heapify(self._heap)

    @property
    def live_tasks(self) -> List[str]:
        return sorted(self._tasks)
