"""Real-process task runtime for the in-process agents of ``LocalMaster``.

The synthetic ``TaskBehavior`` only moves task states along a timeline. ``ProcessTaskBehavior``
makes each agent behave like a Mesos agent with the Mesos containerizer and the default executor:

* **sandbox** per task: ``<work>/<agent host>/frameworks/<fw>/executors/<executor>/tasks/<task id>``
  with ``stdout``/``stderr`` files; ``CommandInfo.uris`` are fetched into it (local paths and
  loopback ``http://`` URLs; anything else is skipped, there is no network);
* **persistent volumes** (``disk.persistence`` on the task's or its executor's resources) live in
  ``<work>/<agent host>/volumes/<persistence id>`` and are linked into the sandbox at their
  ``container_path``, so data survives relaunches on the same reservation and is deleted by a
  ``DESTROY``; host-path and sandbox-path container volumes are linked too; secret volumes and
  secret env vars are resolved through ``secret_resolver``;
* **environment**: the task's ``CommandInfo.environment`` plus ``MESOS_SANDBOX``/``MESOS_TASK_ID``
  and friends, and ``HIP_VISIBLE_DEVICES``/``ROCR_VISIBLE_DEVICES`` from the GPU devices the agent
  assigned (what the Mesos GPU isolator does for a task that asked for ``gpus``);
* **lifecycle**: ``bash -c <cmd>`` in its own session; exit 0 -> ``TASK_FINISHED``, otherwise
  ``TASK_FAILED``; a scheduler KILL sends SIGTERM to the session and SIGKILL after the task's
  ``kill_policy`` grace period -> ``TASK_KILLED``;
* **checks**: the readiness ``check`` command runs in the sandbox (``LocalMaster``'s check loop);
  the ``health_check`` command runs every ``interval_seconds`` after ``delay_seconds``; health
  changes are reported on ``TASK_RUNNING`` updates and ``consecutive_failures`` failures past the
  grace period kill the task (``TASK_KILLED``, ``healthy=false``).

Process start-up and reaping go through ``sdk-agent-launcher`` (``native/agent/launcher.cpp``) when
it is built: the helper creates the sandbox and links its volumes (an ordered list of set-up steps
in the launch request; a task with secret files or URIs to fetch has its sandbox prepared here
first), forks, execs and reaps outside the interpreter, and reports starts and exits back over a
socket. The master does not wait for the fork: STARTING is reported when the helper reports the
process started, as an executor reports it (``SDK_NATIVE_AGENT_LAUNCHER=0``, or no binary:
``subprocess.Popen`` plus a waiter thread per task, as before). Task processes, readiness checks
and health checks all start that way.

Test hooks: ``exec_in_task`` (``dcos task exec``), ``kill_with_pattern`` (``pkill -9 -f`` limited
to the sessions this runtime started) and ``sandbox_of``. Every process this runtime starts is in a
session it owns; ``shutdown()`` kills them all.
"""
from __future__ import annotations

import json
import logging
import os
import re
import shutil
import signal
import subprocess
import threading
import time
import urllib.parse
import urllib.request
from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional, Tuple

from dcos_commons_amd.mesos import protos as P
from dcos_commons_amd.mesos.local_master import TaskBehavior, TaskTiming

LOGGER = logging.getLogger(__name__)
_LOOPBACK = {"127.0.0.1", "localhost", "::1"}
DEFAULT_KILL_GRACE_S = 3.0
EXECUTOR_ARGV0 = "mesos-default-executor"


@dataclass
class _Proc:
    task_id: str
    name: str
    agent_host: str
    sandbox: str
    env: Dict[str, str]
    popen: Optional[subprocess.Popen] = None
    killed: bool = False
    unhealthy: bool = False
    health_stop: threading.Event = field(default_factory=threading.Event)
    exited: threading.Event = field(default_factory=threading.Event)
    rc: Optional[int] = None


def _safe(name: str) -> str:
    return re.sub(r"[^A-Za-z0-9_.-]", "_", name) or "_"


def _session_pids(sid: int) -> List[int]:
    """Live processes whose session id is ``sid`` (the task's own session)."""
    out = []
    for d in os.listdir("/proc"):
        if not d.isdigit():
            continue
        try:
            with open(f"/proc/{d}/stat", "rb") as f:
                stat = f.read().decode("utf-8", "replace")
            # fields after the ")" that closes comm: state ppid pgrp session ...
            rest = stat[stat.rindex(")") + 2:].split()
            if int(rest[3]) == sid:
                out.append(int(d))
        except (OSError, ValueError, IndexError):
            continue
    return out


def _start_ticks(pid: int) -> int:
    try:
        with open(f"/proc/{pid}/stat", "rb") as f:
            stat = f.read().decode("utf-8", "replace")
        return int(stat[stat.rindex(")") + 2:].split()[19])
    except (OSError, ValueError, IndexError):
        return 1 << 62


def _alive(pid: int) -> bool:
    """The process exists and is not a zombie (an orphan whose new parent has not reaped it)."""
    try:
        with open(f"/proc/{pid}/stat", "rb") as f:
            stat = f.read().decode("utf-8", "replace")
        return stat[stat.rindex(")") + 2:].split()[0] != "Z"
    except (OSError, ValueError, IndexError):
        return False


def _cmdline(pid: int) -> str:
    try:
        with open(f"/proc/{pid}/cmdline", "rb") as f:
            return f.read().replace(b"\0", b" ").decode("utf-8", "replace").strip()
    except OSError:
        return ""


class SecretAccessDenied(Exception):
    pass


def secret_accessible(secret_path: str, space: str) -> bool:
    """DC/OS secret spaces: a service at ``/a/b`` may read secrets stored directly under its own
    path or any ancestor path (``a/b/x``, ``a/x``, ``x``), never deeper ones (``a/b/c/x``)."""
    parent = [p for p in secret_path.strip("/").split("/")[:-1] if p]
    own = [p for p in space.strip("/").split("/") if p]
    return own[:len(parent)] == parent


class _RemoteProcess:
    """What the containerizer needs of a ``Popen`` for a process the native launcher started:
    its pid (a session and process-group leader) and its exit status."""

    def __init__(self, pid: int):
        self.pid = pid                  # 0 until the helper reports the fork (an unwaited launch)
        self.returncode: Optional[int] = None
        self._done = threading.Event()
        self._started = threading.Event()
        if pid:
            self._started.set()

    def _set_pid(self, pid: int) -> None:
        self.pid = pid
        self._started.set()

    def _exited(self, rc: int) -> None:
        self.returncode = rc
        self._started.set()
        self._done.set()

    def wait_started(self, timeout: Optional[float] = None) -> int:
        """The pid once the helper has forked the process (0: it never started)."""
        self._started.wait(timeout)
        return self.pid

    def wait(self, timeout: Optional[float] = None) -> Optional[int]:
        self._done.wait(timeout)
        return self.returncode

    def poll(self) -> Optional[int]:
        return self.returncode


class NativeLauncher:
    """Client of ``sdk-agent-launcher``: one helper process per containerizer, one socket, one
    reader thread that turns the helper's events into callbacks. ``launch`` waits at most for the
    fork (the pid), or not at all when given ``on_error``; ``run`` (a check command) returns its
    exit code."""

    def __init__(self, binary: str):
        import socket
        import subprocess as sp

        self._ours, theirs = socket.socketpair()
        self.proc = sp.Popen([binary, "--fd", str(theirs.fileno())], pass_fds=(theirs.fileno(),),
                             stdin=sp.DEVNULL, close_fds=True)
        theirs.close()
        self._send_lock = threading.Lock()
        self._lock = threading.Lock()
        self._seq = 0
        self._waiting: Dict[str, "Future"] = {}            # request id -> started pid / run rc
        self._procs: Dict[str, tuple] = {}      # launch id -> (_RemoteProcess, on_exit, on_error, on_started)
        self._closed = False
        self._stopping = False
        self._reader = threading.Thread(target=self._read_loop, name="agent-launcher-events", daemon=True)
        self._reader.start()

    def _next_id(self) -> str:
        with self._lock:
            self._seq += 1
            return str(self._seq)

    def _request(self, msg: dict) -> "Future":
        from concurrent.futures import Future

        fut: Future = Future()
        with self._lock:
            if self._closed:
                raise OSError("agent launcher is closed")
            self._waiting[msg["id"]] = fut
        line = (json.dumps(msg, separators=(",", ":")) + "\n").encode("utf-8")
        with self._send_lock:
            self._ours.sendall(line)
        return fut

    def launch(self, argv: List[str], exe: str, cwd: str, env: Dict[str, str], stdout: str, stderr: str,
               on_exit: Callable[["_RemoteProcess", int], None], setup: Optional[List[tuple]] = None,
               on_error: Optional[Callable[["_RemoteProcess", str], None]] = None,
               on_started: Optional[Callable[["_RemoteProcess"], None]] = None) -> "_RemoteProcess":
        """Starts the process after the helper has run the sandbox ``setup``, in order:
        ``("d", dir)`` creates a directory with its parents, ``("l", target, link)`` symlinks
        ``link`` to ``target`` unless it exists. ``on_exit(process, rc)`` runs on the event thread when it is
        reaped. Without ``on_error`` this returns once the helper has forked it (a failure raises
        ``OSError``); with it, it returns at once: the pid is filled in when the fork is reported
        (``wait_started``) and ``on_started(process)`` runs on the event thread, or a failed set-up
        or fork calls ``on_error(process, message)`` there instead."""
        rid = self._next_id()
        proc = _RemoteProcess(0)
        with self._lock:
            self._procs[rid] = (proc, on_exit, on_error, on_started)
        msg = {"op": "launch", "id": rid, "argv": argv, "exe": exe, "cwd": cwd, "env": env,
               "stdout": stdout, "stderr": stderr}
        if setup:
            msg["setup"] = [list(step) for step in setup]
        try:
            if on_error is not None:
                self._send(msg)
            else:
                self._request(msg).result(30)
        except BaseException:
            with self._lock:
                pending = self._procs.pop(rid, None)
            if pending is None and on_error is not None:
                # the helper died between registering the launch and sending it: the read loop
                # already popped the entry and reported the failure through on_error, so raising
                # here would report the same task's failure a second time
                return proc
            raise
        return proc

    def _send(self, msg: dict) -> None:
        with self._lock:
            if self._closed:
                raise OSError("agent launcher is closed")
        line = (json.dumps(msg, separators=(",", ":")) + "\n").encode("utf-8")
        with self._send_lock:
            self._ours.sendall(line)

    def run(self, argv: List[str], cwd: str, env: Dict[str, str], timeout_s: float) -> int:
        rid = self._next_id()
        fut = self._request({"op": "run", "id": rid, "argv": argv, "cwd": cwd, "env": env,
                             "timeout_ms": int(timeout_s * 1000) if timeout_s and timeout_s > 0 else 0})
        return int(fut.result())

    def _read_loop(self) -> None:
        buf = b""
        try:
            while True:
                data = self._ours.recv(65536)
                if not data:
                    break
                buf += data
                while b"\n" in buf:
                    line, buf = buf.split(b"\n", 1)
                    if line:
                        self._event(json.loads(line))
        except OSError:
            pass
        with self._lock:
            self._closed = True
            waiting, self._waiting = self._waiting, {}
            unstarted = [(rid, e) for rid, e in self._procs.items() if not e[0].pid and e[2] is not None]
            for rid, _ in unstarted:
                self._procs.pop(rid, None)
            orphans, self._procs = list(self._procs.values()), {}
        if orphans and not self._stopping:
            # the helper died under running processes: they live on (reparented), but their exit
            # status is gone with it. Watch for their end and report it as a kill.
            LOGGER.warning("agent launcher exited with %d processes running: watching them", len(orphans))
            threading.Thread(target=self._watch_orphans, args=(orphans,), name="agent-launcher-orphans",
                             daemon=True).start()
        for fut in waiting.values():
            if not fut.done():
                fut.set_exception(OSError("agent launcher exited"))
        for _, (proc, _, on_error, _) in unstarted:
            proc._exited(127)
            try:
                on_error(proc, "agent launcher exited")
            except Exception:  # noqa: BLE001
                LOGGER.exception("launch error callback failed")

    def _event(self, ev: dict) -> None:
        kind, rid = ev.get("ev"), str(ev.get("id", ""))
        if kind == "exited":
            with self._lock:
                entry = self._procs.pop(rid, None)
            if entry is not None:
                proc, cb = entry[0], entry[1]
                proc._exited(int(ev["rc"]))
                try:
                    cb(proc, int(ev["rc"]))
                except Exception:  # noqa: BLE001
                    LOGGER.exception("exit callback failed")
            return
        with self._lock:
            fut = self._waiting.pop(rid, None)
            entry = self._procs.get(rid)
        if kind == "started" and entry is not None:
            entry[0]._set_pid(int(ev["pid"]))   # set before any exit of it is dispatched (same thread)
            if entry[3] is not None:
                try:
                    entry[3](entry[0])
                except Exception:  # noqa: BLE001
                    LOGGER.exception("launch started callback failed")
        if fut is None:
            if kind == "error":
                if entry is not None and entry[2] is not None:
                    with self._lock:
                        self._procs.pop(rid, None)
                    entry[0]._exited(127)
                    try:
                        entry[2](entry[0], str(ev.get("msg") or "launch failed"))
                    except Exception:  # noqa: BLE001
                        LOGGER.exception("launch error callback failed")
                else:
                    LOGGER.error("agent launcher: %s", ev.get("msg"))
            return
        if kind == "started":
            fut.set_result(int(ev["pid"]))
        elif kind == "ran":
            fut.set_result(int(ev["rc"]))
        else:
            with self._lock:
                self._procs.pop(rid, None)
            fut.set_exception(OSError(ev.get("msg") or "launch failed"))

    @staticmethod
    def _watch_orphans(orphans) -> None:
        live = [(proc, cb) for proc, cb, _, _ in orphans if proc.pid > 0]
        while live:
            still = []
            for proc, cb in live:
                if _alive(proc.pid):
                    still.append((proc, cb))
                    continue
                proc._exited(-signal.SIGKILL)
                try:
                    cb(proc, -signal.SIGKILL)
                except Exception:  # noqa: BLE001
                    LOGGER.exception("exit callback failed")
            live = still
            if live:
                time.sleep(0.05)

    @property
    def closed(self) -> bool:
        """The helper is gone (it exited, or ``close`` was called)."""
        return self._closed

    def close(self) -> None:
        self._stopping = True
        with self._lock:
            self._closed = True
        try:
            self._ours.sendall(b'{"op":"stop"}\n')
        except OSError:
            pass
        try:
            self.proc.wait(2)
        except Exception:  # noqa: BLE001
            self.proc.kill()
        self._ours.close()


def native_launcher_binary() -> Optional[str]:
    """The built helper, unless ``SDK_NATIVE_AGENT_LAUNCHER=0``."""
    if os.environ.get("SDK_NATIVE_AGENT_LAUNCHER", "1").lower() in ("0", "false", "no"):
        return None
    from dcos_commons_amd.ops.build import BUILD

    path = os.path.join(BUILD, "sdk-agent-launcher")
    return path if os.access(path, os.X_OK) else None


class ProcessTaskBehavior(TaskBehavior):
    executes_commands = True

    def __init__(self, work_dir: str, secret_resolver: Optional[Callable[[str], Optional[bytes]]] = None,
                 default_kill_grace_s: float = DEFAULT_KILL_GRACE_S, extra_env: Optional[Dict[str, str]] = None,
                 check_workers: int = 8, resolver: Optional[Callable[[str], Optional[str]]] = None,
                 artifact_resolver: Optional[Callable[[str], Optional[str]]] = None):
        """``resolver(hostname)`` maps cluster DNS names to an address the fetcher can reach
        (``None``: not a cluster name); ``artifact_resolver(uri)`` maps a URI to a local file, or
        to a directory whose contents stand for the extracted archive (e.g. ``bootstrap.zip`` ->
        the native ``sdk-bootstrap`` as ``./bootstrap``)."""
        super().__init__(default=TaskTiming(), check_runner=self._run_readiness_check, check_workers=check_workers)
        self.work_dir = os.path.abspath(work_dir)
        os.makedirs(self.work_dir, exist_ok=True)
        self.secret_resolver = secret_resolver
        self.resolver = resolver
        self.artifact_resolver = artifact_resolver
        self.default_kill_grace_s = default_kill_grace_s
        self.extra_env = dict(extra_env or {})
        # the cluster's metrics service (testing.cluster.metrics.LocalMetrics): each task gets the
        # StatsD address of its own container
        self.metrics = None
        self._procs: Dict[str, _Proc] = {}
        self._lock = threading.Lock()
        self._native = None      # NativeLauncher once started; False: start processes in-process

    # -- paths -----------------------------------------------------------------------
    def _agent_dir(self, host: str) -> str:
        return os.path.join(self.work_dir, _safe(host))

    def volume_dir(self, host: str, persistence_id: str) -> str:
        return os.path.join(self._agent_dir(host), "volumes", _safe(persistence_id))

    def mount_dir(self, host: str, root: str) -> str:
        return os.path.join(self._agent_dir(host), "mounts", _safe(root.strip("/")))

    def sandbox_of(self, task_id: str) -> Optional[str]:
        with self._lock:
            p = self._procs.get(task_id)
        return p.sandbox if p is not None else None

    # -- launch (called on the master's actor thread) --------------------------------
    def launch(self, master, task, agent) -> None:
        info: P.TaskInfo = task.info
        host = agent.spec.hostname
        eid = task.executor_id or "command"
        sandbox = os.path.join(self._agent_dir(host), "frameworks", _safe(task.framework_id), "executors",
                               _safe(eid), "tasks", _safe(info.task_id.value))
        native = self._native_launcher()
        resources = list(info.resources) + self._executor_resources(master, task, agent)
        # with the native helper, the sandbox and its volume links are made by the helper, off the
        # master's thread (secrets and fetched URIs still need this process: done here first)
        plan = self._sandbox_plan(host, sandbox, resources, info) if native is not None else None
        proc = _Proc(info.task_id.value, info.name, host, sandbox, {})
        with self._lock:
            self._procs[proc.task_id] = proc
        epoch = task.epoch
        try:
            space = self._dcos_space(master, task, agent)
            if plan is None:
                os.makedirs(sandbox, exist_ok=True)
                self._link_volumes(host, sandbox, resources)
                self._link_container_volumes(sandbox, info, space)
                self._fetch(sandbox, info.command.uris)
            proc.env = self._environment(master, task, agent, sandbox, space)
            # the task's shell is named like the executor that would run it on Mesos, so a
            # `pkill -f mesos-default-executor` takes the task down with "its executor" (the
            # trailing `exit $?` keeps that shell alive as the command's parent: bash would
            # otherwise exec the last command of the list in its place)
            argv = [EXECUTOR_ARGV0, "-c", (info.command.value or "true") + "\nexit $?"]
            if native is not None:
                proc.popen = native.launch(
                    argv, "/bin/bash", sandbox, proc.env, os.path.join(sandbox, "stdout"),
                    os.path.join(sandbox, "stderr"),
                    on_exit=lambda rp, rc: self._exited(master, task, epoch, proc, rc, rp),
                    setup=plan,
                    on_error=lambda rp, msg: self._launch_failed(master, task, epoch, proc, msg),
                    # STARTING / RUNNING once the process exists, as an executor reports them
                    on_started=lambda rp: master._schedule(0, master._lifecycle_starting, task, epoch,
                                                           self.timing(info)))
            else:
                with open(os.path.join(sandbox, "stdout"), "ab") as out, \
                        open(os.path.join(sandbox, "stderr"), "ab") as err:
                    proc.popen = subprocess.Popen(argv, executable="/bin/bash", cwd=sandbox, env=proc.env,
                                                  stdin=subprocess.DEVNULL, stdout=out, stderr=err,
                                                  start_new_session=True)
        except Exception as e:  # noqa: BLE001
            LOGGER.exception("failed to start %s", info.name)
            master._schedule(0, master._container_failed, task, task.epoch, str(e))
            proc.exited.set()
            return
        if native is None:
            threading.Thread(target=self._wait, args=(master, task, epoch, proc), name=f"wait-{info.name}",
                             daemon=True).start()
            master._schedule(0, master._lifecycle_starting, task, epoch, self.timing(info))

    def _sandbox_plan(self, host: str, sandbox: str, resources: List[P.Resource], info: P.TaskInfo):
        """The sandbox set-up steps for the native helper, in the order ``_link_volumes`` and
        ``_link_container_volumes`` take them: the sandbox, each persistent volume's directory and
        its link at the container path, then host / sandbox path volumes. None when the task also
        needs a secret file or fetched URIs written into its sandbox."""
        if info.command.uris:
            return None
        steps: list = [("d", sandbox)]

        def link(target: str, container_path: str) -> None:
            if container_path and not os.path.isabs(container_path):   # absolute: needs a mount namespace
                steps.append(("l", target, os.path.join(sandbox, container_path)))
        for r in resources:
            if not r.HasField("disk") or not r.disk.HasField("persistence") or not r.disk.persistence.id:
                continue
            if r.disk.HasField("source") and r.disk.source.type == P.Resource.DiskInfo.Source.MOUNT:
                target = os.path.join(self.mount_dir(host, r.disk.source.mount.root), _safe(r.disk.persistence.id))
            else:
                target = self.volume_dir(host, r.disk.persistence.id)
            steps.append(("d", target))
            link(target, r.disk.volume.container_path)
        for v in info.container.volumes:
            src = v.source
            if src.type == P.Volume.Source.SECRET:
                return None
            if src.type == P.Volume.Source.HOST_PATH or v.host_path:
                host_path = src.host_path.path or v.host_path
                if not os.path.isabs(host_path):
                    # a sandbox-relative host path (the SDK's `/tmp` -> `tmp` volume) exists
                    steps.append(("d", os.path.join(sandbox, host_path)))
                link(host_path, v.container_path)
            elif src.type == P.Volume.Source.SANDBOX_PATH:
                target = os.path.join(sandbox, src.sandbox_path.path)
                steps.append(("d", target))
                link(target, v.container_path)
        return steps

    def _launch_failed(self, master, task, epoch: int, proc: _Proc, msg: str) -> None:
        """The helper could not set up the sandbox or fork (on the launcher's event thread)."""
        LOGGER.error("failed to start %s: %s", proc.name, msg)
        proc.health_stop.set()
        proc.exited.set()
        master._schedule(0, master._container_failed, task, epoch, msg)

    def _native_launcher(self) -> Optional[NativeLauncher]:
        if self._native is False:
            return None
        if self._native is None or self._native.closed:
            with self._lock:
                if self._native is not None and self._native is not False and self._native.closed:
                    LOGGER.warning("native agent launcher exited: starting a new one")
                    self._native = None
                if self._native is None:
                    binary = native_launcher_binary()
                    try:
                        self._native = NativeLauncher(binary) if binary else False
                    except OSError as e:
                        LOGGER.warning("native agent launcher unavailable (%s): starting tasks in-process", e)
                        self._native = False
        return self._native or None

    @staticmethod
    def _dcos_space(master, task, agent) -> Optional[str]:
        """The ``DCOS_SPACE`` label of the task's executor (the scheduler's Marathon app path),
        which scopes the secrets the task may read; None when the executor carries none."""
        e = agent.executors.get((task.framework_id, task.executor_id))
        if e is None:
            return None
        return next((l.value for l in e.info.labels.labels if l.key == "DCOS_SPACE"), None)

    @staticmethod
    def _executor_resources(master, task, agent) -> List[P.Resource]:
        e = agent.executors.get((task.framework_id, task.executor_id))
        return list(e.info.resources) if e is not None else []

    def _link(self, target: str, sandbox: str, container_path: str) -> None:
        if not container_path or os.path.isabs(container_path):
            return  # absolute container paths need a mount namespace: not modelled
        link = os.path.join(sandbox, container_path)
        os.makedirs(os.path.dirname(link), exist_ok=True)
        if os.path.lexists(link):
            return
        os.symlink(target, link)

    def _link_volumes(self, host: str, sandbox: str, resources: List[P.Resource]) -> None:
        for r in resources:
            if not r.HasField("disk") or not r.disk.HasField("persistence") or not r.disk.persistence.id:
                continue
            if r.disk.HasField("source") and r.disk.source.type == P.Resource.DiskInfo.Source.MOUNT:
                target = os.path.join(self.mount_dir(host, r.disk.source.mount.root), _safe(r.disk.persistence.id))
            else:
                target = self.volume_dir(host, r.disk.persistence.id)
            os.makedirs(target, exist_ok=True)
            self._link(target, sandbox, r.disk.volume.container_path)

    def _link_container_volumes(self, sandbox: str, info: P.TaskInfo, space: Optional[str] = None) -> None:
        for v in info.container.volumes:
            src = v.source
            if src.type == P.Volume.Source.SECRET:
                data = self._secret(src.secret, space)
                path = os.path.join(sandbox, v.container_path)
                os.makedirs(os.path.dirname(path), exist_ok=True)
                with open(path, "wb") as f:
                    f.write(data or b"")
            elif src.type == P.Volume.Source.HOST_PATH or v.host_path:
                host_path = src.host_path.path or v.host_path
                if not os.path.isabs(host_path):
                    os.makedirs(os.path.join(sandbox, host_path), exist_ok=True)
                self._link(host_path, sandbox, v.container_path)
            elif src.type == P.Volume.Source.SANDBOX_PATH:
                target = os.path.join(sandbox, src.sandbox_path.path)
                os.makedirs(target, exist_ok=True)
                self._link(target, sandbox, v.container_path)

    def _secret(self, secret: P.Secret, space: Optional[str] = None) -> Optional[bytes]:
        """The secret's bytes; a reference outside ``space`` (the task's DCOS_SPACE) is refused."""
        if secret.type == P.Secret.VALUE:
            return secret.value.data
        if self.secret_resolver is None:
            return None
        name = secret.reference.name
        if space is not None and not secret_accessible(name, space):
            raise SecretAccessDenied(f"secret '{name}' is not accessible from DCOS_SPACE '{space}'")
        return self.secret_resolver(name)

    def _fetch(self, sandbox: str, uris) -> None:
        for u in uris:
            parsed = urllib.parse.urlparse(u.value)
            name = u.output_file or os.path.basename(parsed.path) or "download"
            dest = os.path.join(sandbox, name)
            addr = parsed.hostname if parsed.hostname in _LOOPBACK else (
                self.resolver(parsed.hostname) if self.resolver is not None and parsed.hostname else None)
            local = self.artifact_resolver(u.value) if self.artifact_resolver is not None else None
            try:
                if local is not None and os.path.isdir(local):
                    for entry in os.listdir(local):   # the archive's extracted contents
                        src = os.path.join(local, entry)
                        if os.path.isdir(src):
                            shutil.copytree(src, os.path.join(sandbox, entry), dirs_exist_ok=True)
                        else:
                            shutil.copy2(src, os.path.join(sandbox, entry))
                    continue
                if local is not None:
                    shutil.copy2(local, dest)
                elif parsed.scheme in ("", "file"):
                    shutil.copyfile(parsed.path, dest)
                elif parsed.scheme in ("http", "https") and addr is not None:
                    url = u.value.replace(parsed.hostname, addr, 1)
                    with urllib.request.urlopen(url, timeout=10) as resp, open(dest, "wb") as f:
                        shutil.copyfileobj(resp, f)
                else:
                    LOGGER.info("fetcher: skipping %s (no network in the local cluster)", u.value)
                    continue
            except OSError as e:
                LOGGER.warning("fetcher: %s: %s", u.value, e)
                continue
            if u.executable:
                os.chmod(dest, 0o755)
            elif u.extract and re.search(r"\.(tar\.gz|tgz|tar|zip)$", dest):
                try:
                    shutil.unpack_archive(dest, sandbox)
                except (shutil.ReadError, ValueError, OSError) as e:
                    LOGGER.warning("fetcher: cannot extract %s: %s", dest, e)

    def _environment(self, master, task, agent, sandbox: str, space: Optional[str] = None) -> Dict[str, str]:
        env = {k: os.environ[k] for k in ("PATH", "LANG", "LC_ALL", "TZ", "TMPDIR") if k in os.environ}
        env.update(self.extra_env)
        for v in task.info.command.environment.variables:
            if v.type == P.Environment.Variable.SECRET:
                data = self._secret(v.secret, space)
                env[v.name] = data.decode("utf-8", "replace") if data is not None else ""
            else:
                env[v.name] = v.value
        env.update({
            "MESOS_SANDBOX": sandbox, "MESOS_TASK_ID": task.info.task_id.value,
            "MESOS_FRAMEWORK_ID": task.framework_id, "MESOS_AGENT_ID": agent.id,
            "MESOS_EXECUTOR_ID": task.executor_id, "MESOS_CONTAINER_IP": "127.0.0.1",
            "LIBPROCESS_IP": "127.0.0.1", "HOST": agent.spec.hostname, "HOME": sandbox,
        })
        if task.gpu_devices:
            devs = ",".join(str(d) for d in task.gpu_devices)
            env["HIP_VISIBLE_DEVICES"] = devs
            env["ROCR_VISIBLE_DEVICES"] = devs
        for v in task.info.container.volumes:
            # the container's /tmp is the sandbox's `tmp` (PodInfoBuilder adds that volume to
            # every task); without a mount namespace the task is pointed at it through TMPDIR
            if v.container_path == "/tmp" and v.host_path and not os.path.isabs(v.host_path):
                env["TMPDIR"] = os.path.join(sandbox, v.host_path)
        if self.metrics is not None:
            from dcos_commons_amd.mesos.local_master import container_id_for

            env.update(self.metrics.container_env(
                container_id_for(task.info.task_id.value), agent.id,
                {"task_name": task.info.name, "task_id": task.info.task_id.value,
                 "framework_id": task.framework_id, "executor_id": task.executor_id,
                 "hostname": agent.spec.hostname}))
        return env

    # -- process supervision ----------------------------------------------------------
    def _wait(self, master, task, epoch: int, proc: _Proc) -> None:
        rc = proc.popen.wait()
        proc.rc = rc
        proc.health_stop.set()
        # a task's session may leave stragglers (e.g. `sleep &`): the container is torn down
        self._signal_session(proc, signal.SIGKILL)
        proc.exited.set()
        master._schedule(0, master._process_exited, task, epoch, rc, proc.killed, proc.unhealthy)

    def _exited(self, master, task, epoch: int, proc: _Proc, rc: int, remote) -> None:
        """A process the native launcher started was reaped (on the launcher's event thread)."""
        if proc.popen is None:
            proc.popen = remote
        proc.rc = rc
        proc.health_stop.set()
        # stragglers of the task: its process group now, the rest of its session off this thread
        # (a /proc scan costs milliseconds on a busy host and would hold up every other event)
        self._signal_group(proc, signal.SIGKILL)
        proc.exited.set()
        master._schedule(0, master._process_exited, task, epoch, rc, proc.killed, proc.unhealthy)
        threading.Thread(target=self._signal_session, args=(proc, signal.SIGKILL), name=f"reap-{proc.name}",
                         daemon=True).start()

    def started(self, master, task, epoch: int) -> None:
        """Called when the task reports RUNNING: start its health checks."""
        hc = task.info.health_check if task.info.HasField("health_check") else None
        if hc is None or hc.type != P.HealthCheck.COMMAND:
            return
        with self._lock:
            proc = self._procs.get(task.info.task_id.value)
        if proc is None:
            return
        threading.Thread(target=self._health_loop, args=(master, task, epoch, proc, hc),
                         name=f"health-{task.info.name}", daemon=True).start()

    def _health_loop(self, master, task, epoch: int, proc: _Proc, hc: P.HealthCheck) -> None:
        t0 = time.monotonic()
        if proc.health_stop.wait(hc.delay_seconds):
            return
        failures, healthy = 0, None
        while not proc.health_stop.is_set():
            ok = self._run_command(proc, hc.command.value, hc.timeout_seconds) == 0
            if ok:
                failures = 0
            elif time.monotonic() - t0 >= hc.grace_period_seconds:
                failures += 1
            if ok != healthy:
                healthy = ok
                master._schedule(0, master._health_changed, task, epoch, ok)
            if failures >= max(1, hc.consecutive_failures):
                LOGGER.info("%s failed %d consecutive health checks: killing it", proc.name, failures)
                proc.unhealthy = True
                self._terminate(proc, self.default_kill_grace_s)
                return
            if proc.health_stop.wait(max(0.05, hc.interval_seconds)):
                return

    def _run_command(self, proc: _Proc, cmd: str, timeout_s: float) -> int:
        native = self._native_launcher()
        if native is not None:
            try:
                return native.run(["bash", "-c", cmd], proc.sandbox, proc.env, timeout_s)
            except OSError:
                return 127
        try:
            r = subprocess.run(["bash", "-c", cmd], cwd=proc.sandbox, env=proc.env, stdin=subprocess.DEVNULL,
                               stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL,
                               timeout=timeout_s if timeout_s > 0 else None, start_new_session=True)
            return r.returncode
        except subprocess.TimeoutExpired:
            return 124
        except OSError:
            return 127

    def _run_readiness_check(self, task_info: P.TaskInfo, devices) -> bool:
        with self._lock:
            proc = self._procs.get(task_info.task_id.value)
        if proc is None or proc.exited.is_set():
            return False
        check = task_info.check
        return self._run_command(proc, check.command.command.value, check.timeout_seconds) == 0

    # -- kill ---------------------------------------------------------------------------
    def kill(self, master, task) -> bool:
        """Scheduler KILL: True when a live process was signalled (its exit reports KILLED)."""
        with self._lock:
            proc = self._procs.get(task.info.task_id.value)
        if proc is None or proc.popen is None or proc.exited.is_set():
            return False
        proc.killed = True
        grace = self.default_kill_grace_s
        if task.info.HasField("kill_policy") and task.info.kill_policy.HasField("grace_period"):
            grace = task.info.kill_policy.grace_period.nanoseconds / 1e9
        self._terminate(proc, grace)
        return True

    @staticmethod
    def _pid(proc: _Proc) -> int:
        """The task's session leader; 0 when it never started. A launch handed to the native
        helper without waiting may not have reported its fork yet: wait for it (briefly)."""
        p = proc.popen
        if p is None:
            return 0
        if not p.pid and isinstance(p, _RemoteProcess):
            return p.wait_started(5.0)
        return p.pid

    def _signal_session(self, proc: _Proc, sig: int) -> int:
        sid = self._pid(proc)
        if sid <= 0:
            return 0
        n = 0
        for pid in _session_pids(sid):
            try:
                os.kill(pid, sig)
                n += 1
            except ProcessLookupError:
                pass
        return n

    @staticmethod
    def _signal_group(proc: _Proc, sig: int) -> None:
        """The task's process group (its session leader's group: ``bash -c`` and whatever it runs
        without job control), in one ``killpg`` instead of a ``/proc`` scan."""
        pgid = ProcessTaskBehavior._pid(proc)
        if pgid <= 0:       # never started (killpg(0) would signal this process's own group)
            return
        try:
            os.killpg(pgid, sig)
        except (ProcessLookupError, PermissionError):
            pass

    def _terminate(self, proc: _Proc, grace_s: float) -> None:
        """SIGTERM now to the task's process group, from the caller's thread (the master's, on a
        KILL); then, off that thread, SIGTERM to anything else left in the task's session (a
        child that made its own process group), and SIGKILL to the whole session after the grace
        period. Scanning ``/proc`` for the session costs ~10 ms of interpreter time on a busy host,
        which the kill used to spend before the master could go on."""
        proc.health_stop.set()
        self._signal_group(proc, signal.SIGTERM)

        def escalate():
            self._signal_session(proc, signal.SIGTERM)
            if not proc.exited.wait(max(0.0, grace_s)):
                self._signal_group(proc, signal.SIGKILL)
                self._signal_session(proc, signal.SIGKILL)
        threading.Thread(target=escalate, name=f"kill-{proc.name}", daemon=True).start()

    def release(self, task) -> None:
        """The master forgot the task (terminal, torn down, agent gone): the container goes too."""
        with self._lock:
            proc = self._procs.get(task.info.task_id.value)
        if proc is not None and not proc.exited.is_set():
            proc.killed = True
            self._terminate(proc, 0.0)

    def destroy_volumes(self, agent, volumes) -> None:
        for v in volumes:
            if v.HasField("disk") and v.disk.HasField("persistence") and v.disk.persistence.id:
                if v.disk.HasField("source") and v.disk.source.type == P.Resource.DiskInfo.Source.MOUNT:
                    path = os.path.join(self.mount_dir(agent.spec.hostname, v.disk.source.mount.root),
                                        _safe(v.disk.persistence.id))
                else:
                    path = self.volume_dir(agent.spec.hostname, v.disk.persistence.id)
                shutil.rmtree(path, ignore_errors=True)

    # -- test hooks ---------------------------------------------------------------------
    def exec_in_task(self, task_id: str, cmd: str, timeout_s: float = 30.0) -> Tuple[int, str, str]:
        """``dcos task exec``: run ``cmd`` in the task's sandbox with its environment."""
        with self._lock:
            proc = self._procs.get(task_id)
        if proc is None:
            raise KeyError(task_id)
        r = subprocess.run(["bash", "-c", cmd], cwd=proc.sandbox, env=proc.env, stdin=subprocess.DEVNULL,
                           capture_output=True, timeout=timeout_s, start_new_session=True)
        return r.returncode, r.stdout.decode("utf-8", "replace"), r.stderr.decode("utf-8", "replace")

    def kill_with_pattern(self, pattern: str, agent_host: Optional[str] = None, sig: int = signal.SIGKILL,
                          oldest: bool = False) -> int:
        """``pkill [-o] -<sig> -f <pattern>`` over the processes of the tasks this runtime started
        (optionally only on one agent; ``oldest``: only the longest-running match). Returns how
        many processes were signalled."""
        rx = re.compile(pattern)
        with self._lock:
            procs = [p for p in self._procs.values() if not p.exited.is_set()
                     and (agent_host is None or p.agent_host == agent_host)]
        matches = []
        for p in procs:
            sid = self._pid(p)
            if sid <= 0:
                continue
            for pid in _session_pids(sid):
                if rx.search(_cmdline(pid)):
                    matches.append(pid)
        if oldest and matches:
            matches = [min(matches, key=_start_ticks)]
        n = 0
        for pid in matches:
            try:
                os.kill(pid, sig)
                n += 1
            except ProcessLookupError:
                pass
        return n

    def running_task_ids(self) -> List[str]:
        with self._lock:
            return [t for t, p in self._procs.items() if not p.exited.is_set()]

    def shutdown(self) -> None:
        with self._lock:
            procs = list(self._procs.values())
        for p in procs:
            if not p.exited.is_set():
                p.killed = True
                p.health_stop.set()
                self._signal_session(p, signal.SIGKILL)
        for p in procs:
            p.exited.wait(5.0)
        native, self._native = self._native, False
        if native:
            native.close()
