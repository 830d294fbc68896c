"""Marathon stand-in: runs and supervises each service's scheduler as a real OS process.

On DC/OS a service's scheduler is a Marathon app; Marathon restarts it when it exits and rolls it
when its definition changes (``dcos <svc> update``, ``sdk_marathon.update_app``); the scheduler
resumes from ZooKeeper. Here each app's ``cmd`` runs under ``bash -c`` in its own session and
sandbox (``<work>/marathon/<app>/<task id>``), with the app's ``env`` plus what Marathon and the
cluster provide: ``PORT0``/``PORT_API`` (a free loopback port), ``MARATHON_APP_ID``,
``MESOS_SANDBOX``, the Mesos master URL (``SDK_MESOS_MASTER``), the ZooKeeper connect string
(``SDK_ZOOKEEPER``, ``SDK_PERSISTER=zk``) and ``PYTHONPATH`` for this SDK.

* **task ids**: ``<app id reversed and dotted>.<uuid>`` (``/test/integration/hw`` ->
  ``hw.integration.test.<uuid>``), a new one per (re)start, as Marathon does;
* **restart policy**: an exit that was not asked for (crash, ``ProcessExit``, ``kill_scheduler``)
  is followed by a relaunch after ``restart_backoff_s``;
* **deployments**: install/update/restart complete once the new scheduler serves its API.
"""
from __future__ import annotations

import copy
import json
import logging
import os
import signal
import socket
import subprocess
import threading
import time
import urllib.error
import urllib.request
import uuid
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Tuple

LOGGER = logging.getLogger(__name__)
REPO_ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def normalize_app_id(app_id: str) -> str:
    return "/" + app_id.strip("/")


def scheduler_task_prefix(app_id: str) -> str:
    """``/path/to/svc`` -> ``svc.to.path`` (Marathon's task-id mangling of foldered app ids)."""
    parts = app_id.strip("/").split("/")
    return ".".join(reversed(parts))


def free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@dataclass
class MarathonTask:
    id: str
    app_id: str
    host: str
    ports: List[int]
    sandbox: str
    started_at: float
    state: str = "TASK_RUNNING"
    exit_code: Optional[int] = None

    def to_json(self) -> dict:
        return {"id": self.id, "appId": self.app_id, "host": self.host, "ports": list(self.ports),
                "state": self.state, "startedAt": time.strftime("%Y-%m-%dT%H:%M:%S", time.gmtime(self.started_at)),
                "sandbox": self.sandbox}


DEFAULT_APP_ROLE = "slave_public"


@dataclass
class _App:
    id: str
    definition: dict
    version: str
    api_port: int
    proc: Optional[subprocess.Popen] = None
    task: Optional[MarathonTask] = None
    history: List[MarathonTask] = field(default_factory=list)
    stopping: bool = False
    destroyed: bool = False
    restarts: int = 0
    deployed: threading.Event = field(default_factory=threading.Event)
    lock: threading.Lock = field(default_factory=threading.Lock)
    supervisor: Optional[threading.Thread] = None
    running_version: str = ""


class LocalMarathon:
    def __init__(self, cluster, restart_backoff_s: float = 0.5, deploy_timeout_s: float = 60.0):
        self.cluster = cluster
        self.restart_backoff_s = restart_backoff_s
        self.deploy_timeout_s = deploy_timeout_s
        self._apps: Dict[str, _App] = {}
        self._groups: Dict[str, dict] = {}   # top-level group id -> definition ({"enforceRole": bool})
        self._lock = threading.Lock()

    # -- groups and roles (Marathon 1.9 quota support) ---------------------------------------
    def create_group(self, definition: dict) -> None:
        gid = normalize_app_id(definition["id"])
        with self._lock:
            if gid in self._groups:
                raise ValueError(f"Group {gid} is already created. Use PUT to change this group.")
            self._groups[gid] = copy.deepcopy(definition)

    def update_group(self, definition: dict) -> None:
        gid = normalize_app_id(definition["id"])
        with self._lock:
            self._groups.setdefault(gid, {"id": gid}).update(copy.deepcopy(definition))

    def delete_group(self, group_id: str) -> None:
        gid = normalize_app_id(group_id)
        for app_id in [a for a in self.app_ids() if a.startswith(gid + "/")]:
            self.destroy_app(app_id)
        with self._lock:
            self._groups.pop(gid, None)

    def groups(self) -> List[dict]:
        with self._lock:
            return [copy.deepcopy(g) for _, g in sorted(self._groups.items())]

    def app_role(self, app_id: str, requested: Optional[str]) -> Tuple[str, bool]:
        """(role, enforced) of an app: in a top-level group with ``enforceRole`` the group's name is
        the only valid role; otherwise an app may ask for ``slave_public`` (the default) or its
        top-level group's name, and any other role is reset to ``slave_public``."""
        parts = normalize_app_id(app_id).strip("/").split("/")
        group = "/" + parts[0] if len(parts) > 1 else None
        with self._lock:
            g = self._groups.get(group) if group else None
        if g is not None and g.get("enforceRole"):
            return parts[0], True
        if requested and group is not None and requested == parts[0]:
            return requested, False
        return DEFAULT_APP_ROLE, False

    # -- queries ---------------------------------------------------------------------------
    def app_ids(self) -> List[str]:
        with self._lock:
            return sorted(a for a, app in self._apps.items() if not app.destroyed)

    def app_exists(self, app_id: str) -> bool:
        return normalize_app_id(app_id) in self.app_ids()

    def _get(self, app_id: str) -> _App:
        with self._lock:
            app = self._apps.get(normalize_app_id(app_id))
        if app is None or app.destroyed:
            raise KeyError(f"App '{normalize_app_id(app_id)}' does not exist")
        return app

    def get_app(self, app_id: str) -> dict:
        """The app definition as ``GET /v2/apps/<id>`` returns it (``app`` field)."""
        app = self._get(app_id)
        out = copy.deepcopy(app.definition)
        out["id"] = app.id
        out["version"] = app.version
        out["tasks"] = [app.task.to_json()] if app.task is not None and app.task.state == "TASK_RUNNING" else []
        out["tasksRunning"] = len(out["tasks"])
        out["deployments"] = [] if app.deployed.is_set() else [{"id": app.version}]
        return out

    def scheduler_url(self, app_id: str) -> str:
        return f"http://127.0.0.1:{self._get(app_id).api_port}"

    def tasks(self, prefix: str = "") -> List[MarathonTask]:
        with self._lock:
            apps = list(self._apps.values())
        out = []
        for app in apps:
            for t in app.history:
                if t.id.startswith(prefix):
                    out.append(t)
        return out

    def sandbox(self, app_id: str) -> Optional[str]:
        app = self._get(app_id)
        return app.task.sandbox if app.task is not None else None

    # -- lifecycle ---------------------------------------------------------------------------
    def install_app(self, definition: dict, wait: bool = True) -> dict:
        app_id = normalize_app_id(definition["id"])
        with self._lock:
            existing = self._apps.get(app_id)
            if existing is not None and not existing.destroyed:
                raise ValueError(f"An app with id [{app_id}] already exists.")
            app = _App(app_id, copy.deepcopy(definition), uuid.uuid4().hex, free_port())
            self._apps[app_id] = app
        app.supervisor = threading.Thread(target=self._supervise, args=(app,), name=f"marathon{app_id}", daemon=True)
        app.supervisor.start()
        if wait:
            self.wait_for_deployment(app_id)
        return self.get_app(app_id)

    def update_app(self, definition: dict, wait: bool = True) -> dict:
        """Replaces the app definition and rolls the scheduler (``PUT /v2/apps/<id>?force=true``)."""
        app = self._get(definition["id"])
        with app.lock:
            keep = {"id": app.id}
            app.definition = {**copy.deepcopy(definition), **keep}
            app.version = uuid.uuid4().hex
            app.deployed.clear()
        self._bounce(app)
        if wait:
            self.wait_for_deployment(app.id)
        return self.get_app(app.id)

    def restart_app(self, app_id: str, wait: bool = True) -> dict:
        app = self._get(app_id)
        with app.lock:
            app.version = uuid.uuid4().hex
            app.deployed.clear()
        self._bounce(app)
        if wait:
            self.wait_for_deployment(app.id)
        return self.get_app(app.id)

    def destroy_app(self, app_id: str, timeout_s: float = 30.0) -> None:
        app = self._get(app_id)
        app.destroyed = True
        self._stop_process(app, timeout_s)
        if app.supervisor is not None:
            app.supervisor.join(timeout_s)

    def kill_scheduler(self, app_id: str, sig: int = signal.SIGKILL) -> str:
        """Kills the scheduler process without telling Marathon (a crash); returns the task id
        that died. The restart policy relaunches it under a new task id."""
        app = self._get(app_id)
        with app.lock:
            proc, task = app.proc, app.task
        if proc is None or task is None:
            raise RuntimeError(f"{app.id} has no running scheduler")
        os.killpg(proc.pid, sig)
        return task.id

    def kill_with_pattern(self, pattern: str, oldest: bool = False, host: Optional[str] = None) -> int:
        """``pkill -9 -f`` over the scheduler processes (and their children); with ``host``, only
        over those of schedulers placed on that agent."""
        import re

        from dcos_commons_amd.mesos.containerizer import _cmdline, _session_pids, _start_ticks

        rx = re.compile(pattern)
        with self._lock:
            procs = [a.proc for a in self._apps.values() if a.proc is not None and a.proc.poll() is None
                     and (host is None or (a.task is not None and a.task.host == host))]
        matches = [pid for p in procs for pid in _session_pids(p.pid) if rx.search(_cmdline(pid))]
        if oldest and matches:
            matches = [min(matches, key=_start_ticks)]
        n = 0
        for pid in matches:
            try:
                os.kill(pid, signal.SIGKILL)
                n += 1
            except ProcessLookupError:
                pass
        return n

    def wait_for_deployment(self, app_id: str, timeout_s: Optional[float] = None) -> None:
        app = self._get(app_id)
        if not app.deployed.wait(self.deploy_timeout_s if timeout_s is None else timeout_s):
            raise TimeoutError(f"Marathon deployment of {app.id} did not finish; "
                               f"scheduler log tail:\n{self.log_tail(app.id)}")

    def log_tail(self, app_id: str, n: int = 40) -> str:
        app = self._get(app_id)
        if app.task is None:
            return ""
        out = []
        for name in ("stdout", "stderr"):
            try:
                with open(os.path.join(app.task.sandbox, name), "rb") as f:
                    lines = f.read().decode("utf-8", "replace").splitlines()[-n:]
                out.append(f"--- {name} ---\n" + "\n".join(lines))
            except OSError:
                pass
        return "\n".join(out)

    def history_log_tails(self, app_id: str, n: int = 40) -> str:
        """Log tails of every scheduler process the app ever ran (also after it was destroyed)."""
        with self._lock:
            app = self._apps.get(normalize_app_id(app_id))
        if app is None:
            return ""
        out = []
        for t in app.history:
            for name in ("stderr",):
                try:
                    with open(os.path.join(t.sandbox, name), "rb") as f:
                        lines = f.read().decode("utf-8", "replace").splitlines()[-n:]
                    out.append(f"--- {t.id} ({t.state}, exit {t.exit_code}) {name} ---\n" + "\n".join(lines))
                except OSError:
                    pass
        return "\n".join(out)

    def shutdown(self) -> None:
        with self._lock:
            apps = list(self._apps.values())
        for app in apps:
            app.destroyed = True
        for app in apps:
            self._stop_process(app, 10.0)
        for app in apps:
            if app.supervisor is not None:
                app.supervisor.join(10.0)

    # -- process supervision --------------------------------------------------------------
    def _bounce(self, app: _App) -> None:
        """Stop the running scheduler; the supervisor starts the new version."""
        app.stopping = True
        self._stop_process(app, 30.0)

    def _stop_process(self, app: _App, timeout_s: float) -> None:
        with app.lock:
            proc = app.proc
        if proc is None or proc.poll() is not None:
            return
        try:
            os.killpg(proc.pid, signal.SIGTERM)
            proc.wait(timeout=min(timeout_s, 10.0))
        except subprocess.TimeoutExpired:
            os.killpg(proc.pid, signal.SIGKILL)
            proc.wait(timeout=timeout_s)
        except ProcessLookupError:
            pass

    def _environment(self, app: _App, task: MarathonTask) -> Dict[str, str]:
        env = {k: os.environ[k] for k in ("PATH", "LANG", "LC_ALL", "TZ", "TMPDIR", "HOME") if k in os.environ}
        env.update(self.cluster.scheduler_environment())
        secrets = app.definition.get("secrets") or {}
        for k, v in (app.definition.get("env") or {}).items():
            if isinstance(v, dict):  # {"secret": "<name>"} -> app "secrets": {"<name>": {"source": path}}
                source = (secrets.get(v.get("secret", "")) or {}).get("source")
                data = self.cluster.resolve_secret(source) if source else None
                if data is not None:
                    env[k] = data.decode("utf-8", "replace")
                continue
            env[k] = str(v)
        role, enforced = self.app_role(app.id, app.definition.get("role"))
        env.update({
            "MESOS_ALLOCATION_ROLE": role, "MARATHON_APP_ENFORCE_GROUP_ROLE": "true" if enforced else "false",
            "PORT0": str(app.api_port), "PORT_API": str(app.api_port), "PORT": str(app.api_port),
            "PORTS": str(app.api_port), "MARATHON_APP_ID": app.id, "MARATHON_APP_VERSION": app.version,
            "MESOS_TASK_ID": task.id, "MESOS_SANDBOX": task.sandbox, "HOST": task.host,
            "LIBPROCESS_IP": "127.0.0.1",
        })
        if self.cluster.metrics is not None:
            # a scheduler is a Marathon task: its StatsD reporter gets its container's socket
            from dcos_commons_amd.mesos.local_master import container_id_for

            env.update(self.cluster.metrics.container_env(
                container_id_for(task.id), self.cluster.agent_ids.get(task.host, task.host),
                {"task_name": app.id.strip("/"), "task_id": task.id, "framework_id": "marathon",
                 "hostname": task.host}))
        pp = env.get("PYTHONPATH", os.environ.get("PYTHONPATH", ""))
        env["PYTHONPATH"] = REPO_ROOT + (os.pathsep + pp if pp else "")
        return env

    def _start(self, app: _App) -> None:
        tid = f"{scheduler_task_prefix(app.id)}.{uuid.uuid4()}"
        sandbox = os.path.join(self.cluster.work_dir, "marathon", app.id.strip("/").replace("/", "_"), tid)
        os.makedirs(sandbox, exist_ok=True)
        task = MarathonTask(tid, app.id, self._place(app), [app.api_port], sandbox, time.time())
        env = self._environment(app, task)
        self._fetch(app.definition.get("fetch") or [], sandbox)
        cmd = app.definition.get("cmd") or ""
        with open(os.path.join(sandbox, "stdout"), "ab") as out, open(os.path.join(sandbox, "stderr"), "ab") as err:
            proc = subprocess.Popen(["bash", "-c", cmd], cwd=sandbox, env=env, stdin=subprocess.DEVNULL,
                                    stdout=out, stderr=err, start_new_session=True)
        with app.lock:
            app.proc, app.task = proc, task
            app.running_version = app.version
            app.history.append(task)
        LOGGER.info("Marathon started %s (%s, pid %d, api port %d)", app.id, tid, proc.pid, app.api_port)

    def _fetch(self, fetch: list, sandbox: str) -> None:
        """The app's ``fetch`` URIs, as the Mesos fetcher stages them into the scheduler's sandbox,
        from the cluster's artifact store (no network): a directory artifact stands for an
        extracted archive and its contents are copied in; a file is copied, and extracted when it
        is an archive and ``extract`` is not false. URIs the store does not hold (a JRE, the
        libmesos bundle: nothing this SDK's schedulers run) are skipped."""
        import shutil
        import urllib.parse

        for entry in fetch:
            uri = entry.get("uri", "") if isinstance(entry, dict) else str(entry)
            local = self.cluster.resolve_artifact(uri) if uri else None
            if local is None:
                LOGGER.info("marathon fetcher: skipping %s (not in the local artifact store)", uri)
                continue
            if os.path.isdir(local):
                for name in os.listdir(local):
                    src = os.path.join(local, name)
                    if os.path.isdir(src):
                        shutil.copytree(src, os.path.join(sandbox, name), dirs_exist_ok=True)
                    else:
                        shutil.copy2(src, os.path.join(sandbox, name))
                continue
            dest = os.path.join(sandbox, os.path.basename(urllib.parse.urlparse(uri).path) or "download")
            shutil.copy2(local, dest)
            if isinstance(entry, dict) and entry.get("executable"):
                os.chmod(dest, 0o755)
            elif (not isinstance(entry, dict) or entry.get("extract", True)) and \
                    dest.endswith((".zip", ".tar.gz", ".tgz", ".tar")):
                try:
                    shutil.unpack_archive(dest, sandbox)
                except (shutil.ReadError, ValueError, OSError) as e:
                    LOGGER.warning("marathon fetcher: cannot extract %s: %s", dest, e)

    def _place(self, app: _App) -> str:
        """The agent the scheduler task runs on. Without app ``constraints`` that is the loopback
        host (the master node of the stand-in); with them, the first active agent matching all of
        ``[field, LIKE|UNLIKE|CLUSTER|IS, value]`` on ``hostname`` or an agent attribute
        (Marathon's constraint operators; UNIQUE/GROUP_BY/MAX_PER hold for a single instance)."""
        import re

        constraints = app.definition.get("constraints") or []
        if not constraints:
            return "127.0.0.1"
        for a in sorted(self.cluster.agents(), key=lambda a: a["hostname"]):
            if not a["active"]:
                continue
            ok = True
            for c in constraints:
                field, op = c[0], c[1].upper()
                value = c[2] if len(c) > 2 else None
                actual = a["hostname"] if field == "hostname" else a["attributes"].get(field)
                if op in ("LIKE", "UNLIKE"):
                    hit = actual is not None and re.fullmatch(value, actual) is not None
                    ok &= hit if op == "LIKE" else not hit
                elif op in ("CLUSTER", "IS"):
                    ok &= actual == value
            if ok:
                return a["hostname"]
        raise RuntimeError(f"no agent satisfies the constraints {constraints} of {app.id}")

    def _api_up(self, app: _App) -> bool:
        try:
            with urllib.request.urlopen(f"http://127.0.0.1:{app.api_port}/v1/health", timeout=2) as r:
                return r.status < 500
        except urllib.error.HTTPError as e:
            return e.code < 500 or e.code == 503   # any answer from the scheduler means it is serving
        except (urllib.error.URLError, OSError):
            return False

    def _supervise(self, app: _App) -> None:
        while not app.destroyed:
            try:
                self._start(app)
            except RuntimeError as e:   # no agent satisfies the app's constraints (yet): stay waiting
                LOGGER.warning("Marathon: cannot place %s: %s", app.id, e)
                time.sleep(self.restart_backoff_s)
                continue
            proc = app.proc
            while proc.poll() is None:
                # only the process started for the current version completes a deployment (the
                # previous one may still be serving while it is being stopped)
                if not app.deployed.is_set() and app.running_version == app.version and self._api_up(app):
                    app.deployed.set()
                if app.destroyed:
                    break
                time.sleep(0.05)
            rc = proc.wait()
            # the task's command ended: as the Mesos executor destroys the task's container,
            # whatever it left running in its session (the scheduler under a killed shell) goes too
            try:
                os.killpg(proc.pid, signal.SIGKILL)
            except (ProcessLookupError, PermissionError):
                pass
            with app.lock:
                if app.task is not None:
                    app.task.state = "TASK_KILLED" if (app.stopping or app.destroyed) else \
                        ("TASK_FINISHED" if rc == 0 else "TASK_FAILED")
                    app.task.exit_code = rc
            if app.destroyed:
                break
            if app.stopping:
                app.stopping = False
                continue  # a roll: start the new version right away
            app.restarts += 1
            LOGGER.warning("Marathon: scheduler of %s exited with %s; restarting", app.id, rc)
            time.sleep(self.restart_backoff_s)
        with app.lock:
            app.proc = None


def app_json(app: dict) -> str:
    return json.dumps(app, indent=2, sort_keys=True)
