"""A local DC/OS stand-in that runs the SDK's frameworks end to end on one machine.

Reference: the system-integration tier of the reference (``testing/sdk_*.py`` driving
``frameworks/*/tests`` against a live DC/OS cluster). Pieces:

* **ZooKeeper** -- ``testing.zk_server.ZkServer`` (jute wire protocol); schedulers persist to it
  with ``SDK_PERSISTER=zk`` exactly as on DC/OS (``/dcos-service-<name>`` trees, service lock);
* **Mesos master + agents** -- ``LocalMaster`` behind ``HttpMaster`` (Mesos v1 scheduler HTTP
  API); agents carry hostnames, fault domains (region/zone), attributes and optional MI355X GPUs;
  with ``executor="process"`` every task command really runs (``mesos.containerizer``), with
  ``executor="synthetic"`` tasks follow a timeline (``finish_tasks`` names the ones that exit 0);
* **Marathon** -- ``LocalMarathon`` runs every scheduler as a supervised OS process;
* **Cosmos** -- ``LocalCosmos`` installs the universe packages under ``frameworks/*/universe``;
* **DNS** -- names under the cluster TLDs (``*.thisdcos.directory``, ``*.mesos``) resolve to the
  loopback address for the task fetcher;
* **fault injection** -- agent partition/reconnect, agent shutdown, agent decommission (GONE),
  ``pkill``-style kills inside task sessions, scheduler crashes.

``current()`` is the cluster the ``testing.sdk`` helpers act on (``use(cluster)`` sets it).
"""
from __future__ import annotations

import logging
import os
import shutil
import tempfile
import threading
import time
from dataclasses import dataclass, field
from typing import Dict, Iterable, List, Optional, Sequence

from dcos_commons_amd.mesos import protos as P
from dcos_commons_amd.mesos.http_master import HttpMaster
from dcos_commons_amd.mesos.local_master import (TERMINAL, AgentSpec, LocalMaster, TaskBehavior, TaskTiming,
                                                  gpu_agent_specs)
from dcos_commons_amd.testing.cluster.marathon import LocalMarathon
from dcos_commons_amd.testing.cluster.packages import LocalCosmos
from dcos_commons_amd.testing.zk_server import ZkServer

LOGGER = logging.getLogger(__name__)
CLUSTER_DNS_SUFFIXES = (".thisdcos.directory", ".mesos", ".dcos")
DEFAULT_REGION = "us-west-2"
DEFAULT_ZONES = ("us-west-2a", "us-west-2b", "us-west-2c")
# what a DC/OS private agent offers: everything above 1024 except the ports of the agent's own
# services (ZooKeeper 2181/3888, Mesos agent 5051, adminrouter 8080-8081, ...)
DCOS_AGENT_PORTS = ((1025, 2180), (2182, 3887), (3889, 5049), (5052, 8079), (8082, 8180), (8182, 32000))

class _ZkProcess:
    """The ZooKeeper stand-in in its own interpreter (``python -m dcos_commons_amd.testing.zk_server``),
    as ZooKeeper is its own JVM on a cluster: its request handling then does not share the GIL
    with the master, the agents and the bench driving them. Connection drops are not supported."""

    def __init__(self):
        self.proc = None
        self.port = 0

    @property
    def connect_string(self) -> str:
        return f"127.0.0.1:{self.port}"

    def start(self) -> "_ZkProcess":
        import socket
        import subprocess
        import sys

        from dcos_commons_amd.testing.cluster.marathon import REPO_ROOT, free_port

        self.port = free_port()
        env = dict(os.environ, PYTHONPATH=REPO_ROOT)
        self.proc = subprocess.Popen([sys.executable, "-m", "dcos_commons_amd.testing.zk_server", "--port",
                                      str(self.port)], env=env, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
        deadline = time.monotonic() + 30
        while True:
            try:
                socket.create_connection(("127.0.0.1", self.port), timeout=1).close()
                return self
            except OSError:
                if self.proc.poll() is not None or time.monotonic() > deadline:
                    self.stop()
                    raise RuntimeError("the ZooKeeper stand-in process did not start")
                time.sleep(0.05)

    def drop_connections(self) -> None:
        raise NotImplementedError("connection drops need the in-process ZooKeeper stand-in")

    def stop(self) -> None:
        if self.proc is not None and self.proc.poll() is None:
            self.proc.terminate()
            try:
                self.proc.wait(5)
            except Exception:  # noqa: BLE001
                self.proc.kill()
                self.proc.wait(5)


_current: Optional["LocalCluster"] = None
_current_lock = threading.Lock()


def current() -> "LocalCluster":
    if _current is None:
        raise RuntimeError("No local cluster is active: create one with LocalCluster(...).start() and use() it")
    return _current


def use(cluster: Optional["LocalCluster"]) -> None:
    global _current
    with _current_lock:
        _current = cluster


@dataclass
class TaskView:
    """One task as ``dcos task --json`` / ``/mesos/tasks`` show it."""
    id: str
    name: str
    framework_id: str
    framework_name: str
    agent_id: str
    host: str
    state: str
    resources: Dict[str, float]
    labels: Dict[str, str]
    statuses: List[P.TaskStatus] = field(default_factory=list)

    @property
    def is_terminal(self) -> bool:
        return P.TaskState.Value(self.state) in TERMINAL


class _SyntheticBehavior(TaskBehavior):
    """Synthetic lifecycle; tasks whose name ends with one of ``finish_suffixes`` exit 0."""

    def __init__(self, finish_suffixes: Sequence[str], finish_after_s: float = 0.2, honor_check_delays: bool = True):
        super().__init__(TaskTiming(honor_check_delays=honor_check_delays))
        self.finish_suffixes = tuple(finish_suffixes)
        self.finish = TaskTiming(finish_after_s=finish_after_s, exit_state=P.TASK_FINISHED,
                                 honor_check_delays=honor_check_delays)

    def timing(self, task: P.TaskInfo) -> TaskTiming:
        if self.finish_suffixes and task.name.endswith(self.finish_suffixes):
            return self.finish
        return self.default


class LocalCluster:
    def __init__(self, agents: int = 5, agent_specs: Optional[Iterable[AgentSpec]] = None,
                 work_dir: Optional[str] = None, executor: str = "process", allocation_interval_s: float = 0.1,
                 region: str = DEFAULT_REGION, zones: Sequence[str] = DEFAULT_ZONES, gpus_per_agent: int = 0,
                 agent_cpus: float = 8.0, agent_mem: float = 32768.0, agent_disk: float = 65536.0,
                 packages: Optional[Dict[str, str]] = None, scheduler_env: Optional[Dict[str, str]] = None,
                 finish_tasks: Sequence[str] = (), dcos_version: str = "1.13.0", keep_work_dir: bool = False,
                 mount_disks: Sequence[tuple] = (), dcos_security: bool = False, zk_process: bool = False,
                 gpu_probe_service: bool = False, gpu_inventory=None, finish_after_s: float = 0.2,
                 honor_check_delays: bool = True):
        self.work_dir = os.path.abspath(work_dir or tempfile.mkdtemp(prefix="sdk-cluster-"))
        self._own_work_dir = work_dir is None and not keep_work_dir
        self.region = region
        self.dcos_version = dcos_version
        self.extra_scheduler_env = dict(scheduler_env or {})
        self.artifacts: Dict[str, str] = {}   # URI basename -> local file or extracted-archive directory
        self._stage_native_artifacts()
        self.secrets: Dict[str, bytes] = {}
        # DC/OS Enterprise services (IAM login, secrets API, CA) for strict-mode scenarios: the
        # schedulers' TLS artifacts and service-account logins go through them
        self.dcos = None
        if dcos_security:
            from dcos_commons_amd.testing.dcos_fakes import FakeDcosCluster

            self.dcos = FakeDcosCluster(require_auth=True, intermediate_ca=True, version=dcos_version)
        if executor == "process":
            from dcos_commons_amd.mesos.containerizer import ProcessTaskBehavior

            from dcos_commons_amd.testing.cluster.marathon import REPO_ROOT

            # tasks see this SDK's python package (what a fetched artifact provides on DC/OS: e.g.
            # the MI355X readiness probe `python3 -m dcos_commons_amd.ops.gpu_health`) and the
            # host's ROCm/HSA settings
            task_env = {"PYTHONPATH": REPO_ROOT}
            task_env.update({k: v for k, v in os.environ.items()
                             if k.startswith(("HSA_", "ROCM_", "HIP_PLATFORM", "LD_LIBRARY_PATH"))})
            self.behavior = ProcessTaskBehavior(os.path.join(self.work_dir, "agents"),
                                                secret_resolver=self.resolve_secret, resolver=self.resolve,
                                                artifact_resolver=self.resolve_artifact, extra_env=task_env)
        elif executor == "synthetic":
            # finish_after_s: how long a synthetic ONCE/FINISH task runs before it exits 0;
            # honor_check_delays=False starts readiness checks at once (a package's check delay
            # covers a real process's start-up, which a synthetic task does not have)
            self.behavior = _SyntheticBehavior(finish_tasks, finish_after_s, honor_check_delays)
        else:
            raise ValueError(f"executor must be 'process' or 'synthetic', not {executor!r}")
        self.executor = executor
        if agent_specs is None:
            # GPU agents split this node's discovered GPUs (ops.gpu: KFD topology / amd-smi), with
            # their model and xGMI hive as attributes; a driverless node gets synthetic MI355X ones
            agent_specs = gpu_agent_specs(agents, gpus_per_agent, lambda i: f"10.0.0.{i + 1}", inventory=gpu_inventory,
                                          cpus=agent_cpus, mem=agent_mem, disk=agent_disk, ports=DCOS_AGENT_PORTS,
                                          region=region, mount_disks=tuple(mount_disks))
            for i, spec in enumerate(agent_specs):
                spec.zone = zones[i % len(zones)] if zones else None
        self._agent_specs = list(agent_specs)
        domain = P.DomainInfo()
        domain.fault_domain.region.name = region
        domain.fault_domain.zone.name = zones[0] if zones else "local"
        self.master = LocalMaster(allocation_interval_s=allocation_interval_s, behavior=self.behavior, domain=domain)
        self.master.add_status_listener(self._on_status)
        self._tasks: Dict[str, TaskView] = {}
        self._tasks_lock = threading.Lock()
        self.agent_ids: Dict[str, str] = {}  # hostname -> agent id
        self.zk = None  # ZkServer, or a _ZkProcess with zk_process=True
        self.zk_process = zk_process
        # the node's GPU readiness service (ops.probe_service): tasks find it through
        # AMD_GPU_PROBE_SOCKET, and `amd-gpu-ready` checks run against the resident HIP runtime
        if gpu_probe_service and executor != "process":
            raise ValueError("gpu_probe_service needs executor='process' (the checks are task commands)")
        self.gpu_probe_service = gpu_probe_service
        self.probe_service = None
        self.metrics = None   # testing.cluster.metrics.LocalMetrics, from start()
        self.http_master: Optional[HttpMaster] = None
        self.marathon = LocalMarathon(self)
        from dcos_commons_amd.testing.cluster.metronome import LocalMetronome

        self.metronome = LocalMetronome(self)
        self.cosmos = LocalCosmos(self, packages)
        self._started = False

    # -- lifecycle -------------------------------------------------------------------------
    def start(self) -> "LocalCluster":
        self._started = True   # a start that fails part-way is shut down: no ZooKeeper process left behind
        try:
            if self.dcos is not None:
                self.dcos.start()
            self.zk = _ZkProcess().start() if self.zk_process else ZkServer().start()
            if self.gpu_probe_service:
                from dcos_commons_amd.ops.probe_service import ProbeService

                self.probe_service = ProbeService(os.path.join(self.work_dir, "gpu-probe.sock")).start()
                self.behavior.extra_env.update(self.probe_service.task_env)
            from dcos_commons_amd.testing.cluster.metrics import LocalMetrics

            self.metrics = LocalMetrics()
            if hasattr(self.behavior, "metrics"):
                self.behavior.metrics = self.metrics
            self.http_master = HttpMaster(self.master).start()
            for spec in self._agent_specs:
                self.agent_ids[spec.hostname] = self.master.add_agent(spec)
        except BaseException:
            self.shutdown()
            raise
        return self

    def shutdown(self) -> None:
        if not self._started:
            return
        self._started = False
        self.marathon.shutdown()
        self.metronome.shutdown()
        if self.http_master is not None:
            self.http_master.stop()
        self.master.shutdown()
        if self.probe_service is not None:
            self.probe_service.stop()
        if self.metrics is not None:
            self.metrics.stop()
            self.metrics = None
        if self.zk is not None:
            self.zk.stop()
        if self.dcos is not None:
            self.dcos.stop()
        if _current is self:
            use(None)
        if self._own_work_dir:
            shutil.rmtree(self.work_dir, ignore_errors=True)

    def __enter__(self) -> "LocalCluster":
        if not self._started:
            self.start()
        use(self)
        return self

    def __exit__(self, *exc) -> None:
        self.shutdown()

    # -- what Marathon hands every scheduler ---------------------------------------------------
    def scheduler_environment(self) -> Dict[str, str]:
        env = {
            "SDK_MESOS_MASTER": self.http_master.url, "SDK_MESOS_CONTENT_TYPE": "protobuf",
            "SDK_PERSISTER": "zk", "SDK_ZOOKEEPER": self.zk.connect_string,
            "SDK_API_HOST": "127.0.0.1", "DCOS_VERSION": self.dcos_version,
            # a killed scheduler's ZooKeeper lease (and lock) expires within 2 s, not 10
            "SDK_ZK_SESSION_TIMEOUT_MS": "2000",
            "FRAMEWORK_LOG_LEVEL": "INFO",
        }
        if self.dcos is not None:
            env["SDK_DCOS_MASTER_URI"] = self.dcos.url
        env.update(self.extra_scheduler_env)
        return env

    def resolve_secret(self, path: str) -> Optional[bytes]:
        """The DC/OS secret store as Mesos' secret resolver sees it: secrets created through the
        CLI, then (strict mode) those the schedulers wrote through the secrets API, e.g. TLS
        artifacts; values of ``__dcos_base64__``-prefixed secrets are base64-decoded."""
        path = path.strip("/")
        if path in self.secrets:
            return self.secrets[path]
        if self.dcos is None:
            return None
        with self.dcos._lock:
            entry = self.dcos.secrets.get(path)
        if entry is None or "value" not in entry:
            return None
        value = entry["value"]
        if os.path.basename(path).startswith("__dcos_base64__"):
            import base64

            return base64.b64decode(value)
        return value.encode("utf-8") if isinstance(value, str) else value

    def _stage_native_artifacts(self) -> None:
        """``bootstrap.zip`` (every SDK task fetches it) holds this tree's native ``sdk-bootstrap``;
        ``keytab-fix.tar.gz`` (Kerberized hdfs tasks) its native ``keytab-fix``."""
        from dcos_commons_amd.testing.cluster.marathon import REPO_ROOT

        for artifact, built, name in (("bootstrap.zip", "sdk-bootstrap", "bootstrap"),
                                      ("keytab-fix.tar.gz", "keytab-fix", "keytab-fix")):
            binary = os.path.join(REPO_ROOT, "native", "build", built)
            if os.path.exists(binary):
                d = os.path.join(self.work_dir, "artifacts", name)
                os.makedirs(d, exist_ok=True)
                shutil.copy2(binary, os.path.join(d, name))
                self.artifacts[artifact] = d

    def register_artifact(self, basename: str, path: str) -> None:
        """Tasks fetching a URI that ends in ``basename`` get ``path`` (a file, or a directory
        standing for the extracted archive)."""
        self.artifacts[basename] = path

    def resolve_artifact(self, uri: str) -> Optional[str]:
        import urllib.parse

        return self.artifacts.get(os.path.basename(urllib.parse.urlparse(uri).path))

    @staticmethod
    def resolve(hostname: str) -> Optional[str]:
        if hostname in ("localhost", "127.0.0.1") or hostname.endswith(CLUSTER_DNS_SUFFIXES):
            return "127.0.0.1"
        return None

    # -- master views -----------------------------------------------------------------------
    def _on_status(self, framework_id: str, status: P.TaskStatus) -> None:
        # runs on the master's actor thread: master state is consistent here
        tid = status.task_id.value
        with self._tasks_lock:
            view = self._tasks.get(tid)
            if view is None:
                t = self.master._find_task(tid)
                if t is None:
                    return
                fw = self.master.frameworks.get(framework_id)
                agent = self.master.agents.get(t.agent_id)
                res: Dict[str, float] = {}
                for r in t.info.resources:
                    if r.type == P.Value.SCALAR:
                        res[r.name] = res.get(r.name, 0.0) + r.scalar.value
                    elif r.type == P.Value.RANGES:
                        res.setdefault(r.name, 0.0)
                view = TaskView(tid, t.info.name, framework_id, fw.info.name if fw is not None else "",
                                t.agent_id, agent.spec.hostname if agent is not None else "", "TASK_STAGING", res,
                                {l.key: l.value for l in t.info.labels.labels})
                self._tasks[tid] = view
            view.state = P.TaskState.Name(status.state)
            view.statuses.append(status)

    def frameworks(self, include_inactive: bool = False) -> List[dict]:
        def multi(fw) -> bool:
            return any(c.type == P.FrameworkInfo.Capability.MULTI_ROLE for c in fw.info.capabilities)

        def do():
            return [{"id": fid, "name": fw.info.name, "active": fw.connected, "roles": sorted(fw.roles),
                     "webui_url": fw.info.webui_url,
                     "role": None if multi(fw) else (fw.info.role or "*"), "multi_role": multi(fw)}
                    for fid, fw in self.master.frameworks.items() if include_inactive or fw.connected]
        return self.master.call(do)

    def framework_ids(self, name: str) -> List[str]:
        return [f["id"] for f in self.frameworks(include_inactive=True) if f["name"] == name]

    def tasks(self, framework_name: Optional[str] = None, include_terminal: bool = False) -> List[TaskView]:
        with self._tasks_lock:
            views = list(self._tasks.values())
        out = []
        for v in views:
            if framework_name is not None and v.framework_name != framework_name:
                continue
            if not include_terminal and v.is_terminal:
                continue
            out.append(v)
        return sorted(out, key=lambda v: (v.name, v.statuses[0].timestamp if v.statuses else 0.0))

    def task_roles(self, framework_name: str) -> Dict[str, str]:
        """task name -> the role its resources are allocated to (``/mesos/state`` ``tasks[].role``):
        the reservation role of its reserved resources."""
        from dcos_commons_amd.mesos.resource_math import effective_role

        def do():
            out: Dict[str, str] = {}
            for a in self.master.agents.values():
                for t in a.tasks.values():
                    fw = self.master.frameworks.get(t.framework_id)
                    if fw is None or fw.info.name != framework_name or t.status.state in TERMINAL:
                        continue
                    roles = [effective_role(r) for r in t.info.resources]
                    out[t.info.name] = next((r for r in roles if r != "*"), roles[0] if roles else "*")
            return out
        return self.master.call(do)

    def task(self, task_id: str) -> Optional[TaskView]:
        with self._tasks_lock:
            return self._tasks.get(task_id)

    def agents(self) -> List[dict]:
        def do():
            out = []
            for aid, a in self.master.agents.items():
                out.append({"id": aid, "hostname": a.spec.hostname, "active": a.active, "zone": a.spec.zone,
                            "region": a.spec.region, "attributes": dict(a.spec.attributes), "gpus": a.spec.gpus})
            return out
        return self.master.call(do)

    def reserved_resources(self, role: Optional[str] = None) -> List[tuple]:
        """(agent hostname, resource) for every dynamically reserved resource (optionally of one
        role) still held on an agent -- what an uninstall must leave empty."""
        from dcos_commons_amd.mesos.resource_math import effective_role

        out = []
        for a in self.agents():
            for r in self.master.reserved_resources(a["id"]):
                if role is None or effective_role(r) == role:
                    out.append((a["hostname"], r))
        return out

    def dns_enumerate(self) -> dict:
        """Mesos-DNS ``/v1/enumerate``: per framework, each running task's A record
        ``<task>.<framework>.mesos.`` and one SRV record per named discovery port,
        ``_<port name>._<discovery name>._<protocol>.<framework>.mesos.``, pointing at the task's
        address. Tasks without ports only get the A record."""
        def do():
            fws: Dict[str, dict] = {}
            for fid, fw in self.master.frameworks.items():
                fws[fid] = {"name": fw.info.name, "tasks": []}
            for a in self.master.agents.values():
                for t in a.tasks.values():
                    if P.TaskState.Value("TASK_RUNNING") != t.status.state or t.framework_id not in fws:
                        continue
                    fw_name = fws[t.framework_id]["name"].replace("/", "")
                    ip = next((x.ip_address for n in t.networks for x in n.ip_addresses), a.ip)
                    d = t.info.discovery if t.info.HasField("discovery") else None
                    dns_name = d.name if d is not None and d.name else t.info.name
                    records = [{"name": f"{dns_name}.{fw_name}.mesos.", "host": ip, "rtype": "A"}]
                    for port in (d.ports.ports if d is not None else ()):
                        if not port.name:
                            continue
                        proto = port.protocol or "tcp"
                        records.append({"name": f"_{port.name}._{dns_name}._{proto}.{fw_name}.mesos.",
                                        "host": f"{ip}:{port.number}", "rtype": "SRV"})
                    fws[t.framework_id]["tasks"].append({"name": t.info.name, "records": records})
            return {"frameworks": list(fws.values())}
        return self.master.call(do)

    def zk_children(self, path: str = "/") -> List[str]:
        from dcos_commons_amd.storage.zookeeper import ZkClient

        c = ZkClient(self.zk.connect_string).start()
        try:
            return sorted(c.get_children(path))
        finally:
            c.close()

    # -- fault injection ------------------------------------------------------------------
    def _agent(self, host: str) -> str:
        aid = self.agent_ids.get(host)
        if aid is None:
            raise KeyError(f"no agent with hostname {host}")
        return aid

    def partition_agent(self, host: str) -> None:
        self.master.lose_agent(self._agent(host))

    def reconnect_agent(self, host: str) -> None:
        self.master.reconnect_agent(self._agent(host))

    def decommission_agent(self, host: str) -> None:
        """The operator marks the agent GONE (``dcos node decommission``)."""
        self.master.gone_by_operator(self._agent(host))

    def create_testing_volumes(self, count: int = 2, size_mb: float = 10240.0, profile: Optional[str] = None,
                               hosts: Optional[Sequence[str]] = None) -> List[str]:
        """``/dcos/volume<i>`` MOUNT disks on every agent (or on ``hosts``), numbered after the
        ones the agent already has (reference tools/create_testing_volumes.py); returns the roots."""
        roots: List[str] = []
        for host, aid in sorted(self.agent_ids.items()):
            if hosts is not None and host not in hosts:
                continue
            spec = self.master.agents[aid].spec
            start = len(spec.mount_disks)
            disks = [(f"/dcos/volume{start + i}", float(size_mb)) + ((profile,) if profile else ())
                     for i in range(count)]
            self.master.add_mount_disks(aid, disks)
            roots.extend(d[0] for d in disks)
        return roots

    def add_agent(self, spec: AgentSpec) -> str:
        aid = self.master.add_agent(spec)
        self.agent_ids[spec.hostname] = aid
        return aid

    def kill_task_with_pattern(self, pattern: str, agent_host: Optional[str] = None, oldest: bool = False) -> int:
        """``pkill -9 [-o] -f pattern`` on one host (or the master host when ``agent_host`` is None):
        the processes of task sandboxes and of the scheduler processes Marathon runs (those run on
        the loopback host). The cluster's own master and ZooKeeper are in-process: a pattern naming
        them (``mesos-master``, ``QuorumPeerMain``) drops all their connections instead, which is
        what their clients observe when the process dies and is restarted."""
        import re as _re

        if agent_host is None and _re.search(pattern, "mesos-master"):
            self.http_master.drop_streams()
            return 1
        if agent_host is None and _re.search(pattern, "org.apache.zookeeper.server.quorum.QuorumPeerMain"):
            self.zk.drop_connections()
            return 1
        n = 0
        if agent_host in (None, "127.0.0.1", "localhost"):
            n += self.marathon.kill_with_pattern(pattern, oldest=oldest)
            if n and oldest:
                return n
        else:   # a scheduler placed on this agent by its app constraints
            n += self.marathon.kill_with_pattern(pattern, oldest=oldest, host=agent_host)
            if n and oldest:
                return n
        if self.executor == "process" and agent_host not in ("127.0.0.1", "localhost"):
            n += self.behavior.kill_with_pattern(pattern, agent_host, oldest=oldest)
        return n

    def restart_master(self) -> None:
        """Master failover as the schedulers see it: every event stream is cut."""
        self.http_master.drop_streams()

    def fail_task(self, task_id: str, state: int = P.TASK_FAILED) -> None:
        """Synthetic-executor equivalent of killing a task's process."""
        self.master.fail_task(task_id, state)

    def task_exec(self, task_id: str, cmd: str, timeout_s: float = 30.0):
        if self.executor != "process":
            raise RuntimeError("task exec needs the process executor")
        return self.behavior.exec_in_task(task_id, cmd, timeout_s)

    def wait(self, predicate, timeout_s: float = 60.0, interval_s: float = 0.05, what: str = "condition"):
        deadline = time.time() + timeout_s
        while True:
            v = predicate()
            if v:
                return v
            if time.time() >= deadline:
                raise TimeoutError(f"timed out after {timeout_s}s waiting for {what}")
            time.sleep(interval_s)
