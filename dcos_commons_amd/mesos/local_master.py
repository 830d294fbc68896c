"""An in-process Mesos master + agents with a scheduler driver.

This is the cluster the scheduler talks to in tests, the simulation harness and the benchmark
(the reference talks to a real Mesos master through libmesos; none exists here). It models what
the SDK's timing and correctness depend on:

* **allocation** -- every ``allocation_interval_s`` (Mesos ``--allocation_interval``, default
  1 s) each subscribed, unsuppressed framework is offered the unreserved + role-reserved
  resources of every agent that has no outstanding offer and no active decline filter; REVIVE
  clears filters and triggers an immediate allocation;
* **offer operations** -- RESERVE / UNRESERVE / CREATE / DESTROY / LAUNCH_GROUP applied in
  order on the offered resources (``resource_math.ResourceBag``); leftovers go back to the agent
  with the ACCEPT's ``refuse_seconds`` filter;
* **task lifecycle** -- STAGING -> STARTING -> RUNNING (with an empty ``check_status`` when the
  task has a check, then ``exit_code`` once the readiness check passes, honouring
  ``delay_seconds``) -> terminal; KILL -> KILLED; executor resources are released when its last
  task ends; GPUs are assigned by device index (``HIP_VISIBLE_DEVICES`` for the task);
* **reconciliation** (implicit and explicit; an unknown task answers TASK_UNKNOWN to a
  partition-aware framework, TASK_LOST otherwise), **teardown**, and fault injection for
  recovery/MTTR measurements: ``fail_task``, ``send_status``, ``lose_agent`` /
  ``reconnect_agent`` (partition and return), ``gone_by_operator``, ``forget_task``,
  ``rescind_offers`` and ``drop_next_accepts`` (lost ACCEPT).

All state is owned by one dispatcher thread (an actor): driver calls and test hooks enqueue
actions, and scheduler callbacks are delivered from that thread in order.
"""
from __future__ import annotations

import contextlib
import heapq
import itertools
import logging
import threading
import time
import uuid
from concurrent.futures import Future
from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional, Set, Tuple

from dcos_commons_amd.framework.driver import SchedulerDriver
from dcos_commons_amd.mesos import protos as P
from dcos_commons_amd.mesos.resource_math import (
    InsufficientResources,
    ResourceBag,
    effective_role,
    pop_reservation,
    strip_volume,
)
from dcos_commons_amd import trace
from dcos_commons_amd.ops.gpu import select_devices
from dcos_commons_amd.utils import ids

LOGGER = logging.getLogger(__name__)
TERMINAL = {P.TASK_FINISHED, P.TASK_FAILED, P.TASK_KILLED, P.TASK_ERROR, P.TASK_LOST, P.TASK_DROPPED,
            P.TASK_GONE, P.TASK_GONE_BY_OPERATOR}


def scalar(name: str, value: float) -> P.Resource:
    r = P.Resource(name=name, type=P.Value.SCALAR)
    r.scalar.value = value
    return r


def ranges(name: str, intervals) -> P.Resource:
    r = P.Resource(name=name, type=P.Value.RANGES)
    r.ranges.SetInParent()
    for b, e in intervals:
        r.ranges.range.add(begin=b, end=e)
    return r


def text_attribute(name: str, value: str) -> P.Attribute:
    a = P.Attribute(name=name, type=P.Value.TEXT)
    a.text.value = value
    return a


@dataclass
class AgentSpec:
    hostname: str
    cpus: float = 8.0
    mem: float = 32768.0
    disk: float = 65536.0
    ports: Tuple[Tuple[int, int], ...] = ((10000, 20000),)
    gpus: int = 0
    gpu_devices: Optional[List[int]] = None  # physical device indices; default range(gpus)
    attributes: Dict[str, str] = field(default_factory=dict)
    zone: Optional[str] = None
    region: Optional[str] = None
    mount_disks: Tuple[tuple, ...] = ()  # (root, size) or (root, size, profile)
    pre_reserved: Tuple[Tuple[str, str, float], ...] = ()  # (role, resource name, amount)
    # device index -> xGMI hive id / direct xGMI peers (``ops.gpu`` discovery): a ``gpus: N`` task
    # gets N devices of one hive when the agent has them free (``ops.gpu.select_devices``)
    gpu_hives: Optional[Dict[int, str]] = None
    gpu_peers: Optional[Dict[int, Tuple[int, ...]]] = None

    @staticmethod
    def from_gpu_inventory(hostname: str, inventory, devices: Optional[List[int]] = None,
                           attributes: Optional[Dict[str, str]] = None, **kw) -> "AgentSpec":
        """An agent owning ``devices`` (default: all) of a discovered ``ops.gpu.GpuInventory``:
        ``gpus`` is their count, ``gpu_devices`` their indices, and the agent's attributes carry
        their vendor / model / arch / xGMI hive (``GpuInventory.attributes``)."""
        inv = inventory if devices is None else inventory.subset(devices)
        attrs = dict(inv.attributes())
        attrs.update(attributes or {})
        return AgentSpec(hostname=hostname, gpus=inv.count, gpu_devices=[d.index for d in inv.devices],
                         attributes=attrs, gpu_hives=inv.hive_map(),
                         gpu_peers={d.index: tuple(d.xgmi_peers) for d in inv.devices}, **kw)

    def resources(self) -> List[P.Resource]:
        out = []
        for name, amount in (("cpus", self.cpus), ("mem", self.mem), ("disk", self.disk)):
            if amount > 0:
                out.append(scalar(name, amount))
        if self.ports:
            out.append(ranges("ports", self.ports))
        if self.gpus:
            out.append(scalar("gpus", float(self.gpus)))
        for disk in self.mount_disks:
            # (root, size) or (root, size, profile): a profiled disk comes from a CSI volume
            # profile (DC/OS storage "volume_profile"), which MOUNT volumes may ask for by name
            root, size = disk[0], disk[1]
            r = scalar("disk", size)
            r.disk.source.type = P.Resource.DiskInfo.Source.MOUNT
            r.disk.source.mount.root = root
            if len(disk) > 2 and disk[2]:
                r.disk.source.profile = disk[2]
            out.append(r)
        # statically pre-reserved resources come out of the unreserved pool
        bag = ResourceBag(out)
        for role, name, amount in self.pre_reserved:
            bag.subtract(scalar(name, amount))
            r = scalar(name, amount)
            r.reservations.add(type=P.Resource.ReservationInfo.STATIC, role=role)
            bag.add(r)
        return bag.to_resources()

    def domain(self) -> Optional[P.DomainInfo]:
        if not self.zone and not self.region:
            return None
        d = P.DomainInfo()
        d.fault_domain.region.name = self.region or "default-region"
        d.fault_domain.zone.name = self.zone or "default-zone"
        return d


@dataclass
class TaskTiming:
    """Synthetic task lifecycle timing (seconds after the previous event)."""
    starting_s: float = 0.0
    running_s: float = 0.0
    honor_check_delays: bool = True
    check_exec_s: float = 0.0
    finish_after_s: Optional[float] = None  # None: runs until killed
    exit_state: int = P.TASK_FINISHED


class TaskBehavior:
    """Decides the lifecycle of a launched task; override ``timing`` for scenarios.

    ``check_runner(task_info, gpu_devices) -> bool`` executes a task's check (readiness) for real
    (e.g. the HIP GPU probe on the task's devices) on a worker thread; without it checks pass
    synthetically after ``delay_seconds + check_exec_s``.
    """

    def __init__(self, default: Optional[TaskTiming] = None,
                 overrides: Optional[Dict[str, TaskTiming]] = None,
                 check_runner: Optional[Callable[[P.TaskInfo, List[int]], bool]] = None,
                 check_workers: int = 8):
        self.default = default or TaskTiming()
        self.overrides = dict(overrides or {})
        self.check_runner = check_runner
        self._pool = None
        self._workers = check_workers

    def pool(self):
        if self._pool is None:
            from concurrent.futures import ThreadPoolExecutor

            self._pool = ThreadPoolExecutor(max_workers=self._workers, thread_name_prefix="task-check")
        return self._pool

    def prestart(self) -> "TaskBehavior":
        """Start every check worker now. An agent's check executor is already running when a task
        launches; without this the pool starts a thread at each of the first checks, inside the
        launch being timed."""
        import threading as _threading

        pool = self.pool()
        gate = _threading.Barrier(self._workers + 1)
        for _ in range(self._workers):
            pool.submit(gate.wait, 10.0)
        gate.wait(10.0)
        return self

    def timing(self, task: P.TaskInfo) -> TaskTiming:
        for k, v in self.overrides.items():
            if k in task.name:
                return v
        return self.default


@dataclass
class _Task:
    info: P.TaskInfo
    framework_id: str
    executor_id: str
    agent_id: str
    resources: List[P.Resource]
    gpu_devices: List[int]
    status: P.TaskStatus
    epoch: int = 0  # bumps on kill/failure so stale timers are ignored
    # the task's addresses as its statuses report them (``container_status.network_infos``)
    networks: List[P.NetworkInfo] = field(default_factory=list)
    reported_exit: bool = False   # its end came from its agent's runtime (no ``drop`` to send back)
    container_id: str = ""        # what its statuses report as container_status.container_id


def container_id_for(task_id: str) -> str:
    """The container ID a task's statuses report (``container_status.container_id``; the local
    cluster's metrics service files the task's StatsD under it): one per launch, as task IDs are."""
    return str(uuid.uuid5(uuid.NAMESPACE_URL, "mesos-task:" + task_id))


@dataclass
class _Executor:
    info: P.ExecutorInfo
    framework_id: str
    resources: List[P.Resource]
    tasks: Set[str] = field(default_factory=set)


# CNI networks that map container ports to host ports (the container is reached on the agent's address)
BRIDGE_NETWORKS = ("mesos-bridge", "bridge")


class _Agent:
    def __init__(self, agent_id: str, spec: AgentSpec):
        self.id = agent_id
        self.spec = spec
        self.available = ResourceBag(spec.resources())
        self.executors: Dict[Tuple[str, str], _Executor] = {}
        self.tasks: Dict[str, _Task] = {}
        devices = spec.gpu_devices if spec.gpu_devices is not None else list(range(spec.gpus))
        self.free_gpus: List[int] = list(devices)
        self.active = True
        self.check_runner = None  # per-agent check executor (e.g. a remote GPU agent)
        self.index = 0            # position among the master's agents (overlay subnet 9.0.<index>.0/24)
        self._overlay_ips = itertools.count(2)
        self._check_thread = None  # the agent's own thread for inline checks (see check_thread)
        # the agent runs its tasks' lifecycle itself (``mesos.agent_runtime``): an object whose
        # ``send(msg)`` reaches it; its reports come back through ``LocalMaster.runtime_reports``
        self.runtime = None

    def check_thread(self):
        """This agent's check executor: one thread, as a Mesos agent's executor runs its tasks'
        checks. Inline checks (one short native call, e.g. the fused HIP probe) run here, never on
        the master's event thread: a slow or hung probe on one GPU stalls only its own agent, and
        the checks of different agents' GPUs run in parallel."""
        if self._check_thread is None:
            from concurrent.futures import ThreadPoolExecutor

            self._check_thread = ThreadPoolExecutor(max_workers=1, thread_name_prefix=f"check-{self.spec.hostname}")
            self._check_thread.submit(lambda: None).result(10)   # started before any task launches
        return self._check_thread

    def close(self) -> None:
        if self._check_thread is not None:
            self._check_thread.shutdown(wait=False)

    @property
    def ip(self) -> str:
        """The agent's address: its hostname when that is an IPv4 literal (``10.0.0.3``)."""
        parts = self.spec.hostname.split(".")
        if len(parts) == 4 and all(p.isdigit() and int(p) < 256 for p in parts):
            return self.spec.hostname
        return "127.0.0.1"

    def task_networks(self, container: Optional[P.ContainerInfo]) -> List[P.NetworkInfo]:
        """Addresses of a container joining ``container.network_infos``, as Mesos reports them.

        Host networking (no network infos) reports the agent's address with no network name;
        bridge CNI networks with port mappings (``mesos-bridge``) name the network and are reached
        on the agent's address; any other named network is a virtual (overlay) network: the
        container gets its own address from the agent's overlay subnet ``9.0.<agent index>.0/24``
        and the status names the network and carries its labels (DC/OS ``dcos`` overlay,
        reference ``overlay.yml``)."""
        out: List[P.NetworkInfo] = []
        for ni in (container.network_infos if container is not None else ()):
            if not ni.name:
                continue
            n = P.NetworkInfo(name=ni.name)
            if ni.name in BRIDGE_NETWORKS:
                n.ip_addresses.add(ip_address=self.ip)
            else:
                n.ip_addresses.add(ip_address=f"9.0.{self.index % 256}.{next(self._overlay_ips) % 254 + 1}")
            if ni.HasField("labels"):
                n.labels.CopyFrom(ni.labels)
            out.append(n)
        if not out:
            n = P.NetworkInfo()
            n.ip_addresses.add(ip_address=self.ip)
            out.append(n)
        return out

    def info_attributes(self) -> List[P.Attribute]:
        return [text_attribute(k, v) for k, v in sorted(self.spec.attributes.items())]


@dataclass
class _Framework:
    id: str
    info: P.FrameworkInfo
    driver: "LocalSchedulerDriver"
    roles: Set[str]
    suppressed: bool = False
    connected: bool = True
    # agent id -> [(expiry, declined resources)]: Mesos' RefusedOfferFilter -- an agent's offer is
    # filtered only while everything it would contain is within a declined set
    filters: Dict[str, list] = field(default_factory=dict)
    # which of a MULTI_ROLE framework's roles gets the next agent's unreserved resources
    rr: int = 0


@dataclass
class _Offer:
    id: str
    framework_id: str
    agent_id: str
    resources: List[P.Resource]


class LocalMaster:
    def __init__(self, allocation_interval_s: float = 1.0, behavior: Optional[TaskBehavior] = None,
                 domain: Optional[P.DomainInfo] = None, offer_timeout_s: Optional[float] = None,
                 clock: Callable[[], float] = time.monotonic):
        self.allocation_interval_s = allocation_interval_s
        self.behavior = behavior or TaskBehavior()
        # () -> context manager around the delivery of one agent report batch: a network front end
        # (stream_api.StreamMaster) sets one that writes the batch's events to each framework's
        # connection in one write, so its scheduler reads them together
        self.batch_delivery: Callable[[], "contextlib.AbstractContextManager"] = contextlib.nullcontext
        # ProcessTaskBehavior (mesos.containerizer) runs task commands for real
        self._executes = bool(getattr(self.behavior, "executes_commands", False))
        self.domain = domain
        self.offer_timeout_s = offer_timeout_s
        self.clock = clock
        self.master_info = P.MasterInfo(id="local-master-" + uuid.uuid4().hex[:8], hostname="127.0.0.1",
                                        version="1.9.0-local")
        if domain is not None:
            self.master_info.domain.CopyFrom(domain)
        self.agents: Dict[str, _Agent] = {}
        self.frameworks: Dict[str, _Framework] = {}
        self.offers: Dict[str, _Offer] = {}
        self._seq = itertools.count()
        self._heap: List[tuple] = []
        self._cond = threading.Condition()
        self._running = True
        self._thread = threading.Thread(target=self._run, name="LocalMaster", daemon=True)
        self._listeners: List[Callable[[str, P.TaskStatus], None]] = []
        self.accept_calls = 0
        self.dropped_accepts = 0
        self._drop_accepts = 0
        self._drop_rescind_s = 0.5
        self.operations: List[Tuple[str, int]] = []  # (agent id, operation type) in applied order
        self._thread.start()
        self._schedule(self.allocation_interval_s, self._periodic_allocate)

    # -- actor plumbing ----------------------------------------------------------------
    def _schedule(self, delay: float, fn, *args) -> None:
        with self._cond:
            heapq.heappush(self._heap, (self.clock() + max(0.0, delay), next(self._seq), fn, args))
            self._cond.notify()

    def _after(self, delay: float, fn, *args) -> None:
        """A task's next lifecycle step: due now, it runs right here (an agent drives its own task
        from STARTING to RUNNING to its first check without queueing behind every other task's
        events, so the first readiness checks start while later tasks are still launching);
        otherwise it is scheduled."""
        if delay <= 0 and threading.current_thread() is self._thread:
            fn(*args)
        else:
            self._schedule(delay, fn, *args)

    def _run(self) -> None:
        while True:
            with self._cond:
                while self._running and (not self._heap or self._heap[0][0] > self.clock()):
                    timeout = None if not self._heap else max(0.0, self._heap[0][0] - self.clock())
                    self._cond.wait(timeout if timeout is None else min(timeout, 0.5))
                if not self._running:
                    return
                _, _, fn, args = heapq.heappop(self._heap)
            try:
                fn(*args)
            except Exception:  # noqa: BLE001
                LOGGER.exception("LocalMaster action %s failed", getattr(fn, "__name__", fn))

    def call(self, fn, *args, timeout: float = 30.0):
        """Run ``fn`` on the dispatcher thread and return its result (test hooks/queries)."""
        if threading.current_thread() is self._thread:
            return fn(*args)
        fut: Future = Future()

        def run():
            try:
                fut.set_result(fn(*args))
            except Exception as e:  # noqa: BLE001
                fut.set_exception(e)
        self._schedule(0, run)
        return fut.result(timeout)

    def shutdown(self) -> None:
        with self._cond:
            self._running = False
            self._cond.notify_all()
        if threading.current_thread() is not self._thread:
            self._thread.join(timeout=5)
        for a in list(self.agents.values()):
            a.close()
        stop = getattr(self.behavior, "shutdown", None)
        if callable(stop):
            stop()

    def add_status_listener(self, fn: Callable[[str, P.TaskStatus], None]) -> None:
        self._listeners.append(fn)

    # -- cluster management --------------------------------------------------------------
    def add_agent(self, spec: AgentSpec, check_runner=None, runtime=None) -> str:
        """``runtime``: the agent runs its tasks' lifecycle and checks itself (an object with
        ``send(msg)``, see ``mesos.agent_runtime``); the master then only applies ACCEPTs, keeps
        the books and turns the agent's reports into status updates."""
        def do():
            aid = f"agent-{len(self.agents)}-{uuid.uuid4().hex[:6]}"
            self.agents[aid] = _Agent(aid, spec)
            self.agents[aid].check_runner = check_runner
            self.agents[aid].runtime = runtime
            self.agents[aid].index = len(self.agents)
            self._allocate()
            return aid
        aid = self.call(do)
        runner = check_runner if check_runner is not None else self.behavior.check_runner
        if getattr(runner, "inline", False):
            self.agents[aid].check_thread()   # started now, outside any timed launch
        return aid

    def add_mount_disks(self, agent_id: str, disks) -> None:
        """Attach MOUNT disks (``(root, size[, profile])``) to a registered agent, as an agent
        restarted with new ``--resources`` re-registers with them; its tasks keep running."""
        def do():
            a = self.agents[agent_id]
            extra = AgentSpec(hostname=a.spec.hostname, cpus=0, mem=0, disk=0, ports=(),
                              mount_disks=tuple(disks)).resources()
            for r in extra:
                a.available.add(r)
            a.spec.mount_disks = tuple(a.spec.mount_disks) + tuple(disks)
            self._allocate()
        self.call(do)

    def lose_agent(self, agent_id: str, partition_aware: bool = True) -> None:
        """Agent disappears: outstanding offers are rescinded and its tasks go UNREACHABLE/LOST."""
        def do():
            a = self.agents[agent_id]
            a.active = False
            for oid in [o.id for o in self.offers.values() if o.agent_id == agent_id]:
                self._rescind(oid)
            for t in list(a.tasks.values()):
                if t.status.state in TERMINAL:
                    continue
                fw = self.frameworks.get(t.framework_id)
                aware = partition_aware and fw is not None and any(
                    c.type == P.FrameworkInfo.Capability.PARTITION_AWARE for c in fw.info.capabilities)
                self._update(t, P.TASK_UNREACHABLE if aware else P.TASK_LOST, source=P.TaskStatus.SOURCE_MASTER,
                             reason=P.TaskStatus.REASON_AGENT_REMOVED, message="Agent lost")
        self.call(do)

    def fail_task(self, task_id: str, state: int = P.TASK_FAILED, message: str = "injected failure") -> None:
        def do():
            t = self._find_task(task_id)
            if t is None:
                raise KeyError(task_id)
            a = self.agents.get(t.agent_id)
            if a is not None and a.runtime is not None and t.status.state not in TERMINAL:
                # the task dies on its agent, which reports it (as an executor would)
                a.runtime.send({"op": "fail", "task": task_id, "state": state, "message": message,
                                "reason": P.TaskStatus.REASON_COMMAND_EXECUTOR_FAILED})
                return
            self._update(t, state, message=message, reason=P.TaskStatus.REASON_COMMAND_EXECUTOR_FAILED)
        self.call(do)

    def send_status(self, task_id: str, state: int, **fields) -> None:
        def do():
            t = self._find_task(task_id)
            self._update(t, state, **fields)
        self.call(do)

    # -- fault injection (kill/lost/unreachable/gone task, agent loss and return,
    #    offer rescind, dropped ACCEPT) ---------------------------------------------------
    def rescind_offers(self, agent_id: Optional[str] = None) -> int:
        """Rescind every outstanding offer (of one agent); returns how many were rescinded."""
        def do():
            oids = [o.id for o in self.offers.values() if agent_id is None or o.agent_id == agent_id]
            for oid in oids:
                self._rescind(oid)
            return len(oids)
        return self.call(do)

    def drop_next_accepts(self, n: int = 1, rescind_after_s: float = 0.5) -> None:
        """The next ``n`` ACCEPT calls are lost in transit: nothing is applied and the scheduler
        hears nothing. The offers stay outstanding until the master's offer timeout rescinds them
        (``rescind_after_s``), as a real master would after a lost message."""
        def do():
            self._drop_accepts += n
            self._drop_rescind_s = rescind_after_s
        self.call(do)

    def gone_by_operator(self, agent_id: str) -> None:
        """The operator marks an agent GONE: its tasks report TASK_GONE_BY_OPERATOR and the agent
        (with its reservations) is removed for good."""
        def do():
            a = self.agents[agent_id]
            a.active = False
            for oid in [o.id for o in self.offers.values() if o.agent_id == agent_id]:
                self._rescind(oid)
            for t in list(a.tasks.values()):
                if t.status.state not in TERMINAL:
                    self._update(t, P.TASK_GONE_BY_OPERATOR, source=P.TaskStatus.SOURCE_MASTER,
                                 reason=P.TaskStatus.REASON_AGENT_REMOVED, message="Agent marked gone by operator")
            self.agents.pop(agent_id, None)
        self.call(do)

    def reconnect_agent(self, agent_id: str) -> None:
        """A partitioned agent (``lose_agent``) re-registers: tasks that were UNREACHABLE and
        are still alive on it report RUNNING again (Mesos' partition-aware re-registration)."""
        def do():
            a = self.agents[agent_id]
            a.active = True
            for t in list(a.tasks.values()):
                if t.status.state == P.TASK_UNREACHABLE:
                    self._update(t, P.TASK_RUNNING, source=P.TaskStatus.SOURCE_MASTER,
                                 message="Agent re-registered")
            self._allocate()
        self.call(do)

    def forget_task(self, task_id: str) -> None:
        """The master loses all knowledge of a task (e.g. agent wiped while the scheduler was
        down): no status is sent; reconciliation of it answers TASK_UNKNOWN / TASK_LOST."""
        def do():
            t = self._find_task(task_id)
            if t is not None:
                t.epoch += 1
                self._release_task(t)
                self.agents[t.agent_id].tasks.pop(task_id, None)
        self.call(do)

    def task_states(self, framework_id: Optional[str] = None) -> Dict[str, int]:
        def do():
            out = {}
            for a in self.agents.values():
                for tid, t in a.tasks.items():
                    if framework_id is None or t.framework_id == framework_id:
                        out[tid] = t.status.state
            return out
        return self.call(do)

    def tasks_by_name(self, include_terminal: bool = False) -> Dict[str, P.TaskInfo]:
        def do():
            out = {}
            for a in self.agents.values():
                for t in a.tasks.values():
                    if include_terminal or t.status.state not in TERMINAL:
                        out[t.info.name] = t.info
            return out
        return self.call(do)

    def placement(self) -> List[Dict]:
        """Where every live task runs: task name, agent hostname and attributes, and the GPU
        devices the agent assigned it (what ``HIP_VISIBLE_DEVICES`` carries)."""
        def do():
            out = []
            for a in self.agents.values():
                for t in a.tasks.values():
                    if t.status.state not in TERMINAL:
                        out.append({"task": t.info.name, "hostname": a.spec.hostname,
                                    "attributes": dict(a.spec.attributes), "gpu_devices": list(t.gpu_devices)})
            return sorted(out, key=lambda x: x["task"])
        return self.call(do)

    def agent_resources(self, agent_id: str) -> List[P.Resource]:
        return self.call(lambda: self.agents[agent_id].available.to_resources())

    def _held_resources(self, agent_id: str) -> List[P.Resource]:
        """Everything an agent holds: available, offered, and used by executors and live tasks."""
        a = self.agents[agent_id]
        rs = a.available.to_resources()
        for o in self.offers.values():
            if o.agent_id == agent_id:
                rs.extend(o.resources)
        for e in a.executors.values():
            rs.extend(e.resources)
        for t in a.tasks.values():
            if t.status.state not in TERMINAL:
                rs.extend(t.resources)
        return rs

    def reserved_resources(self, agent_id: str) -> List[P.Resource]:
        def do():
            return [r for r in self._held_resources(agent_id) if len(r.reservations) and
                    r.reservations[-1].type == P.Resource.ReservationInfo.DYNAMIC]
        return self.call(do)

    def persistent_volumes(self, agent_id: str) -> List[P.Resource]:
        """Persistent volumes on an agent, whatever their reservation (static or dynamic)."""
        def do():
            return [r for r in self._held_resources(agent_id) if r.HasField("disk") and r.disk.persistence.id]
        return self.call(do)

    # -- framework-facing API (called through LocalSchedulerDriver) -------------------------
    def subscribe(self, driver: "LocalSchedulerDriver", info: P.FrameworkInfo) -> None:
        def do():
            fid = info.id.value if info.HasField("id") and info.id.value else "fw-" + uuid.uuid4().hex
            roles = set(info.roles) if len(info.roles) else {info.role or "*"}
            existing = self.frameworks.get(fid)
            fw = _Framework(fid, info, driver, roles)
            if existing is not None:
                # failover: offers outstanding to the previous scheduler instance are recovered
                # (the new instance never saw them; Mesos rescinds them on failover)
                for oid in [o.id for o in self.offers.values() if o.framework_id == fid]:
                    self._return_offer(oid, 0)
            self.frameworks[fid] = fw
            driver._framework_id = fid
            driver._deliver(lambda s: s.registered(driver, P.FrameworkID(value=fid), self.master_info))
            self._allocate()
        self._schedule(0, do)

    def _fw(self, fid: str) -> Optional[_Framework]:
        fw = self.frameworks.get(fid)
        return fw if fw is not None and fw.connected else None

    def accept(self, fid: str, offer_ids: List[str], ops: List[P.Offer.Operation], refuse_s: float) -> None:
        self._schedule(0, self._accept, fid, list(offer_ids), list(ops), refuse_s)

    def decline(self, fid: str, offer_ids: List[str], refuse_s: float) -> None:
        self._schedule(0, self._decline, fid, list(offer_ids), refuse_s)

    def revive(self, fid: str) -> None:
        def do():
            fw = self._fw(fid)
            if fw is None:
                return
            fw.suppressed = False
            fw.filters.clear()
            self._allocate()
        self._schedule(0, do)

    def suppress(self, fid: str) -> None:
        def do():
            fw = self._fw(fid)
            if fw is not None:
                fw.suppressed = True
        self._schedule(0, do)

    def kill(self, fid: str, task_id: str) -> None:
        self._schedule(0, self._kill, fid, task_id)

    def reconcile(self, fid: str, statuses: List[P.TaskStatus]) -> None:
        self._schedule(0, self._reconcile, fid, list(statuses))

    def teardown(self, fid: str) -> None:
        def do():
            fw = self.frameworks.get(fid)
            if fw is None:
                return
            fw.connected = False
            for oid in [o.id for o in self.offers.values() if o.framework_id == fid]:
                self._return_offer(oid, 0)
            for a in self.agents.values():
                for t in list(a.tasks.values()):
                    if t.framework_id == fid and t.status.state not in TERMINAL:
                        self._update(t, P.TASK_KILLED, reason=P.TaskStatus.REASON_FRAMEWORK_REMOVED, deliver=False)
            del self.frameworks[fid]
        self._schedule(0, do)

    def disconnect(self, fid: str) -> None:
        def do():
            fw = self.frameworks.get(fid)
            if fw is None:
                return
            fw.connected = False
            for oid in [o.id for o in self.offers.values() if o.framework_id == fid]:
                self._return_offer(oid, 0)
        self._schedule(0, do)

    # -- allocation -------------------------------------------------------------------
    def _periodic_allocate(self) -> None:
        self._allocate()
        if self._running:
            self._schedule(self.allocation_interval_s, self._periodic_allocate)

    def _offerable(self, fw: _Framework, r: P.Resource) -> bool:
        return self._alloc_role(fw, effective_role(r)) is not None

    @staticmethod
    def _alloc_role(fw: _Framework, role: str) -> Optional[str]:
        """The framework role that may be allocated a resource reserved for ``role``: the role
        itself, or (hierarchical roles) a sub-role of it, which can then refine the reservation
        (``slave_public`` resources go to a framework subscribed as ``slave_public/<svc>-role``).
        Unreserved resources go to the framework's top-level roles in turn, one agent's offer at
        a time (``fw.rr``), as Mesos' allocator spreads them over a MULTI_ROLE framework's roles:
        a service migrating between its legacy and its group role gets offers for both."""
        if role == "*":
            tops = sorted(r for r in fw.roles if "/" not in r) or sorted(fw.roles)
            return tops[getattr(fw, "rr", 0) % len(tops)]
        if role in fw.roles:
            return role
        return next((r for r in sorted(fw.roles) if r.startswith(role + "/")), None)

    def _allocate(self) -> None:
        now = self.clock()
        for fw in list(self.frameworks.values()):
            if not fw.connected or fw.suppressed:
                continue
            batch: List[P.Offer] = []
            for a in self.agents.values():
                if not a.active:
                    continue
                mine = [r for r in a.available.to_resources() if self._offerable(fw, r)]
                if not mine:
                    continue
                flist = [f for f in fw.filters.get(a.id, []) if f[0] > now]
                if flist:
                    fw.filters[a.id] = flist
                    if any(all(f[1].contains(r) for r in mine) for f in flist):
                        continue
                else:
                    fw.filters.pop(a.id, None)
                for r in mine:
                    a.available.subtract(r)
                for r in mine:
                    r.allocation_info.role = self._alloc_role(fw, effective_role(r))
                fw.rr += 1
                oid = "offer-" + ids.uuid4_hex()
                self.offers[oid] = _Offer(oid, fw.id, a.id, mine)
                o = P.Offer(hostname=a.spec.hostname)
                o.id.value = oid
                o.framework_id.value = fw.id
                o.agent_id.value = a.id
                o.resources.extend(mine)
                o.attributes.extend(a.info_attributes())
                d = a.spec.domain()
                if d is not None:
                    o.domain.CopyFrom(d)
                for (efid, eid), e in a.executors.items():
                    if efid == fw.id:
                        o.executor_ids.add(value=eid)
                batch.append(o)
                if self.offer_timeout_s:
                    self._schedule(self.offer_timeout_s, self._expire_offer, oid)
            if batch:
                fw.driver._deliver(lambda s, b=batch, d=fw.driver: s.resource_offers(d, b))

    def _expire_offer(self, oid: str) -> None:
        if oid in self.offers:
            self._rescind(oid)

    def _rescind(self, oid: str) -> None:
        o = self.offers.get(oid)
        if o is None:
            return
        self._return_offer(oid, 0)
        fw = self.frameworks.get(o.framework_id)
        if fw is not None and fw.connected:
            fw.driver._deliver(lambda s, d=fw.driver: s.offer_rescinded(d, P.OfferID(value=oid)))

    def _return_offer(self, oid: str, refuse_s: float, leftover: Optional[ResourceBag] = None) -> None:
        o = self.offers.pop(oid, None)
        if o is None:
            return
        a = self.agents.get(o.agent_id)
        if a is None:
            return
        rs = leftover.take_all() if leftover is not None else o.resources
        for r in rs:
            r.ClearField("allocation_info")
            a.available.add(r)
        fw = self.frameworks.get(o.framework_id)
        if fw is not None and refuse_s > 0 and rs:
            fw.filters.setdefault(o.agent_id, []).append((self.clock() + refuse_s, ResourceBag(rs)))

    def _decline(self, fid: str, offer_ids: List[str], refuse_s: float) -> None:
        for oid in offer_ids:
            o = self.offers.get(oid)
            if o is not None and o.framework_id == fid:
                self._return_offer(oid, refuse_s)

    # -- ACCEPT -----------------------------------------------------------------------
    def _accept(self, fid: str, offer_ids: List[str], ops: List[P.Offer.Operation], refuse_s: float) -> None:
        self.accept_calls += 1
        if self._drop_accepts > 0:
            self._drop_accepts -= 1
            self.dropped_accepts += 1
            for oid in offer_ids:
                self._schedule(self._drop_rescind_s, self._expire_offer, oid)
            return
        fw = self._fw(fid)
        offers = [self.offers.get(oid) for oid in offer_ids]
        if fw is None or not offers or any(o is None or o.framework_id != fid for o in offers) or \
                len({o.agent_id for o in offers}) != 1:
            # invalid offers: every launched task is dropped
            LOGGER.warning("ACCEPT of framework %s rejected: offers %s are invalid or no longer valid (%d operations "
                           "dropped)", fid, offer_ids, len(ops))
            for op in ops:
                for t in self._op_tasks(op):
                    self._deliver_synthetic(fid, t, P.TASK_DROPPED, P.TaskStatus.REASON_INVALID_OFFERS,
                                            "Offers are invalid or no longer valid")
            return
        agent = self.agents[offers[0].agent_id]
        bag = ResourceBag()
        for o in offers:
            for r in o.resources:
                c = P.Resource()
                c.CopyFrom(r)
                c.ClearField("allocation_info")
                bag.add(c)
        for op in ops:
            self.operations.append((agent.id, op.type))
            try:
                self._apply(fw, agent, bag, op)
            except InsufficientResources as e:
                LOGGER.warning("Operation %s failed on %s: %s", P.Offer.Operation.Type.Name(op.type), agent.id, e)
                for t in self._op_tasks(op):
                    self._deliver_synthetic(fid, t, P.TASK_ERROR, P.TaskStatus.REASON_TASK_INVALID, str(e))
        # first offer returns the leftovers; the others are simply consumed
        for i, oid in enumerate(offer_ids):
            if i == 0:
                self._return_offer(oid, refuse_s, leftover=bag)
            else:
                self.offers.pop(oid, None)

    @staticmethod
    def _op_tasks(op: P.Offer.Operation) -> List[P.TaskInfo]:
        if op.type == P.Offer.Operation.LAUNCH_GROUP:
            return list(op.launch_group.task_group.tasks)
        if op.type == P.Offer.Operation.LAUNCH:
            return list(op.launch.task_infos)
        return []

    @staticmethod
    def _swap_in_place(bag: ResourceBag, pairs) -> None:
        """For each ``(take, give)``: subtract ``take`` from ``bag``, then add ``give``. All or
        nothing: on a shortfall the pairs already applied are undone before the error propagates
        (the result is what applying them to a copy and keeping it on success gives, without
        copying the offer's whole bag for every operation)."""
        done = []
        try:
            for take, give in pairs:
                bag.subtract(take)
                done.append((take, None))
                bag.add(give)
                done[-1] = (take, give)
        except InsufficientResources:
            for take, give in reversed(done):
                if give is not None:
                    bag.subtract(give)
                bag.add(take)
            raise

    def _apply(self, fw: _Framework, agent: _Agent, bag: ResourceBag, op: P.Offer.Operation) -> None:
        T = P.Offer.Operation
        if op.type == T.RESERVE:
            pairs = []
            for r in op.reserve.resources:
                c = P.Resource()
                c.CopyFrom(r)
                c.ClearField("allocation_info")
                pairs.append((pop_reservation(r), c))
            self._swap_in_place(bag, pairs)
        elif op.type == T.UNRESERVE:
            pairs = []
            for r in op.unreserve.resources:
                c = P.Resource()
                c.CopyFrom(r)
                c.ClearField("allocation_info")
                pairs.append((c, pop_reservation(c)))
            self._swap_in_place(bag, pairs)
        elif op.type == T.CREATE:
            trial = bag.copy()
            for v in op.create.volumes:
                trial.subtract(strip_volume(v))
                c = P.Resource()
                c.CopyFrom(v)
                c.ClearField("allocation_info")
                trial.add(c)
            bag._q, bag._proto = trial._q, trial._proto
        elif op.type == T.DESTROY:
            trial = bag.copy()
            for v in op.destroy.volumes:
                c = P.Resource()
                c.CopyFrom(v)
                c.ClearField("allocation_info")
                trial.subtract(c)
                trial.add(strip_volume(c))
            bag._q, bag._proto = trial._q, trial._proto
            if self._executes:
                self.behavior.destroy_volumes(agent, op.destroy.volumes)
        elif op.type == T.LAUNCH_GROUP:
            self._launch_group(fw, agent, bag, op.launch_group.executor, list(op.launch_group.task_group.tasks))
        elif op.type == T.LAUNCH:
            for t in op.launch.task_infos:
                self._launch_group(fw, agent, bag, t.executor if t.HasField("executor") else None, [t])
        else:
            raise InsufficientResources(f"unsupported operation {op.type}")

    @staticmethod
    def _clean(rs) -> List[P.Resource]:
        out = []
        for r in rs:
            c = P.Resource()
            c.CopyFrom(r)
            c.ClearField("allocation_info")
            out.append(c)
        return out

    def _launch_group(self, fw: _Framework, agent: _Agent, bag: ResourceBag, executor: Optional[P.ExecutorInfo],
                      tasks: List[P.TaskInfo]) -> None:
        trial = bag.copy()
        eid = executor.executor_id.value if executor is not None else ""
        key = (fw.id, eid)
        new_exec = executor is not None and key not in agent.executors
        exec_rs = self._clean(executor.resources) if new_exec else []
        trial.subtract_all(exec_rs)
        per_task = []
        for t in tasks:
            rs = self._clean(t.resources)
            trial.subtract_all(rs)
            per_task.append(rs)
        gpus_needed = [int(round(sum(r.scalar.value for r in rs if r.name == "gpus"))) for rs in per_task]
        if sum(gpus_needed) > len(agent.free_gpus):
            raise InsufficientResources("not enough free GPU devices")
        bag._q, bag._proto = trial._q, trial._proto
        if new_exec:
            agent.executors[key] = _Executor(executor, fw.id, exec_rs)
        for t, rs, ng in zip(tasks, per_task, gpus_needed):
            devices = select_devices(agent.free_gpus, ng, agent.spec.gpu_hives, agent.spec.gpu_peers)
            agent.free_gpus = [d for d in agent.free_gpus if d not in devices]
            st = P.TaskStatus(state=P.TASK_STAGING, source=P.TaskStatus.SOURCE_MASTER, timestamp=time.time())
            st.task_id.CopyFrom(t.task_id)
            st.agent_id.value = agent.id
            if eid:
                st.executor_id.value = eid
            task = _Task(t, fw.id, eid, agent.id, rs, devices, st)
            task.networks = agent.task_networks(
                executor.container if executor is not None and executor.HasField("container") else
                (t.container if t.HasField("container") else None))
            agent.tasks[t.task_id.value] = task
            if eid:
                agent.executors[key].tasks.add(t.task_id.value)
            if self._executes:
                self.behavior.launch(self, task, agent)
            elif agent.runtime is not None:
                agent.runtime.send(self._runtime_launch(task, self.behavior.timing(t)))
            else:
                timing = self.behavior.timing(t)
                self._schedule(timing.starting_s, self._lifecycle_starting, task, task.epoch, timing)

    # -- agent-run lifecycle (mesos.agent_runtime) ------------------------------------------
    @staticmethod
    def _runtime_launch(task: _Task, timing: TaskTiming) -> dict:
        info = task.info
        check = None
        if info.HasField("check"):
            check = {"delay": info.check.delay_seconds if timing.honor_check_delays else 0.0,
                     "interval": info.check.interval_seconds or 1.0}
        return {"op": "launch", "task": info.task_id.value, "name": info.name, "devices": list(task.gpu_devices),
                "check": check, "health": info.HasField("health_check"),
                "timing": {"starting": timing.starting_s, "running": timing.running_s,
                           "check_exec": timing.check_exec_s, "finish_after": timing.finish_after_s,
                           "exit_state": timing.exit_state}}

    def runtime_reports(self, agent_id: str, reports: List[dict]) -> None:
        """What an agent running its own tasks reported (any thread): applied in order on the
        dispatcher thread as the status updates Mesos would forward."""
        self._schedule(0, self._apply_runtime_reports, agent_id, list(reports))

    def _apply_runtime_reports(self, agent_id: str, reports: List[dict]) -> None:
        with self.batch_delivery():
            self._apply_reports(agent_id, reports)

    def _apply_reports(self, agent_id: str, reports: List[dict]) -> None:
        a = self.agents.get(agent_id)
        for r in reports:
            t = a.tasks.get(r.get("task")) if a is not None else None
            if t is None or t.status.state in TERMINAL:
                continue
            ev = r.get("event")
            if ev == "starting":
                self._update(t, P.TASK_STARTING)
            elif ev == "running":
                extra = {}
                if t.info.HasField("check"):
                    cs = P.CheckStatusInfo(type=t.info.check.type)
                    cs.command.SetInParent()
                    extra["check_status"] = cs
                if t.info.HasField("health_check"):
                    extra["healthy"] = True
                self._update(t, P.TASK_RUNNING, **extra)
            elif ev == "ready":
                self._lifecycle_ready(t, t.epoch)
            elif ev == "check_failed":
                if t.status.state != P.TASK_RUNNING:
                    continue
                prev = t.status.check_status.command.exit_code if t.status.HasField("check_status") else None
                if prev != 1:
                    cs = P.CheckStatusInfo(type=t.info.check.type)
                    cs.command.exit_code = 1
                    self._update(t, P.TASK_RUNNING, check_status=cs,
                                 reason=P.TaskStatus.REASON_TASK_CHECK_STATUS_UPDATED)
            elif ev == "exited":
                t.reported_exit = True
                fields = {"message": r.get("message", "")}
                if r.get("reason") is not None:
                    fields["reason"] = int(r["reason"])
                self._update(t, int(r.get("state", P.TASK_FINISHED)), **fields)
            else:
                LOGGER.warning("unknown agent report %r", r)

    # -- task lifecycle ----------------------------------------------------------------
    def _lifecycle_starting(self, task: _Task, epoch: int, timing: TaskTiming) -> None:
        if task.epoch != epoch or task.status.state in TERMINAL:
            return
        self._update(task, P.TASK_STARTING)
        self._after(timing.running_s, self._lifecycle_running, task, epoch, timing)

    def _lifecycle_running(self, task: _Task, epoch: int, timing: TaskTiming) -> None:
        if task.epoch != epoch or task.status.state in TERMINAL:
            return
        extra = {}
        info = task.info
        if info.HasField("check"):
            cs = P.CheckStatusInfo(type=info.check.type)
            cs.command.SetInParent()
            extra["check_status"] = cs
        if info.HasField("health_check") and not self._executes:
            extra["healthy"] = True
        self._update(task, P.TASK_RUNNING, **extra)
        if self._executes:
            self.behavior.started(self, task, epoch)
        if info.HasField("check"):
            delay = (info.check.delay_seconds if timing.honor_check_delays else 0.0) + timing.check_exec_s
            if self._check_runner(task) is not None:
                self._after(delay, self._run_check, task, epoch)   # submits to the check pool
            else:
                self._schedule(delay, self._lifecycle_ready, task, epoch)
        if timing.finish_after_s is not None and not self._executes:
            self._schedule(timing.finish_after_s, self._lifecycle_exit, task, epoch, timing.exit_state)

    def _check_runner(self, task: _Task):
        a = self.agents.get(task.agent_id)
        if a is not None and a.check_runner is not None:
            return a.check_runner
        return self.behavior.check_runner

    def _run_check(self, task: _Task, epoch: int) -> None:
        if task.epoch != epoch or task.status.state != P.TASK_RUNNING:
            return
        trace.instant("check_submit", "master", task=task.info.name)
        runner = self._check_runner(task)
        devices = list(task.gpu_devices)
        run_async = getattr(runner, "run_async", None)
        if run_async is not None:
            # the runner reports back by itself (a remote agent's link): no pool thread blocks on it
            def done(ok: bool) -> None:
                self._schedule(0, self._check_result, task, epoch, ok)
            try:
                run_async(task.info, devices, done)
            except Exception:  # noqa: BLE001
                LOGGER.exception("check of %s raised", task.info.name)
                self._schedule(0, self._check_result, task, epoch, False)
            return

        def check() -> bool:
            try:
                with trace.span("readiness_check", "master", task=task.info.name):
                    return bool(runner(task.info, devices))
            except Exception:  # noqa: BLE001
                LOGGER.exception("check of %s raised", task.info.name)
                return False

        agent = self.agents.get(task.agent_id)
        if getattr(runner, "inline", False) and agent is not None:
            # a check that is one short native call (the fused HIP probe, ~0.07 ms with the
            # interpreter released) runs on the agent's own check thread (not on this
            # event thread, where a slow probe would stall every agent's launches and statuses)
            agent.check_thread().submit(lambda: self._schedule(0, self._check_result, task, epoch, check()))
            return
        self.behavior.pool().submit(lambda: self._schedule(0, self._check_result, task, epoch, check()))

    def _check_result(self, task: _Task, epoch: int, ok: bool) -> None:
        if task.epoch != epoch or task.status.state != P.TASK_RUNNING:
            return
        if ok:
            self._lifecycle_ready(task, epoch)
            return
        prev = task.status.check_status.command.exit_code if task.status.HasField("check_status") else None
        if prev != 1:
            cs = P.CheckStatusInfo(type=task.info.check.type)
            cs.command.exit_code = 1
            self._update(task, P.TASK_RUNNING, check_status=cs, reason=P.TaskStatus.REASON_TASK_CHECK_STATUS_UPDATED)
        self._schedule(task.info.check.interval_seconds, self._run_check, task, epoch)

    def _lifecycle_ready(self, task: _Task, epoch: int) -> None:
        if task.epoch != epoch or task.status.state != P.TASK_RUNNING:
            return
        trace.instant("task_ready", "master", task=task.info.name)
        cs = P.CheckStatusInfo(type=task.info.check.type)
        cs.command.exit_code = 0
        extra = {"check_status": cs, "reason": P.TaskStatus.REASON_TASK_CHECK_STATUS_UPDATED}
        if task.info.HasField("health_check"):
            if not self._executes:
                extra["healthy"] = True
            elif task.status.HasField("healthy"):
                extra["healthy"] = task.status.healthy
        self._update(task, P.TASK_RUNNING, **extra)

    def _lifecycle_exit(self, task: _Task, epoch: int, state: int) -> None:
        if task.epoch != epoch or task.status.state in TERMINAL:
            return
        self._update(task, state, message="task exited")

    # -- real-process runtime callbacks (ProcessTaskBehavior) ----------------------------
    def _process_exited(self, task: _Task, epoch: int, rc: int, killed: bool, unhealthy: bool) -> None:
        if task.epoch != epoch or task.status.state in TERMINAL:
            return
        if unhealthy:
            self._update(task, P.TASK_KILLED, healthy=False, reason=P.TaskStatus.REASON_TASK_HEALTH_CHECK_STATUS_UPDATED,
                         message="Task was killed since health check failed")
        elif killed:
            self._update(task, P.TASK_KILLED, message="Command terminated with signal SIGTERM")
        elif rc == 0:
            self._update(task, P.TASK_FINISHED, message="Command exited with status 0")
        else:
            msg = f"Command terminated with signal {-rc}" if rc < 0 else f"Command exited with status {rc}"
            self._update(task, P.TASK_FAILED, message=msg, reason=P.TaskStatus.REASON_COMMAND_EXECUTOR_FAILED)

    def _health_changed(self, task: _Task, epoch: int, healthy: bool) -> None:
        if task.epoch != epoch or task.status.state != P.TASK_RUNNING:
            return
        extra = {"healthy": healthy, "reason": P.TaskStatus.REASON_TASK_HEALTH_CHECK_STATUS_UPDATED}
        if task.status.HasField("check_status"):
            extra["check_status"] = task.status.check_status
        self._update(task, P.TASK_RUNNING, **extra)

    def _container_failed(self, task: _Task, epoch: int, message: str) -> None:
        if task.epoch != epoch or task.status.state in TERMINAL:
            return
        self._update(task, P.TASK_FAILED, message=f"Failed to launch container: {message}",
                     reason=P.TaskStatus.REASON_CONTAINER_LAUNCH_FAILED)

    def _kill(self, fid: str, task_id: str) -> None:
        t = self._find_task(task_id)
        if t is None or t.framework_id != fid:
            st = P.TaskStatus(state=P.TASK_LOST, source=P.TaskStatus.SOURCE_MASTER,
                              reason=P.TaskStatus.REASON_RECONCILIATION, message="Attempted to kill an unknown task",
                              timestamp=time.time())
            st.task_id.value = task_id
            fw = self._fw(fid)
            if fw is not None:
                fw.driver._deliver(lambda s, d=fw.driver: s.status_update(d, st))
            return
        if t.status.state in TERMINAL:
            return
        if not self.agents[t.agent_id].active:
            # Mesos cannot reach the agent: the kill is answered with the task's current
            # (UNREACHABLE/LOST) state and nothing is released until the agent returns.
            st = P.TaskStatus()
            st.CopyFrom(t.status)
            st.message = "Task is unreachable: cannot kill it now"
            st.timestamp = time.time()
            fw = self._fw(fid)
            if fw is not None:
                fw.driver._deliver(lambda s, d=fw.driver: s.status_update(d, st))
            return
        if self._executes and self.behavior.kill(self, t):
            return  # TASK_KILLED is reported when the process has exited
        a = self.agents.get(t.agent_id)
        if a is not None and a.runtime is not None:
            a.runtime.send({"op": "kill", "task": task_id})
            return  # the agent reports TASK_KILLED once it has stopped the task
        self._update(t, P.TASK_KILLED, message="Task killed by scheduler")

    def _find_task(self, task_id: str) -> Optional[_Task]:
        for a in self.agents.values():
            t = a.tasks.get(task_id)
            if t is not None:
                return t
        return None

    def _update(self, task: _Task, state: int, deliver: bool = True, **fields) -> None:
        st = P.TaskStatus(state=state, timestamp=time.time())
        st.task_id.CopyFrom(task.info.task_id)
        st.agent_id.value = task.agent_id
        if task.executor_id:
            st.executor_id.value = task.executor_id
        st.source = fields.pop("source", P.TaskStatus.SOURCE_EXECUTOR)
        cs = fields.pop("check_status", None)
        if cs is not None:
            st.check_status.CopyFrom(cs)
        for k, v in fields.items():
            setattr(st, k, v)
        if task.gpu_devices:
            st.labels.labels.add(key="gpu_devices", value=",".join(str(d) for d in task.gpu_devices))
        if task.networks:
            st.container_status.network_infos.extend(task.networks)
        else:
            st.container_status.network_infos.add().ip_addresses.add(ip_address="127.0.0.1")
        if not task.container_id:
            task.container_id = container_id_for(task.info.task_id.value)
        st.container_status.container_id.value = task.container_id
        st.uuid = ids.uuid4_bytes()
        task.status = st
        if state in TERMINAL:
            task.epoch += 1
            self._release_task(task)
        fw = self.frameworks.get(task.framework_id)
        for fn in self._listeners:
            try:
                fn(task.framework_id, st)
            except Exception:  # noqa: BLE001
                LOGGER.exception("status listener failed")
        if deliver and fw is not None and fw.connected:
            fw.driver._deliver(lambda s, d=fw.driver, st=st: s.status_update(d, st))

    def _release_task(self, task: _Task) -> None:
        if self._executes:
            self.behavior.release(task)
        a = self.agents.get(task.agent_id)
        if a is None:
            return
        if a.runtime is not None and not task.reported_exit:
            # ended by the master (teardown, forget, agent removed): the agent stops tracking it
            a.runtime.send({"op": "drop", "task": task.info.task_id.value})
        for r in task.resources:
            a.available.add(r)
        task.resources = []
        a.free_gpus.extend(task.gpu_devices)
        a.free_gpus.sort()
        task.gpu_devices = []
        key = (task.framework_id, task.executor_id)
        e = a.executors.get(key)
        if e is not None:
            e.tasks.discard(task.info.task_id.value)
            if not e.tasks:
                for r in e.resources:
                    a.available.add(r)
                del a.executors[key]

    def _deliver_synthetic(self, fid: str, t: P.TaskInfo, state: int, reason: int, message: str) -> None:
        fw = self._fw(fid)
        if fw is None:
            return
        st = P.TaskStatus(state=state, source=P.TaskStatus.SOURCE_MASTER, reason=reason, message=message,
                          timestamp=time.time())
        st.task_id.CopyFrom(t.task_id)
        fw.driver._deliver(lambda s, d=fw.driver: s.status_update(d, st))

    def _reconcile(self, fid: str, statuses: List[P.TaskStatus]) -> None:
        fw = self._fw(fid)
        if fw is None:
            return
        out = []
        if not statuses:
            for a in self.agents.values():
                for t in a.tasks.values():
                    if t.framework_id == fid and t.status.state not in TERMINAL:
                        out.append(t.status)
        else:
            for s in statuses:
                t = self._find_task(s.task_id.value)
                if t is not None and t.framework_id == fid:
                    c = P.TaskStatus()
                    c.CopyFrom(t.status)
                    c.reason = P.TaskStatus.REASON_RECONCILIATION
                    out.append(c)
                else:
                    aware = any(c.type == P.FrameworkInfo.Capability.PARTITION_AWARE for c in fw.info.capabilities)
                    st = P.TaskStatus(state=P.TASK_UNKNOWN if aware else P.TASK_LOST, source=P.TaskStatus.SOURCE_MASTER,
                                      reason=P.TaskStatus.REASON_RECONCILIATION, message="Reconciliation: task unknown",
                                      timestamp=time.time())
                    st.task_id.CopyFrom(s.task_id)
                    out.append(st)
        for st in out:
            fw.driver._deliver(lambda s, d=fw.driver, st=st: s.status_update(d, st))


class LocalSchedulerDriver(SchedulerDriver):
    """Driver bound to a ``LocalMaster``; callbacks go to a FrameworkScheduler-like sink."""

    def __init__(self, master: LocalMaster, scheduler, framework_info: P.FrameworkInfo):
        self.master = master
        self.scheduler = scheduler
        self.framework_info = framework_info
        self._framework_id: Optional[str] = None
        self._stopped = threading.Event()
        self.acknowledged: List[bytes] = []

    # deliveries run on the master thread, in order
    def _deliver(self, fn) -> None:
        if self._stopped.is_set():
            return
        try:
            fn(self.scheduler)
        except Exception:  # noqa: BLE001
            LOGGER.exception("Scheduler callback failed")

    @property
    def framework_id(self) -> Optional[str]:
        return self._framework_id

    def start(self) -> None:
        self.master.subscribe(self, self.framework_info)

    def run(self) -> int:
        self.start()
        self._stopped.wait()
        return 0

    def join(self, timeout: Optional[float] = None) -> bool:
        return self._stopped.wait(timeout)

    def accept_offers(self, offer_ids, operations, filters=None) -> None:
        refuse = filters.refuse_seconds if filters is not None else 5.0
        self.master.accept(self._framework_id, [o.value for o in offer_ids], list(operations), refuse)

    def decline_offer(self, offer_id, filters=None) -> None:
        self.decline_offers([offer_id], filters)

    def decline_offers(self, offer_ids, filters=None) -> None:
        refuse = filters.refuse_seconds if filters is not None else 5.0
        self.master.decline(self._framework_id, [o.value for o in offer_ids], refuse)

    def kill_task(self, task_id) -> None:
        self.master.kill(self._framework_id, task_id.value)

    def reconcile_tasks(self, statuses) -> None:
        self.master.reconcile(self._framework_id, list(statuses))

    def revive_offers(self) -> None:
        self.master.revive(self._framework_id)

    def suppress_offers(self) -> None:
        self.master.suppress(self._framework_id)

    def acknowledge_status_update(self, status) -> None:
        if status.uuid:
            self.acknowledged.append(status.uuid)

    def teardown(self) -> None:
        if self._framework_id:
            self.master.teardown(self._framework_id)

    def stop(self, failover: bool = True) -> None:
        if self._framework_id:
            if failover:
                self.master.disconnect(self._framework_id)
            else:
                self.master.teardown(self._framework_id)
        self._stopped.set()


def local_master_from_env(env) -> LocalMaster:
    """An in-process cluster sized from ``SDK_LOCAL_*`` variables (``SDK_MESOS_MASTER=local``)."""
    n = env.get_optional_int("SDK_LOCAL_AGENTS", 3)
    gpus_env = env.get_optional("SDK_LOCAL_AGENT_GPUS", "0")
    master = LocalMaster(allocation_interval_s=env.get_optional_double("SDK_LOCAL_ALLOCATION_INTERVAL_S", 1.0))
    specs = gpu_agent_specs(n, gpus_env, lambda i: f"agent-{i}.local")
    for spec in specs:
        spec.cpus = env.get_optional_double("SDK_LOCAL_AGENT_CPUS", 8.0)
        spec.mem = env.get_optional_double("SDK_LOCAL_AGENT_MEM", 32768.0)
        spec.disk = env.get_optional_double("SDK_LOCAL_AGENT_DISK", 65536.0)
        master.add_agent(spec)
    return master


def gpu_agent_specs(agents: int, gpus_per_agent, hostname, inventory=None, **kw) -> List[AgentSpec]:
    """``agents`` GPU agent specs built from node discovery (``ops.gpu``).

    ``gpus_per_agent="auto"``: the agents share this one node and split its discovered GPUs in
    contiguous blocks (one agent per GPU on an 8-GPU node). An int: every agent stands for a node
    of its own with that many GPUs (a simulated cluster): the first ones of this node's inventory,
    or of ``inventory``. Each agent's ``gpu_devices``, attributes (``gpu_model``, ``xgmi_hive``,
    ...) and device topology come from the inventory; a node with fewer GPUs than asked for (no
    driver here) gets a synthetic MI355X inventory of the right size."""
    from dcos_commons_amd.ops import gpu as G

    if gpus_per_agent == "auto":
        inv = inventory if inventory is not None else G.node_inventory()
        per = inv.count // agents if agents else 0
        blocks = [[d.index for d in inv.devices[i * per:(i + 1) * per]] for i in range(agents)]
    else:
        per = int(gpus_per_agent or 0)
        inv = inventory if inventory is not None else (G.node_inventory(per) if per else None)
        if per and inv.count < per:
            raise ValueError(f"{per} GPUs per agent, the inventory has {inv.count}")
        blocks = [[d.index for d in inv.devices[:per]] for _ in range(agents)] if per else []
    out = []
    for i in range(agents):
        name = hostname(i) if callable(hostname) else f"{hostname}-{i}"
        if per:
            out.append(AgentSpec.from_gpu_inventory(name, inv, devices=blocks[i], **kw))
        else:
            out.append(AgentSpec(hostname=name, **kw))
    return out
