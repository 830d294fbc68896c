"""Implementation of the simulation harness (see package docstring)."""
from __future__ import annotations

import os
import random
import uuid
from dataclasses import dataclass, field
from typing import Callable, Dict, Iterable, List, Optional

from dcos_commons_amd.framework import task_killer
from dcos_commons_amd.framework.driver import SchedulerDriver
from dcos_commons_amd.framework.framework_config import FrameworkConfig
from dcos_commons_amd.framework.framework_scheduler import FrameworkScheduler
from dcos_commons_amd.framework.process_exit import ProcessExit
from dcos_commons_amd.http.api import Router
from dcos_commons_amd.mesos import protos as P
from dcos_commons_amd.offer.resources import get_resource_id
from dcos_commons_amd.offer.taskdata.labels import env_to_map
from dcos_commons_amd.scheduler.plan.status import Status
from dcos_commons_amd.scheduler.scheduler_builder import SchedulerBuilder
from dcos_commons_amd.scheduler.scheduler_config import SchedulerConfig
from dcos_commons_amd.specification.yaml.mappers import ServiceSpecGenerator
from dcos_commons_amd.specification.yaml.raw import RawServiceSpec
from dcos_commons_amd.state.framework_store import FrameworkStore
from dcos_commons_amd.state.state_store import StateStore
from dcos_commons_amd.storage.mem_persister import MemPersister

Op = P.Offer.Operation
TEST_FRAMEWORK_ID = "test-framework-id"


# ---------------------------------------------------------------------------------------
# recording driver + cluster state


class RecordingDriver(SchedulerDriver):
    def __init__(self):
        self.accepts: List["AcceptEntry"] = []
        self.declines: List[tuple] = []  # (offer id, refuse seconds)
        self.kills: List[str] = []
        self.reconciles: List[List[P.TaskStatus]] = []
        self.revives = 0
        self.suppresses = 0
        self.teardowns = 0
        self.stopped = False

    def accept_offers(self, offer_ids, operations, filters=None):
        self.accepts.append(AcceptEntry([o.value for o in offer_ids], list(operations)))

    def decline_offer(self, offer_id, filters=None):
        self.declines.append((offer_id.value, filters.refuse_seconds if filters is not None else None))

    def decline_offers(self, offer_ids, filters=None):
        for o in offer_ids:
            self.decline_offer(o, filters)

    def kill_task(self, task_id):
        self.kills.append(task_id.value)

    def reconcile_tasks(self, statuses):
        self.reconciles.append(list(statuses))

    def revive_offers(self):
        self.revives += 1

    def suppress_offers(self):
        self.suppresses += 1

    def acknowledge_status_update(self, status):
        pass

    def teardown(self):
        self.teardowns += 1

    def stop(self, failover=True):
        self.stopped = True


@dataclass
class AcceptEntry:
    offer_ids: List[str]
    operations: List[P.Offer.Operation]

    def of_type(self, t) -> List[P.Offer.Operation]:
        return [o for o in self.operations if o.type == t]

    def launched_tasks(self) -> List[P.TaskInfo]:
        out = []
        for o in self.of_type(Op.LAUNCH_GROUP):
            out.extend(o.launch_group.task_group.tasks)
        for o in self.of_type(Op.LAUNCH):
            out.extend(o.launch.task_infos)
        return out

    def executors(self) -> List[P.ExecutorInfo]:
        return [o.launch_group.executor for o in self.of_type(Op.LAUNCH_GROUP)]

    def unreserved(self) -> List[P.Resource]:
        out = []
        for o in self.of_type(Op.UNRESERVE):
            out.extend(o.unreserve.resources)
        return out


@dataclass
class ClusterState:
    spec: object
    driver: RecordingDriver
    router: Router
    sent_offers: List[P.Offer] = field(default_factory=list)
    # task name -> (agent id, hostname) of its last launch
    task_agents: Dict[str, tuple] = field(default_factory=dict)

    def accepts_for_pod(self, pod_name: str) -> List[AcceptEntry]:
        return [a for a in self.driver.accepts if any(t.name.startswith(pod_name + "-") for t in a.launched_tasks())]

    def last_launched(self, task_name: str) -> Optional[P.TaskInfo]:
        for a in reversed(self.driver.accepts):
            for t in a.launched_tasks():
                if t.name == task_name:
                    return t
        return None

    def last_offer(self) -> Optional[P.Offer]:
        return self.sent_offers[-1] if self.sent_offers else None


# ---------------------------------------------------------------------------------------
# ticks


class SimulationTick:
    description = ""

    def __repr__(self):
        return f"{type(self).__name__}({self.description})"


class Send(SimulationTick):
    def __init__(self, fn: Callable[["_Sim"], None], description: str):
        self.fn = fn
        self.description = description

    def send(self, sim: "_Sim") -> None:
        self.fn(sim)

    @staticmethod
    def register() -> "Send":
        def fn(sim):
            master = P.MasterInfo(id="test-master-id", ip=1, port=2)
            sim.framework.registered(sim.driver, P.FrameworkID(value=TEST_FRAMEWORK_ID), master)
        return Send(fn, "Framework registration completed")

    @staticmethod
    def offer_builder(pod_type: str) -> "SendOffer":
        return SendOffer(pod_type)

    @staticmethod
    def task_status(task_name: str, state: int) -> "SendTaskStatus":
        return SendTaskStatus(task_name, state)

    @staticmethod
    def replace_pod(pod_name: str) -> "Send":
        return Send(lambda sim: sim.http_ok(sim.state.router.post(f"/v1/pod/{pod_name}/replace")),
                    f"Replace pod: {pod_name}")

    @staticmethod
    def restart_pod(pod_name: str) -> "Send":
        return Send(lambda sim: sim.http_ok(sim.state.router.post(f"/v1/pod/{pod_name}/restart")),
                    f"Restart pod: {pod_name}")

    @staticmethod
    def http(method: str, path: str, body=b"", expect_status: Optional[int] = None) -> "Send":
        def fn(sim):
            r = sim.state.router.dispatch(method, path, body if isinstance(body, bytes) else str(body).encode())
            if expect_status is not None and r.status != expect_status:
                raise AssertionError(f"{method} {path}: expected HTTP {expect_status}, got {r.status}: {r.payload()!r}")
        return Send(fn, f"{method} {path}")

    @staticmethod
    def drive_plan(plan: str = "deploy", max_rounds: int = 40, pods: Optional[List[str]] = None) -> "Send":
        """Plays the cluster until ``plan`` is COMPLETE: each round offers fresh resources for every pod
        type (new host each time) plus reoffers of every launched pod instance, answers each new
        launch with RUNNING (+ readiness passed) or FINISHED for FINISH/ONCE goals, and issues a plan
        ``continue`` when a round makes no progress (canary strategies wait for the operator)."""
        def fn(sim):
            from dcos_commons_amd.specification.specs import GoalState

            answered = set()
            hosts = iter(range(10 ** 6))
            stalled = 0
            for _ in range(max_rounds):
                p = sim.scheduler.get_plan(plan)
                if p is None:
                    raise AssertionError(f"no plan {plan}")
                if p.get_status() == Status.COMPLETE:
                    return
                before = len(answered)
                for pod in sim.state.spec.pods:
                    if pods is not None and pod.type not in pods:
                        continue
                    SendOffer(pod.type).set_hostname(f"auto-{next(hosts)}").build().send(sim)
                    for i in range(pod.count):
                        if sim.state.accepts_for_pod(f"{pod.type}-{i}"):
                            (SendOffer(pod.type).set_pod_index_to_reoffer(i).add_unreserved_resources()
                             .set_hostname(f"auto-{next(hosts)}").build().send(sim))
                for a in list(sim.driver.accepts):
                    for t in a.launched_tasks():
                        if t.task_id.value in answered:
                            continue
                        answered.add(t.task_id.value)
                        goal = _task_goal(sim.state.spec, t.name)
                        if goal in (GoalState.FINISH, GoalState.ONCE):
                            SendTaskStatus(t.name, P.TASK_FINISHED).set_task_id(t.task_id.value).send(sim)
                        else:
                            (SendTaskStatus(t.name, P.TASK_RUNNING).set_task_id(t.task_id.value)
                             .set_readiness_check_exit_code(0).send(sim))
                if len(answered) == before:
                    stalled += 1
                    sim.state.router.post(f"/v1/plans/{plan}/continue")
                    for ph in p.get_children():
                        if ph.get_status() in (Status.WAITING, Status.PENDING) or ph.is_interrupted():
                            sim.state.router.post(f"/v1/plans/{plan}/continue?phase={ph.get_name()}")
                    if stalled > 5:
                        break
                else:
                    stalled = 0
            p = sim.scheduler.get_plan(plan)
            raise AssertionError(f"plan {plan} is {p.get_status()} after {max_rounds} rounds: "
                                 + "; ".join(f"{ph.get_name()}={[(s.get_name(), str(s.get_status())) for s in ph.get_children()]}"
                                             for ph in p.get_children()))
        return Send(fn, f"drive plan {plan} to completion")

    @staticmethod
    def empty_offers() -> "Send":
        return Send(lambda sim: sim.framework.resource_offers(sim.driver, []), "Nudge offer processing")


class SendOffer(Send):
    def __init__(self, pod_type: str):
        self.pod_type = pod_type
        self.pod_to_reuse: Optional[str] = None
        self.hostname = "test-hostname"
        self.count = 1
        self.agent_id: Optional[str] = None
        self.extra: List[P.Resource] = []
        self.attributes: Dict[str, str] = {}
        self.with_unreserved = False

    def add_unreserved_resources(self) -> "SendOffer":
        """With a reoffer: also include unreserved resources for the pod type (e.g. for sidecar tasks
        with their own resource set that launch next to an existing executor)."""
        self.with_unreserved = True
        return self

    def set_pod_index_to_reoffer(self, index: int) -> "SendOffer":
        self.pod_to_reuse = f"{self.pod_type}-{index}"
        return self

    def set_hostname(self, hostname: str) -> "SendOffer":
        self.hostname = hostname
        return self

    def set_count(self, count: int) -> "SendOffer":
        self.count = count
        return self

    def set_agent_id(self, agent_id: str) -> "SendOffer":
        self.agent_id = agent_id
        return self

    def add_resources(self, *resources: P.Resource) -> "SendOffer":
        self.extra.extend(resources)
        return self

    def set_attributes(self, **attrs) -> "SendOffer":
        self.attributes.update(attrs)
        return self

    def build(self) -> "SendOffer":
        self.description = (f"{self.count} reserved offer(s) for pod={self.pod_to_reuse}" if self.pod_to_reuse
                            else f"{self.count} unreserved offer(s) for pod type={self.pod_type}")
        return self

    @staticmethod
    def _unreserved(name: str, value: P.Value, mount_root: Optional[str] = None,
                    pre_reserved_role: Optional[str] = None, profile: Optional[str] = None) -> P.Resource:
        """An unreserved resource, or with ``pre_reserved_role`` one statically reserved to that role
        (refinement form: a STATIC entry at the bottom of ``reservations``, as an agent started with
        ``--resources=...(role)`` offers it). ``profile`` marks a MOUNT disk as coming from that CSI
        volume profile, so ``profiles: [...]`` volumes can match it."""
        role = pre_reserved_role if pre_reserved_role not in (None, "", "*") else None
        r = P.Resource(name=name, type=value.type) if role else P.Resource(name=name, type=value.type, role="*")
        if role:
            r.reservations.add(type=P.Resource.ReservationInfo.STATIC, role=role)
        if value.type == P.Value.SCALAR:
            r.scalar.CopyFrom(value.scalar)
        elif value.type == P.Value.RANGES:
            r.ranges.CopyFrom(value.ranges)
        if mount_root is not None:
            r.disk.source.type = P.Resource.DiskInfo.Source.MOUNT
            r.disk.source.mount.root = mount_root
            if profile:
                r.disk.source.profile = profile
        return r

    def _offer(self, sim: "_Sim") -> P.Offer:
        pod = sim.state.spec.pod(self.pod_type)
        if pod is None:
            raise ValueError(f"No PodSpec found with type={self.pod_type}: types={[p.type for p in sim.state.spec.pods]}")
        o = P.Offer(hostname=self.hostname)
        o.id.value = str(uuid.uuid4())
        o.framework_id.value = TEST_FRAMEWORK_ID
        agent = self.agent_id
        if self.pod_to_reuse:
            by_id: Dict[str, P.Resource] = {}
            executors = set()
            for a in sim.state.accepts_for_pod(self.pod_to_reuse):
                # every reservation made for the pod (incl. resource sets of tasks not launched yet),
                # superseded below by launched tasks' copies, which carry volume persistence
                for op in a.of_type(Op.RESERVE):
                    for r in op.reserve.resources:
                        by_id[get_resource_id(r) or str(uuid.uuid4())] = r
                for e in a.executors():
                    for r in e.resources:
                        by_id[get_resource_id(r) or str(uuid.uuid4())] = r
                    executors.add(e.executor_id.value)
                for t in a.launched_tasks():
                    if not t.name.startswith(self.pod_to_reuse + "-"):
                        continue
                    agent = agent or t.agent_id.value
                    for r in list(t.resources) + list(t.executor.resources):
                        rid = get_resource_id(r)
                        by_id[rid or str(uuid.uuid4())] = r
                    executors.add(t.executor.executor_id.value)
            o.resources.extend(by_id.values())
            for e in sorted(x for x in executors if x):
                o.executor_ids.add(value=e)
        if not self.pod_to_reuse or self.with_unreserved:
            from dcos_commons_amd.specification.specs import VolumeType

            pre_role = getattr(pod, "pre_reserved_role", None)

            def vol(v):
                mount = "/mnt/" + v.container_path if v.type == VolumeType.MOUNT else None
                profile = v.profiles[0] if mount is not None and v.profiles else None
                return self._unreserved("disk", v.value, mount, pre_role, profile)
            for v in pod.volumes:
                o.resources.add().CopyFrom(vol(v))
            from dcos_commons_amd.specification.specs import PortSpec

            dynamic_ports = False
            for t in pod.tasks:
                for r in t.resource_set.resources:
                    if isinstance(r, PortSpec) and r.port == 0:
                        # agents offer port *ranges*: dynamic ports are claimed from them
                        dynamic_ports = True
                        for rg in r.ranges:
                            o.resources.add().CopyFrom(self._unreserved("ports", _ranges(rg.begin, rg.end),
                                                                        pre_reserved_role=pre_role))
                        continue
                    o.resources.add().CopyFrom(self._unreserved(r.name, r.value, pre_reserved_role=pre_role))
                for v in t.resource_set.volumes:
                    o.resources.add().CopyFrom(vol(v))
            if dynamic_ports:
                o.resources.add().CopyFrom(self._unreserved("ports", _ranges(10000, 10999), pre_reserved_role=pre_role))
            for name, value in sim.cfg.executor_resources().items():
                o.resources.add().CopyFrom(self._unreserved(name, value, pre_reserved_role=pre_role))
        o.resources.extend(self.extra)
        o.agent_id.value = agent or ("test-agent-" + str(uuid.uuid4()))
        for k, v in sorted(self.attributes.items()):
            a = o.attributes.add(name=k, type=P.Value.TEXT)
            a.text.value = v
        return o

    def send(self, sim: "_Sim") -> None:
        offers = [self._offer(sim) for _ in range(self.count)]
        sim.state.sent_offers.extend(offers)
        sim.framework.resource_offers(sim.driver, offers)


def _task_goal(spec, task_name: str):
    """Goal of the TaskSpec behind a ``<pod>-<index>-<task>`` instance name."""
    for pod in spec.pods:
        prefix = pod.type + "-"
        if not task_name.startswith(prefix):
            continue
        rest = task_name[len(prefix):]
        idx, _, name = rest.partition("-")
        if not idx.isdigit():
            continue
        for t in pod.tasks:
            if t.name == name:
                return t.goal
    return None


def _ranges(begin: int, end: int) -> P.Value:
    val = P.Value(type=P.Value.RANGES)
    val.ranges.range.add(begin=begin, end=end)
    return val


def _scalar(v: float) -> P.Value:
    val = P.Value(type=P.Value.SCALAR)
    val.scalar.value = v
    return val


class SendTaskStatus(Send):
    def __init__(self, task_name: str, state: int):
        self.task_name = task_name
        self.state = state
        self.readiness_exit: Optional[int] = None
        self.task_id: Optional[str] = None
        self.healthy: Optional[bool] = None
        self.ip: Optional[str] = None
        self.description = f"{P.TaskState.Name(state)} for task {task_name}"

    def set_readiness_check_exit_code(self, code: int) -> "SendTaskStatus":
        self.readiness_exit = code
        return self

    def set_check_pending(self) -> "SendTaskStatus":
        """An empty ``check_status`` (no exit code yet): what Mesos attaches to the first RUNNING
        update of a task that has a check."""
        self.readiness_exit = -1
        return self

    def set_task_id(self, task_id: str) -> "SendTaskStatus":
        self.task_id = task_id
        return self

    def set_healthy(self, healthy: bool) -> "SendTaskStatus":
        self.healthy = healthy
        return self

    def set_ip(self, ip: str) -> "SendTaskStatus":
        self.ip = ip
        return self

    def build(self) -> "SendTaskStatus":
        return self

    def send(self, sim: "_Sim") -> None:
        tid = self.task_id
        agent = None
        last = sim.state.last_launched(self.task_name)
        if last is None:  # launched by an earlier scheduler run: use the persisted TaskInfo
            last = StateStore(sim.persister, sim.namespace).fetch_task(self.task_name)
        if tid is None:
            if last is None:
                raise AssertionError(f"No task named {self.task_name} was launched")
            tid = last.task_id.value
        if last is not None:
            agent = last.agent_id.value
        st = P.TaskStatus(state=self.state, message="This is a test status")
        st.task_id.value = tid
        if agent:
            st.agent_id.value = agent
        if self.readiness_exit is not None:
            st.check_status.type = P.CheckInfo.COMMAND
            st.check_status.command.SetInParent()
            if self.readiness_exit >= 0:
                st.check_status.command.exit_code = self.readiness_exit
        if self.healthy is not None:
            st.healthy = self.healthy
        if self.ip is not None:
            st.container_status.network_infos.add().ip_addresses.add(ip_address=self.ip)
        sim.framework.status_update(sim.driver, st)


class Expect(SimulationTick):
    def __init__(self, fn: Callable[["_Sim"], None], description: str):
        self.fn = fn
        self.description = description

    def expect(self, sim: "_Sim") -> None:
        self.fn(sim)

    @staticmethod
    def declined_last_offer() -> "Expect":
        def fn(sim):
            last = sim.state.last_offer()
            assert last is not None, "no offer was sent"
            declined = {d[0] for d in sim.driver.declines}
            assert last.id.value in declined, f"offer {last.id.value} was not declined (declines: {declined})"
        return Expect(fn, "declined the last offer")

    @staticmethod
    def launched_tasks(*task_names: str, accepts_to_check: int = 1) -> "Expect":
        def fn(sim):
            entries = sim.driver.accepts[-accepts_to_check:] if sim.driver.accepts else []
            launched = sorted(t.name for a in entries for t in a.launched_tasks())
            assert launched == sorted(task_names), f"expected launch of {sorted(task_names)}, got {launched}"
            for a in entries:
                for t in a.launched_tasks():
                    sim.state.task_agents[t.name] = (t.agent_id.value, None)
        return Expect(fn, f"launched tasks {list(task_names)}")

    @staticmethod
    def unreserved_tasks(*task_names: str) -> "Expect":
        """The latest ACCEPT that unreserves anything released every reservation the named tasks
        held before it."""
        def fn(sim):
            accepts = sim.driver.accepts
            idx = next((i for i in range(len(accepts) - 1, -1, -1) if accepts[i].unreserved()), None)
            assert idx is not None, "no UNRESERVE was issued"
            ids = set()
            for name in task_names:
                prev = None
                for a in accepts[:idx]:
                    for x in a.launched_tasks():
                        if x.name == name:
                            prev = x
                assert prev is not None, f"task {name} was not launched before the UNRESERVE"
                ids.update(get_resource_id(r) for r in prev.resources)
            unreserved = {get_resource_id(r) for r in accepts[idx].unreserved()}
            missing = ids - unreserved
            assert not missing, f"resources of {task_names} not unreserved: {missing}"
        return Expect(fn, f"unreserved resources of {list(task_names)}")

    @staticmethod
    def task_name_killed(task_name: str, total_times: int = 1) -> "Expect":
        def fn(sim):
            n = sum(1 for k in sim.driver.kills if k.split("__")[-2:-1] == [task_name] or
                    k.startswith(task_name + "__") or f"__{task_name}__" in k)
            assert n == total_times, f"{task_name} killed {n} times, expected {total_times}"
        return Expect(fn, f"{task_name} killed {total_times}x")

    @staticmethod
    def task_name_not_killed(task_name: str) -> "Expect":
        return Expect.task_name_killed(task_name, 0)

    @staticmethod
    def reconciled_implicitly() -> "Expect":
        return Expect(lambda sim: _assert(any(len(r) == 0 for r in sim.driver.reconciles), "no implicit reconcile"),
                      "implicit reconciliation")

    @staticmethod
    def reconciled_explicitly(*task_names: str) -> "Expect":
        def fn(sim):
            store = StateStore(sim.persister)
            want = {store.fetch_task(n).task_id.value for n in task_names}
            got = {s.task_id.value for r in sim.driver.reconciles for s in r}
            assert want <= got, f"explicit reconcile missing {want - got}"
        return Expect(fn, f"explicit reconciliation of {list(task_names)}")

    @staticmethod
    def revived_offers(total_times: int) -> "Expect":
        return Expect(lambda sim: _assert(sim.driver.revives == total_times,
                                          f"revives={sim.driver.revives}, expected {total_times}"),
                      f"revived {total_times}x")

    @staticmethod
    def suppressed_offers(total_times: int) -> "Expect":
        return Expect(lambda sim: _assert(sim.driver.suppresses == total_times,
                                          f"suppresses={sim.driver.suppresses}, expected {total_times}"),
                      f"suppressed {total_times}x")

    @staticmethod
    def all_plans_complete() -> "Expect":
        def fn(sim):
            bad = {p.get_name(): str(p.get_status()) for p in sim.scheduler.get_plans() if not p.is_complete()}
            assert not bad, f"incomplete plans: {bad}"
        return Expect(fn, "all plans complete")

    @staticmethod
    def plan_status(plan: str, status: Status) -> "Expect":
        def fn(sim):
            p = sim.scheduler.get_plan(plan)
            assert p is not None, f"no plan {plan}"
            assert p.get_status() == status, f"plan {plan} is {p.get_status()}, expected {status}"
        return Expect(fn, f"plan {plan} is {status}")

    @staticmethod
    def step_status(plan: str, phase: str, step: str, status: Status) -> "Expect":
        def fn(sim):
            p = sim.scheduler.get_plan(plan)
            ph = next((x for x in p.get_children() if x.get_name() == phase), None)
            assert ph is not None, f"no phase {phase} in {plan}: {[x.get_name() for x in p.get_children()]}"
            st = next((x for x in ph.get_children() if x.get_name() == step), None)
            assert st is not None, f"no step {step} in {plan}/{phase}: {[x.get_name() for x in ph.get_children()]}"
            assert st.get_status() == status, f"{plan}/{phase}/{step} is {st.get_status()}, expected {status}"
        return Expect(fn, f"{plan}/{phase}/{step} is {status}")

    @staticmethod
    def deploy_step_status(phase: str, step: str, status: Status) -> "Expect":
        return Expect.step_status("deploy", phase, step, status)

    @staticmethod
    def recovery_step_status(phase: str, step: str, status: Status) -> "Expect":
        return Expect.step_status("recovery", phase, step, status)

    @staticmethod
    def step_count(plan: str, count: int) -> "Expect":
        def fn(sim):
            p = sim.scheduler.get_plan(plan)
            n = sum(len(ph.get_children()) for ph in p.get_children())
            assert n == count, f"{plan} has {n} steps, expected {count}"
        return Expect(fn, f"{plan} has {count} steps")

    @staticmethod
    def deploy_step_count(count: int) -> "Expect":
        return Expect.step_count("deploy", count)

    @staticmethod
    def recovery_step_count(count: int) -> "Expect":
        return Expect.step_count("recovery", count)

    @staticmethod
    def known_tasks(*task_names: str) -> "Expect":
        def fn(sim):
            names = sorted(StateStore(sim.persister, sim.namespace).fetch_task_names())
            assert names == sorted(task_names), f"known tasks {names}, expected {sorted(task_names)}"
        return Expect(fn, f"known tasks {list(task_names)}")

    @staticmethod
    def task_env(task_name: str, key: str, value: str) -> "Expect":
        def fn(sim):
            t = StateStore(sim.persister, sim.namespace).fetch_task(task_name)
            env = env_to_map(t.command.environment)
            assert env.get(key) == value, f"{task_name} env {key}={env.get(key)!r}, expected {value!r}"
        return Expect(fn, f"{task_name} env {key}={value}")

    @staticmethod
    def same_pod(*task_names: str) -> "Expect":
        def fn(sim):
            store = StateStore(sim.persister, sim.namespace)
            execs = {store.fetch_task(n).executor.executor_id.value for n in task_names}
            assert len(execs) == 1, f"tasks {task_names} do not share an executor: {execs}"
        return Expect(fn, f"same pod {list(task_names)}")

    @staticmethod
    def http(method: str, path: str, status: int, check: Optional[Callable] = None) -> "Expect":
        def fn(sim):
            r = sim.state.router.dispatch(method, path)
            assert r.status == status, f"{method} {path}: HTTP {r.status}, expected {status}: {r.payload()[:300]!r}"
            if check is not None:
                check(r)
        return Expect(fn, f"{method} {path} -> {status}")

    @staticmethod
    def that(fn: Callable[["_Sim"], None], description: str = "custom") -> "Expect":
        return Expect(fn, description)


def _assert(cond: bool, msg: str) -> None:
    if not cond:
        raise AssertionError(msg)


# ---------------------------------------------------------------------------------------
# runner


@dataclass
class _Sim:
    framework: FrameworkScheduler
    scheduler: object
    driver: RecordingDriver
    state: ClusterState
    persister: object
    cfg: SchedulerConfig
    namespace: Optional[str] = None

    @staticmethod
    def http_ok(resp) -> None:
        if resp.status >= 300:
            raise AssertionError(f"HTTP {resp.status}: {resp.payload()!r}")


@dataclass
class TaskConfig:
    pod_type: str
    task_name: str
    config_name: str
    content: str


@dataclass
class ServiceTestResult:
    persister: object
    cluster_state: ClusterState
    scheduler: object
    sim: _Sim
    service_spec: object = None
    raw_service_spec: object = None
    scheduler_environment: Dict[str, str] = field(default_factory=dict)
    task_configs: List[TaskConfig] = field(default_factory=list)

    def get_task_config(self, pod_type: str, task_name: str, config_name: str) -> str:
        for c in self.task_configs:
            if (c.pod_type, c.task_name, c.config_name) == (pod_type, task_name, config_name):
                return c.content
        raise KeyError(f"no config {config_name} for {pod_type}/{task_name}: "
                       f"{[(c.pod_type, c.task_name, c.config_name) for c in self.task_configs]}")


# Sandbox variables Mesos provides to every task (ServiceTestRunner.DCOS_TASK_ENVVARS)
DCOS_TASK_ENVVARS = {"MESOS_SANDBOX": "/path/to/mesos/sandbox", "MESOS_CONTAINER_IP": "999.987.654.321",
                     "STATSD_UDP_HOST": "999.123.456.789", "STATSD_UDP_PORT": "99999"}


class ServiceTestRunner:
    """Builds a scheduler from a YAML spec (or a ServiceSpec) and plays ticks against it."""

    def __init__(self, spec_path: Optional[str] = None, spec=None, raw=None, universe_dir: Optional[str] = None):
        self.spec_path = spec_path
        self.spec = spec
        self.raw = raw
        self.universe_dir = universe_dir
        self.env: Dict[str, str] = {}
        self.scheduler_env: Dict[str, str] = {}
        self.options: Dict[str, str] = {}
        self.build_params: Dict[str, str] = {}
        self.pod_env: Dict[str, Dict[str, str]] = {}
        self.validators: List = []
        self.recovery_factory = None
        self.persister = None
        self.template_dir: Optional[str] = None
        self.customize: Optional[Callable[[SchedulerBuilder], None]] = None
        self.reader = None
        self.prior_accepts: List = []

    @staticmethod
    def for_framework(name: str, spec_file: str = "svc.yml", root: Optional[str] = None) -> "ServiceTestRunner":
        """Spec + Universe package of ``frameworks/<name>`` (the reference's default runner layout).

        ``root`` points at another framework tree instead, e.g. the reference's unchanged
        ``frameworks/<name>``: there the spec lives in ``src/main/dist`` (ServiceTestRunner.java
        ``getDistDir``), here in ``specs``."""
        if root is None:
            root = os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))),
                                "frameworks", name)
        spec_dir = os.path.join(root, "specs")
        if not os.path.isdir(spec_dir):
            spec_dir = os.path.join(root, "src", "main", "dist")
        return ServiceTestRunner(os.path.join(spec_dir, spec_file), universe_dir=os.path.join(root, "universe"))

    def set_options(self, *key_vals, **options) -> "ServiceTestRunner":
        """Universe package options, e.g. ``set_options("service.user", "foo")``."""
        if len(key_vals) % 2:
            raise ValueError("expected key/value pairs")
        self.options.update({key_vals[i]: str(key_vals[i + 1]) for i in range(0, len(key_vals), 2)})
        self.options.update({k: str(v) for k, v in options.items()})
        return self

    def set_build_template_params(self, **params) -> "ServiceTestRunner":
        self.build_params.update({k: str(v) for k, v in params.items()})
        return self

    def set_pod_env(self, pod_type: str, env: Optional[Dict[str, str]] = None, **kw) -> "ServiceTestRunner":
        """Task env for rendering ``pod_type``'s config templates (values Main would inject)."""
        d = self.pod_env.setdefault(pod_type, {})
        d.update({k: str(v) for k, v in dict(env or {}, **kw).items()})
        return self

    def set_custom_validators(self, validators) -> "ServiceTestRunner":
        self.validators = list(validators)
        return self

    def set_recovery_manager_factory(self, factory) -> "ServiceTestRunner":
        self.recovery_factory = factory
        return self

    def set_env(self, env: Dict[str, str]) -> "ServiceTestRunner":
        self.env.update({k: str(v) for k, v in env.items()})
        return self

    def set_scheduler_env(self, **env) -> "ServiceTestRunner":
        self.scheduler_env.update({k: str(v) for k, v in env.items()})
        return self

    def set_state(self, previous) -> "ServiceTestRunner":
        """Resume from a previous run (scheduler restart / config update tests): a persister, or a
        ``ServiceTestResult`` whose cluster state (prior accepts/reservations) is carried over too,
        like ``ClusterState.withUpdatedConfig`` in the reference runner."""
        if isinstance(previous, ServiceTestResult):
            self.persister = previous.persister
            self.prior_accepts = list(previous.sim.driver.accepts)
        else:
            self.persister = previous
        return self

    def set_config_template_dir(self, path: str) -> "ServiceTestRunner":
        self.template_dir = path
        return self

    def set_template_reader(self, reader) -> "ServiceTestRunner":
        self.reader = reader
        return self

    def set_builder_customizer(self, fn: Callable[[SchedulerBuilder], None]) -> "ServiceTestRunner":
        self.customize = fn
        return self

    def scheduler_environment(self) -> Dict[str, str]:
        env: Dict[str, str] = {}
        if self.universe_dir is not None:
            from dcos_commons_amd.testing.cosmos import render_scheduler_environment

            env.update(render_scheduler_environment(self.universe_dir, self.options, self.build_params))
        env.update(self.env)
        env.update(self.scheduler_env)
        return env

    def _build(self):
        sched_env = self.scheduler_environment()
        cfg_env = dict(sched_env) if self.universe_dir is not None else {}
        cfg_env.update({"PORT_API": "0", "SDK_EVENT_DRIVEN": "false", "SDK_OFFER_HOLD_S": "0"})
        from dcos_commons_amd.testing import profiles

        cfg_env.update(profiles.ACTIVE)     # the suite's flag profile; a test's own flags win
        cfg_env.update(self.scheduler_env)
        if "DCOS_SERVICE_ACCOUNT_CREDENTIAL" not in cfg_env:
            # the reference runner's mocked SchedulerConfig hands out a (null) token provider
            # without failing (ServiceTestRunner.java:296), so TLS specs pass TLSRequiresServiceAccount
            cfg_env.setdefault("SDK_DCOS_AUTH_TOKEN", "service-test-runner-token")
        cfg = SchedulerConfig.for_testing(**cfg_env)
        raw = self.raw
        spec = self.spec
        render_env = sched_env if self.universe_dir is not None else self.env
        if spec is None:
            rb = RawServiceSpec.new_builder(self.spec_path).set_env(render_env)
            if self.universe_dir is not None:
                rb.enable_strict_rendering()
            raw = rb.build()
            gen = ServiceSpecGenerator(raw, cfg, self.template_dir or os.path.dirname(os.path.abspath(self.spec_path)),
                                       render_env)
            if self.reader is not None:
                gen.reader = self.reader
            spec = gen.build()
        persister = self.persister if self.persister is not None else MemPersister()
        builder = SchedulerBuilder(spec, cfg, persister)
        if raw is not None:
            builder.set_plans_from(raw)
        if self.validators:
            builder.set_custom_config_validators(self.validators)
        if self.recovery_factory is not None:
            builder.set_recovery_manager_factory(self.recovery_factory)
        if self.customize is not None:
            self.customize(builder)
        self._last = (raw, sched_env)
        return cfg, spec, persister, builder

    def _task_configs(self, spec, cfg) -> List[TaskConfig]:
        """Renders every config template of pod index 0 strictly (reference Test 4)."""
        from dcos_commons_amd.offer.evaluate.pod_info_builder import get_task_environment
        from dcos_commons_amd.specification.specs import PodInstance, PortSpec
        from dcos_commons_amd.specification.yaml.template_utils import render_mustache_throw_if_missing

        out: List[TaskConfig] = []
        rng = random.Random(0)
        for pod in spec.pods:
            pi = PodInstance(pod, 0)
            for task in pod.tasks:
                env = get_task_environment(spec.name, pi, task, cfg)
                env.update(DCOS_TASK_ENVVARS)
                # a pod whose placement names zones/regions only launches on offers that carry a
                # fault domain, so its tasks always see ZONE/REGION (PodInfoBuilder adds them)
                if env.get("PLACEMENT_REFERENCED_ZONE") == "true":
                    env.setdefault("ZONE", "test-zone")
                if env.get("PLACEMENT_REFERENCED_REGION") == "true":
                    env.setdefault("REGION", "test-region")
                for r in task.resource_set.resources:
                    if isinstance(r, PortSpec) and r.env_key:
                        env[r.env_key] = str(r.port or rng.randrange(32768, 61000))
                env.update(self.pod_env.get(pod.type, {}))
                for c in task.config_files:
                    content = render_mustache_throw_if_missing(
                        f"pod={pod.type} task={task.name} config={c.name}", c.template_content, env)
                    out.append(TaskConfig(pod.type, task.name, c.name, content))
        return out

    def run(self, ticks: Iterable[SimulationTick] = ()) -> ServiceTestResult:
        ProcessExit.set_test_mode(True)
        task_killer.reset(executor_enabled=False)
        cfg, spec, persister, builder = self._build()
        task_configs = self._task_configs(spec, cfg) if self.universe_dir is not None or self.pod_env else []
        scheduler = builder.build()
        fc = FrameworkConfig.from_service_spec(spec)
        roles = set(fc.pre_reserved_roles) | {fc.role}
        framework = FrameworkScheduler(roles, cfg, persister, FrameworkStore(persister), scheduler).disable_threading()
        framework.set_api_server_started()
        driver = RecordingDriver()
        driver.accepts.extend(self.prior_accepts)
        router = Router(scheduler.get_http_endpoints())
        state = ClusterState(spec, driver, router)
        sim = _Sim(framework, scheduler, driver, state, persister, cfg, getattr(scheduler, "namespace", None))
        for i, tick in enumerate(ticks):
            try:
                if isinstance(tick, Send):
                    tick.send(sim)
                elif isinstance(tick, Expect):
                    tick.expect(sim)
                else:
                    raise TypeError(f"unknown tick {tick!r}")
            except AssertionError as e:
                raise AssertionError(f"tick {i} ({tick.description}) failed: {e}") from e
        task_killer.reset(executor_enabled=True)
        raw, sched_env = self._last
        return ServiceTestResult(persister, state, scheduler, sim, spec, raw, sched_env, task_configs)
