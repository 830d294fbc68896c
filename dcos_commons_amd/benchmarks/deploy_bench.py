"""Deploy wall-clock + pod-recovery MTTR benchmark (the BASELINE.json headline metric).

One *cycle* on a fresh cluster and fresh state:
  1. start the helloworld scheduler and time until ``GET /v1/plans/deploy`` answers 200
     (deploy plan COMPLETE: every pod RUNNING and, for GPU pods, its readiness check -- the HIP
     device probe on the GPU it was given -- passed);
  2. inject ``TASK_FAILED`` into pod ``hello-0`` and time until it is back (new task RUNNING +
     ready) and the ``recovery`` plan is COMPLETE (MTTR, transient restart);
  3. ``POST /v1/pod/hello-0/replace`` and time the same way (MTTR, permanent replace);
  4. tear the scheduler down.

Cluster: ``n_agents`` agents, each owning one MI355X (``gpus: 1``, ``HIP_VISIBLE_DEVICES``
pinned by device index); helloworld ``gpu.yml`` with one pod per agent (``hostname:UNIQUE``).
The ``reference`` profile replays the reference scheduler's timing constants on the same harness
(5 s offer poll, long declines + 5 s-throttled revives, no event-driven wake-up).
"""
from __future__ import annotations

import os
import time
from dataclasses import dataclass
from typing import Callable, Dict, List, Optional

from dcos_commons_amd.framework.process_exit import ProcessExit
from dcos_commons_amd.mesos import protos as P
from dcos_commons_amd.mesos.local_master import AgentSpec, LocalMaster, LocalSchedulerDriver, TaskBehavior, TaskTiming
from dcos_commons_amd.offer.taskdata.labels import TaskLabelReader
from dcos_commons_amd.scheduler.scheduler_builder import SchedulerBuilder
from dcos_commons_amd.scheduler.scheduler_config import SchedulerConfig
from dcos_commons_amd.scheduler.scheduler_runner import SchedulerRunner
from dcos_commons_amd.specification.yaml.mappers import ServiceSpecGenerator
from dcos_commons_amd.specification.yaml.raw import RawServiceSpec
from dcos_commons_amd.storage.mem_persister import MemPersister

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
SPECS = os.path.join(ROOT, "frameworks", "helloworld", "specs")

PROFILES = {
    # this framework: event-driven offer loop, bounded offer holding
    "mi355x": {},  # framework defaults: event-driven wake-ups, 10 s offer holding, 1 s revive spacing
    # the reference's cadence on the same harness
    "reference": {"SDK_EVENT_DRIVEN": "false", "SDK_OFFER_HOLD_S": "0", "SDK_OFFER_WAIT_S": "5",
                  "SDK_REVIVE_INTERVAL_S": "5", "SDK_REVIVE_BURST_INTERVAL_S": "5",
                  "SDK_RESERVATION_GC_ALL_OFFERS": "false",
                  "SDK_FAST_UNSUPPRESS": "false", "SDK_MERGE_AGENT_OFFERS": "false",
                  "SDK_LAUNCH_RECONCILE_S": "0", "SDK_UNKNOWN_AS_LOST": "false", "SDK_STREAM_LAUNCHES": "false",
                  "SDK_REVIVE_ONLY_UNMATCHED": "false", "SDK_GC_GEN0_THRESHOLD": "0",
                  "SDK_STATUS_CYCLE_WAIT_MS": "0"},
}


@dataclass
class CycleResult:
    deploy_s: float            # from the scheduler's construction (SchedulerRunner.run) to deploy COMPLETE
    mttr_restart_s: float
    mttr_replace_s: float
    total_s: float
    deploy_from_subscribed_s: float = 0.0   # BASELINE.md protocol: from SUBSCRIBED to deploy COMPLETE


def helloworld_env(n_pods: int, gpus_per_pod: int, probe_cmd: str) -> Dict[str, str]:
    return {
        "FRAMEWORK_NAME": "hello-world", "FRAMEWORK_PRINCIPAL": "hello-world-principal", "FRAMEWORK_USER": "nobody",
        "HELLO_COUNT": str(n_pods), "HELLO_PLACEMENT": '[["hostname", "UNIQUE"]]', "HELLO_CPUS": "0.1",
        "HELLO_GPUS": str(gpus_per_pod), "HELLO_MEM": "252", "HELLO_DISK": "25", "SLEEP_DURATION": "1000",
        "GPU_PROBE_CMD": probe_cmd, "WORLD_COUNT": "0", "WORLD_PLACEMENT": "", "WORLD_CPUS": "0.2",
        "WORLD_MEM": "512", "WORLD_DISK": "25", "WORLD_READINESS_CHECK_INTERVAL": "5",
        "WORLD_READINESS_CHECK_DELAY": "0", "WORLD_READINESS_CHECK_TIMEOUT": "10",
    }


def reference_spec(name: str) -> Optional[str]:
    """Path of the reference's unchanged helloworld example ``name`` (e.g. ``gpu_resource.yml``),
    from $SDK_REFERENCE_ROOT, the reference checkout or the staged ``ref_inputs/`` copy."""
    for root in (os.environ.get("SDK_REFERENCE_ROOT", ""), "/root/reference", os.path.join(ROOT, "ref_inputs")):
        p = os.path.join(root, "frameworks", "helloworld", "src", "main", "dist", name) if root else ""
        if p and os.path.isfile(p):
            return p
    return None


def agent_specs_from_inventory(devices: List[int], inventory=None, hostname="mi355x-agent-{i}") -> List[AgentSpec]:
    """One agent per entry of ``devices`` (a device index of this node), its resources and
    attributes (``gpu_model``, ``gpu_arch``, ``xgmi_hive``) from node discovery (``ops.gpu``):
    the devices this node really has, or a synthetic MI355X inventory where there is no driver."""
    from dcos_commons_amd.ops import gpu as G

    inv = inventory if inventory is not None else G.node_inventory(max(devices) + 1 if devices else 0)
    return [AgentSpec.from_gpu_inventory(hostname.format(i=i), inv, devices=[dev], cpus=16, mem=65536, disk=100000)
            for i, dev in enumerate(devices)]


def agent_spec_from_registration(info: Dict, index: int) -> AgentSpec:
    """The agent a remote rank registered over ``parallel.agent_link``: its hostname, the device
    indices it serves and its discovered inventory (``GpuInventory.to_dict``)."""
    from dcos_commons_amd.ops import gpu as G

    inv = G.GpuInventory.from_dict(info["inventory"])
    return AgentSpec.from_gpu_inventory(info.get("hostname") or f"mi355x-agent-{index}", inv,
                                        devices=list(info["devices"]), cpus=16, mem=65536, disk=100000)


class _LocalCluster:
    """This interpreter's LocalMaster (agents' task lifecycles included)."""

    def __init__(self, master: LocalMaster):
        self.master = master

    def driver(self, sched, info):
        return LocalSchedulerDriver(self.master, sched, info)

    def placement(self):
        return self.master.placement()

    def fail_task(self, task_id: str) -> None:
        self.master.fail_task(task_id)

    def shutdown(self) -> None:
        self.master.shutdown()


class _RemoteCluster:
    """A fresh master in the master process (``mesos.master_process``), same agents."""

    def __init__(self, client, allocation_interval_s: float):
        from dcos_commons_amd.mesos.stream_api import StreamSchedulerDriver

        self.client = client
        self.address = client.call("reset", allocation_interval_s=allocation_interval_s)["stream"]
        self._driver_cls = StreamSchedulerDriver

    def driver(self, sched, info):
        return self._driver_cls(self.address, sched, info)

    def placement(self):
        return self.client.call("placement")

    def fail_task(self, task_id: str) -> None:
        self.client.call("fail_task", task_id=task_id)

    def shutdown(self) -> None:
        pass


class DeployBench:
    def __init__(self, n_agents: int, profile: str = "mi355x", spec_file: str = "gpu.yml",
                 check_runner: Optional[Callable[[P.TaskInfo, List[int]], bool]] = None,
                 gpu_devices: Optional[List[int]] = None, allocation_interval_s: float = 1.0,
                 timeout_s: float = 120.0, agent_runners: Optional[List[Callable]] = None,
                 extra_env: Optional[Dict[str, str]] = None, agent_specs: Optional[List[AgentSpec]] = None,
                 spec_env: Optional[Dict[str, str]] = None, master_client=None):
        self.n = n_agents
        # ``mesos.master_process.MasterClient``: the master runs in a process of its own and the
        # agents run their tasks themselves (the scheduler subscribes over ``mesos.stream_api``);
        # None: the master and every agent's task lifecycle run in this interpreter
        self.master_client = master_client
        self.extra_env = dict(extra_env or {})  # scheduler flag overrides on top of the profile
        self.spec_env = dict(spec_env or {})    # spec rendering overrides (e.g. WORLD_COUNT)
        self.profile = profile
        # a file of frameworks/helloworld/specs, or an absolute path (the reference's examples)
        self.spec_file = spec_file
        self.check_runner = check_runner
        self.gpu_devices = gpu_devices if gpu_devices is not None else list(range(n_agents))
        self.agent_specs = agent_specs if agent_specs is not None else (
            [] if master_client is not None else agent_specs_from_inventory(self.gpu_devices))
        if master_client is None and len(self.agent_specs) != n_agents:
            raise ValueError(f"{len(self.agent_specs)} agent specs for {n_agents} agents")
        self.last_placement: List[Dict] = []  # LocalMaster.placement() once the last deploy completed
        self.allocation_interval_s = allocation_interval_s
        self.timeout_s = timeout_s
        self.agent_runners = agent_runners  # per-agent check runner (remote GPU agents)
        # the agents' check executors outlive a cycle, as they outlive a scheduler on a real cluster
        self.behavior = None if master_client is not None else TaskBehavior(
            TaskTiming(), check_runner=self.check_runner, check_workers=max(8, n_agents)).prestart()

    # -- helpers ---------------------------------------------------------------------------
    def _wait(self, pred, what: str, event=None) -> float:
        """Until ``pred()``. With ``event`` (the scheduler's status-processed event) the predicate
        is re-checked whenever a status has been processed (and every 5 ms regardless), so the
        observer neither lags the completing status by a poll period nor competes with the
        scheduler for the interpreter between statuses."""
        t0 = time.perf_counter()
        while True:
            if event is not None:
                event.clear()
            if pred():
                return time.perf_counter() - t0
            if time.perf_counter() - t0 > self.timeout_s:
                raise TimeoutError(f"timed out after {self.timeout_s}s waiting for {what}")
            if event is not None:
                event.wait(0.005)
            else:
                time.sleep(0.001)

    @staticmethod
    def _plan_done(scheduler, name: str) -> bool:
        """What ``GET /v1/plans/<name>`` reports as 200 (COMPLETE, no errors), read straight from
        the plan instead of rendering the plan JSON through the API router on every 1 ms poll (the
        poller would otherwise compete with the scheduler it is timing)."""
        plan = scheduler.get_plan(name)
        return plan is not None and not plan.has_errors() and plan.is_complete()

    @staticmethod
    def _pod_ready(state_store, task_name: str, old_task_id: Optional[str]) -> bool:
        info = state_store.fetch_task_shared(task_name)    # the observer only reads it
        st = state_store.fetch_status(task_name)
        if info is None or st is None or st.state != P.TASK_RUNNING:
            return False
        if old_task_id is not None and st.task_id.value == old_task_id:
            return False
        if st.task_id.value != info.task_id.value:
            return False
        return TaskLabelReader(info).is_readiness_check_succeeded(st)

    @staticmethod
    def _expect_api(router, plan: str) -> None:
        r = router.get(f"/v1/plans/{plan}")
        if r.status != 200:
            raise RuntimeError(f"/v1/plans/{plan} answered {r.status} after the plan completed")

    def _make_master(self) -> "_Cluster":
        if self.master_client is not None:
            return _RemoteCluster(self.master_client, self.allocation_interval_s)
        master = LocalMaster(allocation_interval_s=self.allocation_interval_s, behavior=self.behavior)
        for i, spec in enumerate(self.agent_specs):
            master.add_agent(spec, check_runner=self.agent_runners[i] if self.agent_runners else None)
        return _LocalCluster(master)

    # -- one cycle -------------------------------------------------------------------------
    def run_cycle(self) -> CycleResult:
        ProcessExit.set_test_mode(True)
        t_cycle = time.perf_counter()
        env = helloworld_env(self.n, 1, "amd-gpu-probe --readiness")
        env.update(self.spec_env)
        overrides = dict(PROFILES[self.profile])
        overrides.update(self.extra_env)
        overrides.update({"PORT_API": "0", "SDK_PERSISTER": "mem"})
        cfg = SchedulerConfig.for_testing(**overrides)
        path = self.spec_file if os.path.isabs(self.spec_file) else os.path.join(SPECS, self.spec_file)
        raw = RawServiceSpec.new_builder(path).set_env(env).build()
        spec = ServiceSpecGenerator(raw, cfg, os.path.dirname(path), env).build()
        master = self._make_master()
        builder = SchedulerBuilder(spec, cfg, MemPersister()).set_plans_from(raw)
        marks = {}

        def driver_factory(sched, info):
            # SUBSCRIBED reaches the scheduler as its `registered` callback: the start of the
            # BASELINE.md deploy window (the scheduler's construction and API server come before)
            orig = sched.registered

            def registered(*a, **k):
                marks.setdefault("subscribed", time.perf_counter())
                return orig(*a, **k)
            sched.registered = registered
            return master.driver(sched, info)
        runner = SchedulerRunner(builder, driver_factory=driver_factory)
        try:
            t0 = time.perf_counter()
            runner.run(block=False)
            router = runner.framework_runner.api_server.router
            state_store = runner.scheduler.state_store
            sched = runner.scheduler
            ev = sched.status_processed
            self._wait(lambda: self._plan_done(sched, "deploy"), "deploy plan COMPLETE", ev)
            t_done = time.perf_counter()
            deploy_s = t_done - t0
            deploy_sub = t_done - marks.get("subscribed", t0)
            self._expect_api(router, "deploy")
            self.last_placement = master.placement()

            # failures are injected in steady state: deploy finished and the offer loop has gone
            # idle (suppressed), as for a pod that fails long after its service deployed
            rm = runner.framework_runner.framework_scheduler.offer_processor.revive_manager
            self._wait(lambda: rm.is_suppressed, "scheduler idle after deploy")

            # transient restart MTTR
            old = state_store.fetch_task("hello-0-server").task_id.value
            t1 = time.perf_counter()
            master.fail_task(old)
            self._wait(lambda: self._pod_ready(state_store, "hello-0-server", old) and
                       self._plan_done(sched, "recovery"), "restart recovery", ev)
            mttr_restart = time.perf_counter() - t1
            self._expect_api(router, "recovery")

            self._wait(lambda: rm.is_suppressed, "scheduler idle after restart")

            # permanent replace MTTR
            old = state_store.fetch_task("hello-0-server").task_id.value
            t2 = time.perf_counter()
            r = router.post("/v1/pod/hello-0/replace")
            if r.status != 200:
                raise RuntimeError(f"replace failed: {r.status} {r.payload()!r}")
            self._wait(lambda: self._pod_ready(state_store, "hello-0-server", old) and
                       self._plan_done(sched, "recovery"), "replace recovery", ev)
            mttr_replace = time.perf_counter() - t2
            self._expect_api(router, "recovery")
        finally:
            runner.stop()
            master.shutdown()
        return CycleResult(deploy_s, mttr_restart, mttr_replace, time.perf_counter() - t_cycle, deploy_sub)
