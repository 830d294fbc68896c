"""Framework-level benchmarks for the remaining BASELINE.json configs (the headline helloworld
deploy/MTTR bench lives in ``deploy_bench``):

* **cassandra, 3 nodes** -- deploy plan COMPLETE wall-clock (serial ``node`` phase plus the ONCE
  ``init_system_keyspaces`` step), then ``POST /v1/pod/node-<i>/replace`` until the replacement
  server is RUNNING + ready and the recovery plan is COMPLETE. The recovery phase must come from
  ``CassandraRecoveryPlanOverrider`` (``-Dcassandra.replace_address=<old ip>`` on the new server's
  command; reference: frameworks/cassandra/.../CassandraRecoveryPlanOverrider.java:66-101).
* **hdfs, HA layout** (3 journal, 2 name with zkfc, 3 data) -- deploy plan COMPLETE wall-clock
  (multi-step phases: ``journal`` bootstrap + node, ``name`` format/bootstrap/zkfc-format + node/zkfc,
  ``data``), then a configuration change rolled out by a scheduler restart: the ``update`` plan
  (journal serial -> name ``[[node, zkfc]]`` -> data serial; reference frameworks/hdfs/src/main/dist/
  svc.yml:566-611) replaces deploy and is timed until COMPLETE with every task relaunched.

Both run the real scheduler (offer loop, plan engine, state store, HTTP API) against the in-process
Mesos master (``LocalMaster``) with synthetic task payloads: RUNNING tasks start at once, ONCE/FINISH
tasks exit FINISHED at once and readiness checks pass without their configured delays, so the numbers
are scheduler cost, not Cassandra/HDFS start-up time. ``profile="reference"`` replays the
reference's offer cadence (5 s poll, throttled revives; see ``deploy_bench.PROFILES``).
"""
from __future__ import annotations

import os
import time
from dataclasses import dataclass
from typing import Dict, List, Optional

from dcos_commons_amd.framework.process_exit import ProcessExit
from dcos_commons_amd.mesos import protos as P
from dcos_commons_amd.mesos.local_master import AgentSpec, LocalMaster, LocalSchedulerDriver, TaskBehavior, TaskTiming
from dcos_commons_amd.offer.taskdata.labels import TaskLabelReader
from dcos_commons_amd.scheduler.scheduler_config import SchedulerConfig
from dcos_commons_amd.scheduler.scheduler_runner import SchedulerRunner
from dcos_commons_amd.state.state_store_utils import get_deployment_was_completed
from dcos_commons_amd.storage.mem_persister import MemPersister

from .deploy_bench import PROFILES

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

# task-name fragments of the ONCE/FINISH tasks: they exit FINISHED right after RUNNING
_FINISHING = ("init_system_keyspaces", "-bootstrap", "-format")


@dataclass
class FrameworkCycle:
    framework: str
    deploy_s: float
    second_s: float          # cassandra: replace-node MTTR; hdfs: rolling config update
    second_name: str
    tasks: int
    total_s: float

    def as_dict(self) -> Dict[str, float]:
        return {"framework": self.framework, "deploy_s": round(self.deploy_s, 6),
                self.second_name: round(self.second_s, 6), "tasks": self.tasks, "total_s": round(self.total_s, 6)}


def _behavior() -> TaskBehavior:
    finish = TaskTiming(finish_after_s=0.0, honor_check_delays=False)
    return TaskBehavior(TaskTiming(honor_check_delays=False), overrides={k: finish for k in _FINISHING})


# Where the reference's unchanged framework packages are looked for: $SDK_REFERENCE_ROOT, the
# reference checkout, or a staged copy of its frameworks/ (scripts/stage_reference_inputs.sh; the GPU
# box gets only the repository tree, so the copy travels in a gitignored directory of it).
REFERENCE_ROOTS = (os.environ.get("SDK_REFERENCE_ROOT", ""), "/root/reference", os.path.join(ROOT, "ref_inputs"))


def reference_framework_root(framework: str) -> Optional[str]:
    for root in REFERENCE_ROOTS:
        d = os.path.join(root, "frameworks", framework) if root else ""
        if d and os.path.isfile(os.path.join(d, "src", "main", "dist", "svc.yml")):
            return d
    return None


def framework_root(framework: str, spec_set: str) -> str:
    """``spec_set="reference"``: the reference's unchanged ``svc.yml`` (+ config templates) and
    ``universe/`` package; ``"repo"``: this repository's rewritten, lighter package."""
    if spec_set == "reference":
        root = reference_framework_root(framework)
        if root is None:
            raise FileNotFoundError(f"no reference frameworks/{framework} found in {REFERENCE_ROOTS}")
        return root
    if spec_set != "repo":
        raise ValueError(f"unknown spec set {spec_set!r}")
    return os.path.join(ROOT, "frameworks", framework)


def spec_path(root: str) -> str:
    repo_layout = os.path.join(root, "specs", "svc.yml")
    return repo_layout if os.path.isfile(repo_layout) else os.path.join(root, "src", "main", "dist", "svc.yml")


def _scheduler_env(root: str, **extra: str) -> Dict[str, str]:
    from dcos_commons_amd.testing.cosmos import render_scheduler_environment

    env = render_scheduler_environment(os.path.join(root, "universe"), {}, {})
    env.update(extra)
    return env


class FrameworkBench:
    def __init__(self, framework: str, profile: str = "mi355x", allocation_interval_s: float = 1.0,
                 timeout_s: float = 120.0, spec_set: str = "reference"):
        if framework not in ("cassandra", "hdfs"):
            raise ValueError(f"unknown framework {framework!r}")
        self.framework = framework
        self.spec_set = spec_set
        self.root = framework_root(framework, spec_set)
        self.profile = profile
        self.allocation_interval_s = allocation_interval_s
        self.timeout_s = timeout_s

    # -- helpers ---------------------------------------------------------------------------
    def _wait(self, pred, what: str, event=None) -> float:
        """Until ``pred()``; with the scheduler's status-processed ``event`` the predicate is
        re-checked when a status lands (and every 5 ms), as in ``DeployBench._wait``."""
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
        """What ``GET /v1/plans/<name>`` answers 200 for, read from the plan itself (rendering the
        plan JSON on every poll competed with the scheduler being timed)."""
        plan = scheduler.get_plan(name)
        return plan is not None and not plan.has_errors() and plan.is_complete()

    @staticmethod
    def _expect_api(api, name: str) -> None:
        r = api.get(f"/v1/plans/{name}")
        if r.status != 200:
            raise RuntimeError(f"/v1/plans/{name} answered {r.status} after the plan completed")

    def _config(self) -> SchedulerConfig:
        overrides = dict(PROFILES[self.profile])
        overrides.update({"PORT_API": "0", "SDK_PERSISTER": "mem"})
        return SchedulerConfig.for_testing(**overrides)

    def _master(self, agents: int) -> LocalMaster:
        master = LocalMaster(allocation_interval_s=self.allocation_interval_s, behavior=_behavior())
        for i in range(agents):
            master.add_agent(AgentSpec(hostname=f"agent-{i}", cpus=32, mem=262144, disk=2_000_000,
                                       ports=((1025, 32000),)))  # cassandra/hdfs use fixed ports
        return master

    def _builder(self, env: Dict[str, str], cfg: SchedulerConfig, persister):
        spec = spec_path(self.root)
        if self.framework == "cassandra":
            from dcos_commons_amd.models import cassandra as m
        else:
            from dcos_commons_amd.models import hdfs as m
        return m.create_scheduler_builder(spec, cfg, env, persister)

    @staticmethod
    def _ready(state_store, task_name: str, old_task_id: Optional[str]) -> bool:
        info = state_store.fetch_task_shared(task_name)    # the observer only reads it
        st = state_store.fetch_status(task_name)
        if info is None or st is None or st.state != P.TASK_RUNNING:
            return False
        if st.task_id.value != info.task_id.value or (old_task_id is not None and st.task_id.value == old_task_id):
            return False
        return TaskLabelReader(info).is_readiness_check_succeeded(st)

    def _start(self, master, env, cfg, persister):
        runner = SchedulerRunner(self._builder(env, cfg, persister),
                                 driver_factory=lambda s, info: LocalSchedulerDriver(master, s, info))
        runner.run(block=False)
        return runner

    # -- cycles ----------------------------------------------------------------------------
    def run_cycle(self) -> FrameworkCycle:
        ProcessExit.set_test_mode(True)
        return self._cassandra() if self.framework == "cassandra" else self._hdfs()

    def _cassandra(self) -> FrameworkCycle:
        t_cycle = time.perf_counter()
        env = _scheduler_env(self.root, NODE_COUNT="3")
        cfg, persister, master = self._config(), MemPersister(), self._master(3)
        runner = None
        try:
            t0 = time.perf_counter()
            runner = self._start(master, env, cfg, persister)
            api, store = runner.framework_runner.api_server.router, runner.scheduler.state_store
            sched = runner.scheduler
            ev = sched.status_processed
            self._wait(lambda: self._plan_done(sched, "deploy"), "cassandra deploy COMPLETE", ev)
            deploy_s = time.perf_counter() - t0
            self._expect_api(api, "deploy")
            rm = runner.framework_runner.framework_scheduler.offer_processor.revive_manager
            self._wait(lambda: rm.is_suppressed, "scheduler idle after deploy")

            # replace a seed node (node-1 of 3 is a seed with the default SEED_COUNT of 2)
            old = store.fetch_task("node-1-server").task_id.value
            t1 = time.perf_counter()
            r = api.post("/v1/pod/node-1/replace")
            if r.status != 200:
                raise RuntimeError(f"replace failed: {r.status} {r.payload()!r}")
            self._wait(lambda: self._ready(store, "node-1-server", old) and
                       self._plan_done(sched, "recovery"), "cassandra replace recovery", ev)
            replace_s = time.perf_counter() - t1
            self._expect_api(api, "recovery")
            cmd = store.fetch_task("node-1-server").command.value
            if "-Dcassandra.replace_address=" not in cmd:
                raise RuntimeError("replacement did not go through CassandraRecoveryPlanOverrider")
            tasks = sum(1 for n in store.fetch_task_names()
                        if (store.fetch_status(n) or P.TaskStatus()).state == P.TASK_RUNNING)
        finally:
            if runner is not None:
                runner.stop()
            master.shutdown()
        return FrameworkCycle("cassandra", deploy_s, replace_s, "mttr_replace_node_s", tasks,
                              time.perf_counter() - t_cycle)

    def _hdfs(self) -> FrameworkCycle:
        t_cycle = time.perf_counter()
        env = _scheduler_env(self.root)
        cfg, persister, master = self._config(), MemPersister(), self._master(8)
        runner = None
        try:
            t0 = time.perf_counter()
            runner = self._start(master, env, cfg, persister)
            api = runner.framework_runner.api_server.router
            sched = runner.scheduler
            self._wait(lambda: self._plan_done(sched, "deploy"), "hdfs deploy COMPLETE", sched.status_processed)
            deploy_s = time.perf_counter() - t0
            self._expect_api(api, "deploy")
            store = runner.scheduler.state_store
            # the scheduler records deploy completion on its next status pass; a later config
            # change is then rolled out by the update plan instead of re-running deploy
            self._wait(lambda: get_deployment_was_completed(store), "deploy-completed marker")
            running = [n for n in store.fetch_task_names()
                       if (store.fetch_status(n) or P.TaskStatus()).state == P.TASK_RUNNING]
            before = {n: store.fetch_task(n).task_id.value for n in running}
            runner.stop()
            runner = None

            # configuration change routed to every task (TASKCFG_ALL_*): the update plan restarts all
            env2 = dict(env, TASKCFG_ALL_BENCH_ROLLOUT="2")
            t1 = time.perf_counter()
            runner = self._start(master, env2, cfg, persister)
            api, store = runner.framework_runner.api_server.router, runner.scheduler.state_store
            plan = runner.scheduler.get_plan("deploy")
            if plan is None or [p.get_name() for p in plan.get_children()] != ["journal", "name", "data"]:
                raise RuntimeError("update plan was not selected for the configuration change: %r" % (
                    plan and [p.get_name() for p in plan.get_children()],))
            sched = runner.scheduler
            self._wait(lambda: self._plan_done(sched, "deploy") and
                       all(self._ready(store, n, old) for n, old in before.items()), "hdfs rolling update",
                       sched.status_processed)
            update_s = time.perf_counter() - t1
            self._expect_api(api, "deploy")
            tasks = len(before)
        finally:
            if runner is not None:
                runner.stop()
            master.shutdown()
        return FrameworkCycle("hdfs", deploy_s, update_s, "rolling_update_s", tasks, time.perf_counter() - t_cycle)


def main(argv: Optional[List[str]] = None) -> int:
    import argparse
    import json
    import statistics

    ap = argparse.ArgumentParser(description="cassandra / hdfs framework benchmarks (BASELINE configs 3 and 4)")
    ap.add_argument("--framework", choices=["cassandra", "hdfs", "all"], default="all")
    ap.add_argument("--profile", choices=sorted(PROFILES), default="mi355x")
    ap.add_argument("--cycles", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1,
                    help="untimed cycles first: the first scheduler built in a process also pays one-time "
                         "imports and caches, which a scheduler pays once at process start, before SUBSCRIBE")
    ap.add_argument("--allocation-interval", type=float, default=1.0)
    ap.add_argument("--specs", choices=["reference", "repo", "both"], default="both",
                    help="reference: the reference's unchanged svc.yml + universe/ (the BASELINE configs); "
                         "repo: this repository's rewritten packages")
    args = ap.parse_args(argv)
    spec_sets = ["reference", "repo"] if args.specs == "both" else [args.specs]
    runs = [(fw, ss) for fw in (["cassandra", "hdfs"] if args.framework == "all" else [args.framework])
            for ss in spec_sets]
    for fw, ss in runs:
        if ss == "reference" and reference_framework_root(fw) is None:
            print(json.dumps({"framework": fw, "specs": ss, "skipped": "reference package not found"}), flush=True)
            continue
        bench = FrameworkBench(fw, args.profile, args.allocation_interval, spec_set=ss)
        for _ in range(args.warmup):
            bench.run_cycle()
        cycles = [bench.run_cycle() for _ in range(args.cycles)]
        second = cycles[0].second_name

        def stat(vals):
            return {"mean": round(sum(vals) / len(vals), 6), "median": round(statistics.median(vals), 6),
                    "min": round(min(vals), 6), "max": round(max(vals), 6)}
        out = {"framework": fw, "specs": ss, "spec_path": spec_path(bench.root), "profile": args.profile,
               "cycles": args.cycles, "warmup": args.warmup, "tasks": cycles[0].tasks,
               "deploy_s": stat([c.deploy_s for c in cycles]),
               second: stat([c.second_s for c in cycles]),
               "data": "synthetic task payloads (LocalMaster), readiness delays not honoured"}
        print(json.dumps(out), flush=True)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
