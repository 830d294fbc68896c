"""Deploy wall-clock and pod-recovery MTTR on the local DC/OS stand-in: the scheduler as its own
OS process, talking to the Mesos master over the v1 scheduler HTTP API, persisting to ZooKeeper.

``deploy_bench`` (the ``bench.py`` headline) runs the scheduler, the master and the agents in one
interpreter with an in-memory persister. This bench runs the same helloworld ``gpu.yml`` service the
way it runs on a cluster (``testing.cluster.LocalCluster``, SURVEY §4 system-integration tier):

* the service is installed through the Cosmos stand-in and its scheduler is started by the Marathon
  stand-in as a separate process (``python -m dcos_commons_amd.models.helloworld``);
* the scheduler subscribes to the master over HTTP (RecordIO event stream, protobuf calls,
  acknowledgements) and keeps its state in ZooKeeper (jute wire protocol, ``SDK_PERSISTER=zk``);
* with ``executor="process"`` every task is a real process in an agent sandbox, and the readiness
  check is a real command run by the agent (``--probe-cmd``; on an MI355X box
  ``native/build/amd-gpu-probe --readiness`` runs the HIP probe on the pod's device, starting a HIP
  runtime per check; with ``--probe-service`` the node's readiness service ``amd-gpu-probed``
  keeps one runtime resident and the check is ``native/build/amd-gpu-ready``).

Timing follows BASELINE.md: deploy is measured from the master accepting the framework's SUBSCRIBE
to ``GET /v1/plans/deploy`` answering 200 (the scheduler process start-up and imports are outside
the window, as they are for the reference). Restart MTTR: from an injected ``TASK_FAILED`` to the
new task RUNNING and ready with ``/v1/plans/recovery`` at 200; replace MTTR: from
``POST /v1/pod/hello-0/replace`` to the same.

    python -m dcos_commons_amd.benchmarks.cluster_bench --agents 1 --cycles 3
"""
from __future__ import annotations

import argparse
import http.client
import json
import logging
import statistics
import threading
import time
import urllib.error
import urllib.parse
import urllib.request
from typing import Callable, Dict, List, Optional

from dcos_commons_amd.mesos import protos as P

PACKAGE = "hello-world"
DEFAULT_PROBE = 'test -n "$HIP_VISIBLE_DEVICES"'
POLL_S = 0.001


class _Watch:
    """Master-side observations, from the bench process (the master runs here, the scheduler
    does not): when a framework subscribed, and each task's latest status."""

    def __init__(self, cluster):
        self.cond = threading.Condition()
        self.subscribed: Dict[str, float] = {}
        self.statuses: Dict[str, P.TaskStatus] = {}
        master = cluster.master
        orig = master.subscribe

        def subscribe(driver, info, _orig=orig):
            with self.cond:
                self.subscribed.setdefault(info.name, time.perf_counter())
                self.cond.notify_all()
            return _orig(driver, info)

        master.subscribe = subscribe
        master.add_status_listener(self._on_status)

    def _on_status(self, framework_id: str, status: P.TaskStatus) -> None:
        with self.cond:
            self.statuses[status.task_id.value] = status
            self.cond.notify_all()

    def wait(self, pred: Callable[[], bool], timeout_s: float, what: str) -> None:
        deadline = time.monotonic() + timeout_s
        with self.cond:
            while not pred():
                left = deadline - time.monotonic()
                if left <= 0:
                    raise TimeoutError(f"timed out waiting for {what}")
                self.cond.wait(min(left, 0.05))


def _ready(status: Optional[P.TaskStatus]) -> bool:
    """RUNNING with the readiness check's exit code 0 reported (or no check at all)."""
    if status is None or status.state != P.TASK_RUNNING:
        return False
    if not status.HasField("check_status"):
        return True
    cmd = status.check_status.command
    return cmd.HasField("exit_code") and cmd.exit_code == 0


def _get(url: str) -> int:
    try:
        with urllib.request.urlopen(url, timeout=5) as r:
            return r.status
    except urllib.error.HTTPError as e:
        return e.code
    except OSError:
        return 0


def _post(url: str) -> int:
    req = urllib.request.Request(url, data=b"", method="POST")
    try:
        with urllib.request.urlopen(req, timeout=5) as r:
            return r.status
    except urllib.error.HTTPError as e:
        return e.code


class ClusterBench:
    def __init__(self, agents: int = 1, executor: str = "process", probe_cmd: str = DEFAULT_PROBE,
                 allocation_interval_s: float = 1.0, timeout_s: float = 120.0, profile_env: Optional[dict] = None,
                 probe_service: bool = False):
        from dcos_commons_amd.testing.cluster import LocalCluster, use

        self.n = agents
        self.probe_cmd = probe_cmd
        self.timeout_s = timeout_s
        env = {"SDK_LOCK_WAIT_S": "1"}
        env.update(profile_env or {})
        # ZooKeeper in its own process, as on a cluster (the master and agents stay in this one)
        self.cluster = LocalCluster(agents=agents, gpus_per_agent=1, executor=executor, zk_process=True,
                                    allocation_interval_s=allocation_interval_s, scheduler_env=env,
                                    gpu_probe_service=probe_service).start()
        use(self.cluster)
        self.watch = _Watch(self.cluster)
        self._seq = 0

    def close(self) -> None:
        self.cluster.shutdown()

    def _task(self, svc: str, name: str) -> Optional[str]:
        """The current task id of ``name`` (e.g. ``hello-0-server``) of service ``svc``."""
        best = None
        for t in self.cluster.tasks(svc):
            if t.name == name:
                best = t.id
        return best

    def _wait_plan(self, base: str, plan: str) -> float:
        """Polls ``GET /v1/plans/<plan>`` until it answers 200, over one keep-alive connection (a
        new connection per poll would cost the scheduler a connection thread every millisecond,
        taken from the status processing being measured)."""
        deadline = time.monotonic() + self.timeout_s
        u = urllib.parse.urlsplit(base)
        conn = http.client.HTTPConnection(u.hostname, u.port, timeout=5)
        try:
            while time.monotonic() < deadline:
                try:
                    conn.request("GET", f"/v1/plans/{plan}")
                    r = conn.getresponse()
                    r.read()
                    if r.status == 200:
                        return time.perf_counter()
                except (OSError, http.client.HTTPException):
                    conn.close()
                time.sleep(POLL_S)
        finally:
            conn.close()
        raise TimeoutError(f"/v1/plans/{plan} never answered 200")

    def _wait_idle(self, svc: str) -> None:
        """Until the service's scheduler has suppressed offers (gone idle), as a pod that fails
        long after its service deployed finds it (``deploy_bench`` injects failures the same way)."""
        def idle():
            return any(fw.info.name == svc and fw.suppressed for fw in list(self.cluster.master.frameworks.values()))
        deadline = time.monotonic() + self.timeout_s
        while not idle():
            if time.monotonic() > deadline:
                raise TimeoutError(f"{svc} never suppressed offers")
            time.sleep(0.005)

    def _wait_replaced(self, svc: str, old: str) -> None:
        def done():
            tid = self._task(svc, "hello-0-server")
            return tid is not None and tid != old and _ready(self.watch.statuses.get(tid))
        self.watch.wait(done, self.timeout_s, "hello-0 back")

    def run_cycle(self) -> Dict[str, float]:
        from dcos_commons_amd.testing.sdk import sdk_install

        self._seq += 1
        svc = f"hello-bench-{self._seq}"
        opts = {"service": {"yaml": "gpu", "mi355x_probe": {"command": self.probe_cmd}},
                "hello": {"count": self.n, "gpus": 1, "placement": '[["hostname", "UNIQUE"]]'},
                "world": {"count": 0}}
        sdk_install.install(PACKAGE, svc, 0, additional_options=opts, wait_for_deployment=False,
                            wait_for_all_conditions=False)
        self.watch.wait(lambda: svc in self.watch.subscribed, self.timeout_s, f"{svc} SUBSCRIBE")
        t0 = self.watch.subscribed[svc]
        base = self.cluster.marathon.scheduler_url(svc)
        names = [f"hello-{i}-server" for i in range(self.n)]
        self.watch.wait(lambda: all(_ready(self.watch.statuses.get(self._task(svc, n) or "")) for n in names),
                        self.timeout_s, f"{svc} pods ready")
        deploy = self._wait_plan(base, "deploy") - t0
        # failures are injected in steady state: deployed, and the scheduler idle (suppressed)
        self._wait_idle(svc)
        old = self._task(svc, "hello-0-server")
        t1 = time.perf_counter()
        self.cluster.fail_task(old)
        self._wait_replaced(svc, old)
        restart = self._wait_plan(base, "recovery") - t1
        self._wait_idle(svc)
        old = self._task(svc, "hello-0-server")
        t2 = time.perf_counter()
        if _post(f"{base}/v1/pod/hello-0/replace") != 200:
            raise RuntimeError("pod replace was refused")
        self._wait_replaced(svc, old)
        replace = self._wait_plan(base, "recovery") - t2
        sdk_install.uninstall(PACKAGE, svc)
        return {"deploy_s": deploy, "mttr_restart_s": restart, "mttr_replace_s": replace}


# The stand-in cluster runs the master, every agent and the bench in this one interpreter, whose
# threads hand the interpreter lock to each other at most every switch interval while one of them
# is busy. On a cluster they are separate native processes. Same-box A/B
# (profiles/cluster_helper_setup_ab_r05_box.txt): 0.5 ms instead of Python's 5 ms took the 8-pod
# deploy 30.0 -> 27.7 ms (lower in each of the 4 rounds); 1 pod within the spread.
CLUSTER_SWITCH_INTERVAL_MS = 0.5


def readiness_label(probe_cmd: str, probe_service: bool) -> str:
    """What gates a pod's readiness in a row, so a row whose check is a shell ``test`` is never
    read as a GPU-checked one."""
    if probe_service:
        return "GPU readiness: amd-gpu-ready -> node service amd-gpu-probed (HIP MFMA/HBM probe on the pod's GPU)"
    if "amd-gpu-probe" in probe_cmd:
        return "GPU readiness: amd-gpu-probe binary per check (HIP runtime started per check)"
    return "no GPU readiness (the check only tests that HIP_VISIBLE_DEVICES was injected)"


def main(argv: Optional[List[str]] = None) -> int:
    from dcos_commons_amd.benchmarks.deploy_bench import PROFILES

    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--agents", type=int, default=1, help="agents = pods (hostname UNIQUE)")
    ap.add_argument("--cycles", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--executor", choices=["process", "synthetic"], default="process")
    ap.add_argument("--probe-cmd", default=DEFAULT_PROBE, help="the pods' readiness check command")
    ap.add_argument("--profile", choices=sorted(PROFILES), default="mi355x")
    ap.add_argument("--allocation-interval", type=float, default=1.0)
    ap.add_argument("--probe-service", action="store_true",
                    help="run the node's GPU readiness service; the default check becomes amd-gpu-ready")
    ap.add_argument("--scheduler-env", action="append", default=[], metavar="KEY=VALUE",
                    help="extra environment for the scheduler process (repeatable), e.g. for same-box A/Bs")
    ap.add_argument("--cluster-switch-interval-ms", type=float, default=CLUSTER_SWITCH_INTERVAL_MS,
                    help="interpreter switch interval of this process (the master, its agents and the "
                         "bench; on a cluster these are separate native processes); 0: Python's 5 ms")
    args = ap.parse_args(argv)
    if args.cluster_switch_interval_ms > 0:
        import sys

        sys.setswitchinterval(args.cluster_switch_interval_ms / 1000.0)
    if args.probe_service and args.probe_cmd == DEFAULT_PROBE:
        from dcos_commons_amd.ops.probe_service import CLIENT_BINARY

        args.probe_cmd = CLIENT_BINARY
    logging.basicConfig(level=logging.ERROR)
    env = dict(PROFILES[args.profile])
    env.update(kv.split("=", 1) for kv in args.scheduler_env)
    bench = ClusterBench(args.agents, args.executor, args.probe_cmd, args.allocation_interval,
                         profile_env=env, probe_service=args.probe_service)
    served = None
    try:
        for _ in range(args.warmup):
            bench.run_cycle()
        cycles = [bench.run_cycle() for _ in range(args.cycles)]
        if bench.cluster.probe_service is not None:
            served = bench.cluster.probe_service.served()
    finally:
        bench.close()

    def stat(key):
        vals = [c[key] for c in cycles]
        return {"mean": round(statistics.mean(vals), 6), "min": round(min(vals), 6), "max": round(max(vals), 6)}

    print(json.dumps({"bench": "cluster", "agents": args.agents, "pods": args.agents, "cycles": args.cycles,
                      "executor": args.executor, "probe_cmd": args.probe_cmd, "profile": args.profile,
                      "allocation_interval_s": args.allocation_interval, "probe_service": args.probe_service,
                      "scheduler_env": dict(kv.split("=", 1) for kv in args.scheduler_env),
                      "cluster_switch_interval_ms": args.cluster_switch_interval_ms or None,
                      "probe_service_checks": served,
                      "readiness": readiness_label(args.probe_cmd, args.probe_service),
                      "deploy_s": stat("deploy_s"), "mttr_restart_s": stat("mttr_restart_s"),
                      "mttr_replace_s": stat("mttr_replace_s"),
                      "data": "scheduler process + v1 HTTP API + ZooKeeper; helloworld gpu.yml, gpus:1 per pod"}),
          flush=True)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
