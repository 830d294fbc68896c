"""python scripts/dev/cluster_timeline.py [pods] [cycles]: master-side timeline of cluster-mode deploys
(ClusterBench: scheduler process over the v1 HTTP API, ZooKeeper process, real task processes).

Wraps the LocalMaster entry points the scheduler process drives (subscribe, offers sent, ACCEPTs,
launches, status updates, check results, acknowledgements) and prints, for the last cycle, each
event's offset from SUBSCRIBE in ms. The deploy window ends where /v1/plans/deploy answers 200.
"""
import json
import logging
import sys
import urllib.request
import threading
import time

from dcos_commons_amd.benchmarks import cluster_bench as CB
from dcos_commons_amd.mesos import protos as P
from dcos_commons_amd.mesos.local_master import LocalMaster

pods = int(sys.argv[1]) if len(sys.argv) > 1 else 8
cycles = int(sys.argv[2]) if len(sys.argv) > 2 else 2
logging.basicConfig(level=logging.ERROR)
sys.setswitchinterval(CB.CLUSTER_SWITCH_INTERVAL_MS / 1000.0)    # as cluster_bench runs
events = []
lock = threading.Lock()


def mark(what, t=None):
    with lock:
        events.append((time.perf_counter() if t is None else t, what))


def wrap(name, label):
    orig = getattr(LocalMaster, name)

    def f(self, *a, **kw):
        t0, c0 = time.perf_counter(), time.thread_time()
        try:
            return orig(self, *a, **kw)
        finally:
            what = label(*a) if callable(label) else label
            mark(f"{what} ({(time.perf_counter() - t0) * 1e3:.2f} ms, cpu {(time.thread_time() - c0) * 1e3:.2f} ms)",
                 t0)
    setattr(LocalMaster, name, f)


wrap("_accept", lambda fid, oids, ops, refuse: f"accept {len(oids)} offer(s) {len(ops)} op(s)")
wrap("_decline", lambda fid, oids, refuse: f"decline {len(oids)}")
wrap("_allocate", "allocate")
wrap("_revive" if hasattr(LocalMaster, "_revive") else "revive", "revive")
wrap("_check_result", lambda task, epoch, ok: f"check {task.info.name} ok={ok}")
orig_update = LocalMaster._update


def update(self, task, state, deliver=True, **kw):
    mark(f"status {task.info.name} {P.TaskState.Name(state)}")
    return orig_update(self, task, state, deliver, **kw)


LocalMaster._update = update

bench = CB.ClusterBench(pods, profile_env={"SDK_TRACE": "1"})
sched_trace = {}
from dcos_commons_amd.testing.sdk import sdk_install  # noqa: E402

_uninstall = sdk_install.uninstall


def uninstall(pkg, svc, *a, **kw):
    """Read the scheduler's spans (its own process) before it goes away."""
    url = bench.cluster.marathon.scheduler_url(svc) + "/v1/debug/trace?clear=true"
    with urllib.request.urlopen(url, timeout=5) as r:
        sched_trace.clear()
        sched_trace.update(json.loads(r.read()))
    return _uninstall(pkg, svc, *a, **kw)


sdk_install.uninstall = uninstall
try:
    for _ in range(cycles):
        with lock:
            events.clear()
        t_end = None
        orig_wait = bench._wait_plan

        def wait_plan(base, plan, _o=orig_wait):
            t = _o(base, plan)
            if plan == "deploy":
                mark("GET /v1/plans/deploy -> 200")
            return t
        bench._wait_plan = wait_plan
        r = bench.run_cycle()
        bench._wait_plan = orig_wait
    svc = f"hello-bench-{bench._seq}"
    t0 = bench.watch.subscribed[svc]
    print(f"# {pods} pods, deploy {r['deploy_s'] * 1000:.1f} ms")
    epoch = sched_trace["otherData"]["epoch_monotonic_ns"] / 1e9
    names = {ev["tid"]: ev["args"]["name"] for ev in sched_trace["traceEvents"] if ev.get("ph") == "M"}
    for ev in sched_trace["traceEvents"]:
        if ev.get("ph") != "X" or ev["cat"] == "persister" and ev["dur"] < 200:
            continue
        t = epoch + ev["ts"] / 1e6
        args = ",".join(f"{k}={v}" for k, v in (ev.get("args") or {}).items())
        events.append((t, f"    [sched {names.get(ev['tid'], ev['tid'])}] {ev['name']} {ev['dur'] / 1e3:.2f} ms {args}"))
    for t, what in sorted(events):
        if t < t0 - 0.001:
            continue
        print(f"{(t - t0) * 1000:8.2f}  {what}")
        if what.startswith("GET /v1/plans/deploy"):
            break
finally:
    bench.close()
