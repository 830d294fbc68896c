"""Per-span timeline of one traced deploy in the split topology (master process, one agent process
per pod, scheduler here over the framed stream): python scripts/dev/split_timeline.py N [--probe].

Prints the scheduler process's spans (offer cycle, evaluations, accepts, status batches) relative
to the deploy's start, each with its thread's CPU time, and the scheduler threads' CPU shares."""
import argparse
import collections
import os
import subprocess
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
os.environ.setdefault("SDK_TRACE", "1")
import logging  # noqa: E402

logging.disable(logging.WARNING)
from dcos_commons_amd import trace  # noqa: E402
from dcos_commons_amd.mesos import master_process as MP  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("n", type=int)
ap.add_argument("--probe", action="store_true")
ap.add_argument("--cycles", type=int, default=5)
ap.add_argument("--agent0", choices=["process", "thread"], default="process",
                help="agent 0 in a process of its own, or on a thread of the scheduler's process (as bench.py's "
                     "default)")
ap.add_argument("--spans", default="",
                help="comma-separated module:Qual.name callables to trace as spans (e.g. "
                     "dcos_commons_amd.http.server:ApiServer.start)")
args = ap.parse_args()


def _wrap_spans(spec: str) -> None:
    import functools
    import importlib

    for item in filter(None, spec.split(",")):
        mod_name, qual = item.split(":")
        owner = importlib.import_module(mod_name)
        parts = qual.split(".")
        for p in parts[:-1]:
            owner = getattr(owner, p)
        raw = owner.__dict__.get(parts[-1]) if isinstance(owner, type) else getattr(owner, parts[-1])
        fn = raw.__func__ if isinstance(raw, (staticmethod, classmethod)) else raw

        def make(fn=fn, name=parts[-1] if parts[-1] != "__init__" else parts[-2]):
            @functools.wraps(fn)
            def w(*a, **k):
                with trace.span(name, "dev"):
                    return fn(*a, **k)
            return w
        w = make()
        setattr(owner, parts[-1], type(raw)(w) if isinstance(raw, (staticmethod, classmethod)) else w)

proc, ports = MP.spawn()
client = MP.MasterClient("127.0.0.1", ports["control"])
root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
first = 1 if args.agent0 == "thread" else 0
kids = [subprocess.Popen([sys.executable, "-m", "dcos_commons_amd.parallel.agent_process", "--port",
                          str(ports["agents"]), "--rank", str(i), "--device", "0", "--probe",
                          "on" if args.probe else "off"], cwd=root) for i in range(first, args.n)]
if first:
    from dcos_commons_amd.benchmarks.runner import _local_agent_info, _start_agent_thread  # noqa: E402
    from dcos_commons_amd.parallel.agent_process import check_for  # noqa: E402

    _start_agent_thread("127.0.0.1", ports["agents"], _local_agent_info(0, 0, 0), check_for(0, args.probe))
client.call("agents", n=args.n)

cpu = collections.defaultdict(float)
lock = threading.Lock()
orig_run = threading.Thread.run


def run(self, *a, **k):
    t0 = time.thread_time()
    try:
        return orig_run(self, *a, **k)
    finally:
        with lock:
            cpu[self.name.split("-")[0] if self.name.startswith("Thread") else self.name] += time.thread_time() - t0


threading.Thread.run = run
import dcos_commons_amd.benchmarks.deploy_bench as DB  # noqa: E402

_orig = DB.SchedulerRunner.run


def _run(self, *a, **k):
    trace.TRACER.instant("deploy_start")
    return _orig(self, *a, **k)


DB.SchedulerRunner.run = _run
_wrap_spans(args.spans)
b = DB.DeployBench(args.n, master_client=client)
for _ in range(3):
    b.run_cycle()
deploys = []
for _ in range(args.cycles):
    deploys.append(b.run_cycle().deploy_s)
trace.TRACER.clear()
r = b.run_cycle()
time.sleep(0.3)
print("deploy ms: traced %.2f; untraced-loop mean %.2f" % (r.deploy_s * 1e3, sum(deploys) / len(deploys) * 1e3))
ev = sorted(trace.TRACER.events(), key=lambda e: e["ts"])
t0 = [e["ts"] for e in ev if e["name"] == "deploy_start"][0]
end = r.deploy_s * 1e6 + 300
tids, agg, cnt = {}, collections.defaultdict(float), collections.Counter()
for e in ev:
    rel = e["ts"] - t0
    if rel < 0 or rel > end:
        continue
    tid = tids.setdefault(e.get("tid"), len(tids))
    d = e.get("dur", 0)
    agg[e["name"]] += d
    cnt[e["name"]] += 1
    a = {k: v for k, v in (e.get("args") or {}).items() if k != "task"}
    print("%7.2f +%6.2f t%d %-14s %s" % (rel / 1e3, d / 1e3, tid, e["name"], a))
for k in agg:
    print("  %-16s %3d %8.2f ms" % (k, cnt[k], agg[k] / 1e3))
client.call("shutdown")
proc.wait(10)
for k in kids:
    k.wait(10)
