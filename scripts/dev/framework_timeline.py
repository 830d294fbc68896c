"""Per-span timeline of one traced framework deploy (SDK_TRACE=1):
python scripts/dev/framework_timeline.py cassandra|hdfs [reference|repo] [-v]."""
import collections
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from dcos_commons_amd import trace  # noqa: E402
import dcos_commons_amd.benchmarks.framework_bench as FB  # noqa: E402

fw = sys.argv[1] if len(sys.argv) > 1 else "hdfs"
specs = sys.argv[2] if len(sys.argv) > 2 and not sys.argv[2].startswith("-") else "reference"
_orig = FB.FrameworkBench._start


def _start(self, *a, **k):
    trace.TRACER.instant("scheduler_start")
    return _orig(self, *a, **k)


FB.FrameworkBench._start = _start
b = FB.FrameworkBench(fw, spec_set=specs)
for _ in range(2):
    b.run_cycle()
trace.TRACER.clear()
r = b.run_cycle()
print(r.as_dict())
ev = sorted(trace.TRACER.events(), key=lambda e: e["ts"])
t0 = [e["ts"] for e in ev if e["name"] == "scheduler_start"][0]
end = t0 + r.deploy_s * 1e6 + 500
tids = {}
for e in ev:
    if e["ts"] < t0 or e["ts"] > end:
        continue
    tid = tids.setdefault(e["tid"], len(tids))
    if e["cat"] == "persister" and "-v" not in sys.argv:
        continue
    a = {k: (v.split("__")[1] if isinstance(v, str) and "__" in v else v) for k, v in e.get("args", {}).items()}
    print(f"{(e['ts'] - t0) / 1000:8.2f} +{e.get('dur', 0) / 1000:6.2f} t{tid} {e['name']:14s} {a}")
agg = collections.defaultdict(lambda: [0, 0.0])
for e in ev:
    if t0 <= e["ts"] <= end:
        x = agg[e["name"]]
        x[0] += 1
        x[1] += e.get("dur", 0) / 1000
for k, v in sorted(agg.items(), key=lambda kv: -kv[1][1]):
    print(f"  {k:28s} {v[0]:4d} {v[1]:7.2f} ms")
