"""cProfile of every thread during one framework bench phase (the hdfs rolling update, or the
cassandra replace): python scripts/dev/prof_framework.py hdfs|cassandra [reference|repo] [N].
PROF_WHOLE_CYCLE=1 profiles the whole cycle instead (deploy included), with the LocalMaster's threads;
PROF_OUT=<file> dumps the merged stats.

The profilers start when the phase's scheduler starts (hdfs: the second ``_start`` of a cycle),
including in threads started afterwards, and their stats are merged; the top N functions by
cumulative and by own time are printed."""
import cProfile
import os
import pstats
import sys
import threading

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import dcos_commons_amd.benchmarks.framework_bench as FB  # noqa: E402

fw = sys.argv[1] if len(sys.argv) > 1 else "hdfs"
specs = sys.argv[2] if len(sys.argv) > 2 else "reference"
top = int(sys.argv[3]) if len(sys.argv) > 3 else 40
profiles = []
state = {"on": False, "starts": 0}


def _thread_hook(*_):
    if not state["on"]:
        return
    p = cProfile.Profile()
    profiles.append(p)
    p.enable()


_orig = FB.FrameworkBench._start


def _start(self, *a, **k):
    state["starts"] += 1
    if state["arm"] and state["starts"] == (2 if fw == "hdfs" else 1) and not state["on"]:
        state["on"] = True
        threading.setprofile(_thread_hook)
        p = cProfile.Profile()
        profiles.append(p)
        p.enable()
    return _orig(self, *a, **k)


FB.FrameworkBench._start = _start
b = FB.FrameworkBench(fw, spec_set=specs)
state["arm"] = False
for _ in range(2):
    b.run_cycle()
state.update(arm=True, starts=0)
if os.environ.get("PROF_WHOLE_CYCLE"):     # also the master's and agents' threads, from the cycle's start
    state["on"] = True
    threading.setprofile(_thread_hook)
    _p = cProfile.Profile()
    profiles.append(_p)
    _p.enable()
r = b.run_cycle()
state["on"] = False
threading.setprofile(None)
for p in profiles:
    p.disable()
print(r.as_dict())
stats = None
for p in profiles:
    try:
        stats = pstats.Stats(p) if stats is None else stats.add(p)
    except TypeError:       # a profiler that never recorded anything
        pass
if os.environ.get("PROF_OUT"):
    stats.dump_stats(os.environ["PROF_OUT"])
stats.sort_stats("cumulative").print_stats(top)
stats.sort_stats("tottime").print_stats(top)
