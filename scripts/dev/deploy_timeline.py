"""Per-span timeline of one traced deploy (SDK_TRACE=1): python scripts/dev/deploy_timeline.py N [--gpu|--fake-probe] [--restart] [-v]."""
import os, sys, time, collections
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from dcos_commons_amd import trace
from dcos_commons_amd.benchmarks.deploy_bench import DeployBench
n = int(sys.argv[1]) if len(sys.argv) > 1 else 8
import dcos_commons_amd.benchmarks.deploy_bench as DB
_orig = DB.SchedulerRunner.run
def _run(self, *a, **k):
    trace.TRACER.instant("deploy_start")
    return _orig(self, *a, **k)
DB.SchedulerRunner.run = _run
import dcos_commons_amd.mesos.local_master as LM
_orig_fail = LM.LocalMaster.fail_task
def _fail(self, *a, **k):
    trace.TRACER.instant("restart_start")
    return _orig_fail(self, *a, **k)
LM.LocalMaster.fail_task = _fail
gpu = '--gpu' in sys.argv
if gpu:
    from dcos_commons_amd.benchmarks.runner import gpu_check_runner
    b = DeployBench(n, check_runner=gpu_check_runner(), gpu_devices=[0]*n)
elif '--fake-probe' in sys.argv:   # a 0.2 ms GIL-releasing check, the fused probe's cost
    b = DeployBench(n, check_runner=lambda t, d: (time.sleep(0.0002), True)[1], gpu_devices=[0] * n)
else:
    b = DeployBench(n)
for _ in range(3): b.run_cycle()
trace.TRACER.clear()
t0 = (time.perf_counter_ns() - trace.TRACER._epoch_ns) / 1e3
r = b.run_cycle()
print("deploy ms %.2f  restart ms %.2f" % (r.deploy_s * 1000, r.mttr_restart_s * 1000))
ev = sorted(trace.TRACER.events(), key=lambda e: e['ts'])
restart = '--restart' in sys.argv
t0 = [e['ts'] for e in ev if e['name'] == ('restart_start' if restart else 'deploy_start')][0]
tids = {}
end = (r.mttr_restart_s if '--restart' in sys.argv else r.deploy_s) * 1e6 + 500
for e in ev:
    rel = e['ts'] - t0
    if rel < 0: continue
    if rel > end: break
    tid = tids.setdefault(e['tid'], len(tids))
    if e['cat'] == 'persister' and '-v' not in sys.argv: continue
    a = e.get('args', {})
    a = {k: (v.split('__')[1] if isinstance(v, str) and '__' in v else v) for k, v in a.items()}
    print(f"{rel/1000:7.2f} +{e.get('dur',0)/1000:6.2f} t{tid} {e['name']:14s} {a}")
agg = collections.defaultdict(lambda: [0, 0.0])
for e in ev:
    if e['ts'] - t0 > end or e['ts'] < t0: continue
    x = agg[e['name']]; x[0] += 1; x[1] += e.get('dur', 0) / 1000
for k, v in sorted(agg.items(), key=lambda kv: -kv[1][1]): print(f"  {k:28s} {v[0]:4d} {v[1]:7.2f} ms")
