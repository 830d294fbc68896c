"""Profile of the LocalMaster ACCEPT handling in cluster mode (ClusterBench, 8 pods, 3 cycles): python scripts/dev/prof_master_accept.py"""
import cProfile, pstats, sys, logging, io
sys.path.insert(0, "/root/repo")
logging.basicConfig(level=logging.ERROR)
from dcos_commons_amd.benchmarks import cluster_bench as CB
from dcos_commons_amd.mesos.local_master import LocalMaster
prof = cProfile.Profile()
orig = LocalMaster._accept
def acc(self, *a, **kw):
    prof.enable()
    try:
        return orig(self, *a, **kw)
    finally:
        prof.disable()
LocalMaster._accept = acc
b = CB.ClusterBench(8)
try:
    for _ in range(3):
        b.run_cycle()
finally:
    b.close()
s = io.StringIO()
pstats.Stats(prof, stream=s).sort_stats(sys.argv[1] if len(sys.argv) > 1 else "cumulative").print_stats(40)
print(s.getvalue()[:7000])
