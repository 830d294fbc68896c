"""cProfile of the scheduler side of an N-pod split-topology deploy (master process, one agent
process per pod): python scripts/dev/prof_split_cycle.py N [--cycles C] [--sort tottime].

Profiles the offer-loop cycles and the status callbacks (each on its own thread, merged)."""
import argparse
import cProfile
import logging
import os
import pstats
import subprocess
import sys
import threading

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
logging.disable(logging.WARNING)
from dcos_commons_amd.framework import framework_scheduler as FS  # noqa: E402
from dcos_commons_amd.framework import offer_processing as OP  # noqa: E402
from dcos_commons_amd.mesos import master_process as MP  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("n", type=int)
ap.add_argument("--cycles", type=int, default=30)
ap.add_argument("--sort", default="tottime")
ap.add_argument("--limit", type=int, default=45)
ap.add_argument("--callers", default="", help="also print the callers of functions matching this pattern")
args = ap.parse_args()

proc, ports = MP.spawn()
client = MP.MasterClient("127.0.0.1", ports["control"])
root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
kids = [subprocess.Popen([sys.executable, "-m", "dcos_commons_amd.parallel.agent_process", "--port",
                          str(ports["agents"]), "--rank", str(i), "--device", "0", "--probe", "off"], cwd=root)
        for i in range(args.n)]
client.call("agents", n=args.n)

profiles = []
on = threading.Event()
local = threading.local()


def wrap(fn):
    def inner(*a, **k):
        if not on.is_set():
            return fn(*a, **k)
        p = getattr(local, "p", None)
        if p is None:
            p = local.p = cProfile.Profile()
            profiles.append(p)
        p.enable()
        try:
            return fn(*a, **k)
        finally:
            p.disable()
    return inner


OP.OfferProcessor.process_queued_offers = wrap(OP.OfferProcessor.process_queued_offers)
for name in ("status_update", "status_updates"):
    if hasattr(FS.FrameworkScheduler, name):
        setattr(FS.FrameworkScheduler, name, wrap(getattr(FS.FrameworkScheduler, name)))
import dcos_commons_amd.benchmarks.deploy_bench as DB  # noqa: E402

b = DB.DeployBench(args.n, master_client=client)
for _ in range(3):
    b.run_cycle()
on.set()
ds = [b.run_cycle().deploy_s for _ in range(args.cycles)]
on.clear()
print("deploy ms mean %.2f (profiled)" % (sum(ds) / len(ds) * 1e3))
st = pstats.Stats(profiles[0])
for p in profiles[1:]:
    st.add(p)
st.sort_stats(args.sort).print_stats(args.limit)
if args.callers:
    st.print_callers(args.callers)
client.call("shutdown")
proc.wait(10)
for k in kids:
    k.wait(10)
