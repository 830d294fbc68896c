"""Single-thread microbenchmark of the offer-evaluation hot path: one
``get_client_status`` + ``offers`` pass of the helloworld ``gpu.yml`` scheduler over N fresh
agents' offers, N pods deployed in parallel. Prints ms per pass and per pod; ``--profile`` adds a
cProfile table of the pass.

    python scripts/offer_eval_bench.py --pods 8 --reps 50 [--profile]
"""
import argparse
import cProfile
import io
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from dcos_commons_amd.benchmarks.deploy_bench import SPECS, helloworld_env  # noqa: E402
from dcos_commons_amd.framework import driver  # noqa: E402
from dcos_commons_amd.mesos import protos as P  # noqa: E402
from dcos_commons_amd.mesos.local_master import AgentSpec  # noqa: E402
from dcos_commons_amd.scheduler.scheduler_builder import SchedulerBuilder  # noqa: E402
from dcos_commons_amd.scheduler.scheduler_config import SchedulerConfig  # noqa: E402
from dcos_commons_amd.specification.yaml.mappers import ServiceSpecGenerator  # noqa: E402
from dcos_commons_amd.specification.yaml.raw import RawServiceSpec  # noqa: E402
from dcos_commons_amd.storage.mem_persister import MemPersister  # noqa: E402
from dcos_commons_amd.testing.harness import RecordingDriver  # noqa: E402


def offers(n):
    out = []
    for i in range(n):
        spec = AgentSpec(hostname=f"agent-{i}", cpus=16, mem=65536, disk=100000, gpus=1)
        o = P.Offer(hostname=spec.hostname)
        o.id.value, o.agent_id.value, o.framework_id.value = f"offer-{i}", f"agent-{i}", "fw-1"
        for r in spec.resources():
            r.allocation_info.role = "hello-world-role"
            o.resources.add().CopyFrom(r)
        out.append(o)
    return out


def one_pass(n, prof=None):
    env = helloworld_env(n, 1, "true")
    cfg = SchedulerConfig.for_testing(PORT_API="0")
    raw = RawServiceSpec.new_builder(os.path.join(SPECS, "gpu.yml")).set_env(env).build()
    spec = ServiceSpecGenerator(raw, cfg, SPECS, env).build()
    persister = MemPersister()
    sched = SchedulerBuilder(spec, cfg, persister).set_plans_from(raw).build()
    driver.set_driver(RecordingDriver())
    sched.framework_store.store_framework_id(P.FrameworkID(value="fw-1"))
    sched.registered(False)
    os_ = offers(n)
    if prof:
        prof.enable()
    t0 = time.perf_counter()
    sched.get_client_status()
    resp = sched.offers(os_)
    dt = time.perf_counter() - t0
    if prof:
        prof.disable()
    launched = sum(1 for r in resp.recommendations if type(r).__name__ == "LaunchOfferRecommendation")
    assert launched == n, (launched, n)
    return dt


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pods", type=int, default=8)
    ap.add_argument("--reps", type=int, default=30)
    ap.add_argument("--profile", action="store_true")
    ap.add_argument("--sort", default="tottime", help="cProfile sort key (tottime, cumulative)")
    a = ap.parse_args()
    one_pass(a.pods)
    prof = cProfile.Profile() if a.profile else None
    ts = []
    for _ in range(a.reps):
        ts.append(one_pass(a.pods, prof))
    ts.sort()
    med = ts[len(ts) // 2] * 1000
    print(f"pods={a.pods} median pass {med:.2f} ms, {med / a.pods:.3f} ms/pod (min {ts[0] * 1000:.2f})")
    if prof:
        out = io.StringIO()
        pstats.Stats(prof, stream=out).sort_stats(a.sort).print_stats(40)
        print(out.getvalue())


if __name__ == "__main__":
    main()
