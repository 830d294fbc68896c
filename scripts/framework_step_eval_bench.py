"""Microbenchmark of one cassandra/hdfs step's offer evaluation (``OfferEvaluator.evaluate`` for the
first deploy step against fresh agent offers), on the reference's unchanged package or this repo's.

    python scripts/framework_step_eval_bench.py hdfs [--specs reference|repo] [--reps 200] [--profile]
"""
import argparse
import cProfile
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from dcos_commons_amd.benchmarks import framework_bench as FB  # noqa: E402
from dcos_commons_amd.framework import driver  # noqa: E402
from dcos_commons_amd.mesos import protos as P  # noqa: E402
from dcos_commons_amd.mesos.local_master import AgentSpec  # noqa: E402
from dcos_commons_amd.scheduler.scheduler_config import SchedulerConfig  # noqa: E402
from dcos_commons_amd.storage.mem_persister import MemPersister  # noqa: E402
from dcos_commons_amd.testing.harness import RecordingDriver  # noqa: E402


def offers(n, role):
    out = []
    for i in range(n):
        spec = AgentSpec(hostname=f"agent-{i}", cpus=32, mem=262144, disk=2_000_000, ports=((1025, 32000),))
        o = P.Offer(hostname=spec.hostname)
        o.id.value, o.agent_id.value, o.framework_id.value = f"offer-{i}", f"agent-{i}", "fw-1"
        for r in spec.resources():
            r.allocation_info.role = role
            o.resources.add().CopyFrom(r)
        out.append(o)
    return out


def setup(framework, specs):
    root = FB.framework_root(framework, specs)
    env = FB._scheduler_env(root)
    cfg = SchedulerConfig.for_testing(PORT_API="0")
    if framework == "cassandra":
        from dcos_commons_amd.models import cassandra as m
    else:
        from dcos_commons_amd.models import hdfs as m
    t0 = time.perf_counter()
    sched = m.create_scheduler_builder(FB.spec_path(root), cfg, env, MemPersister()).build()
    build_ms = (time.perf_counter() - t0) * 1e3
    driver.set_driver(RecordingDriver())
    sched.framework_store.store_framework_id(P.FrameworkID(value="fw-1"))
    sched.registered(False)
    step = sched.plan_coordinator.get_candidates()[0]
    req = step.get_pod_instance_requirement()
    return sched.plan_scheduler.offer_evaluator, req, build_ms, sched.service_spec.role


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("framework", choices=["cassandra", "hdfs"])
    ap.add_argument("--specs", choices=["reference", "repo"], default="reference")
    ap.add_argument("--reps", type=int, default=200)
    ap.add_argument("--offers", type=int, default=4)
    ap.add_argument("--profile", action="store_true")
    ap.add_argument("--sort", default="tottime")
    ap.add_argument("--cold", action="store_true", help="drop the evaluator's PodInfoBuilder templates before "
                                                         "each rep (a deploy evaluates every pod instance cold)")
    args = ap.parse_args()
    ev, req, build_ms, role = setup(args.framework, args.specs)
    os_ = offers(args.offers, role)
    for _ in range(20):
        ev.evaluate(req, os_)
    prof = cProfile.Profile() if args.profile else None
    if prof:
        prof.enable()
    t0 = time.perf_counter()
    for _ in range(args.reps):
        if args.cold:
            ev._templates.clear()
        recs = ev.evaluate(req, os_)
    dt = (time.perf_counter() - t0) / args.reps * 1e3
    if prof:
        prof.disable()
    print(f"{args.framework} {args.specs}{' cold' if args.cold else ''}: step {req.pod_instance.name}:{list(req.tasks_to_launch)} "
          f"evaluate {dt:.3f} ms ({len(recs)} recs, {args.offers} offers); scheduler build {build_ms:.1f} ms")
    if prof:
        pstats.Stats(prof).sort_stats(args.sort).print_stats(35)


if __name__ == "__main__":
    main()
