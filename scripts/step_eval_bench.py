"""Microbenchmark of ONE step's offer evaluation (``OfferEvaluator.evaluate`` for a helloworld
``gpu.yml`` pod against one fresh agent offer), the per-pod unit of a deploy's offer cycle.

    python scripts/step_eval_bench.py --reps 2000 [--profile] [--sort tottime]
"""
import argparse
import cProfile
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from dcos_commons_amd.benchmarks.deploy_bench import SPECS, helloworld_env  # noqa: E402
from dcos_commons_amd.framework import driver  # noqa: E402
from dcos_commons_amd.mesos import protos as P  # noqa: E402
from dcos_commons_amd.scheduler.scheduler_builder import SchedulerBuilder  # noqa: E402
from dcos_commons_amd.scheduler.scheduler_config import SchedulerConfig  # noqa: E402
from dcos_commons_amd.specification.yaml.mappers import ServiceSpecGenerator  # noqa: E402
from dcos_commons_amd.specification.yaml.raw import RawServiceSpec  # noqa: E402
from dcos_commons_amd.storage.mem_persister import MemPersister  # noqa: E402
from dcos_commons_amd.testing.harness import RecordingDriver  # noqa: E402

from offer_eval_bench import offers  # noqa: E402


def setup():
    env = helloworld_env(1, 1, "true")
    cfg = SchedulerConfig.for_testing(PORT_API="0")
    raw = RawServiceSpec.new_builder(os.path.join(SPECS, "gpu.yml")).set_env(env).build()
    spec = ServiceSpecGenerator(raw, cfg, SPECS, env).build()
    sched = SchedulerBuilder(spec, cfg, MemPersister()).set_plans_from(raw).build()
    driver.set_driver(RecordingDriver())
    sched.framework_store.store_framework_id(P.FrameworkID(value="fw-1"))
    sched.registered(False)
    step = sched.plan_coordinator.get_candidates()[0]
    req = step.get_pod_instance_requirement()
    evaluator = sched.plan_scheduler.offer_evaluator
    return evaluator, req, offers(1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=2000)
    ap.add_argument("--profile", action="store_true")
    ap.add_argument("--sort", default="tottime")
    ap.add_argument("--cold", action="store_true", help="drop the evaluator's PodInfoBuilder templates before "
                                                         "each evaluation (a deploy evaluates each pod index once)")
    a = ap.parse_args()
    evaluator, req, os_ = setup()
    assert evaluator.evaluate(req, os_)
    for _ in range(200):
        evaluator.evaluate(req, os_)
    prof = cProfile.Profile() if a.profile else None
    if prof:
        prof.enable()
    chunk = max(1, a.reps // 20)
    best, total, done = float("inf"), 0.0, 0
    while done < a.reps:
        t0 = time.process_time()  # CPU time of this (single-threaded) loop: steadier than wall time
        for _ in range(chunk):
            if a.cold:
                evaluator._templates.clear()
            evaluator.evaluate(req, os_)
        dt = time.process_time() - t0
        best, total, done = min(best, dt / chunk), total + dt, done + chunk
    if prof:
        prof.disable()
    # the minimum over chunks is the stable figure on a shared machine; the mean is reported too
    print(f"{best * 1e6:.1f} us per step evaluation (best chunk of {chunk}; mean {total / done * 1e6:.1f} us, "
          f"{done} reps)")
    if prof:
        pstats.Stats(prof).sort_stats(a.sort).print_stats(35)


if __name__ == "__main__":
    main()
