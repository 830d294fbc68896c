"""Microbenchmark of task-status handling (``AbstractScheduler.task_status``) during a helloworld
``gpu.yml`` deploy: N pods are launched from one offer pass, then each task's STARTING, RUNNING and
RUNNING-with-readiness-passed updates are fed in; reports CPU time per status update.

    python scripts/status_bench.py --pods 8 --reps 30 [--profile]
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
from dcos_commons_amd.offer.taskdata import labels as L  # noqa: E402
from dcos_commons_amd.scheduler.scheduler_builder import SchedulerBuilder  # noqa: E402
from dcos_commons_amd.scheduler.scheduler_config import SchedulerConfig  # noqa: E402
from dcos_commons_amd.specification.yaml.mappers import ServiceSpecGenerator  # noqa: E402
from dcos_commons_amd.specification.yaml.raw import RawServiceSpec  # noqa: E402
from dcos_commons_amd.storage.mem_persister import MemPersister  # noqa: E402
from dcos_commons_amd.testing.harness import RecordingDriver  # noqa: E402

from offer_eval_bench import offers  # noqa: E402


def launched_scheduler(n):
    env = helloworld_env(n, 1, "true")
    cfg = SchedulerConfig.for_testing(PORT_API="0")
    raw = RawServiceSpec.new_builder(os.path.join(SPECS, "gpu.yml")).set_env(env).build()
    spec = ServiceSpecGenerator(raw, cfg, SPECS, env).build()
    sched = SchedulerBuilder(spec, cfg, MemPersister()).set_plans_from(raw).build()
    driver.set_driver(RecordingDriver())
    sched.framework_store.store_framework_id(P.FrameworkID(value="fw-1"))
    sched.registered(False)
    sched.get_client_status()
    sched.offers(offers(n))
    return sched


def statuses(sched):
    out = []
    for stage in ("STARTING", "RUNNING", "READY"):
        for info in sched.state_store.fetch_tasks():
            s = P.TaskStatus(state=P.TASK_STARTING if stage == "STARTING" else P.TASK_RUNNING)
            s.task_id.CopyFrom(info.task_id)
            if stage == "READY":
                s.labels.labels.add(key=L.READINESS_CHECK_PASSED_LABEL, value="true")
            out.append(s)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pods", type=int, default=8)
    ap.add_argument("--reps", type=int, default=30)
    ap.add_argument("--profile", action="store_true")
    ap.add_argument("--sort", default="tottime")
    a = ap.parse_args()
    prof = cProfile.Profile() if a.profile else None
    best, total, count = float("inf"), 0.0, 0
    for _ in range(a.reps):
        sched = launched_scheduler(a.pods)
        sts = statuses(sched)
        if prof:
            prof.enable()
        t0 = time.process_time()
        for s in sts:
            sched.task_status(s)
        dt = time.process_time() - t0
        if prof:
            prof.disable()
        assert sched.plan_coordinator.get_plan_managers()[0].get_plan().is_complete()
        best, total, count = min(best, dt / len(sts)), total + dt, count + len(sts)
    print(f"{best * 1e6:.1f} us per status update (best rep; mean {total / count * 1e6:.1f} us, "
          f"{a.pods} pods x 3 updates x {a.reps} reps)")
    if prof:
        pstats.Stats(prof).sort_stats(a.sort).print_stats(35)


if __name__ == "__main__":
    main()
