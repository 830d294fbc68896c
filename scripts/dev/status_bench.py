"""Microbenchmark of the scheduler's status path: a helloworld gpu.yml scheduler launches N pods
(offer pass + write-ahead record, as a deploy does), then handles their STARTING, RUNNING and
readiness updates in one batch (``FrameworkScheduler.status_updates`` -> ``process_status_updates``).
Prints us per status; ``--profile`` adds a cProfile table of the batches.

    python scripts/dev/status_bench.py --pods 8 --reps 100 [--profile]
"""
import argparse
import cProfile
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from offer_eval_bench import offers  # noqa: E402

from dcos_commons_amd.benchmarks.deploy_bench import SPECS, helloworld_env  # noqa: E402
from dcos_commons_amd.framework import driver  # noqa: E402
from dcos_commons_amd.framework.framework_scheduler import FrameworkScheduler  # noqa: E402
from dcos_commons_amd.mesos import protos as P  # noqa: E402
from dcos_commons_amd.offer.recommendations import LaunchOfferRecommendation  # noqa: E402
from dcos_commons_amd.scheduler.scheduler_builder import SchedulerBuilder  # noqa: E402
from dcos_commons_amd.scheduler.scheduler_config import SchedulerConfig  # noqa: E402
from dcos_commons_amd.specification.yaml.mappers import ServiceSpecGenerator  # noqa: E402
from dcos_commons_amd.specification.yaml.raw import RawServiceSpec  # noqa: E402
from dcos_commons_amd.storage.mem_persister import MemPersister  # noqa: E402
from dcos_commons_amd.testing.harness import RecordingDriver  # noqa: E402


def statuses_for(recs):
    out = []
    for r in recs:
        if not isinstance(r, LaunchOfferRecommendation):
            continue
        t = r.task_info
        for state, ready in ((P.TASK_STARTING, False), (P.TASK_RUNNING, False), (P.TASK_RUNNING, True)):
            st = P.TaskStatus(state=state, source=P.TaskStatus.SOURCE_EXECUTOR, uuid=os.urandom(16))
            st.task_id.CopyFrom(t.task_id)
            st.agent_id.CopyFrom(r.offer.agent_id)
            if state == P.TASK_RUNNING and t.HasField("check"):
                st.check_status.type = t.check.type
                st.check_status.command.SetInParent()
                if ready:
                    st.check_status.command.exit_code = 0
            out.append(st)
    # the order an agent reports them: every pod's STARTING, RUNNING, then readiness
    return sorted(out, key=lambda s: (s.state, s.check_status.command.HasField("exit_code")))


def one(n, prof=None):
    env = helloworld_env(n, 1, "true")
    cfg = SchedulerConfig.for_testing(PORT_API="0")
    raw = RawServiceSpec.new_builder(os.path.join(SPECS, "gpu.yml")).set_env(env).build()
    spec = ServiceSpecGenerator(raw, cfg, SPECS, env).build()
    persister = MemPersister()
    sched = SchedulerBuilder(spec, cfg, persister).set_plans_from(raw).build()
    driver.set_driver(RecordingDriver())
    sched.framework_store.store_framework_id(P.FrameworkID(value="fw-1"))
    sched.registered(False)
    sched.get_client_status()
    resp = sched.offers(offers(n))
    fs = FrameworkScheduler([], cfg, persister, sched.framework_store, sched)
    sts = statuses_for(resp.recommendations)
    if prof:
        prof.enable()
    t0 = time.perf_counter()
    fs.status_updates(None, sts)
    dt = time.perf_counter() - t0
    if prof:
        prof.disable()
    assert sched.get_plan("deploy").is_complete(), "the batch did not complete the deploy"
    return dt, len(sts)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pods", type=int, default=8)
    ap.add_argument("--reps", type=int, default=100)
    ap.add_argument("--profile", action="store_true")
    a = ap.parse_args()
    prof = cProfile.Profile() if a.profile else None
    for _ in range(5):
        one(a.pods)
    per = sorted(dt / n for dt, n in (one(a.pods, prof) for _ in range(a.reps)))
    print(f"pods={a.pods}: median {per[len(per) // 2] * 1e6:.1f} us per status (min {per[0] * 1e6:.1f})")
    if prof:
        pstats.Stats(prof).sort_stats("cumtime").print_stats(45)


if __name__ == "__main__":
    main()
