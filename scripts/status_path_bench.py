"""Microbenchmark of the scheduler's status path (``FrameworkScheduler.status_update`` ->
``DefaultScheduler.process_status_update`` -> plan updates) for a helloworld ``gpu.yml`` deploy of
N pods whose tasks are launched: one RUNNING status with a passed readiness check per call.

    python scripts/status_path_bench.py [--pods 8] [--reps 2000] [--profile]
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
from dcos_commons_amd.framework.framework_scheduler import FrameworkScheduler  # noqa: E402
from dcos_commons_amd.mesos import protos as P  # noqa: E402
from dcos_commons_amd.scheduler.scheduler_builder import SchedulerBuilder  # noqa: E402
from dcos_commons_amd.scheduler.scheduler_config import SchedulerConfig  # noqa: E402
from dcos_commons_amd.specification.yaml.mappers import ServiceSpecGenerator  # noqa: E402
from dcos_commons_amd.specification.yaml.raw import RawServiceSpec  # noqa: E402
from dcos_commons_amd.state.framework_store import FrameworkStore  # noqa: E402
from dcos_commons_amd.storage.mem_persister import MemPersister  # noqa: E402
from dcos_commons_amd.testing.harness import RecordingDriver  # noqa: E402

from offer_eval_bench import offers  # noqa: E402


def setup(n):
    env = helloworld_env(n, 1, "true")
    cfg = SchedulerConfig.for_testing(PORT_API="0", SDK_EVENT_DRIVEN="false")
    raw = RawServiceSpec.new_builder(os.path.join(SPECS, "gpu.yml")).set_env(env).build()
    spec = ServiceSpecGenerator(raw, cfg, SPECS, env).build()
    persister = MemPersister()
    sched = SchedulerBuilder(spec, cfg, persister).set_plans_from(raw).build()
    d = RecordingDriver()
    driver.set_driver(d)
    fw = FrameworkScheduler({spec.role}, cfg, persister, FrameworkStore(persister), sched).disable_threading()
    fw.registered(d, P.FrameworkID(value="fw-1"), P.MasterInfo(id="m", ip=1, port=2))
    fw.set_api_server_started()
    fw.resource_offers(d, offers(n))
    statuses = []
    for a in d.accepts:
        for op in a.operations if hasattr(a, "operations") else []:
            pass
    for t in sched.state_store.fetch_tasks():
        s = P.TaskStatus(state=P.TASK_RUNNING, source=P.TaskStatus.SOURCE_EXECUTOR)
        s.task_id.CopyFrom(t.task_id)
        s.check_status.type = P.CheckInfo.COMMAND
        s.check_status.command.exit_code = 0
        statuses.append(s)
    return fw, d, statuses


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pods", type=int, default=8)
    ap.add_argument("--reps", type=int, default=2000)
    ap.add_argument("--profile", action="store_true")
    ap.add_argument("--sort", default="tottime")
    a = ap.parse_args()
    fw, d, statuses = setup(a.pods)
    assert len(statuses) == a.pods, len(statuses)
    for i in range(200):
        fw.status_update(d, statuses[i % len(statuses)])
    prof = cProfile.Profile() if a.profile else None
    if prof:
        prof.enable()
    chunk = max(1, a.reps // 20)
    best, done = float("inf"), 0
    while done < a.reps:
        t0 = time.process_time()
        for i in range(chunk):
            fw.status_update(d, statuses[i % len(statuses)])
        best, done = min(best, (time.process_time() - t0) / chunk), done + chunk
    if prof:
        prof.disable()
    print(f"{best * 1e6:.1f} us per status update ({a.pods} pods)")
    if prof:
        pstats.Stats(prof).sort_stats(a.sort).print_stats(35)


if __name__ == "__main__":
    main()
