"""The scheduler builds its first evaluation's templates between registering and its first offers
(``DefaultScheduler.prewarm`` -> ``OfferEvaluator.prewarm``, run by the offer thread at start):
the first pod's evaluation then builds no PodInfoBuilder and no reservation template, and what it
launches is what an evaluation without the prewarm launches."""
import os

from dcos_commons_amd.benchmarks.deploy_bench import SPECS, helloworld_env
from dcos_commons_amd.framework import driver
from dcos_commons_amd.mesos import protos as P
from dcos_commons_amd.mesos.local_master import AgentSpec
from dcos_commons_amd.offer import resources as R
from dcos_commons_amd.offer.evaluate import pod_info_builder as PIB
from dcos_commons_amd.offer.recommendations import LaunchOfferRecommendation
from dcos_commons_amd.offer.taskdata.labels import env_to_map
from dcos_commons_amd.scheduler.scheduler_builder import SchedulerBuilder
from dcos_commons_amd.scheduler.scheduler_config import SchedulerConfig
from dcos_commons_amd.specification.yaml.mappers import ServiceSpecGenerator
from dcos_commons_amd.specification.yaml.raw import RawServiceSpec
from dcos_commons_amd.storage.mem_persister import MemPersister
from dcos_commons_amd.testing.harness import RecordingDriver


def _offer(i):
    spec = AgentSpec(hostname=f"agent-{i}", cpus=16, mem=65536, disk=100000, gpus=1)
    o = P.Offer(hostname=spec.hostname)
    o.id.value, o.agent_id.value, o.framework_id.value = f"offer-{i}", f"agent-{i}", "fw"
    for r in spec.resources():
        r.allocation_info.role = "hello-world-role"
        o.resources.add().CopyFrom(r)
    return o


def _scheduler(fid):
    env = helloworld_env(2, 1, "true")
    cfg = SchedulerConfig.for_testing(PORT_API="0", SDK_OFFER_PREWARM="true")
    raw = RawServiceSpec.new_builder(os.path.join(SPECS, "gpu.yml")).set_env(env).build()
    spec = ServiceSpecGenerator(raw, cfg, SPECS, env).build()
    sched = SchedulerBuilder(spec, cfg, MemPersister()).set_plans_from(raw).build()
    driver.set_driver(RecordingDriver())
    sched.framework_store.store_framework_id(P.FrameworkID(value=fid))
    sched.registered(False)
    return sched


def _launch(sched):
    step = sched.plan_coordinator.get_candidates()[0]
    recs = sched.plan_scheduler.offer_evaluator.evaluate(step.get_pod_instance_requirement(), [_offer(0)])
    return [r for r in recs if isinstance(r, LaunchOfferRecommendation)][0].task_info, recs


def test_first_evaluation_after_prewarm_builds_nothing(monkeypatch):
    cold_info, cold_recs = _launch(_scheduler("fw-cold"))
    sched = _scheduler("fw-warm")
    sched.prewarm()
    builds = []
    orig_init, orig_from_spec = PIB.PodInfoBuilder.__init__, R.ResourceBuilder.from_spec

    def count_init(self, *a, **k):
        builds.append("PodInfoBuilder")
        orig_init(self, *a, **k)

    def count_from_spec(*a, **k):
        builds.append("ResourceBuilder.from_spec")
        return orig_from_spec(*a, **k)
    monkeypatch.setattr(PIB.PodInfoBuilder, "__init__", count_init)
    monkeypatch.setattr(R.ResourceBuilder, "from_spec", staticmethod(count_from_spec))
    info, recs = _launch(sched)
    assert builds == []
    # the same launch as without the prewarm, up to the generated ids
    assert [type(r).__name__ for r in recs] == [type(r).__name__ for r in cold_recs]
    assert info.name == cold_info.name and len(info.resources) == len(cold_info.resources)
    strip = lambda e: {k: v for k, v in env_to_map(e).items()}   # noqa: E731
    assert strip(info.command.environment) == strip(cold_info.command.environment)


def test_prewarm_is_idempotent_and_fails_only_quietly():
    sched = _scheduler("fw-1")
    _launch(sched)
    sched.prewarm()
    sched.prewarm()
    # before a framework ID is stored the evaluator cannot build anything: prewarm raises, and
    # the offer thread (OfferProcessor._loop) logs that at debug level and goes on
    env = helloworld_env(1, 1, "true")
    cfg = SchedulerConfig.for_testing(PORT_API="0", SDK_OFFER_PREWARM="true")
    raw = RawServiceSpec.new_builder(os.path.join(SPECS, "gpu.yml")).set_env(env).build()
    spec = ServiceSpecGenerator(raw, cfg, SPECS, env).build()
    fresh = SchedulerBuilder(spec, cfg, MemPersister()).set_plans_from(raw).build()
    try:
        fresh.prewarm()
        raised = False
    except RuntimeError:
        raised = True
    assert raised


def test_prewarm_stops_when_offers_are_queued(monkeypatch):
    """The offer thread's ``stop()`` turns true once offers are queued: the prewarm builds
    nothing more and the cycle starts."""
    sched = _scheduler("fw-stop")
    builds = []
    orig = PIB.PodInfoBuilder.__init__

    def count(self, *a, **k):
        builds.append(1)
        orig(self, *a, **k)
    monkeypatch.setattr(PIB.PodInfoBuilder, "__init__", count)
    sched.prewarm(lambda: True)
    assert builds == []
    asked = []

    def after_template():           # let the template through, stop before the reservations
        asked.append(1)
        return len(asked) > 2
    sched.prewarm(after_template)
    assert builds == [1]


def test_prewarm_is_off_by_default(monkeypatch):
    env = helloworld_env(1, 1, "true")
    cfg = SchedulerConfig.for_testing(PORT_API="0")
    raw = RawServiceSpec.new_builder(os.path.join(SPECS, "gpu.yml")).set_env(env).build()
    spec = ServiceSpecGenerator(raw, cfg, SPECS, env).build()
    sched = SchedulerBuilder(spec, cfg, MemPersister()).set_plans_from(raw).build()
    sched.prewarm()         # returns before touching anything (no framework ID needed)
