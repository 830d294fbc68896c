"""``PodInfoBuilder.for_instance``: a pod instance's task templates moved from another instance of
the same pod must be exactly what a fresh build gives (every TaskInfo and the ExecutorInfo, byte for
byte), for every pod of every shipped package and helloworld scenario, and of the reference's
unchanged cassandra / hdfs packages when the tree is present. Where the move cannot be exact it must
say so (None) rather than differ; the packages whose deploys matter must never need that."""
import os
import uuid

import pytest

from dcos_commons_amd.http import endpoint_utils
from dcos_commons_amd.mesos import protos as P
from dcos_commons_amd.offer.evaluate.pod_info_builder import PodInfoBuilder
from dcos_commons_amd.scheduler.plan.pod_instance_requirement import PodInstanceRequirement
from dcos_commons_amd.scheduler.scheduler_config import SchedulerConfig
from dcos_commons_amd.specification.specs import PodInstance
from dcos_commons_amd.state.goal_state_override import GoalStateOverride
from dcos_commons_amd.testing import ServiceTestRunner
from dcos_commons_amd.testing.cluster import reference_packages

import test_cassandra
import test_hdfs
import test_helloworld_scenarios as HW

TARGET = uuid.UUID("12345678-1234-5678-1234-567812345678")
FID = P.FrameworkID(value="fw-template-test")
CFG = SchedulerConfig.for_testing()


def _build(spec, pod, index, env=None, overrides=None):
    req = PodInstanceRequirement(PodInstance(pod, index), [t.name for t in pod.tasks], env)
    return PodInfoBuilder(req, spec.name, TARGET, endpoint_utils.template_url_factory(spec.name, CFG), CFG, (), FID,
                          overrides or {})


def _wire(b):
    return ({n: t.SerializeToString(deterministic=True) for n, t in b.task_builders.items()},
            b.executor_builder.SerializeToString(deterministic=True), b.pod_instance, b.assigned_overlay_ports)


def _check_spec(spec, must_move=True, indices=(0, 1, 2, 7, 9, 10, 11, 12, 99, 100)):
    for pod in spec.pods:
        for env, overrides in (({}, {}), ({"EXTRA": "1"}, {pod.tasks[0].name: GoalStateOverride.PAUSED})):
            base = _build(spec, pod, 10, env, overrides)
            for i in indices:
                moved = base.for_instance(PodInstance(pod, i))
                if moved is None:
                    assert not must_move, (spec.name, pod.type, i)
                    continue
                assert _wire(moved) == _wire(_build(spec, pod, i, env, overrides)), (spec.name, pod.type, i)
            # the template itself is untouched by the moves
            assert _wire(base) == _wire(_build(spec, pod, 10, env, overrides))


@pytest.mark.parametrize("spec_file", sorted(f for f in HW.ALL if f not in HW.RENDER_ONLY))
def test_helloworld_scenarios(spec_file):
    r = ServiceTestRunner(os.path.join(HW.SPECS, spec_file)).set_env(HW.ENV).set_scheduler_env(
        SDK_REVIVE_INTERVAL_S="0")
    _check_spec(r.run().service_spec)


def test_shipped_cassandra_and_hdfs():
    _check_spec(test_cassandra.runner().run().service_spec)
    _check_spec(test_hdfs.runner().run().service_spec)


def test_reference_cassandra_and_hdfs():
    root = reference_packages.reference_root()
    if root is None:
        pytest.skip("no reference tree")
    for fw in ("cassandra", "hdfs"):
        r = ServiceTestRunner.for_framework(fw, root=os.path.join(root, "frameworks", fw))
        mod = test_cassandra if fw == "cassandra" else test_hdfs
        base = mod.runner()
        r.pod_env, r.validators, r.recovery_factory, r.customize = (base.pod_env, base.validators,
                                                                    base.recovery_factory, base.customize)
        r.set_scheduler_env(SDK_REVIVE_INTERVAL_S="0")
        _check_spec(r.run().service_spec)


def test_a_name_that_does_not_sort_into_its_slot_is_refused():
    """An environment variable named between the old and the new task name: the task-name
    variable would have to move, so the template is rebuilt instead."""
    r = ServiceTestRunner(os.path.join(HW.SPECS, "svc.yml")).set_env(HW.ENV).set_scheduler_env(
        SDK_REVIVE_INTERVAL_S="0")
    spec = r.run().service_spec
    pod = spec.pod("hello")
    base = _build(spec, pod, 1)
    env = base.task_builders["server"].command.environment
    env.variables.add(name="hello-1-server-z", value="x")
    # keep the environment sorted as a build would
    items = sorted(((v.name, v.value) for v in env.variables))
    del env.variables[:]
    for k, v in items:
        env.variables.add(name=k, value=v)
    assert base.for_instance(PodInstance(pod, 2)) is None       # hello-2-server > hello-1-server-z
