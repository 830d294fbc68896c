"""Conformance against the reference's own, unchanged inputs.

* Every helloworld example spec in the reference's ``frameworks/helloworld/src/main/dist`` is
  rendered with the reference's ``universe/`` package defaults plus the per-spec scheduler env of
  ``ServiceTest.testExampleSpecs`` (frameworks/helloworld/src/test/java/.../ServiceTest.java:986-1023),
  and then deployed to COMPLETE in the simulator. The reference test only renders; deploying goes
  further. The specs whose resources generic offers lack get offers that carry them: statically
  pre-reserved resources (``pre-reserved*.yml``), profiled MOUNT disks (``*profile-mount-volume.yml``),
  and a DC/OS CA stand-in for ``tls.yml``.
* cassandra: the reference's unchanged ``svc.yml`` + ``universe/`` deploy, then replace a seed node
  through ``CassandraRecoveryPlanOverrider`` (``replace_address``).
* hdfs: the reference's unchanged ``svc.yml`` + ``universe/`` deploy, then a configuration change
  is rolled out by the ``update`` plan (frameworks/hdfs/src/main/dist/svc.yml:566-611).

Skipped when the reference tree is absent (the GPU box has none)."""
import os

import pytest

from dcos_commons_amd.mesos import protos as P
from dcos_commons_amd.models import cassandra as C
from dcos_commons_amd.models import hdfs as H
from dcos_commons_amd.scheduler.plan.status import Status
from dcos_commons_amd.specification.yaml import raw as R
from dcos_commons_amd.testing import Expect, Send, ServiceTestRunner

REF = os.environ.get("SDK_REFERENCE_ROOT", "/root/reference")
REF_FW = os.path.join(REF, "frameworks")
HELLO = os.path.join(REF_FW, "helloworld")
DIST = os.path.join(HELLO, "src", "main", "dist")

pytestmark = pytest.mark.skipif(not os.path.isdir(DIST), reason="reference tree not present")

# ServiceTest.java:989-1005: the extra scheduler env some examples need
EXAMPLE_ENV = {
    "secrets.yml": dict(HELLO_SECRET1="hello-world/secret1", HELLO_SECRET2="hello-world/secret2",
                        WORLD_SECRET1="hello-world/secret1", WORLD_SECRET2="hello-world/secret2",
                        WORLD_SECRET3="hello-world/secret3"),
    "custom_steps.yml": dict(DEPLOY_STRATEGY="serial", DEPLOY_STEPS="[[first, second, third]]"),
    "pod-profile-mount-volume.yml": dict(HELLO_VOLUME_PROFILE="xfs"),
    "profile-mount-volume.yml": dict(HELLO_VOLUME_PROFILE="xfs"),
    "svc.yml": dict(HELLO_LABELS="label1:label-value1"),
}
EXAMPLES = sorted(f for f in os.listdir(DIST) if f.endswith(".yml")) if os.path.isdir(DIST) else []


def test_every_reference_example_is_covered():
    # the reference ships 37 example specs; a silently shrinking list would hide regressions
    assert len(EXAMPLES) == 37, EXAMPLES
    assert {"gpu_resource.yml", "graceful-shutdown.yml", "pod-profile-mount-volume.yml", "tls.yml"} <= set(EXAMPLES)


@pytest.fixture
def dcos_ca(monkeypatch):
    from dcos_commons_amd.ops import build
    from dcos_commons_amd.testing.dcos_fakes import FakeDcosCluster

    try:
        build.build_cpp_tools()
    except Exception as e:  # noqa: BLE001
        pytest.skip(f"native toolchain unavailable: {e}")
    cluster = FakeDcosCluster(intermediate_ca=True).start()
    monkeypatch.setenv("SDK_DCOS_MASTER_URI", cluster.url)
    yield cluster
    cluster.stop()


def _example_runner(spec):
    r = ServiceTestRunner(os.path.join(DIST, spec), universe_dir=os.path.join(HELLO, "universe"))
    return r.set_scheduler_env(SDK_REVIVE_INTERVAL_S="0", **EXAMPLE_ENV.get(spec, {}))


@pytest.mark.parametrize("spec", [s for s in EXAMPLES if s != "tls.yml"])
def test_reference_example_deploys_unchanged(spec):
    res = _example_runner(spec).run([Send.register(), Send.drive_plan("deploy"),
                                     Expect.plan_status("deploy", Status.COMPLETE)])
    assert res.service_spec.pods  # rendered and built through the strict (universe) path


def test_reference_tls_example_deploys_with_a_ca(dcos_ca):
    cred = dcos_ca.add_service_account("hello-world")
    r = _example_runner("tls.yml").set_scheduler_env(DCOS_SERVICE_ACCOUNT_CREDENTIAL=cred,
                                                     SDK_DCOS_MASTER_URI=dcos_ca.url)
    r.run([Send.register(), Send.drive_plan("deploy"), Expect.plan_status("deploy", Status.COMPLETE)])
    assert dcos_ca.signed  # certificates really were issued by the CA stand-in


def test_gpu_resource_example_requests_a_gpu_and_ignores_the_container_block(caplog):
    """gpu_resource.yml carries a pod-level ``container:`` block that RawPod ignores
    (``@JsonIgnoreProperties(ignoreUnknown = true)``, RawPod.java:18)."""
    seen = {}

    def check(sim):
        for a in sim.driver.accepts:
            for t in a.launched_tasks():
                seen[t.name] = [r.scalar.value for r in t.resources if r.name == "gpus"]

    with caplog.at_level("WARNING", logger=R.__name__):
        _example_runner("gpu_resource.yml").run([Send.register(), Send.drive_plan("deploy"),
                                                 Expect.that(check, "gpus on the task")])
    assert seen["hello-0-server"] == [1.0]
    assert any("container" in rec.getMessage() and "pods.hello" in rec.getMessage() for rec in caplog.records)


def test_only_pods_are_lenient():
    """Which Raw* levels ignore unknown keys: only RawPod (RawPod.java:18); the other 20 Raw*
    classes keep Jackson's FAIL_ON_UNKNOWN_PROPERTIES."""
    assert R.LENIENT_LEVELS == frozenset({"pod"})
    base = "name: s\npods:\n  p:\n    count: 1\n    tasks:\n      t:\n        goal: RUNNING\n        cmd: x\n" \
           "        cpus: 1\n        memory: 1\n"
    assert "bogus" not in R.RawServiceSpec.from_string(base.replace("    count: 1\n", "    count: 1\n    bogus: 2\n")) \
        .pods["p"]
    for bad in (base + "        bogus: 1\n",  # task
                base + "bogus: 1\n",  # service
                base.replace("name: s\n", "name: s\nscheduler:\n  bogus: 1\n"),  # scheduler
                base + "        health-check:\n          cmd: x\n          bogus: 1\n",
                base + "plans:\n  deploy:\n    bogus: 1\n",
                base + "plans:\n  deploy:\n    phases:\n      ph:\n        pod: p\n        bogus: 1\n"):
        with pytest.raises(R.RawSpecError, match="bogus"):
            R.RawServiceSpec.from_string(bad)


# -- cassandra and hdfs: the reference's unchanged packages --------------------------------
def _cassandra_runner():
    return (ServiceTestRunner.for_framework("cassandra", root=os.path.join(REF_FW, "cassandra"))
            .set_pod_env("node", {"LOCAL_SEEDS": "foo,bar"})
            .set_custom_validators(C.custom_validators())
            .set_recovery_manager_factory(C.CassandraRecoveryPlanOverriderFactory(2))
            .set_builder_customizer(lambda b: b.set_custom_resources([C.SeedsResource(["foo", "bar"])]))
            .set_scheduler_env(SDK_REVIVE_INTERVAL_S="0"))


def _hdfs_runner(**env):
    r = ServiceTestRunner.for_framework("hdfs", root=os.path.join(REF_FW, "hdfs"))
    for pod in ("journal", "name", "data"):
        r.set_pod_env(pod, SERVICE_ZK_ROOT="/dcos-service-hdfs", DECODED_AUTH_TO_LOCAL="")
    return (r.set_recovery_manager_factory(H.HdfsRecoveryPlanOverriderFactory())
            .set_custom_validators([H.HDFSZoneValidator()])
            .set_builder_customizer(lambda b: setattr(b, "original_service_spec",
                                                      H.with_placement_rules(b.original_service_spec)))
            .set_scheduler_env(SDK_REVIVE_INTERVAL_S="0", **env))


def test_reference_cassandra_package_renders_every_plan_and_template():
    r = _cassandra_runner().run()
    node = r.service_spec.pod("node")
    assert node.count == 3 and len(node.tasks) == 13
    assert sorted(r.raw_service_spec.plans) == ["backup-azure", "backup-s3", "cleanup", "deploy", "repair",
                                                "replace", "restore-azure", "restore-s3"]
    # the reference template joins local and remote seeds (cassandra.yaml:12)
    assert '- seeds: "foo,bar,"' in r.get_task_config("node", "server", "cassandra")


def test_reference_cassandra_deploys_and_replaces_a_seed_node():
    from test_cassandra import _deploy_ticks, _launched_server_cmd

    cmd = {}

    def check(sim):
        steps = [s.get_name() for ph in sim.scheduler.get_plan("recovery").get_children() for s in ph.get_children()]
        assert steps == ["node-0:[server]", "node-1:[server]", "node-2:[server]"], steps
        cmd["server"] = _launched_server_cmd(sim, "node-0-server")

    _cassandra_runner().run(_deploy_ticks() + [
        Send.replace_pod("node-0"),
        Expect.task_name_killed("node-0-server"),
        Send.task_status("node-0-server", P.TASK_KILLED).build(),
        Send.offer_builder("node").set_hostname("host-new").build(),
        Expect.launched_tasks("node-0-server"),
        Expect.that(check, "CassandraRecoveryPlanOverrider phase"),
    ])
    assert "-Dcassandra.replace_address=10.0.0.1" in cmd["server"]


def test_reference_hdfs_deploys_then_rolls_out_an_update():
    from test_hdfs import deploy_ticks

    first = _hdfs_runner().run(deploy_ticks() + [Send.empty_offers()])
    assert sorted(first.raw_service_spec.plans) == ["deploy", "replace", "update"]
    before = {t.name: t.task_id.value for a in first.sim.driver.accepts for t in a.launched_tasks()}

    def update_selected(sim):
        plan = sim.scheduler.get_plan("deploy")
        assert [ph.get_name() for ph in plan.get_children()] == ["journal", "name", "data"]
        assert plan.get_status() != Status.COMPLETE

    def relaunched(sim):
        after = {t.name: t.task_id.value for a in sim.driver.accepts for t in a.launched_tasks()}
        for name in ("journal-0-node", "name-0-node", "name-1-zkfc", "data-2-node"):
            assert after[name] != before[name], name

    (_hdfs_runner(TASKCFG_ALL_CONFORMANCE_ROLLOUT="2").set_state(first)
     .run([Send.register(), Expect.that(update_selected, "update plan serves as deploy"),
           Send.drive_plan("deploy"), Expect.plan_status("deploy", Status.COMPLETE),
           Expect.that(relaunched, "every node relaunched")]))


def _spec_json(spec_path: str) -> dict:
    """The ServiceSpec ``spec_path`` builds when rendered with the reference helloworld package's
    universe defaults (the strict rendering path), as JSON."""
    import json

    r = ServiceTestRunner(spec_path, universe_dir=os.path.join(HELLO, "universe")).set_scheduler_env(
        SDK_REVIVE_INTERVAL_S="0")
    _, spec, _, _ = r._build()
    return json.loads(spec.to_json_string())


def test_repo_gpu_resource_builds_the_reference_scenario():
    """``frameworks/helloworld/specs/gpu_resource.yml`` (the spec the bench's ``reference_spec``
    row runs where no reference tree exists) builds the same ServiceSpec as the reference's
    unchanged ``dist/gpu_resource.yml``: same pods, resources, volumes, commands, health and
    readiness checks, placement and default (serial) deploy. (The reference's pod-level
    ``container:`` block is ignored by RawPod, so it contributes nothing to compare.)"""
    repo_spec = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                             "frameworks", "helloworld", "specs", "gpu_resource.yml")
    ours, theirs = _spec_json(repo_spec), _spec_json(os.path.join(DIST, "gpu_resource.yml"))
    assert ours == theirs
    pods = {p["type"]: p for p in ours["pod-specs"]}
    hello, world = pods["hello"]["task-specs"][0], pods["world"]["task-specs"][0]
    gpus = [r["value"]["scalar"]["value"] for r in hello["resource-set"]["resource-specifications"]
            if r["name"] == "gpus"]
    assert gpus == [1.0] and hello["health-check-spec"]
    assert [v["container-path"] for v in hello["resource-set"]["volume-specifications"]] == ["hello-container-path"]
    assert len(world["resource-set"]["volume-specifications"]) == 2 and world["readiness-check-spec"]
