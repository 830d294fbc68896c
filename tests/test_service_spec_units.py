"""ServiceSpec content checks on the reference's own spec fixtures, plus the spec value types.

Mirrors sdk/scheduler/src/test/java/com/mesosphere/sdk/specification/{DefaultServiceSpecTest,
DefaultVolumeSpecTest,RLimitSpecTest,DefaultHealthCheckSpecTest,ReplacementFailurePolicyTest,
DefaultPodSpecTest,DefaultTaskSpecTest,PlanGeneratorTest}.java and yaml/{TemplateUtilsTest,
YAMLServiceSpecFactoryTest}.java. ``test_specification`` already parses every valid fixture
(round-tripping its JSON) and rejects every invalid one; this suite checks what the parsed specs
contain and the exact errors of the invalid ones. Fixtures are read in place from the reference
tree (sdk/scheduler/src/test/resources).
"""
import json
import os

import pytest

import testutils as U
from conftest import reference_path
from dcos_commons_amd.dcos import capabilities
from dcos_commons_amd.scheduler.plan.factories import DefaultStepFactory, PlanGenerator
from dcos_commons_amd.scheduler.scheduler_builder import SchedulerBuilder
from dcos_commons_amd.scheduler.scheduler_config import SchedulerConfig
from dcos_commons_amd.specification import specs as S
from dcos_commons_amd.specification.yaml import mappers
from dcos_commons_amd.specification.yaml import template_utils as TU
from dcos_commons_amd.specification.yaml.raw import RawServiceSpec, RawSpecError
from dcos_commons_amd.state.config_store import ConfigStore
from dcos_commons_amd.state.state_store import StateStore
from dcos_commons_amd.storage.mem_persister import MemPersister

FIXTURES = reference_path("sdk", "scheduler", "src", "test", "resources")
CFG = SchedulerConfig.for_testing()
pytestmark = pytest.mark.skipif(FIXTURES is None, reason="reference fixtures not present")

TEMPLATES = {"config-one.conf.mustache": "hello", "config-two.xml.mustache": "hey",
             "config-three.conf.mustache": "hi"}


class Reader:
    def read(self, path):
        return TEMPLATES.get(os.path.basename(path), f"template for {path}")


def raw(name, env=None):
    return RawServiceSpec.new_builder(os.path.join(FIXTURES, name)).set_env(env or {}).build()


def spec(name, env=None, reader=True):
    g = mappers.ServiceSpecGenerator(raw(name, env), CFG, FIXTURES, env or {})
    if reader:
        g.reader = Reader()
    return g.build()


def ports(s, pod=0, task=0):
    return [r for r in s.pods[pod].tasks[task].resource_set.resources if r.name == "ports"]


def build_scheduler(s, gpus):
    saved = capabilities.get_instance()
    capabilities.override_capabilities(capabilities.Capabilities().with_overrides(
        supports_gpu_resource=gpus, supports_cni_networking=True, supports_domains=True))
    try:
        return SchedulerBuilder(s, CFG, MemPersister()).build()
    finally:
        capabilities.override_capabilities(saved)


# ---------------------------------------------------------------------------------------
# valid specs


def test_valid_exhaustive_and_minimal():
    assert spec("valid-exhaustive.yml") is not None
    assert spec("valid-minimal.yml") is not None


@pytest.mark.parametrize("name,gpus", [
    ("valid-simple.yml", False), ("valid-gpu-resource.yml", True), ("valid-gpu-resourceset.yml", True),
    ("valid-profile-mount-volume.yml", False), ("readiness-check.yml", False),
    ("valid-automatic-cni-port-forwarding.yml", False),
])
def test_valid_specs_build_a_scheduler(name, gpus):
    s = build_scheduler(spec(name), gpus)
    assert s.plan_coordinator.get_plan_managers()


def test_gpu_specs_request_gpus():
    for name in ("valid-gpu-resource.yml", "valid-gpu-resourceset.yml"):
        assert spec(name).uses_gpus()
    assert not spec("valid-simple.yml").uses_gpus()


def test_port_env_keys():
    p = ports(spec("valid-envkey-ports.yml"))
    assert [(x.port_name, x.port, x.env_key) for x in p] == [
        ("name1", 8080, "key1"), ("name2", 8088, None), ("name3", 8089, None)]


def test_seccomp_settings():
    pod = spec("seccomp-unconfined.yml").pods[0]
    assert pod.seccomp_unconfined and pod.seccomp_profile_name is None
    for name in ("seccomp-profile-name.yml", "valid-seccomp-info.yml"):
        pod = spec(name).pods[0]
        assert not pod.seccomp_unconfined and pod.seccomp_profile_name == "foobar"


def test_invalid_seccomp_both_settings():
    with pytest.raises(Exception):
        spec("invalid-seccomp-info.yml")


def test_shared_memory():
    pod = spec("valid-shared-memory-pod.yml").pods[0]
    assert pod.shared_memory == S.IpcMode.PRIVATE and pod.shared_memory_size == 1024
    s = spec("valid-shm-spec.yml")
    pod = s.pods[0]
    assert pod.shared_memory == S.IpcMode.PRIVATE and pod.shared_memory_size == 1024
    t1, t2, t3 = pod.tasks[:3]
    assert (t1.shared_memory, t1.shared_memory_size) == (S.IpcMode.PRIVATE, 256)
    assert (t2.shared_memory, t2.shared_memory_size) == (S.IpcMode.SHARE_PARENT, None)
    assert (t3.shared_memory, t3.shared_memory_size) == (S.IpcMode.SHARE_PARENT, None)


@pytest.mark.parametrize("name", ["invalid-share-parent-pod.yml", "invalid-share-parent-shm-size.yml"])
def test_invalid_share_parent(name):
    with pytest.raises(ValueError):
        spec(name)


def test_port_ranges():
    p = ports(spec("ranges.yml"))
    assert len(p) == 2
    assert (p[0].port_name, p[0].env_key) == ("name1", "key1")
    assert [(r.begin, r.end) for r in p[0].ranges] == [(1, 21), (2000, 5050)]
    assert p[1].port_name == "name2"
    # a missing begin is MIN_PORT, a missing end MAX_PORT (RangeSpec.java:26-27)
    assert [(r.begin, r.end) for r in p[1].ranges] == [(S.RangeSpec.MIN_PORT, 21), (5000, S.RangeSpec.MAX_PORT)]


def test_multiple_ports():
    http, another = ports(spec("valid-multiple-ports.yml"))
    assert [(r.begin, r.end) for r in http.value.ranges.range] == [(8080, 8080)]
    assert [(r.begin, r.end) for r in another.value.ranges.range] == [(8088, 8088)]


def test_duplicate_ports_rejected():
    with pytest.raises(ValueError, match="Task has multiple ports with value 8080"):
        spec("invalid-duplicate-ports.yml")


def test_duplicate_port_names_rejected():
    with pytest.raises(ValueError, match=r"Service has duplicate advertised ports across tasks: "
                                         r"\[across-pods, across-tasks, in-resource-set\]"):
        spec("invalid-duplicate-port-names.yml")


def test_readiness_check():
    rc = spec("readiness-check.yml").pods[0].tasks[0].readiness_check
    assert rc is not None
    assert (rc.command, rc.interval, rc.delay, rc.timeout) == ("./readiness-check", 5, 0, 10)


def test_bridge_network_port_forwarding():
    r = raw("valid-automatic-cni-port-forwarding.yml")
    nets = {p: (r.pods[p].get("networks") or {}) for p in r.pods}
    assert len((nets["pod-type"]["mesos-bridge"] or {}).get("host-ports", []) or []) == 0
    s = spec("valid-automatic-cni-port-forwarding.yml")
    assert len(s.pods) == 3
    maps = [dict(p.networks[0].port_mappings) for p in s.pods]
    assert maps == [{8080: 8080}, {8080: 8080, 8081: 8081}, {4040: 8080, 4041: 8081}]
    assert all(len(p.networks) == 1 for p in s.pods)


def test_port_mapping_network_keeps_port_resources():
    s = spec("valid-automatic-cni-port-forwarding.yml")
    assert s.pods[0].networks[0].name == "mesos-bridge"
    for pod in s.pods:
        for t in pod.tasks:
            want = 2 if pod.type == "meta-data-with-port-mapping" else 1
            assert len([r for r in t.resource_set.resources if r.name == "ports"]) == want


def test_task_kill_grace_period():
    assert spec("valid-task-kill-grace-period-seconds.yml").pods[0].tasks[0].kill_grace_period == 15
    assert spec("valid-minimal.yml").pods[0].tasks[0].kill_grace_period == 0  # the reference default
    with pytest.raises(ValueError):
        spec("invalid-task-kill-grace-period-seconds.yml")


@pytest.mark.parametrize("name,field", [
    ("invalid-pod-name.yml", "meta-data"), ("invalid-duplicate-count.yml", "count"),
    ("invalid-task-name.yml", "meta-data-task"), ("invalid-resource-set-name.yml", "data-store-resources"),
])
def test_duplicate_yaml_fields(name, field):
    with pytest.raises(Exception, match=f"Duplicate field '{field}'"):
        spec(name)


def test_duplicate_dns_names_across_pods():
    with pytest.raises(ValueError, match="Tasks in different pods cannot share DNS names"):
        spec("invalid-task-dns.yml")


def test_host_volume_mode():
    pod = spec("valid-host-volume.yml").pods[0]
    assert pod.host_volumes
    for hv in pod.host_volumes:
        assert (hv.container_path, hv.host_path, hv.mode) == ("host-volume-etc", "/etc", "RO")


def test_volume_and_volumes_rejected():
    with pytest.raises(ValueError, match="Both 'volume' and 'volumes'"):
        spec("invalid-volume-and-volumes.yml")


def test_missing_config_template_file():
    with pytest.raises(FileNotFoundError):
        spec("invalid-config-file.yml", reader=False)


def test_invalid_plan_steps_fail_at_build():
    r = raw("invalid-plan-steps.yml")
    s = mappers.ServiceSpecGenerator(r, CFG, FIXTURES, {}).build()
    with pytest.raises(Exception):
        SchedulerBuilder(s, CFG, MemPersister()).set_plans_from(r).build()


def test_duplicate_pod_types_and_task_names_rejected_on_construction():
    from dataclasses import replace

    s = spec("valid-exhaustive.yml")
    with pytest.raises(ValueError):
        S.ServiceSpec.create(s.name, list(s.pods) + [s.pods[0]], s.role, s.principal)
    pod = s.pods[0]
    with pytest.raises(ValueError):
        replace(pod, tasks=tuple(pod.tasks) + (pod.tasks[0],)).validate()


def test_duplicate_container_definition_rejected():
    with pytest.raises(ValueError):
        spec("invalid-duplicate-container-definition.yml")


def test_image_and_labels():
    assert spec("valid-image.yml").pods[0].image == "group/image"
    labels = spec("valid-task-labels.yml").pods[0].tasks[0].labels
    assert labels["label1"] == "label1-value" and labels["label2"] == "path:/"


@pytest.mark.parametrize("name", [
    "invalid-task-labels-format.yml", "invalid-task-labels-blank.yml", "invalid-image-null.yml",
    "invalid-network.yml", "invalid-network-labels-format.yml", "invalid-network-labels-blank.yml",
    "invalid-scalar-cpu-resource.yml", "invalid-scalar-mem-resource.yml", "invalid-scalar-disk-resource.yml",
    "invalid-rlimit-name.yml", "invalid-vip-port-name-collision.yml", "invalid-task-resources.yml",
])
def test_invalid_specs(name):
    with pytest.raises(Exception):
        spec(name)


def test_networks():
    s = spec("valid-network.yml")
    net = s.pods[0].networks[0]
    assert net.name == "dcos"
    assert len(ports(s)) == 2
    assert dict(net.labels) == {"key1": "val1", "key2": "val2a:val2b"}


def test_zookeeper_connection():
    assert spec("valid-minimal.yml").zookeeper_connection == S.MESOS_MASTER_ZK_CONNECTION_STRING == \
        "master.mesos:2181"
    assert spec("valid-customzk.yml").zookeeper_connection == "custom.master.mesos:2181"


def _pod(user):
    return S.PodSpec(type="p", count=1, tasks=(S.TaskSpec("t", S.GoalState.RUNNING, spec("valid-minimal.yml")
                                                          .pods[0].tasks[0].resource_set),), user=user)


@pytest.mark.parametrize("service_user,pod_user,expected", [
    (None, "user", "user"),                              # from the pod
    ("service-user", "pod-user", "service-user"),        # the service wins
    (None, None, S.DEFAULT_SERVICE_USER),                # the default
])
def test_service_user_resolution(service_user, pod_user, expected):
    assert S.ServiceSpec.create("svc", [_pod(pod_user)], user=service_user).user == expected
    assert S.DEFAULT_SERVICE_USER == "root"


def test_old_finished_goal_reads_as_once():
    assert S.GoalState.parse_persisted("ONCE") == S.GoalState.ONCE
    assert S.GoalState.parse_persisted("FINISHED") == S.GoalState.ONCE


def test_finished_goal_rejected_in_yaml():
    with pytest.raises(ValueError) as e:
        spec("valid-finished.yml")
    assert str(e.value) == ("Unsupported GoalState FINISHED in task meta-data-task, expected one of: "
                            "[UNKNOWN, RUNNING, FINISH, ONCE]")


def test_unknown_placement_rule_types_fail_the_loopback():
    from dataclasses import replace

    class CustomRule:
        def filter(self, offer, pod_instance, tasks):
            raise NotImplementedError

        def to_dict(self):
            return {"@type": "NotARegisteredRule"}

    s = spec("valid-minimal.yml")
    bad = replace(s, pods=(replace(s.pods[0], placement_rule=CustomRule()),))
    with pytest.raises(Exception):
        S.loopback_check(bad)


# ---------------------------------------------------------------------------------------
# DefaultVolumeSpec


@pytest.mark.parametrize("path", ["", " ", "/path/to/volume0", "@?test", "-test"])
def test_invalid_mount_volume_paths(path):
    with pytest.raises(ValueError):
        S.VolumeSpec.create_mount_volume(1000, path, [], "role", "*", "principal")


@pytest.mark.parametrize("path,ok", [("path-0_1-path", True), ("path", True), ("path/path", False),
                                     ("path-0/1-path", False)])
def test_root_volume_paths(path, ok):
    if ok:
        S.VolumeSpec.create_root_volume(1000, path, "role", "*", "principal")
    else:
        with pytest.raises(ValueError):
            S.VolumeSpec.create_root_volume(1000, path, "role", "*", "principal")


@pytest.mark.parametrize("profiles,ok", [
    ([], True), (["test"], True), (["test", "0"], True), (["test", "_.-"], True),
    (["test", None], False), (["test", ""], False), (["test", " "], False), (["test", "a/b"], False),
    (["test", "@?"], False), (["test", "a" * 129], False), (["test", "test"], False),
])
def test_mount_volume_profiles(profiles, ok):
    if ok:
        v = S.VolumeSpec.create_mount_volume(1000, "path", profiles, "role", "*", "principal")
        assert list(v.profiles) == profiles
    else:
        with pytest.raises((ValueError, TypeError)):
            S.VolumeSpec.create_mount_volume(1000, "path", profiles, "role", "*", "principal")


# ---------------------------------------------------------------------------------------
# RLimitSpec, health checks, replacement policy, VIPs


def test_rlimits():
    r = S.RLimitSpec("RLIMIT_AS", 0, 1)
    r.validate()
    assert (r.name, r.soft, r.hard) == ("RLIMIT_AS", 0, 1)
    S.RLimitSpec("RLIMIT_AS", -1, -1).validate()  # unlimited


@pytest.mark.parametrize("name,soft,hard", [
    ("NONSENSE", 0, 1), ("RLIMIT_AS", 0, -1), ("RLIMIT_AS", 1, 0), ("RLIMIT_AS", -2, -2), ("RLIMIT_AS", -1, 0),
    ("RLIMIT_AS", 0, None),
])
def test_invalid_rlimits(name, soft, hard):
    with pytest.raises(ValueError):
        S.RLimitSpec(name, soft, hard).validate()


def test_health_check_validation():
    S.HealthCheckSpec("echo true", 1, 0, 0, 0, 0).validate()
    with pytest.raises(ValueError):
        S.HealthCheckSpec("", -1, -1, -1, -1, -1).validate()


def _hc_json(**grace):
    d = {"command": "some-command", "max-consecutive-failures": 4, "delay": 0, "interval": 15, "timeout": 10}
    d.update(grace)
    return d


@pytest.mark.parametrize("grace", [
    {"gracePeriod": 120},                          # old: camelCase only
    {"grace-period": 120, "gracePeriod": 130},     # both: grace-period wins
    {"grace-period": 120},                         # future: new key only
])
def test_health_check_grace_period_compatibility(grace):
    hc = S.HealthCheckSpec.from_dict(_hc_json(**grace))
    assert hc.grace_period == 120
    # both keys are written so an older scheduler can still read the config
    assert hc.to_dict() == _hc_json(**{"grace-period": 120, "gracePeriod": 120})
    assert list(hc.to_dict()) == list(_hc_json(**{"grace-period": 120, "gracePeriod": 120}))


def test_replacement_failure_policy():
    S.ReplacementFailurePolicy(0, 0).validate()
    with pytest.raises(ValueError):
        S.ReplacementFailurePolicy(-1, -1).validate()
    assert S.ReplacementFailurePolicy().permanent_failure_timeout_mins == 20


def test_named_vip_ports():
    s = spec("valid-exhaustive.yml")
    vips = [r for p in s.pods for t in p.tasks for r in t.resource_set.resources if isinstance(r, S.NamedVIPSpec)]
    assert vips and all(v.vip_name and v.vip_port > 0 for v in vips)


# ---------------------------------------------------------------------------------------
# pod / task spec copies, plan generation, templates


def test_pod_and_task_specs_survive_a_json_round_trip():
    s = spec("valid-exhaustive.yml")
    for pod in s.pods:
        assert S.PodSpec.from_dict(json.loads(json.dumps(pod.to_dict()))) == pod
        for t in pod.tasks:
            assert S.TaskSpec.from_dict(json.loads(json.dumps(t.to_dict()))) == t


def test_custom_phases():
    r = raw("custom-phases.yml")
    s = mappers.ServiceSpecGenerator(r, CFG, FIXTURES, {}).build()
    persister = MemPersister()
    gen = PlanGenerator(DefaultStepFactory(ConfigStore(S.loopback_check(s), persister), StateStore(persister)))
    expected = [
        [["server"]] * 3,
        [["once"]] * 3,
        [["once"], ["server"]] * 3,
        [["once", "server"]] * 3,
        [["once", "server"]] * 3,
        [["once"], ["server"]] * 3,
        [["once"], ["server"], ["server"], ["once"], ["server"]],
        [["server"], ["once"], ["once"], ["server"], ["server"], ["once"]],
    ]
    assert r.plans
    for name, raw_plan in r.plans.items():
        plan = gen.generate(raw_plan, name, s.pods)
        assert len(plan.get_children()) == 8
        for phase, want in zip(plan.get_children(), expected):
            assert [st.get_pod_instance_requirement().tasks_to_launch for st in phase.get_children()] == want


def _read(name):
    with open(os.path.join(FIXTURES, name)) as f:
        return f.read()


def test_render_exhaustive_template():
    text = _read("test-render.yml")
    assert "size: {{VOL_SIZE}}" in text
    assert "size: 1024" in TU.render_mustache_throw_if_missing("test-render.yml", text, {"VOL_SIZE": "1024"})


def test_missing_value_renders_empty_and_is_reported():
    missing = []
    out = TU.render_mustache("testTemplate", "hello this is a {{missing-parameter}}. thanks for reading bye", {},
                             missing)
    assert out == "hello this is a . thanks for reading bye"
    assert [(m.name, m.line) for m in missing] == [("missing-parameter", 1)]


def test_missing_values_raise_with_lines():
    env = {"bar": "baz", "baz": "foo", "foo": "bar"}
    with pytest.raises(TU.MustacheError) as e:
        TU.render_mustache_throw_if_missing(
            "testTemplate",
            "hello this is {{a_missing_parameter}},\nand {{another_missing_parameter}}. thanks for reading bye", env)
    msg = str(e.value)
    assert msg.startswith("Missing 2 values when rendering testTemplate:\n")
    assert "- Missing values: [a_missing_parameter@L1, another_missing_parameter@L2]" in msg


@pytest.mark.parametrize("template,expected", [
    ("hello this is an {{#missing_parameter}}ignored string{{/missing_parameter}}. thanks for reading bye",
     "hello this is an . thanks for reading bye"),
    ("hello this is an {{^missing_parameter}}included string{{/missing_parameter}}. thanks for reading bye",
     "hello this is an included string. thanks for reading bye"),
])
def test_missing_section_names_do_not_fail(template, expected):
    assert TU.render_mustache_throw_if_missing("testTemplate", template, {}) == expected


@pytest.mark.parametrize("value,present,absent", [
    ("true", ["cmd: ./enabled true"], ["cmd: ./disabled"]),
    ("false", ["cmd: ./disabled false"], ["cmd: ./enabled"]),
    ("", ["cmd: ./disabled"], ["cmd: ./disabled false", "cmd: ./enabled"]),
])
def test_sections_follow_the_env_value(value, present, absent):
    text = _read("test-render-inverted.yml")
    assert "ENABLED" in text
    out = TU.render_mustache_throw_if_missing("test-render-inverted.yml", text, {"ENABLED": value})
    for p in present:
        assert p in out
    for a in absent + ["ENABLED"]:
        assert a not in out


def test_raw_spec_from_file_with_env():
    assert raw("valid-exhaustive.yml", {"PORT_API": str(U.PORT_API_VALUE)}) is not None


def test_health_check_json_matches_the_reference_layout():
    from dcos_commons_amd.config.serialization import to_json_string

    hc = S.HealthCheckSpec.from_dict(_hc_json(gracePeriod=120))
    assert to_json_string(hc) == (
        '{\n  "command" : "some-command",\n  "max-consecutive-failures" : 4,\n  "delay" : 0,\n'
        '  "interval" : 15,\n  "timeout" : 10,\n  "grace-period" : 120,\n  "gracePeriod" : 120\n}')


def test_value_json_fast_path_matches_the_protobuf_json_mapping():
    """specs.value_to_json short-cuts scalar/range values; it must emit exactly what the generic
    protobuf JSON mapping does (persisted configs are compared byte for byte)."""
    from dcos_commons_amd.mesos import protos as P
    from dcos_commons_amd.specification.specs import ranges_value, scalar_value, value_to_json

    cases = [scalar_value(0.1), scalar_value(256), scalar_value(0.0), ranges_value([(1, 2), (10, 20)]),
             ranges_value([]), ranges_value([(0, 2 ** 63)]), P.Value(type=P.Value.SCALAR),
             P.Value(type=P.Value.RANGES), P.Value()]
    s = P.Value(type=P.Value.SET)
    s.set.item.extend(["a", "b"])
    t = P.Value(type=P.Value.TEXT)
    t.text.value = "x"
    for v in cases + [s, t]:
        assert value_to_json(v) == P.to_json(v), v
