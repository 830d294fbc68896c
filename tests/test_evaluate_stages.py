"""Offer-evaluation stage units: ports (static, dynamic, overlay, ranges, pre-reserved roles,
stickiness), named VIPs on host/overlay/bridge networks, launch labels and fault-domain env,
executor-ID matching, the simple-resource reservation helper, prior-port lookup, MOUNT volume
creation, placement-rule stages and TLS artifact mounting.

Mirrors sdk/scheduler/src/test/java/com/mesosphere/sdk/offer/evaluate/{PortEvaluationStageTest,
NamedVIPEvaluationStageTest,LaunchEvaluationStageTest,ExecutorEvaluationStageTest,
OfferEvaluationUtilsTest,TaskPortLookupTest,VolumeEvaluationStageTest,
PlacementRuleEvaluationStageTest,TLSEvaluationStageTest}.java. Pods are written as service YAML
and run through the spec mapper, so the stages see exactly the specs a scheduler would.
"""
import dataclasses
import textwrap
import uuid

import pytest

import testutils as U
from dcos_commons_amd.dcos import constants as dcos
from dcos_commons_amd.http.endpoint_utils import template_url_factory
from dcos_commons_amd.mesos import protos as P
from dcos_commons_amd.offer import values as V
from dcos_commons_amd.offer.evaluate.pod_info_builder import PodInfoBuilder
from dcos_commons_amd.offer.evaluate.placement import AgentRule
from dcos_commons_amd.offer.evaluate.security import CertificateNamesGenerator, TLSArtifact, TLSArtifactPaths
from dcos_commons_amd.offer.evaluate.stages import (ExecutorEvaluationStage, LaunchEvaluationStage,
                                                    NamedVIPEvaluationStage, PlacementRuleEvaluationStage,
                                                    PortEvaluationStage, TLSEvaluationStage, VolumeEvaluationStage,
                                                    evaluate_simple_resource)
from dcos_commons_amd.offer.recommendations import ReserveOfferRecommendation, UnreserveOfferRecommendation
from dcos_commons_amd.offer.resource_pool import MesosResourcePool
from dcos_commons_amd.offer.resources import MesosResource, ResourceBuilder, get_framework_id, get_namespace
from dcos_commons_amd.offer.taskdata import labels as L
from dcos_commons_amd.scheduler.plan.pod_instance_requirement import PodInstanceRequirement
from dcos_commons_amd.scheduler.scheduler_config import SchedulerConfig
from dcos_commons_amd.specification.specs import (ANY_ROLE, NamedVIPSpec, PodInstance, PortSpec, RangeSpec,
                                                  ResourceSpec, ranges_value)
from dcos_commons_amd.specification.yaml import mappers
from dcos_commons_amd.specification.yaml.raw import RawServiceSpec

CFG = SchedulerConfig.for_testing()
FRAMEWORK_ID = U.FRAMEWORK_ID.value
TASK = U.TASK_NAME          # "test-task-name"
POD = U.POD_TYPE            # "pod-type"


def _pod_spec(body):
    text = (f"name: {U.SERVICE_NAME}\nscheduler:\n  principal: {U.PRINCIPAL}\npods:\n"
            + textwrap.indent(textwrap.dedent(body), "  "))
    return mappers.ServiceSpecGenerator(RawServiceSpec.from_string(text), CFG, "/tmp", {}).build().pods[0]


def _task_yaml(extra="", ports=None, cpus=1.0):
    out = f"{POD}:\n  count: 1\n{extra}  tasks:\n    {TASK}:\n      goal: RUNNING\n      cmd: ./cmd\n      cpus: {cpus}\n"
    if ports:
        out += "      ports:\n" + textwrap.indent(textwrap.dedent(ports), "        ")
    return out


def _builder(pod_spec, current_tasks=(), index=0):
    req = PodInstanceRequirement(PodInstance(pod_spec, index), [t.name for t in pod_spec.tasks])
    return PodInfoBuilder(req, U.SERVICE_NAME, uuid.uuid4(), template_url_factory, CFG, list(current_tasks),
                          U.FRAMEWORK_ID, {})


def _pool(offer, role=ANY_ROLE):
    return MesosResourcePool(offer, role)


def _port_spec(pod_spec):
    return next(r for r in pod_spec.tasks[0].resource_set.resources if isinstance(r, PortSpec))


def _ports_spec(pod_spec):
    return [r for r in pod_spec.tasks[0].resource_set.resources if isinstance(r, PortSpec)]


def _stage(spec, resource_id=None, cls=PortEvaluationStage, framework_id=FRAMEWORK_ID):
    return cls(spec, [TASK], resource_id, None, framework_id)


def _task(builder):
    return builder.get_task_builder(TASK)


def _env(env):
    return {v.name: v.value for v in env.variables}


def _discovery_port(task, name, number):
    assert task.discovery.visibility == P.DiscoveryInfo.CLUSTER  # DEFAULT_TASK_DISCOVERY_VISIBILITY
    ports = [p for p in task.discovery.ports.ports if p.name == name]
    assert len(ports) == 1, f"no port {name} in {task.discovery.ports}"
    assert ports[0].number == number


# ---------------------------------------------------------------------------------------
# PortEvaluationStage


def test_port_resource_is_ignored_on_overlay():
    pod = _pod_spec(_task_yaml("  networks:\n    dcos: {}\n",
                               "overlay-port-name:\n  port: 80\n  env-key: PORT_TEST_IGNORED\n"))
    b = _builder(pod)
    outcome = _stage(_port_spec(pod)).evaluate(_pool(U.get_offer([U.unreserved_ports(10000, 10000)])), b)
    assert outcome.passing and outcome.get_offer_recommendations() == []
    t = _task(b)
    _discovery_port(t, "overlay-port-name", 80)
    assert len(t.resources) == 0
    assert _env(t.command.environment)["PORT_TEST_IGNORED"] == "80"


def test_dynamic_port_on_overlay():
    pod = _pod_spec(_task_yaml("  networks:\n    dcos: {}\n",
                               "dyn-port-name:\n  port: 0\n  env-key: PORT_TEST_DYNAMIC_OVERLAY\n"))
    b = _builder(pod)
    outcome = _stage(_port_spec(pod)).evaluate(_pool(U.get_offer([U.unreserved_ports(10000, 10000)])), b)
    assert outcome.passing and outcome.get_offer_recommendations() == []
    t = _task(b)
    _discovery_port(t, "dyn-port-name", dcos.OVERLAY_DYNAMIC_PORT_RANGE_START)
    assert dcos.OVERLAY_DYNAMIC_PORT_RANGE_START == 1025
    assert len(t.resources) == 0
    assert _env(t.command.environment)["PORT_TEST_DYNAMIC_OVERLAY"] == "1025"


def test_dynamic_overlay_port_skips_the_explicitly_requested_one():
    pod = _pod_spec(_task_yaml("  networks:\n    dcos: {}\n", f"""\
        explicit-port:
          port: {dcos.OVERLAY_DYNAMIC_PORT_RANGE_START}
          env-key: PORT_TEST_EXPLICIT
        dynamic-port:
          port: 0
          env-key: PORT_TEST_DYNAMIC
        """))
    b = _builder(pod)
    assert len(b.assigned_overlay_ports) == 1
    offer = U.get_offer([U.unreserved_ports(10000, 10000)])
    explicit, dynamic = _ports_spec(pod)
    for spec in (explicit, dynamic):
        outcome = _stage(spec).evaluate(_pool(offer), b)
        assert outcome.passing and outcome.get_offer_recommendations() == []
    assert len(b.assigned_overlay_ports) == 2
    t = _task(b)
    _discovery_port(t, "explicit-port", 1025)
    _discovery_port(t, "dynamic-port", 1026)
    assert len(t.resources) == 0
    env = _env(t.command.environment)
    assert (env["PORT_TEST_EXPLICIT"], env["PORT_TEST_DYNAMIC"]) == ("1025", "1026")


CHECKS = {
    "health": """\
        health-check:
          cmd: /bin/true
          interval: 5
          grace-period: 30
          max-consecutive-failures: 3
          delay: 0
          timeout: 10
    """,
    "readiness": """\
        readiness-check:
          cmd: /bin/true
          interval: 5
          delay: 0
          timeout: 10
    """,
}


@pytest.mark.parametrize("check", ["health", "readiness"])
@pytest.mark.parametrize("overlay", [False, True])
def test_port_env_var_reaches_the_checks(check, overlay):
    body = _task_yaml("  networks:\n    dcos: {}\n" if overlay else "",
                      "test-port:\n  port: 10000\n  env-key: PORT_TEST_PORT\n")
    body += textwrap.indent(textwrap.dedent(CHECKS[check]), "      ")
    pod = _pod_spec(body)
    b = _builder(pod)
    outcome = _stage(_port_spec(pod)).evaluate(_pool(U.complete_offer([U.unreserved_ports(10000, 10000)])), b)
    assert outcome.passing
    recs = outcome.get_offer_recommendations()
    if overlay:
        assert recs == []
    else:
        assert len(recs) == 1
        op = recs[0].get_operation()
        assert op.type == P.Offer.Operation.RESERVE
        rg = op.reserve.resources[0].ranges.range[0]
        assert (rg.begin, rg.end) == (10000, 10000)
    t = b.get_task_builders()[0]
    assert _env(t.command.environment)["PORT_TEST_PORT"] == "10000"
    check_env = t.health_check.command.environment if check == "health" else t.check.command.command.environment
    assert [v.value for v in check_env.variables if v.name == "PORT_TEST_PORT"] == ["10000"]


def _dynamic_pod(extra="", ranges=None):
    ports = "TEST:\n  port: 0\n  env-key: PORT_TEST\n"
    if ranges:
        ports += "  ranges:\n" + "".join(
            f"    - begin: {b}\n" + (f"      end: {e}\n" if e is not None else "") for b, e in ranges)
    return _pod_spec(_task_yaml(extra, ports))


def test_dynamic_port_is_sticky_until_permanent_replacement():
    pod = _dynamic_pod()
    spec = _port_spec(pod)
    b = _builder(pod)
    assert _stage(spec).evaluate(_pool(U.get_offer([U.unreserved_ports(10000, 10050)])), b).passing
    _discovery_port(_task(b), "TEST", 10000)  # the lowest available port
    current = P.TaskInfo()
    current.CopyFrom(_task(b))

    # restart: the prior port must come back; an offer without it fails
    without_prior = U.get_offer([U.unreserved_ports(10001, 10050)])
    assert not _stage(spec).evaluate(_pool(without_prior), _builder(pod, [current])).passing

    # permanent replacement forgets the prior port
    L.TaskLabelWriter(current).set_permanently_failed().apply()
    assert _stage(spec).evaluate(_pool(without_prior), _builder(pod, [current])).passing


PUBLIC = "slave_public"
PUBLIC_POD = "  pre-reserved-role: slave_public\n"


def test_dynamic_port_with_pre_reserved_role_needs_that_role():
    pod = _dynamic_pod(PUBLIC_POD)
    assert _port_spec(pod).pre_reserved_role == PUBLIC
    assert not _stage(_port_spec(pod)).evaluate(
        _pool(U.get_offer([U.unreserved_ports(10000, 10050)])), _builder(pod)).passing


def _public_offer(begin, end):
    return U.complete_offer([U.prereserved_port(begin, end, PUBLIC)], pre_reserved_role=PUBLIC)


@pytest.mark.parametrize("offered,ranges,passing", [
    ((23, 5050), None, True),
    ((23, 5050), [(25, 600)], True),               # port 25 matches
    ((23, 5050), [(6000, 8000)], False),           # nothing in range
    ((23, 5050), [(6000, 8000), (2, 21)], False),  # in neither range
    ((3000, 5050), [(1024, None)], True),          # unbounded upper end
    ((3000, 5050), [(2000, 3000)], True),          # inclusive upper bound
    ((3000, 5050), [(5050, 6000)], True),          # inclusive lower bound
])
def test_dynamic_port_ranges_with_pre_reserved_role(offered, ranges, passing):
    pod = _dynamic_pod(PUBLIC_POD, ranges)
    b = _builder(pod)
    outcome = _stage(_port_spec(pod)).evaluate(_pool(_public_offer(*offered), PUBLIC), b)
    assert outcome.passing is passing
    if passing and ranges:
        lo = max(offered[0], ranges[0][0])
        _discovery_port(_task(b), "TEST", lo)


def test_unbounded_range_spec_ends_at_max_port():
    pod = _dynamic_pod(ranges=[(1024, None)])
    assert _port_spec(pod).ranges == (RangeSpec(1024, RangeSpec.MAX_PORT),)


# ---------------------------------------------------------------------------------------
# NamedVIPEvaluationStage


def _vip_spec(task_port, networks):
    return NamedVIPSpec(name="ports", value=ranges_value([(task_port, task_port)]), role=U.ROLE,
                        principal=U.PRINCIPAL, pre_reserved_role=ANY_ROLE,
                        env_key=f"{U.PORT_ENV_NAME}_VIP_{task_port}", port_name=f"test-vip-{task_port}",
                        visibility=P.DiscoveryInfo.EXTERNAL, network_names=tuple(networks), protocol="sctp",
                        vip_name="test-vip", vip_port=80)


def _vip_builder(task_port, networks):
    extra = "".join(f"  networks:\n    {n}: {{}}\n" for n in networks)
    pod = _pod_spec(_task_yaml(extra, f"test-vip-{task_port}:\n  port: {task_port}\n  vip:\n    port: 80\n"))
    rs = pod.tasks[0].resource_set
    rs = dataclasses.replace(rs, resources=tuple(r for r in rs.resources if not isinstance(r, PortSpec))
                             + (_vip_spec(task_port, networks),))
    pod = dataclasses.replace(pod, tasks=(dataclasses.replace(pod.tasks[0], resource_set=rs),))
    return _builder(pod)


@pytest.mark.parametrize("task_port,network,resources,scope,number", [
    (10000, None, 1, None, 10000),
    (80, "dcos", 0, "container", 80),                                      # overlay: no port resource
    (10000, "mesos-bridge", 1, "host", 10000),                             # bridge still reserves
    (0, "dcos", 0, "container", dcos.OVERLAY_DYNAMIC_PORT_RANGE_START),    # dynamic overlay port
])
def test_vip_discovery_info(task_port, network, resources, scope, number):
    networks = [network] if network else []
    b = _vip_builder(task_port, networks)
    stage = NamedVIPEvaluationStage(_vip_spec(task_port, networks), [TASK], None, None, None)
    assert stage.evaluate(_pool(U.get_offer([U.unreserved_ports(10000, 10000)])), b).passing
    t = _task(b)
    assert t.discovery.name == f"{POD}-0-{TASK}"
    assert t.discovery.visibility == P.DiscoveryInfo.CLUSTER
    assert len(t.resources) == resources
    port = t.discovery.ports.ports[0]
    assert (port.number, port.protocol) == (number, "sctp")
    labels = list(port.labels.labels)
    assert len(labels) == (1 if scope is None else 2)
    assert labels[0].key.startswith("VIP_") and labels[0].value == "test-vip:80"
    assert L.get_vips_from_labels(port) == [("test-vip", 80)]
    if scope is not None:
        assert (labels[1].key, labels[1].value) == ("network-scope", scope)


# ---------------------------------------------------------------------------------------
# LaunchEvaluationStage


def _launch_builder():
    return _builder(_pod_spec(_task_yaml().replace("cpus: 1.0\n", "cpus: 1.0\n      labels: label1:label1-value\n")))


def test_launch_passes_with_sorted_labels():
    b = _launch_builder()
    offer = U.get_offer([U.unreserved_cpus(2.0)])
    assert LaunchEvaluationStage(U.SERVICE_NAME, TASK, True).evaluate(_pool(offer), b).passing
    labels = [(l.key, l.value) for l in _task(b).labels.labels]
    assert [k for k, _ in labels] == ["index", "label1", "offer_attributes", "offer_hostname",
                                      "target_configuration", "task_type"]
    values = dict(labels)
    assert values["index"] == "0" and values["label1"] == "label1-value"
    assert values["offer_attributes"] == "" and values["offer_hostname"] == U.HOSTNAME
    assert len(values["target_configuration"]) == 36 and values["task_type"] == POD


def test_launch_injects_region_and_zone():
    b = _launch_builder()
    offer = U.get_offer([U.unreserved_cpus(2.0)])
    offer.domain.CopyFrom(U.LOCAL_DOMAIN_INFO)
    LaunchEvaluationStage(U.SERVICE_NAME, TASK, True).evaluate(_pool(offer), b)
    env = _env(_task(b).command.environment)
    assert env[L.REGION_TASKENV] == U.LOCAL_REGION and env[L.ZONE_TASKENV] == U.ZONE


def test_launch_without_domain_injects_nothing():
    b = _launch_builder()
    LaunchEvaluationStage(U.SERVICE_NAME, TASK, True).evaluate(_pool(U.get_offer([U.unreserved_cpus(2.0)])), b)
    env = _env(_task(b).command.environment)
    assert L.REGION_TASKENV not in env and L.ZONE_TASKENV not in env


def test_launch_recommendations():
    b = _launch_builder()
    outcome = LaunchEvaluationStage(U.SERVICE_NAME, TASK, True).evaluate(_pool(U.get_offer()), b)
    kinds = [type(r).__name__ for r in outcome.get_offer_recommendations()]
    assert kinds == ["LaunchOfferRecommendation", "StoreTaskInfoRecommendation"]
    assert _task(b).task_id.value.startswith(f"{U.SERVICE_NAME}__{POD}-0-{TASK}__")
    outcome = LaunchEvaluationStage(U.SERVICE_NAME, TASK, False).evaluate(_pool(U.get_offer()), _launch_builder())
    assert [type(r).__name__ for r in outcome.get_offer_recommendations()] == ["StoreTaskInfoRecommendation"]


# ---------------------------------------------------------------------------------------
# ExecutorEvaluationStage


EXECUTOR_ID = P.ExecutorID(value=f"{POD}__{uuid.uuid4()}")


def test_offer_without_the_expected_executor_is_rejected():
    b = _launch_builder()
    outcome = ExecutorEvaluationStage(U.SERVICE_NAME, EXECUTOR_ID).evaluate(_pool(U.complete_offer()), b)
    assert not outcome.passing


def test_offer_with_the_expected_executor_is_accepted():
    b = _launch_builder()
    offer = U.complete_offer()
    offer.executor_ids.add().CopyFrom(EXECUTOR_ID)
    assert ExecutorEvaluationStage(U.SERVICE_NAME, EXECUTOR_ID).evaluate(_pool(offer), b).passing
    assert b.get_executor_builder().executor_id == EXECUTOR_ID


def test_new_executor_gets_a_generated_id():
    b = _launch_builder()
    assert ExecutorEvaluationStage(U.SERVICE_NAME, None).evaluate(_pool(U.complete_offer()), b).passing
    assert b.get_executor_builder().executor_id.value.startswith(f"{U.SERVICE_NAME}__{POD}__")


# ---------------------------------------------------------------------------------------
# OfferEvaluationUtils.evaluateSimpleResource


RESOURCE = "blocks"


class FakePool:
    """Answers consume calls from a table keyed on (method, amount, resource id / role)."""

    def __init__(self, reserved=None, merged=None):
        self.offer = U.get_offer()
        self.reserved = reserved or {}
        self.merged = merged or {}

    def consume_reserved(self, name, value, resource_id):
        assert name == RESOURCE
        return self.reserved.get((value.scalar.value, resource_id))

    def consume_reservable_merged(self, name, value, role):
        assert name == RESOURCE and role == ANY_ROLE
        return self.merged.get(value.scalar.value)


def _blocks(v):
    return ResourceSpec(name=RESOURCE, value=U.scalar_value(v), role="svc-role", principal="svc-principal")


def _reserved_blocks(v, rid, ns, fid):
    return MesosResource(ResourceBuilder.from_spec(_blocks(v), rid, ns, fid).build())


def _unreserved_blocks(v):
    return MesosResource(ResourceBuilder.from_unreserved_value(RESOURCE, U.scalar_value(v)).build())


LABELS = [(None, None), ("foo", FRAMEWORK_ID)]


@pytest.mark.parametrize("ns,fid", LABELS)
@pytest.mark.parametrize("existing", [False, True])
def test_simple_resource_insufficient(existing, ns, fid):
    rid = str(uuid.uuid4()) if existing else None
    res = evaluate_simple_resource(object(), _blocks(5), rid, ns, FakePool(), fid)
    assert not res.outcome.passing and res.outcome.get_offer_recommendations() == [] and res.resource_id is None


def _check_labels(resource, ns, fid):
    assert get_namespace(resource) == ns
    assert get_framework_id(resource) == fid


@pytest.mark.parametrize("ns,fid", LABELS)
@pytest.mark.parametrize("existing", [False, True])
def test_simple_resource_sufficient(existing, ns, fid):
    rid = str(uuid.uuid4()) if existing else None
    pool = FakePool(reserved={(5.0, rid): _reserved_blocks(5, rid, ns, fid)} if existing else None,
                    merged=None if existing else {5.0: _unreserved_blocks(5)})
    res = evaluate_simple_resource(object(), _blocks(5), rid, ns, pool, fid)
    assert res.outcome.passing
    if existing:
        assert res.outcome.get_offer_recommendations() == [] and res.resource_id == rid
    else:
        rec = res.outcome.get_offer_recommendations()[0]
        assert isinstance(rec, ReserveOfferRecommendation) and res.resource_id is not None
        r = rec.get_operation().reserve.resources[0]
        assert r.scalar.value == 5.0
        _check_labels(r, ns, fid)


@pytest.mark.parametrize("ns,fid", LABELS)
@pytest.mark.parametrize("extra_available", [True, False])
def test_simple_resource_increase(extra_available, ns, fid):
    rid = str(uuid.uuid4())
    pool = FakePool(reserved={(5.0, rid): _reserved_blocks(4, rid, ns, fid)},
                    merged={1.0: _unreserved_blocks(1)} if extra_available else None)
    res = evaluate_simple_resource(object(), _blocks(5), rid, ns, pool, fid)
    assert res.outcome.passing is extra_available
    if not extra_available:
        assert res.outcome.get_offer_recommendations() == [] and res.resource_id is None
        return
    rec = res.outcome.get_offer_recommendations()[0]
    assert isinstance(rec, ReserveOfferRecommendation) and res.resource_id == rid
    r = rec.get_operation().reserve.resources[0]
    assert r.scalar.value == 1.0
    _check_labels(r, ns, fid)


@pytest.mark.parametrize("ns,fid", LABELS)
def test_simple_resource_decrease(ns, fid):
    rid = str(uuid.uuid4())
    pool = FakePool(reserved={(4.0, rid): _reserved_blocks(5, rid, ns, fid)})
    res = evaluate_simple_resource(object(), _blocks(4), rid, ns, pool, fid)
    assert res.outcome.passing
    rec = res.outcome.get_offer_recommendations()[0]
    assert isinstance(rec, UnreserveOfferRecommendation) and res.resource_id == rid
    r = rec.get_operation().unreserve.resources[0]
    assert r.scalar.value == 1.0
    _check_labels(r, ns, fid)


# ---------------------------------------------------------------------------------------
# TaskPortLookup (PodInfoBuilder.get_prior_port_for_task)


def test_prior_port_lookup():
    pod = _dynamic_pod()
    spec = dataclasses.replace(_port_spec(pod), port_name="new-test-port")
    empty = P.TaskInfo(name=f"{POD}-0-{TASK}")
    assert _builder(pod, [empty]).get_prior_port_for_task(TASK, spec) is None
    with_port = P.TaskInfo()
    with_port.CopyFrom(empty)
    with_port.discovery.visibility = P.DiscoveryInfo.CLUSTER
    with_port.discovery.ports.ports.add(name="new-test-port", number=12345)
    assert _builder(pod, [with_port]).get_prior_port_for_task(TASK, spec) == 12345


# ---------------------------------------------------------------------------------------
# VolumeEvaluationStage


def _mount_pod(size):
    return _pod_spec(_task_yaml().replace(
        "cpus: 1.0\n", f"cpus: 1.0\n      volume:\n        path: {U.CONTAINER_PATH}\n        type: MOUNT\n"
                       f"        size: {size}\n"))


def test_mount_volume_create_succeeds():
    offered = U.unreserved_mount_volume(2000)
    pod = _mount_pod(1000)
    stage = VolumeEvaluationStage.get_new(pod.tasks[0].resource_set.volumes[0], [TASK], None, FRAMEWORK_ID)
    outcome = stage.evaluate(_pool(U.complete_offer([offered])), _builder(pod))
    assert outcome.passing
    reserve, create = outcome.get_offer_recommendations()
    assert reserve.get_operation().type == P.Offer.Operation.RESERVE
    r = reserve.get_operation().reserve.resources[0]
    assert r.name == "disk" and r.scalar == offered.scalar  # a MOUNT disk is taken whole
    rid = L.labels_to_map(r.reservations[-1].labels)["resource_id"]
    assert rid
    assert create.get_operation().type == P.Offer.Operation.CREATE
    v = create.get_operation().create.volumes[0]
    assert v.name == "disk" and v.scalar == offered.scalar
    assert L.labels_to_map(v.reservations[-1].labels)["resource_id"] == rid
    assert v.disk.persistence.id != ""


def test_mount_volume_too_small_fails():
    pod = _mount_pod(2000)
    stage = VolumeEvaluationStage.get_new(pod.tasks[0].resource_set.volumes[0], [TASK], None, FRAMEWORK_ID)
    outcome = stage.evaluate(_pool(U.complete_offer([U.unreserved_mount_volume(1000)])), _builder(pod))
    assert not outcome.passing and outcome.get_offer_recommendations() == []


# ---------------------------------------------------------------------------------------
# PlacementRuleEvaluationStage


@pytest.mark.parametrize("agent,passing", [("test-agent", True), ("other-agent", False)])
def test_placement_rule_stage(agent, passing):
    offer = U.complete_offer([U.unreserved_cpus(1.0)])
    offer.agent_id.value = agent
    pool = _pool(offer)
    rule = AgentRule.require("test-agent")
    pod = dataclasses.replace(_pod_spec(_task_yaml()), placement_rule=rule)
    assert PlacementRuleEvaluationStage([], rule).evaluate(pool, _builder(pod)).passing is passing
    merged = pool.unreserved_merged_pool()
    assert len(merged) == 3 and abs(merged["cpus"].scalar.value - 1.1) < 0.01  # nothing consumed


# ---------------------------------------------------------------------------------------
# TLSEvaluationStage


class RecordingUpdater:
    def __init__(self, error=None):
        self.calls = []
        self.error = error

    def update(self, paths, names, tls_name):
        self.calls.append(tls_name)
        if self.error is not None:
            raise self.error


def _tls_builder(tls_type):
    return _builder(_pod_spec(_task_yaml() + textwrap.indent(textwrap.dedent(f"""\
        transport-encryption:
          - name: test-tls
            type: {tls_type}
        """), "      ")))


def _tls_paths(b):
    pi = b.pod_instance
    names = CertificateNamesGenerator(U.SERVICE_NAME, pi.pod.tasks[0], pi, CFG)
    return TLSArtifactPaths("test-namespace", f"{POD}-0-{TASK}", names.sans_hash())


def _secret_at(container, path):
    for v in container.volumes:
        if v.container_path == path:
            return v.source.secret.reference.name
    return None


def _tls_stage(updater):
    return TLSEvaluationStage(U.SERVICE_NAME, TASK, "test-namespace", updater, CFG)


@pytest.mark.parametrize("tls_type,mounted,absent", [
    ("TLS", [TLSArtifact.CERTIFICATE, TLSArtifact.CA_CERTIFICATE, TLSArtifact.PRIVATE_KEY],
     [TLSArtifact.KEYSTORE, TLSArtifact.TRUSTSTORE]),
    ("KEYSTORE", [TLSArtifact.KEYSTORE, TLSArtifact.TRUSTSTORE],
     [TLSArtifact.CERTIFICATE, TLSArtifact.CA_CERTIFICATE, TLSArtifact.PRIVATE_KEY]),
])
def test_tls_artifacts_are_mounted(tls_type, mounted, absent):
    updater = RecordingUpdater()
    b = _tls_builder(tls_type)
    assert _tls_stage(updater).evaluate(_pool(U.get_offer([U.unreserved_cpus(2.0)])), b).passing
    assert updater.calls == ["test-tls"]
    assert len(b.get_executor_builder().container.volumes) == 0
    paths = _tls_paths(b)
    container = _task(b).container
    for a in mounted:
        assert _secret_at(container, a.mount_path("test-tls")) == paths.get_secret_store_path(a, "test-tls")
    for a in absent:
        assert _secret_at(container, a.mount_path("test-tls")) is None


def test_tls_update_failure_fails_the_offer():
    b = _tls_builder("TLS")
    stage = _tls_stage(RecordingUpdater(IOError("test")))
    assert not stage.evaluate(_pool(U.get_offer([U.unreserved_cpus(2.0)])), b).passing


def test_repeated_tls_evaluation_adds_no_volumes():
    b = _tls_builder("TLS")
    stage = _tls_stage(RecordingUpdater())
    offer = U.get_offer([U.unreserved_cpus(2.0)])
    assert stage.evaluate(_pool(offer), b).passing
    before = len(_task(b).container.volumes)
    assert stage.evaluate(_pool(offer), b).passing
    assert len(_task(b).container.volumes) == before


def test_task_without_tls_passes_untouched():
    updater = RecordingUpdater()
    b = _launch_builder()
    assert _tls_stage(updater).evaluate(_pool(U.get_offer()), b).passing and updater.calls == []


def test_pod_info_builder_clone_is_an_independent_fresh_build():
    pod = _pod_spec(_task_yaml(ports="""\
        http:
          port: 0
    """))
    proto = _builder(pod)
    fresh = _builder(pod)
    a, b = proto.clone(), proto.clone()
    a.get_task_builder(TASK).command.value = "changed"
    a.add_assigned_overlay_port(1234)
    a.get_executor_builder().executor_id.value = "exec"
    assert b.get_task_builder(TASK).command.value == fresh.get_task_builder(TASK).command.value == "./cmd"
    assert not b.is_assigned_overlay_port(1234) and not proto.is_assigned_overlay_port(1234)
    assert proto.get_executor_builder().executor_id.value == ""
    # labels other than the target configuration (random per build here) match a fresh build
    assert b.get_task_builder(TASK).name == fresh.get_task_builder(TASK).name
    assert b.get_task_builder(TASK).container == fresh.get_task_builder(TASK).container
