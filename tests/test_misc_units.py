"""Small reference units not pinned elsewhere: strict YAML maps, property (de)serializers, VIP
specs, multi-service template URLs, agent/hostname/zone/region/invalid placement rules, the
ZoneValidator and TaskEnvCannotChange transition matrices, the API server's routing and DNS
check, the multi-service schema check, and step state across a scheduler restart.

Mirrors sdk/scheduler/src/test/java/com/mesosphere/sdk/{specification/yaml/WriteOnceLinkedHashMapTest,
http/types/StringPropertyDeserializerTest, state/JsonSerializerTest, specification/DefaultVipSpecTest,
http/endpoints/{ArtifactResourceTest,MultiArtifactResourceTest}, offer/evaluate/placement/{AgentRuleTest,HostnameRuleTest,
ZoneRuleTest,RegionRuleTest,InvalidPlacementRuleTest}, specification/validation/ZoneValidatorTest,
config/validate/TaskEnvCannotChangeTest, framework/ApiServerTest, scheduler/multi/MultiServiceRunnerTest}.java
and frameworks/helloworld/.../SchedulerRestartServiceTest.java.
"""
import json
import os
import threading
import urllib.error
import urllib.request
import uuid

import pytest

import testutils as U
from dcos_commons_amd.config import validate as V
from dcos_commons_amd.http import endpoint_utils
from dcos_commons_amd.http.api import Route, plain
from dcos_commons_amd.http.server import ApiServer, resolve_scheduler_dns
from dcos_commons_amd.mesos import protos as P
from dcos_commons_amd.offer.evaluate import placement as PL
from dcos_commons_amd.scheduler.multi import MultiServiceRunner
from dcos_commons_amd.scheduler.plan.status import Status
from dcos_commons_amd.scheduler.scheduler_config import SchedulerConfig
from dcos_commons_amd.specification.specs import SpecValidationError, VipSpec
from dcos_commons_amd.specification.yaml.raw import RawSpecError, load_yaml_strict
from dcos_commons_amd.state.serializer import JsonSerializer, StringPropertyDeserializer
from dcos_commons_amd.storage.mem_persister import MemPersister
from dcos_commons_amd.testing import Expect, Send, ServiceTestRunner
from test_config_validators import _task, spec

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

# ---------------------------------------------------------------------------------------
# strict YAML maps, serializers, VIP specs


def test_yaml_maps_are_write_once():
    assert load_yaml_strict("a: b\nc: d\n") == {"a": "b", "c": "d"}
    with pytest.raises(RawSpecError):
        load_yaml_strict("a: b\na: d\n")


def test_string_property_deserializer_shows_the_stored_json():
    assert StringPropertyDeserializer().to_json_string("key", JsonSerializer().serialize(False)) == "false"


@pytest.mark.parametrize("value,cls", [(12, int), ("dcos dcos dcos", str), (False, bool)])
def test_json_serializer_round_trip(value, cls):
    s = JsonSerializer()
    assert s.deserialize(s.serialize(value), cls) == value


def test_json_serializer_rejects_broken_json():
    with pytest.raises(ValueError):
        JsonSerializer().deserialize(b'" broken json', str)


def test_vip_spec():
    vip = VipSpec(application_port=0, vip_name="mysvc.mesos", vip_port=0)
    assert VipSpec.from_dict(json.loads(json.dumps(vip.to_dict()))) == vip
    with pytest.raises(SpecValidationError):
        VipSpec(application_port=-1, vip_name="", vip_port=-1)


# ---------------------------------------------------------------------------------------
# multi-service template URLs

ARTIFACT_CFG = SchedulerConfig.for_testing(PORT_API=1234, SERVICE_TLD="some.tld", MARATHON_NAME="test-marathon")


@pytest.mark.parametrize("service,host", [("svc-name", "svc-name"), ("/path/to/svc-name", "svc-name-to-path")])
def test_standalone_template_url(service, host):
    """ArtifactResourceTest: a single service's templates come from its own /v1/artifacts."""
    config_id = uuid.uuid4()
    url = endpoint_utils.template_url_factory(service, ARTIFACT_CFG)(config_id, "some-pod", "some-task", "some-config")
    assert url == (f"http://{host}.test-marathon.some.tld:1234/v1/artifacts/template/"
                   f"{config_id}/some-pod/some-task/some-config")


@pytest.mark.parametrize("framework,service,host,path", [
    ("fwk-name", "job-name", "fwk-name", "job-name"),
    ("/path/to/fwk-name", "/path/to/job-name", "fwk-name-to-path", "path.to.job-name"),
])
def test_multi_service_template_url(framework, service, host, path):
    config_id = uuid.uuid4()
    url = endpoint_utils.template_url_factory(framework, ARTIFACT_CFG, prefix=service)(
        config_id, "some-pod", "some-task", "some-config")
    assert url == (f"http://{host}.test-marathon.some.tld:1234/v1/service/{path}/artifacts/template/"
                   f"{config_id}/some-pod/some-task/some-config")


# ---------------------------------------------------------------------------------------
# agent / hostname / zone / region / invalid rules

AGENTS = ["agent-1-uuid", "agent-2-uuid", "agent-3-uuid"]
HOSTS = ["host-1-uuid", "host-2-uuid", "host-3-uuid"]
POD = type("PodInstance", (), {"name": "type-0", "index": 0})()


def _offer_on(agent=U.AGENT_ID.value, host=U.HOSTNAME):
    o = U.get_offer([U.unreserved_cpus(1.0), U.unreserved_mem(256), U.unreserved_disk(100)], hostname=host)
    o.agent_id.value = agent
    return o


def _passing(rule, offers):
    return [rule.filter(o, POD, []).passing for o in offers]


def _round_trips(rule):
    return PL.placement_rule_from_dict(json.loads(json.dumps(rule.to_dict()))) == rule


@pytest.mark.parametrize("chosen", [(0,), (1,), (0, 2), (1, 2)])
def test_agent_rule_require_and_avoid(chosen):
    offers = [_offer_on(agent=a) for a in AGENTS]
    ids = [AGENTS[i] for i in chosen]
    want = [i in chosen for i in range(3)]
    assert _passing(PL.AgentRule.require(*ids), offers) == want
    assert _passing(PL.AgentRule.avoid(*ids), offers) == [not w for w in want]
    assert _round_trips(PL.AgentRule.require(*ids)) and _round_trips(PL.AgentRule.avoid(*ids))


@pytest.mark.parametrize("chosen", [(0,), (1,), (0, 2), (1, 2)])
def test_hostname_rule_require_and_avoid(chosen):
    offers = [_offer_on(host=h) for h in HOSTS]
    matchers = [PL.ExactMatcher(HOSTS[i]) for i in chosen]
    want = [i in chosen for i in range(3)]
    assert _passing(PL.HostnameRuleFactory.require(*matchers), offers) == want
    assert _passing(PL.HostnameRuleFactory.avoid(*matchers), offers) == [not w for w in want]
    assert _passing(PL.HostnameRuleFactory.require(matchers), offers) == want  # a collection works too
    assert _round_trips(PL.HostnameRuleFactory.require(*matchers))
    assert _round_trips(PL.HostnameRuleFactory.avoid(*matchers))


@pytest.mark.parametrize("cls,key", [(PL.ZoneRule, U.ZONE), (PL.RegionRule, U.LOCAL_REGION)])
def test_zone_and_region_rule_keys(cls, key):
    rule = cls(PL.ExactMatcher(key))
    assert _round_trips(rule)
    assert rule.keys(U.empty_offer()) == []
    with_domain = U.empty_offer()
    with_domain.domain.CopyFrom(U.LOCAL_DOMAIN_INFO)
    assert rule.keys(with_domain) == [key]
    assert rule.filter(with_domain, POD, []).passing and not rule.filter(U.empty_offer(), POD, []).passing


def test_invalid_placement_rule_round_trips_and_never_passes():
    rule = PL.InvalidPlacementRule("constraint", "exception")
    assert _round_trips(rule)
    assert not rule.filter(_offer_on(), POD, []).passing


# ---------------------------------------------------------------------------------------
# ZoneValidator and TaskEnvCannotChange transition matrices

_PLACEMENTS = {
    "empty": "",
    "zones": "placement: '[[\"@zone\", \"GROUP_BY\", \"3\"]]'\n",
    "hosts": "placement: '[[\"hostname\", \"IS\", \"hostname\"]]'\n",
}


@pytest.mark.parametrize("old,new,n", [
    (None, "zones", 0), ("empty", "empty", 0), ("empty", "zones", 1), ("empty", "hosts", 0),
    ("zones", "hosts", 1), ("hosts", "zones", 1), ("zones", "zones", 0), ("hosts", "hosts", 0),
])
def test_zone_validator_transitions(old, new, n):
    def mk(p):
        return spec({"pod-type": (1, _PLACEMENTS[p], _task("test-task-name"))})

    assert len(V.ZoneValidator("pod-type").validate(None if old is None else mk(old), mk(new))) == n


def _env(v):
    return spec({"pod": (1, "", _task("task", extra=f"env:\n  SOME_ENV: '{v}'\n" if v is not None else ""))})


_STATES = {"unset": None, "empty": "", "val": "val", "val2": "val2"}
_PAIRS = [("unset", "unset"), ("unset", "empty"), ("unset", "val"), ("empty", "unset"), ("empty", "empty"),
          ("empty", "val"), ("val", "unset"), ("val", "empty"), ("val", "val"), ("val", "val2"), ("val2", "val")]
_U2S, _S2U = V.TaskEnvCannotChange.ALLOW_UNSET_TO_SET, V.TaskEnvCannotChange.ALLOW_SET_TO_UNSET


@pytest.mark.parametrize("rules,expected", [
    ((), [0, 0, 1, 0, 0, 1, 1, 1, 0, 1, 1]),
    ((_U2S,), [0, 0, 0, 0, 0, 0, 1, 1, 0, 1, 1]),
    ((_S2U,), [0, 0, 1, 0, 0, 1, 0, 0, 0, 1, 1]),
    ((_U2S, _S2U), [0, 0, 0, 0, 0, 0, 0, 0, 0, 1, 1]),
])
def test_task_env_transition_matrix(rules, expected):
    v = V.TaskEnvCannotChange("pod", "task", "SOME_ENV", *rules)
    specs = {k: _env(val) for k, val in _STATES.items()}
    for k in ("unset", "empty", "val"):
        assert v.validate(None, specs[k]) == []
    assert [len(v.validate(specs[a], specs[b])) for a, b in _PAIRS] == expected


# ---------------------------------------------------------------------------------------
# API server


def test_scheduler_dns_resolution():
    assert resolve_scheduler_dns("localhost", "127.0.0.1")
    assert not resolve_scheduler_dns("localhost", "10.255.255.1")  # resolves, but to another address
    assert not resolve_scheduler_dns("no-such-host.invalid", "127.0.0.1")


class _Plans:
    def routes(self):
        return [Route("GET", "/v1/plans/{plan}", lambda r: plain(f"Service Plan: {r.params['plan']}")),
                Route("GET", "/v1/pod/{name}/info", lambda r: plain(f"Service Pod: {r.params['name']}")),
                Route("GET", "/v1/service/{svc}/plans/{plan}",
                      lambda r: plain(f"{r.params['svc']} Plan: {r.params['plan']}")),
                Route("GET", "/v1/service/{svc}/pod/{name}/info",
                      lambda r: plain(f"{r.params['svc']} Pod: {r.params['name']}"))]


def test_api_server_endpoint_handling():
    started = threading.Event()
    srv = ApiServer.start(SchedulerConfig.for_testing(), [_Plans()], started.set, port=0)
    try:
        assert started.wait(30)
        expected = {
            "/v1/metrics": "", "/v1/metrics/prometheus": "",
            "/v1/plans/foo": "Service Plan: foo", "/v1/plans/bar": "Service Plan: bar",
            "/v1/pod/foo/info": "Service Pod: foo", "/v1/pod/bar/info": "Service Pod: bar",
            "/v1/service/fast/plans/foo": "fast Plan: foo", "/v1/service/slow/plans/bar": "slow Plan: bar",
            "/v1/service/path/to/svc/plans/foo": None,  # slashes in a service name are not routed
            "/v1/service/fast/pod/foo/info": "fast Pod: foo", "/v1/service/slow/pod/foo/info": "slow Pod: foo",
            "/v1/service/path/to/svc/pod/foo/info": None,
        }
        for path, body in expected.items():
            try:
                with urllib.request.urlopen(f"http://127.0.0.1:{srv.port}{path}", timeout=10) as r:
                    status, text = r.status, r.read().decode()
            except urllib.error.HTTPError as e:
                status, text = e.code, ""
            if body is None:
                assert status == 404, path
            else:
                assert status == 200, path
                assert body == "" or text == body, path
    finally:
        srv.stop()


# ---------------------------------------------------------------------------------------
# multi-service schema check


@pytest.mark.parametrize("stored,ok", [(b"123", False), (b"1", False), (b"2", True), (None, True)])
def test_multi_service_runner_checks_the_schema_version(stored, ok):
    persister = MemPersister()
    if stored is not None:
        persister.set("SchemaVersion", stored)
    if ok:
        MultiServiceRunner(None, None, persister, None)
        assert persister.get("SchemaVersion") == b"2"
    else:
        with pytest.raises(ValueError, match=stored.decode()):
            MultiServiceRunner(None, None, persister, None)


# ---------------------------------------------------------------------------------------
# step state across a scheduler restart

SVC = os.path.join(ROOT, "frameworks", "helloworld", "specs", "svc.yml")
ENV = dict(FRAMEWORK_NAME="hello-world", FRAMEWORK_PRINCIPAL="hello-world-principal", FRAMEWORK_USER="nobody",
           HELLO_COUNT="1", HELLO_PLACEMENT='[["hostname", "UNIQUE"]]', HELLO_CPUS="0.1", HELLO_MEM="252",
           HELLO_DISK="25", SLEEP_DURATION="1000", WORLD_COUNT="1", WORLD_PLACEMENT='[["hostname", "UNIQUE"]]',
           WORLD_CPUS="0.2", WORLD_MEM="512", WORLD_DISK="25", WORLD_READINESS_CHECK_INTERVAL="5",
           WORLD_READINESS_CHECK_DELAY="0", WORLD_READINESS_CHECK_TIMEOUT="10")


def _runner():
    return ServiceTestRunner(SVC).set_env(ENV).set_scheduler_env(SDK_REVIVE_INTERVAL_S="0")


@pytest.mark.parametrize("readiness_exit,after_check,after_restart", [
    (1, Status.STARTED, Status.PENDING),   # a failing readiness check is re-run after the restart
    (0, Status.COMPLETE, Status.COMPLETE),
])
def test_readiness_outcome_survives_a_scheduler_restart(readiness_exit, after_check, after_restart):
    step = "world-0:[server]"
    first = _runner().run([
        Send.register(),
        Expect.reconciled_implicitly(),
        Send.offer_builder("hello").build(),
        Expect.launched_tasks("hello-0-server"),
        Send.offer_builder("world").build(),
        Expect.declined_last_offer(),
        Send.task_status("hello-0-server", P.TASK_RUNNING).build(),
        Send.offer_builder("world").build(),
        Expect.launched_tasks("world-0-server"),
        Expect.deploy_step_status("world", step, Status.STARTING),
        Send.task_status("world-0-server", P.TASK_RUNNING).set_readiness_check_exit_code(readiness_exit).build(),
        Expect.deploy_step_status("world", step, after_check),
        Send.offer_builder("world").build(),
        Expect.declined_last_offer(),
    ])
    _runner().set_state(first).run([
        Send.register(),
        Expect.reconciled_explicitly("hello-0-server", "world-0-server"),
        Expect.deploy_step_status("world", step, after_restart),
    ])
