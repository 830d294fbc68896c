"""Configuration validators and spec-level path validation.

Behavior pinned against the reference's config/validate test suite
(sdk/scheduler/src/test/java/com/mesosphere/sdk/config/validate/*Test.java): one test group per
validator, including the old=None (first deployment) cases, the capability-gated checks
(DefaultCapabilitiesTestSuite overrides) and VerifyHostVolumePathTest / VerifySecretFilePathTest.
Specs are built from YAML through the real raw→spec mappers.
"""
import dataclasses
import textwrap

import pytest

from dcos_commons_amd.config import validate as V
from dcos_commons_amd.dcos import capabilities
from dcos_commons_amd.offer.evaluate import placement as PL
from dcos_commons_amd.scheduler.scheduler_config import SchedulerConfig
from dcos_commons_amd.specification import specs as S
from dcos_commons_amd.specification.yaml import mappers
from dcos_commons_amd.specification.yaml.raw import RawServiceSpec

CFG = SchedulerConfig.for_testing()


def _task(name="server", cpus=0.1, extra=""):
    return textwrap.indent(textwrap.dedent(f"""\
        {name}:
          goal: RUNNING
          cmd: sleep 1000
          cpus: {cpus}
          memory: 32
        """) + textwrap.indent(textwrap.dedent(extra), "  "), "      ")


def spec(pods=None, name="svc", user=None, extra_top=""):
    """``pods`` maps pod type -> (count, extra pod yaml, task yaml)."""
    pods = pods or {"hello": (1, "", _task())}
    body = [f"name: {name}"]
    if user:
        body.append(f"scheduler:\n  principal: p\n  user: {user}")
    body.append("pods:")
    for t, (count, extra, tasks) in pods.items():
        body.append(f"  {t}:\n    count: {count}")
        if extra:
            body.append(textwrap.indent(textwrap.dedent(extra).rstrip("\n"), "    "))
        body.append("    tasks:\n" + tasks.rstrip("\n"))
    text = "\n".join(body) + "\n" + extra_top
    raw = RawServiceSpec.from_string(text)
    return mappers.ServiceSpecGenerator(raw, CFG, "/tmp", {}).build()


@pytest.fixture
def caps():
    """Capabilities.overrideCapabilities for one test."""
    saved = capabilities.get_instance()

    def set_(**kw):
        capabilities.override_capabilities(capabilities.Capabilities().with_overrides(**kw))
    yield set_
    capabilities.override_capabilities(saved)


def errs(validator, old, new):
    return validator.validate(old, new)


# ---------------------------------------------------------------------------------------
# ServiceNameCannotContainDoubleUnderscores / ServiceNameCannotBreakDNS


def renamed(s, **kw):
    return dataclasses.replace(s, **kw)


def test_double_underscore_name():
    v = V.ServiceNameCannotContainDoubleUnderscores()
    assert errs(v, None, spec(name="ok-name")) == []
    e = errs(v, None, renamed(spec(name="ok-name"), name="bad__name"))
    assert len(e) == 1 and "double underscores" in e[0].message and not e[0].is_fatal()


@pytest.mark.parametrize("name,n_errors", [
    ("a" * 63, 0),
    ("a" * 64, 1),
    ("/folder/" + "a" * 56, 0),      # slashes removed before counting: 62
    ("/" + "a" * 63, 0),
    ("/fo/" + "a" * 62, 1),
])
def test_service_name_dns_length(name, n_errors):
    assert len(errs(V.ServiceNameCannotBreakDNS(), None, spec(name=name))) == n_errors


def test_service_name_dns_only_checked_on_first_deploy():
    long = spec(name="a" * 70)
    assert errs(V.ServiceNameCannotBreakDNS(), long, long) == []


# ---------------------------------------------------------------------------------------
# PodSpecsCannotShrink


def test_pods_cannot_shrink():
    v = V.PodSpecsCannotShrink()
    two = spec({"hello": (2, "", _task())})
    one = spec({"hello": (1, "", _task())})
    assert errs(v, None, one) == []
    assert errs(v, one, two) == []                      # grow ok
    e = errs(v, two, one)
    assert len(e) == 1 and "has 1 tasks, expected >=2 tasks" in e[0].message


def test_pods_can_shrink_with_allow_decommission():
    v = V.PodSpecsCannotShrink()
    two = spec({"hello": (2, "allow-decommission: true\n", _task())})
    one = spec({"hello": (1, "allow-decommission: true\n", _task())})
    assert errs(v, two, one) == []


def test_pod_type_cannot_disappear_unless_decommissionable():
    v = V.PodSpecsCannotShrink()
    both = spec({"hello": (1, "", _task()), "world": (1, "", _task())})
    only_hello = spec({"hello": (1, "", _task())})
    e = errs(v, both, only_hello)
    assert len(e) == 1 and "missing PodSpec named 'world'" in e[0].message
    both_dec = spec({"hello": (1, "", _task()), "world": (1, "allow-decommission: true\n", _task())})
    assert errs(v, both_dec, only_hello) == []


# ---------------------------------------------------------------------------------------
# PodSpecsCannotUseUnsupportedFeatures / TaskSpecsCannotUseUnsupportedFeatures


def test_gpu_requires_capability(caps):
    gpu = spec({"hello": (1, "", _task(extra="gpus: 1\n"))})
    caps(supports_gpu_resource=True)
    assert errs(V.PodSpecsCannotUseUnsupportedFeatures(), None, gpu) == []
    caps(supports_gpu_resource=False)
    e = errs(V.PodSpecsCannotUseUnsupportedFeatures(), None, gpu)
    assert len(e) == 1 and "GPU" in e[0].message
    assert errs(V.PodSpecsCannotUseUnsupportedFeatures(), None, spec()) == []


def test_rlimits_require_capability(caps):
    rl = spec({"hello": (1, "rlimits:\n  RLIMIT_NOFILE:\n    soft: 128000\n    hard: 128000\n", _task())})
    caps(supports_rlimits=False)
    e = errs(V.PodSpecsCannotUseUnsupportedFeatures(), None, rl)
    assert [x.new_value for x in e] == ["rlimits"]
    caps(supports_rlimits=True)
    assert errs(V.PodSpecsCannotUseUnsupportedFeatures(), None, rl) == []


def test_secrets_require_capability(caps):
    env_secret = spec({"hello": (1, "secrets:\n  s1:\n    secret: path/s1\n    env-key: S1\n", _task())})
    file_secret = spec({"hello": (1, "secrets:\n  s1:\n    secret: path/s1\n    file: conf/s1\n", _task())})
    caps(supports_env_based_secrets=False, supports_file_based_secrets=True)
    assert len(errs(V.PodSpecsCannotUseUnsupportedFeatures(), None, env_secret)) == 1
    assert errs(V.PodSpecsCannotUseUnsupportedFeatures(), None, file_secret) == []
    caps(supports_env_based_secrets=True, supports_file_based_secrets=False)
    assert errs(V.PodSpecsCannotUseUnsupportedFeatures(), None, env_secret) == []
    assert len(errs(V.PodSpecsCannotUseUnsupportedFeatures(), None, file_secret)) == 1


def test_pre_reserved_role_requires_capability(caps):
    pr = spec({"hello": (1, "pre-reserved-role: slave_public\n", _task())})
    caps(supports_pre_reserved_resources=False)
    assert len(errs(V.PodSpecsCannotUseUnsupportedFeatures(), None, pr)) == 1
    caps(supports_pre_reserved_resources=True)
    assert errs(V.PodSpecsCannotUseUnsupportedFeatures(), None, pr) == []


def test_shm_requires_capability(caps):
    pod_shm = spec({"hello": (1, "ipc-mode: PRIVATE\nshm-size: 64\n", _task())})
    caps(supports_shm=False)
    assert len(errs(V.PodSpecsCannotUseUnsupportedFeatures(), None, pod_shm)) == 1
    caps(supports_shm=True)
    assert errs(V.PodSpecsCannotUseUnsupportedFeatures(), None, pod_shm) == []
    assert errs(V.TaskSpecsCannotUseUnsupportedFeatures(), None, spec()) == []


# ---------------------------------------------------------------------------------------
# PodSpecsCannotChangeNetworkRegime


def _net(name):
    return f"networks:\n  {name}:\n    host-ports: [8080]\n    container-ports: [80]\n" if name != "dcos" else \
        "networks:\n  dcos: {}\n"


def test_network_regime_cannot_change():
    v = V.PodSpecsCannotChangeNetworkRegime()
    host = spec({"hello": (1, "", _task())})
    overlay = spec({"hello": (1, _net("dcos"), _task())})
    assert errs(v, None, overlay) == []
    assert errs(v, host, host) == []
    assert errs(v, overlay, overlay) == []
    e = errs(v, host, overlay)
    assert len(e) == 1 and "changing its host ports requirements" in e[0].message
    assert len(errs(v, overlay, host)) == 1


def test_port_mapping_on_network_without_support_is_rejected():
    # The YAML mapper already refuses this; the validator guards specs built in code.
    v = V.PodSpecsCannotChangeNetworkRegime()
    old = spec({"hello": (1, _net("dcos"), _task())})
    pod = old.pods[0]
    mapped = dataclasses.replace(old, pods=[dataclasses.replace(
        pod, networks=(S.NetworkSpec("dcos", ((8080, 80),)),))])
    e = errs(v, old, mapped)
    assert any("do not support port mapping" in x.message for x in e)


# ---------------------------------------------------------------------------------------
# PreReservationCannotChange / UserCannotChange / RegionCannotChange / role


def test_pre_reservation_cannot_change():
    v = V.PreReservationCannotChange()
    a = spec({"hello": (1, "pre-reserved-role: slave_public\n", _task())})
    b = spec({"hello": (1, "pre-reserved-role: other\n", _task())})
    none = spec({"hello": (1, "", _task())})
    assert errs(v, None, a) == []
    assert errs(v, a, a) == []
    assert len(errs(v, a, b)) == 1
    assert len(errs(v, none, a)) == 1
    assert len(errs(v, a, none)) == 1


def test_service_user_cannot_change():
    v = V.UserCannotChange()
    root = spec(user="root")
    nobody = spec(user="nobody")
    assert errs(v, None, root) == []
    assert errs(v, root, root) == []
    e = errs(v, root, nobody)
    assert e and all(x.is_fatal() for x in e)
    assert "Cannot change user of deployed service from 'root' to 'nobody'" in e[0].message


def test_pod_user_cannot_change():
    v = V.UserCannotChange()
    base = spec(user="root")
    a = renamed(base, pods=[dataclasses.replace(base.pods[0], user="alice")])
    b = renamed(base, pods=[dataclasses.replace(base.pods[0], user="bob")])
    e = errs(v, a, b)
    assert len(e) == 1 and "existing pod type user from 'alice' to 'bob'" in e[0].message and e[0].is_fatal()


def test_region_cannot_change():
    v = V.RegionCannotChange()
    a, b = spec(), spec()
    assert errs(v, None, a) == []
    assert errs(v, a, b) == []
    e = errs(v, a, renamed(b, region="us-west-2"))
    assert len(e) == 1 and e[0].config_field == "region"


def test_role_validators_selection():
    assert [type(v).__name__ for v in V.get_role_validators(False, False)] == ["TaskVolumesCannotChange"]
    assert [type(v).__name__ for v in V.get_role_validators(True, False)] == [
        "ServiceRoleCannotChangeOnIncompleteDeployment"]
    assert V.get_role_validators(True, True) == []


def test_service_role_cannot_change_on_incomplete_deployment():
    v = V.ServiceRoleCannotChangeOnIncompleteDeployment()
    a = spec()
    b = S.ServiceSpec.from_json_bytes(a.to_json_bytes())
    assert errs(v, a, b) == []
    e = errs(v, a, renamed(b, role="new-role"))
    assert len(e) == 1 and e[0].is_fatal()


# ---------------------------------------------------------------------------------------
# TaskVolumesCannotChange


def _vol(path="data", size=100, type_="ROOT"):
    return f"volume:\n  path: {path}\n  type: {type_}\n  size: {size}\n"


def test_task_volumes_cannot_change():
    v = V.TaskVolumesCannotChange()
    a = spec({"hello": (1, "", _task(extra=_vol()))})
    bigger = spec({"hello": (1, "", _task(extra=_vol(size=200)))})
    moved = spec({"hello": (1, "", _task(extra=_vol(path="other")))})
    novol = spec({"hello": (1, "", _task())})
    assert errs(v, None, a) == []
    assert errs(v, a, a) == []
    assert len(errs(v, a, bigger)) == 1
    assert len(errs(v, a, moved)) == 1
    assert len(errs(v, a, novol)) == 1
    assert len(errs(v, novol, a)) == 1
    # a brand-new task may bring volumes
    grown = spec({"hello": (1, "", _task() + _task("other", extra=_vol()))})
    assert errs(v, novol, grown) == []


# ---------------------------------------------------------------------------------------
# PlacementRuleIsValid / DomainCapabilityValidator / ZoneValidator


def test_placement_rule_is_valid():
    v = V.PlacementRuleIsValid()
    good = spec({"hello": (1, "placement: '[[\"hostname\", \"UNIQUE\"]]'\n", _task())})
    bad = spec({"hello": (1, "placement: 'rack-id:FOO:foo'\n", _task())})
    nested_bad = spec({"hello": (1, "placement: 'hostname:UNIQUE,rack:MAX_PER:x'\n", _task())})
    assert errs(v, None, good) == []
    assert errs(v, None, spec()) == []
    assert len(errs(v, None, bad)) == 1
    assert len(errs(v, None, nested_bad)) == 1


def test_domain_capability(caps):
    zone = spec({"hello": (1, "placement: '[[\"@zone\", \"GROUP_BY\", \"2\"]]'\n", _task())})
    region = spec({"hello": (1, "placement: '[[\"@region\", \"IS\", \"us-west\"]]'\n", _task())})
    plain = spec({"hello": (1, "placement: '[[\"hostname\", \"UNIQUE\"]]'\n", _task())})
    caps(supports_domains=True)
    assert errs(V.DomainCapabilityValidator(), None, zone) == []
    caps(supports_domains=False)
    assert len(errs(V.DomainCapabilityValidator(), None, zone)) == 1
    assert len(errs(V.DomainCapabilityValidator(), None, region)) == 1
    assert errs(V.DomainCapabilityValidator(), None, plain) == []


def test_zone_validator():
    with_zone = spec({"hello": (1, "placement: '[[\"@zone\", \"GROUP_BY\", \"2\"]]'\n", _task())})
    without = spec({"hello": (1, "placement: '[[\"hostname\", \"UNIQUE\"]]'\n", _task())})
    v = V.ZoneValidator("hello")
    assert errs(v, None, with_zone) == []
    assert errs(v, with_zone, with_zone) == []
    assert errs(v, without, without) == []
    assert len(errs(v, without, with_zone)) == 1
    assert len(errs(v, with_zone, without)) == 1
    assert errs(V.ZoneValidator("absent"), with_zone, without) == []
    with pytest.raises(ValueError):
        V.ZoneValidator("hello").validate(with_zone, spec({"other": (1, "", _task())}))


# ---------------------------------------------------------------------------------------
# TaskEnvCannotChange


def _env_spec(value):
    extra = f"env:\n  MY_VAR: '{value}'\n" if value is not None else ""
    return spec({"hello": (1, "", _task(extra=extra))})


@pytest.mark.parametrize("old,new,rules,n", [
    ("a", "a", (), 0),
    ("a", "b", (), 1),
    (None, "b", (), 1),
    (None, "b", (V.TaskEnvCannotChange.ALLOW_UNSET_TO_SET,), 0),
    ("a", None, (), 1),
    ("a", None, (V.TaskEnvCannotChange.ALLOW_SET_TO_UNSET,), 0),
    (None, None, (), 0),
    ("a", "b", (V.TaskEnvCannotChange.ALLOW_UNSET_TO_SET, V.TaskEnvCannotChange.ALLOW_SET_TO_UNSET), 1),
])
def test_task_env_cannot_change(old, new, rules, n):
    v = V.TaskEnvCannotChange("hello", "server", "MY_VAR", *rules)
    assert len(errs(v, _env_spec(old), _env_spec(new))) == n
    assert errs(v, None, _env_spec(new)) == []


def test_task_env_cannot_change_missing_task_is_an_error():
    v = V.TaskEnvCannotChange("hello", "server", "MY_VAR")
    with pytest.raises(ValueError):
        v.validate(_env_spec("a"), spec({"hello": (1, "", _task("other"))}))


# ---------------------------------------------------------------------------------------
# TLSRequiresServiceAccount


class _Cfg:
    def __init__(self, ok):
        self.ok = ok

    def dcos_auth_token_provider(self):
        if not self.ok:
            raise RuntimeError("no service account")
        return object()


def test_tls_requires_service_account():
    tls = spec({"hello": (1, "", _task(extra="transport-encryption:\n  - name: server\n    type: TLS\n"))})
    assert errs(V.TLSRequiresServiceAccount(_Cfg(True)), None, tls) == []
    assert len(errs(V.TLSRequiresServiceAccount(_Cfg(False)), None, tls)) == 1
    assert errs(V.TLSRequiresServiceAccount(_Cfg(False)), None, spec()) == []


# ---------------------------------------------------------------------------------------
# the default validator list and error rendering


def test_default_validators_and_error_text():
    names = [type(v).__name__ for v in V.get_validators(CFG)]
    assert names == [
        "ServiceNameCannotContainDoubleUnderscores", "PodSpecsCannotShrink", "PodSpecsCannotUseUnsupportedFeatures",
        "PodSpecsCannotChangeNetworkRegime", "PreReservationCannotChange", "UserCannotChange",
        "TLSRequiresServiceAccount", "DomainCapabilityValidator", "PlacementRuleIsValid", "RegionCannotChange",
        "ServiceNameCannotBreakDNS", "TaskSpecsCannotUseUnsupportedFeatures"]
    e = V.ConfigValidationError.transition_error("f", "1", "2", "msg", True)
    assert str(e) == "Field: 'f'; Transition: '1' => '2'; Message: 'msg'; Fatal: true"
    e = V.ConfigValidationError.value_error("f", "v", "msg")
    assert str(e) == "Field: 'f'; Value: 'v'; Message: 'msg'; Fatal: false"


def test_every_default_validator_accepts_an_unchanged_spec():
    s = spec({"hello": (2, "placement: 'hostname:UNIQUE'\n", _task(extra=_vol()))})
    for v in V.get_validators(CFG) + V.get_role_validators(False, False):
        assert v.validate(None, s) == [], type(v).__name__
        assert v.validate(s, s) == [], type(v).__name__


# ---------------------------------------------------------------------------------------
# VerifyHostVolumePathTest / VerifySecretFilePathTest


@pytest.mark.parametrize("host,container,ok", [
    ("", "etc", False),
    ("/etc", "", False),
    (" ", "etc", False),
    ("/etc", " ", False),
    ("/etc", "/etc", False),
    ("/etc", "etc", True),
    ("/etc/abc", "etc/abc", True),
    ("./etc", "etc", False),
    (None, "etc", False),
])
def test_host_volume_paths(host, container, ok):
    def make():
        hv = S.HostVolumeSpec(host, container, "RW")
        hv.validate()
    if ok:
        make()
    else:
        with pytest.raises(Exception):
            make()


@pytest.mark.parametrize("secret,env_key,file_path,ok", [
    ("secret/path", "KEY", "", True),
    ("secret/path", "KEY", " ", False),
    ("secret/path", "KEY", "/path/to/file", False),
    ("secret/path", "KEY", "@?test", False),
    ("secret/path", "KEY", "-test", False),
    ("secret/path", "KEY", ".test", True),
    ("secret/path", "KEY", "somePath/someFile.test", True),
    ("secret/path", "KEY", "file", True),
    ("secret/path", "KEY", "file-0/file1/file-2/file3/file_4", True),
    ("file-0/file1/file-2/file3/file_4", "KEY", "file", True),
    ("file", "KEY", "file", True),
    ("file", "", "file", True),
])
def test_secret_file_paths(secret, env_key, file_path, ok):
    def make():
        S.SecretSpec(secret, env_key, file_path).validate()
    if ok:
        make()
    else:
        with pytest.raises(Exception):
            make()


def test_placement_parse_is_what_the_validator_sees():
    s = spec({"hello": (1, "placement: 'hostname:MAX_PER:2'\n", _task())})
    assert isinstance(s.pods[0].placement_rule, PL.MaxPerHostnameRule)
