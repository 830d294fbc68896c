"""FrameworkInfo construction and role selection.

Mirrors the reference's framework/FrameworkRunnerTest.java (sdk/scheduler/src/test/java/com/
mesosphere/sdk/framework/): the minimal and exhaustive FrameworkInfo (name, user, principal,
2-week failover timeout, checkpointing, ID on re-registration, web UI URL, capabilities in order)
and the role matrix over {pre-reserved roles, quota (group) role vs legacy role, Marathon
enforce-group-role, role migration}: which role(s) the framework subscribes with and when it
turns MULTI_ROLE on. Also the driver factory's credential rules (SchedulerDriverFactoryTest.java).
"""
import pytest

from dcos_commons_amd.dcos import capabilities as caps
from dcos_commons_amd.framework import scheduler_driver_factory as F
from dcos_commons_amd.framework.env_store import EnvStore
from dcos_commons_amd.framework.framework_config import FrameworkConfig
from dcos_commons_amd.framework.framework_runner import FrameworkRunner
from dcos_commons_amd.mesos import protos as P
from dcos_commons_amd.scheduler.scheduler_config import SchedulerConfig

Cap = P.FrameworkInfo.Capability
FID = P.FrameworkID(value="test-framework-id")
NONE_CAPS = caps.Capabilities(supports_pre_reserved_resources=False, supports_gpu_resource=False,
                              supports_domains=False, supports_partition_awareness=False)


@pytest.fixture(autouse=True)
def capabilities():
    caps.override_capabilities(NONE_CAPS)
    yield
    caps.override_capabilities(None)


def minimal(**extra):
    env = {"FRAMEWORK_NAME": "/path/to/test-service", "PACKAGE_NAME": "test-package", "PACKAGE_VERSION": "1.5",
           "PACKAGE_BUILD_TIME_EPOCH_MS": "1234567890"}
    env.update(extra)
    return env


def runner(env, gpus=False, regions=False):
    store = EnvStore.from_map(env)
    return FrameworkRunner(SchedulerConfig(store), FrameworkConfig.from_env_store(store), gpus, regions)


def _common(info, user="root", principal="/path/to/test-service-principal"):
    assert info.name == "/path/to/test-service"
    assert info.user == user and info.principal == principal
    assert info.failover_timeout == pytest.approx(1209600)
    assert info.checkpoint


def test_minimal_info_initial_and_relaunch():
    r = runner(minimal())
    info = r.get_framework_info(None)
    _common(info)
    assert not info.HasField("id")
    assert info.role == "path__to__test-service-role" and list(info.roles) == []
    assert list(info.capabilities) == [] and not info.HasField("webui_url")
    info = r.get_framework_info(FID)
    _common(info)
    assert info.id == FID and info.role == "path__to__test-service-role"


def test_exhaustive_info():
    caps.override_capabilities(NONE_CAPS.with_overrides(supports_gpu_resource=True,
                                                        supports_pre_reserved_resources=True, supports_domains=True))
    env = minimal(FRAMEWORK_PRINCIPAL="custom-principal", FRAMEWORK_USER="custom-user",
                  FRAMEWORK_PRERESERVED_ROLES="role1,role2,role3", FRAMEWORK_WEB_URL="custom-url")
    info = runner(env, gpus=True, regions=True).get_framework_info(FID)
    _common(info, user="custom-user", principal="custom-principal")
    assert info.id == FID and not info.HasField("role")
    assert set(info.roles) == {"path__to__test-service-role", "role1", "role2", "role3"}
    assert [c.type for c in info.capabilities] == [Cap.MULTI_ROLE, Cap.GPU_RESOURCES, Cap.RESERVATION_REFINEMENT,
                                                   Cap.REGION_AWARE]
    assert info.webui_url == "custom-url"


def test_partition_awareness_capability():
    caps.override_capabilities(NONE_CAPS.with_overrides(supports_partition_awareness=True))
    info = runner(minimal()).get_framework_info(None)
    assert [c.type for c in info.capabilities] == [Cap.PARTITION_AWARE]


def test_gpu_and_region_capabilities_need_both_usage_and_cluster_support():
    caps.override_capabilities(NONE_CAPS.with_overrides(supports_gpu_resource=True, supports_domains=True))
    assert list(runner(minimal()).get_framework_info(None).capabilities) == []  # not using GPUs/regions
    caps.override_capabilities(NONE_CAPS)
    assert list(runner(minimal(), gpus=True, regions=True).get_framework_info(None).capabilities) == []


# {pre-reserved roles, quota role (MESOS_ALLOCATION_ROLE usable), enforce group role, migration}
@pytest.mark.parametrize("case,alloc,enforce,prereserved,migrate,roles,role,n_caps", [
    ("TTTT", "path", "true", True, "true",
     {"path", "path__to__test-service-role", "role1", "role2", "role3"}, None, 2),
    ("FTFT", "path", "false", False, "true", {"path", "path__to__test-service-role"}, None, 1),
    # slave_public is Marathon's reset value: legacy role, but migration still adds the group role
    ("FFFT", "slave_public", "false", False, "true", {"path", "path__to__test-service-role"}, None, 1),
    ("TTTF", "path", "true", True, "false", {"path", "role1", "role2", "role3"}, None, 2),
    ("FTFF", "path", "false", False, "false", set(), "path", 0),
    ("TFFF", "slave_public", "false", True, "false",
     {"path__to__test-service-role", "role1", "role2", "role3"}, None, 2),
    ("FFFF", "slave_public", "false", False, "false", set(), "path__to__test-service-role", 0),
])
def test_role_matrix(case, alloc, enforce, prereserved, migrate, roles, role, n_caps):
    caps.override_capabilities(NONE_CAPS.with_overrides(supports_pre_reserved_resources=prereserved))
    env = minimal(MESOS_ALLOCATION_ROLE=alloc, MARATHON_APP_ENFORCE_GROUP_ROLE=enforce,
                  ENABLE_ROLE_MIGRATION=migrate)
    if prereserved:
        env["FRAMEWORK_PRERESERVED_ROLES"] = "role1,role2,role3"
    info = runner(env).get_framework_info(FID)
    _common(info)
    assert info.id == FID
    assert set(info.roles) == roles and len(info.roles) == len(roles)
    if role is None:
        assert not info.HasField("role")
    else:
        assert info.role == role
    assert len(info.capabilities) == n_caps
    assert (Cap.MULTI_ROLE in [c.type for c in info.capabilities]) == bool(roles)
    assert not info.HasField("webui_url")


def test_enforced_group_role_requires_an_allocation_role():
    with pytest.raises(Exception):
        runner(minimal(MARATHON_APP_ENFORCE_GROUP_ROLE="true"))


@pytest.mark.parametrize("name,namespaced", [("/path/to/svc", "path"), ("path/svc", "path"), ("svc", None),
                                              ("/svc", None)])
def test_namespaced_role_is_the_top_level_group(name, namespaced):
    fc = FrameworkConfig.from_env_store(EnvStore.from_map({"FRAMEWORK_NAME": name}))
    assert fc.namespaced_role() == namespaced
    assert fc.non_namespaced_role().endswith("-role")


def test_explicit_namespace_overrides_the_environment():
    store = EnvStore.from_map(minimal(MESOS_ALLOCATION_ROLE="path"))
    assert FrameworkConfig.from_env_store(store).role == "path"
    assert FrameworkConfig.from_env_store(store, None).role == "path__to__test-service-role"
    assert FrameworkConfig.from_env_store(store, "other").role == "other"


def test_prereserved_roles_are_deduplicated_in_order():
    fc = FrameworkConfig.from_env_store(EnvStore.from_map(minimal(FRAMEWORK_PRERESERVED_ROLES="b,a,b,c")))
    assert fc.pre_reserved_roles == ["b", "a", "c"]


# ---------------------------------------------------------------------------------------
# SchedulerDriverFactory (reference framework/SchedulerDriverFactoryTest.java)


SECRET = b"sekrit"
WITHOUT_PRINCIPAL = P.FrameworkInfo(user="Foo", name="Bar")
EMPTY_PRINCIPAL = P.FrameworkInfo(user="Foo", name="Bar", principal="")
WITH_PRINCIPAL = P.FrameworkInfo(user="Foo", name="Bar", principal="fake-principal")


class RecordingFactory(F.SchedulerDriverFactory):
    def __init__(self):
        self.calls = []

    def create_internal(self, scheduler, framework_info, master_url, credential, scheduler_config):
        self.calls.append(credential)
        return None


def _cfg(sidechannel):
    env = {"DCOS_SERVICE_ACCOUNT_CREDENTIAL": '{"uid": "svc", "private_key": "k"}'} if sidechannel else {}
    return SchedulerConfig.for_testing(**env)


@pytest.mark.parametrize("sidechannel,secret,has_credential,has_secret", [
    (False, None, False, False),
    (True, None, True, False),
    (False, SECRET, True, True),
    (True, SECRET, True, True),  # a secret wins over the side channel
])
def test_driver_credential_modes(sidechannel, secret, has_credential, has_secret):
    f = RecordingFactory()
    assert f.create(object(), WITH_PRINCIPAL, "fake-master-url", _cfg(sidechannel), secret) is None
    (cred,) = f.calls
    assert (cred is not None) == has_credential
    if cred is not None:
        assert cred.principal == "fake-principal"
        assert (cred.secret == "sekrit") == has_secret and bool(cred.secret) == has_secret


@pytest.mark.parametrize("info", [EMPTY_PRINCIPAL, WITHOUT_PRINCIPAL])
def test_missing_principal_is_fine_without_auth(info):
    f = RecordingFactory()
    f.create(object(), info, "fake-master-url", _cfg(False))
    assert f.calls == [None]


@pytest.mark.parametrize("info", [EMPTY_PRINCIPAL, WITHOUT_PRINCIPAL])
@pytest.mark.parametrize("sidechannel,secret", [(True, None), (False, SECRET), (True, SECRET)])
def test_auth_without_a_principal_is_rejected(info, sidechannel, secret):
    with pytest.raises(ValueError, match="lacks required principal"):
        RecordingFactory().create(object(), info, "fake-master-url", _cfg(sidechannel), secret)


@pytest.mark.parametrize("v1_supported,requested,expected", [
    (True, "V1", "V1"), (True, "V0", "V0"), (False, "V1", "V0"), (False, "V0", "V0")])
def test_api_version_selection(v1_supported, requested, expected):
    c = NONE_CAPS.with_overrides(supports_v1_api_by_default=v1_supported)
    assert F.select_api_version(requested, c) == expected


def test_http_driver_authorization_headers():
    from dcos_commons_amd.mesos.http_driver import V1HttpSchedulerDriver

    basic = V1HttpSchedulerDriver("http://m:5050", object(), WITH_PRINCIPAL,
                                  credential=P.Credential(principal="p", secret="s"))
    assert basic._headers("application/x-protobuf")["Authorization"] == "Basic cDpz"
    side = V1HttpSchedulerDriver("http://m:5050", object(), WITH_PRINCIPAL, credential=P.Credential(principal="p"),
                                 token_provider=lambda: "jwt-value")
    assert side._headers("application/x-protobuf")["Authorization"] == "token=jwt-value"
    none = V1HttpSchedulerDriver("http://m:5050", object(), WITH_PRINCIPAL)
    assert "Authorization" not in none._headers("application/x-protobuf")


def test_sidechannel_driver_gets_an_iam_token_provider(monkeypatch):
    from dcos_commons_amd.mesos import http_driver

    cfg = SchedulerConfig.for_testing(DCOS_SERVICE_ACCOUNT_CREDENTIAL='{"uid": "svc", "private_key": "k"}',
                                      SDK_DCOS_AUTH_TOKEN="a.eyJleHAiOiAxfQ.c")
    monkeypatch.setattr(http_driver, "resolve_master_url", lambda u: u)
    d = F.SchedulerDriverFactory().create(object(), WITH_PRINCIPAL, "http://m:5050", cfg)
    assert d.credential.principal == "fake-principal" and not d.credential.secret
    assert d._headers("application/json")["Authorization"] == "token=a.eyJleHAiOiAxfQ.c"
