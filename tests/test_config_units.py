"""Configuration units: the configuration updater, the TASKCFG env router, the YAML configuration
loader and the configuration value types.

Mirrors sdk/scheduler/src/test/java/com/mesosphere/sdk/config/{ConfigurationUpdaterTest,
DefaultTaskEnvRouterTest,YAMLConfigurationLoaderTest}.java: a changed config is stored and targeted,
an unchanged one keeps its target, a config failing validation keeps the old target and reports the
errors, and user changes (service or pod level, with the unset-means-root rule) stop the scheduler.
"""
import dataclasses
import textwrap
import uuid

import pytest

import testutils as U
from dcos_commons_amd.config import serialization as SU
from dcos_commons_amd.config import validate as V
from dcos_commons_amd.config.configuration_updater import DefaultConfigurationUpdater
from dcos_commons_amd.config.task_env_router import TaskEnvRouter
from dcos_commons_amd.mesos import protos as P
from dcos_commons_amd.offer.taskdata.labels import TaskLabelReader, TaskLabelWriter
from dcos_commons_amd.scheduler.scheduler_config import SchedulerConfig
from dcos_commons_amd.specification import specs as S
from dcos_commons_amd.specification.yaml import mappers
from dcos_commons_amd.specification.yaml.raw import RawServiceSpec
from dcos_commons_amd.state.config_store import ConfigStore, ConfigStoreException
from dcos_commons_amd.state.state_store import StateStore
from dcos_commons_amd.storage.mem_persister import MemPersister
from dcos_commons_amd.storage.persister import Reason

CFG = SchedulerConfig.for_testing()
TARGET_ID, NEW_ID, UNKNOWN_ID = uuid.uuid4(), uuid.uuid4(), uuid.uuid4()


def _pod(pod_type, count, task, cpus):
    return textwrap.dedent(f"""\
        {pod_type}:
          count: {count}
          tasks:
            {task}:
              goal: RUNNING
              cmd: echo {task}
              cpus: {cpus}
              memory: 1000
        """)


def _spec(*pods, user=S.DEFAULT_SERVICE_USER):
    text = f"name: test-service\nscheduler:\n  principal: {U.PRINCIPAL}\n  user: {user}\npods:\n" + \
        textwrap.indent("".join(pods), "  ")
    spec = mappers.ServiceSpecGenerator(RawServiceSpec.from_string(text), CFG, "/tmp", {}).build()
    # TestPodFactory pods run as the test service user (a builder-only pod field, not a YAML key)
    return _with_pod_users(spec, U.SERVICE_USER)


def _with_pod_users(spec, user):
    return dataclasses.replace(spec, pods=tuple(dataclasses.replace(p, user=user) for p in spec.pods))


ORIGINAL = _spec(_pod("POD-A", 1, "A", 1.0), _pod("POD-B", 2, "B", 2.0))
UPDATED = _spec(_pod("POD-A", 1, "A", 2.0), _pod("POD-B", 2, "B", 2.0))
BAD_UPDATE = _spec(_pod("POD-A", 1, "A", 1.0), _pod("POD-B", 1, "B", 2.0))  # shrinks POD-B


class FakeConfigStore:
    """The ConfigStore calls the updater makes, with the reference test's stubbed answers."""

    def __init__(self, target=ORIGINAL, extra=None):
        self.configs = {TARGET_ID: target}
        self.configs.update(extra or {})
        self.target = TARGET_ID
        self.stored = []
        self.targets = []
        self.cleared = []

    def get_target_config(self):
        if self.target is None:
            raise ConfigStoreException(Reason.NOT_FOUND, "no target")
        return self.target

    def fetch(self, cid):
        if cid not in self.configs:
            raise ConfigStoreException(Reason.NOT_FOUND, str(cid))
        return self.configs[cid]

    def store(self, config):
        self.stored.append(config)
        self.configs[NEW_ID] = config
        return NEW_ID

    def set_target_config(self, cid):
        self.targets.append(cid)
        self.target = cid

    def list(self):
        return list(self.configs)

    def clear(self, cid):
        self.cleared.append(cid)
        self.configs.pop(cid, None)


def _updater(store, validators=None):
    if validators is None:
        validators = V.get_validators(CFG)
    return DefaultConfigurationUpdater(StateStore(MemPersister()), store, validators)


def test_changed_config_without_validators_is_targeted():
    store = FakeConfigStore()
    result = _updater(store, []).update_configuration(UPDATED)
    assert store.targets == [NEW_ID]
    assert result.target_id == NEW_ID and result.errors == []


def test_changed_config_passing_validation_is_targeted_and_unused_configs_are_cleared():
    store = FakeConfigStore(extra={UNKNOWN_ID: ORIGINAL})
    result = _updater(store).update_configuration(UPDATED)
    assert store.targets == [NEW_ID]
    assert result.target_id == NEW_ID and result.errors == []
    # no task references the old target or the unknown config: both are garbage-collected
    assert set(store.cleared) == {TARGET_ID, UNKNOWN_ID}


def test_same_config_keeps_the_target():
    store = FakeConfigStore(extra={NEW_ID: UPDATED})
    result = _updater(store).update_configuration(ORIGINAL)
    assert result.target_id == TARGET_ID and result.errors == []
    assert store.stored == [] and store.targets == []


def test_invalid_config_keeps_the_target_and_reports_errors():
    store = FakeConfigStore()
    result = _updater(store).update_configuration(BAD_UPDATE)
    assert result.target_id == TARGET_ID
    assert len(result.errors) == 1 and "Transition: '2' => '1'" in str(result.errors[0])
    assert store.targets == []


def test_invalid_first_config_is_fatal():
    store = FakeConfigStore()
    store.target = None
    store.configs = {}
    shrinker = V.ConfigValidator()
    shrinker.validate = lambda old, new: [V.ConfigValidationError.value_error("f", "v", "always invalid")]
    with pytest.raises(ConfigStoreException, match="without any prior target configuration"):
        _updater(store, [shrinker]).update_configuration(ORIGINAL)


def _without_pod_users(spec):
    return dataclasses.replace(spec, pods=tuple(dataclasses.replace(p, user=None) for p in spec.pods))


def test_user_set_at_pod_level_but_not_at_service_level():
    # the stored spec leaves the service user unset; it is read as root
    store = FakeConfigStore(target=dataclasses.replace(ORIGINAL, user=None))
    result = _updater(store).update_configuration(ORIGINAL)
    assert result.target_id == TARGET_ID and result.errors == []


def test_unset_pod_users_default_to_root_and_cannot_become_another_user():
    store = FakeConfigStore(target=_without_pod_users(ORIGINAL))
    # the new spec's pods run as service-user: the old (unset = root) pods cannot change user
    with pytest.raises(ConfigStoreException, match="Cannot change existing pod type user"):
        _updater(store).update_configuration(ORIGINAL)


def test_unset_pod_users_may_become_explicit_root():
    store = FakeConfigStore(target=_without_pod_users(ORIGINAL))
    result = _updater(store).update_configuration(_with_pod_users(ORIGINAL, S.DEFAULT_SERVICE_USER))
    assert result.target_id == TARGET_ID and result.errors == []


def test_service_user_cannot_change():
    store = FakeConfigStore()
    with pytest.raises(ConfigStoreException, match="Cannot change user of deployed service"):
        _updater(store).update_configuration(dataclasses.replace(ORIGINAL, user="nobody"))


def test_tasks_on_an_equivalent_config_are_relabelled_to_the_new_target():
    """Only count changes (ignored by the pod comparison): the running task's config label moves to
    the new target and the old config is kept only while something still references it."""
    persister = MemPersister()
    state = StateStore(persister)
    store = ConfigStore(S.loopback_check(ORIGINAL), persister)
    old_id = store.store(ORIGINAL)
    store.set_target_config(old_id)
    info = U.with_labels(U.get_task_info([], name="POD-A-0-A", task_id=U.to_task_id("test-service", "POD-A-0-A")),
                         lambda w: (w.set_type("POD-A"), w.set_index(0), w.set_target_configuration(old_id)))
    state.store_tasks([info])
    grown = _spec(_pod("POD-A", 2, "A", 1.0), _pod("POD-B", 2, "B", 2.0))
    result = DefaultConfigurationUpdater(state, store, V.get_validators(CFG)).update_configuration(grown)
    assert result.target_id != old_id and result.errors == []
    assert TaskLabelReader(state.fetch_task("POD-A-0-A")).get_target_configuration() == result.target_id
    assert store.list() == [result.target_id]


def test_tasks_on_a_different_config_keep_their_label():
    persister = MemPersister()
    state = StateStore(persister)
    store = ConfigStore(S.loopback_check(ORIGINAL), persister)
    old_id = store.store(ORIGINAL)
    store.set_target_config(old_id)
    info = U.with_labels(U.get_task_info([], name="POD-A-0-A", task_id=U.to_task_id("test-service", "POD-A-0-A")),
                         lambda w: (w.set_type("POD-A"), w.set_index(0), w.set_target_configuration(old_id)))
    state.store_tasks([info])
    result = DefaultConfigurationUpdater(state, store, V.get_validators(CFG)).update_configuration(UPDATED)
    assert TaskLabelReader(state.fetch_task("POD-A-0-A")).get_target_configuration() == old_id
    assert sorted(map(str, store.list())) == sorted([str(old_id), str(result.target_id)])


# ---------------------------------------------------------------------------------------
# TaskEnvRouter


TEST_ENV = {
    "TASKCFG_A_ONE": "TWO", "TASKCFG_A_THREE": "FOUR", "TASKCFG_A_B_FIVE": "SIX", "TASKCFG_B_SEVEN": "EIGHT",
    "TASKCFG_C_NINE": "TEN", "TASKCFG_ALL_FOO": "BAR", "TASKCFG_ALL_BAR": "BAZ", "TASKCFG_IGNORED": "FOO",
    "IGNORED": "BAR",
}
GLOBAL = {"FOO": "BAR", "BAR": "BAZ"}


def test_router_empty():
    r = TaskEnvRouter({})
    assert all(r.get_config(p) == {} for p in "abcde")


def test_router_mixed():
    r = TaskEnvRouter(TEST_ENV)
    assert r.get_config("a") == r.get_config("A")  # case insensitive
    assert r.get_config("a") == dict(GLOBAL, ONE="TWO", THREE="FOUR", B_FIVE="SIX")
    assert r.get_config("b") == dict(GLOBAL, SEVEN="EIGHT")
    assert r.get_config("c") == dict(GLOBAL, NINE="TEN")
    assert r.get_config("d") == GLOBAL and r.get_config("e") == GLOBAL


def test_router_pod_type_mapping():
    r = TaskEnvRouter(TEST_ENV)
    expected = r.get_config("A_B")
    assert len(expected) == 3
    for name in ("A-B", "A.B", "a_b", "a.b"):
        assert r.get_config(name) == expected


def test_router_priorities():
    r = (TaskEnvRouter(TEST_ENV)
         .set_all_pods_env("NOT_IGNORED", "VAL")
         .set_all_pods_env("ONE", "FOUR")          # loses to TASKCFG_A_ONE in pod a
         .set_pod_env("A", "NOT_IGNORED", "VAL2")  # beats the all-pods value in pod a
         .set_pod_env("A", "THREE", "EIGHT"))      # loses to TASKCFG_A_THREE
    assert r.get_config("a") == r.get_config("A")
    assert r.get_config("a") == dict(GLOBAL, NOT_IGNORED="VAL2", ONE="TWO", THREE="FOUR", B_FIVE="SIX")
    assert r.get_config("b") == dict(GLOBAL, NOT_IGNORED="VAL", ONE="FOUR", SEVEN="EIGHT")
    assert r.get_config("c") == dict(GLOBAL, NOT_IGNORED="VAL", ONE="FOUR", NINE="TEN")
    assert r.get_config("d") == dict(GLOBAL, NOT_IGNORED="VAL", ONE="FOUR")


# ---------------------------------------------------------------------------------------
# YAMLConfigurationLoader, configuration types, serialization


@dataclasses.dataclass
class TestConfig:
    __test__ = False
    name: str = ""
    count: int = 0


def test_yaml_loader(tmp_path):
    p = tmp_path / "test.yml"
    p.write_text("name: DCOS\ncount: 1")
    cfg = SU.load_config_from_env(TestConfig, str(p))
    assert (cfg.name, cfg.count) == ("DCOS", 1)


def test_yaml_loader_substitutes_the_environment(tmp_path):
    p = tmp_path / "test.yml"
    p.write_text("name: ${SVC_NAME}\ncount: ${COUNT:-3}\nliteral: $${SVC_NAME}\nkept: ${UNSET_VAR}\n")
    cfg = SU.load_config_from_env(None, str(p), {"SVC_NAME": "hello-${SUFFIX}", "SUFFIX": "world"})
    assert cfg == {"name": "hello-world", "count": 3, "literal": "${SVC_NAME}", "kept": "${UNSET_VAR}"}


def test_string_configuration():
    c = SU.StringConfiguration('say "hi"')
    assert c.get_bytes() == b'say "hi"'
    assert c.to_json_string() == '{ "string": "say \\"hi\\"" }'
    assert SU.StringConfiguration.Factory().parse(c.get_bytes()) == c
    assert SU.StringConfiguration.Comparator().equals(c, SU.StringConfiguration('say "hi"'))
    store = ConfigStore(SU.StringConfiguration.Factory(), MemPersister())
    cid = store.store(c)
    assert store.fetch(cid) == c


def test_recovery_configuration_round_trip():
    rc = SU.RecoveryConfiguration(60, 30, True)
    d = rc.to_dict()
    assert d == {"recover-in-place-grace-period-secs": 60, "min-delay-between-recoveries-secs": 30,
                 "enable-replacement": True}
    assert SU.RecoveryConfiguration.from_dict(d) == rc and rc.is_replacement_enabled()
    assert SU.from_json_string(SU.to_json_string(rc.to_dict()), SU.RecoveryConfiguration) == rc


def test_jackson_style_json():
    assert SU.to_json_string({"a": 1, "b": [1, 2], "c": {}, "d": []}) == \
        '{\n  "a" : 1,\n  "b" : [ 1, 2 ],\n  "c" : { },\n  "d" : [ ]\n}'
    assert SU.from_yaml_string(SU.to_yaml_string({"x": [1, {"y": "z"}]})) == {"x": [1, {"y": "z"}]}
    assert SU.to_yaml_string_or_empty(object()) == "" or isinstance(SU.to_yaml_string_or_empty(object()), str)
