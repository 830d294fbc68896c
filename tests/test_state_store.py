"""StateStore / ConfigStore / FrameworkStore / StateStoreUtils semantics (reference:
state/StateStoreTest, ConfigStoreTest, StateStoreUtilsTest). The checkpoint layout (node paths) is
part of the contract -- a scheduler must be able to resume from a reference-written tree."""
import uuid

import pytest

from dcos_commons_amd.mesos import protos as P
from dcos_commons_amd.state import state_store_utils as SU
from dcos_commons_amd.state.config_store import ConfigStore, ConfigStoreException
from dcos_commons_amd.state.framework_store import FrameworkStore
from dcos_commons_amd.state.goal_state_override import GoalStateOverride, OverrideProgress, OverrideStatus
from dcos_commons_amd.state.state_store import StateStore, StateStoreException
from dcos_commons_amd.storage.mem_persister import MemPersister
from dcos_commons_amd.storage.persister import Reason


def task(name, tid=None, agent="agent-1"):
    t = P.TaskInfo(name=name)
    t.task_id.value = tid if tid is not None else f"svc__{name}__{uuid.uuid4()}"
    t.agent_id.value = agent
    return t


def status(t, state=P.TASK_RUNNING, **kw):
    s = P.TaskStatus(state=state, **kw)
    s.task_id.CopyFrom(t.task_id)
    return s


@pytest.fixture
def persister():
    return MemPersister()


@pytest.fixture
def store(persister):
    return StateStore(persister)


def test_root_and_namespaced_layout(persister):
    t = task("hello-0-server")
    StateStore(persister).store_tasks([t])
    StateStore(persister, "path/to/svc").store_tasks([t])
    assert persister.get("Tasks/hello-0-server/TaskInfo") == t.SerializeToString()
    assert persister.get("Services/path__to__svc/Tasks/hello-0-server/TaskInfo") == t.SerializeToString()
    StateStore(persister).store_property("k", b"v")
    assert persister.get("Properties/k") == b"v"


def test_store_fetch_clear_tasks(store):
    assert store.fetch_tasks() == [] and store.fetch_task_names() == []
    assert store.fetch_task("missing") is None
    a, b = task("a"), task("b")
    store.store_tasks([a, b])
    store.store_tasks([a])  # repeated store is idempotent
    assert sorted(store.fetch_task_names()) == ["a", "b"]
    assert store.fetch_task("a") == a
    store.clear_task("a")
    store.clear_task("a")  # clearing a missing task is silent
    assert store.fetch_task_names() == ["b"]


def test_large_batches_are_split(store):
    big = [task(f"t{i}") for i in range(5)]
    for t in big:
        t.data = b"x" * 400_000  # 2 MB total > 1 MB per transaction
    store.store_tasks(big)
    assert len(store.fetch_tasks()) == 5


def test_status_lifecycle(store):
    t = task("a")
    store.store_tasks([t])
    assert store.fetch_status("a") is None and store.fetch_statuses() == []
    store.store_status("a", status(t, P.TASK_RUNNING))
    assert store.fetch_status("a").state == P.TASK_RUNNING
    store.store_status("a", status(t, P.TASK_FAILED))
    # LOST/GONE/DROPPED/UNKNOWN/UNREACHABLE after a terminal state are stale and rejected
    for late in (P.TASK_LOST, P.TASK_UNREACHABLE, P.TASK_UNKNOWN):
        with pytest.raises(StateStoreException) as e:
            store.store_status("a", status(t, late))
        assert e.value.reason == Reason.LOGIC_ERROR
    assert [s.state for s in store.fetch_statuses()] == [P.TASK_FAILED]


def test_status_with_mismatched_task_id_rejected_unless_staging(store):
    t = task("a")
    store.store_tasks([t])
    store.store_status("a", status(t))
    other = task("a")
    with pytest.raises(StateStoreException) as e:
        store.store_status("a", status(other, P.TASK_RUNNING))
    assert e.value.reason == Reason.NOT_FOUND
    store.store_status("a", status(other, P.TASK_STAGING))  # a relaunch
    assert store.fetch_status("a").task_id == other.task_id


@pytest.mark.parametrize("bad", ["", "  ", "a/b"])
def test_property_key_validation(store, bad):
    with pytest.raises(StateStoreException):
        store.store_property(bad, b"v")
    with pytest.raises(StateStoreException):
        store.fetch_property(bad)


def test_properties(store):
    assert store.fetch_property_keys() == []
    store.store_property("a", b"1")
    store.store_properties({"b": b"2", "c": b""})
    assert sorted(store.fetch_property_keys()) == ["a", "b", "c"]
    assert store.fetch_property("b") == b"2"
    store.clear_property("a")
    store.clear_property("a")
    with pytest.raises(StateStoreException) as e:
        store.fetch_property("a")
    assert e.value.reason == Reason.NOT_FOUND
    with pytest.raises(StateStoreException):
        store.store_property("big", b"x" * (1024 * 1024 + 1))


def test_goal_state_override_round_trip(store, persister):
    assert store.fetch_goal_override_status("a") == OverrideStatus.INACTIVE
    st = GoalStateOverride.PAUSED.new_status(OverrideProgress.PENDING)
    store.store_goal_override_status("a", st)
    assert store.fetch_goal_override_status("a") == st
    assert persister.get("Tasks/a/Metadata/goal-state-override") == b"PAUSED"
    assert persister.get("Tasks/a/Metadata/override-status") == b"PENDING"
    store.store_goal_override_status("a", OverrideStatus.INACTIVE)
    assert store.fetch_goal_override_status("a") == OverrideStatus.INACTIVE


def test_delete_all_data_if_namespaced(persister):
    root, ns = StateStore(persister), StateStore(persister, "svc")
    root.store_property("k", b"v")
    ns.store_property("k", b"v")
    root.delete_all_data_if_namespaced()
    ns.delete_all_data_if_namespaced()
    assert root.fetch_property("k") == b"v"
    assert ns.fetch_property_keys() == []


def test_repair_task_ids(persister):
    store = StateStore(persister)
    t = task("a")
    store.store_tasks([t])
    st = status(t)
    st.task_id.value = "svc__a__stale"
    persister.set("Tasks/a/TaskStatus", st.SerializeToString())
    repaired = StateStore(persister)  # repair runs at construction
    # the TaskInfo adopts the status' TaskID and the task is marked failed so it is relaunched
    assert repaired.fetch_task("a").task_id.value == "svc__a__stale"
    assert repaired.fetch_status("a").state == P.TASK_FAILED
    # a task with no status at all is assumed failed
    StateStore(persister).store_tasks([task("b")])
    assert StateStore(persister).fetch_status("b").state == P.TASK_FAILED


def test_state_store_utils(store):
    assert not SU.is_uninstalling(store)
    SU.set_uninstalling(store)
    assert SU.is_uninstalling(store)
    assert not SU.get_deployment_was_completed(store)
    SU.set_deployment_was_completed(store)
    assert SU.get_deployment_was_completed(store)
    t = task("a")
    st = status(t)
    st.container_status.network_infos.add().ip_addresses.add(ip_address="10.0.0.1")
    SU.store_task_status_as_property(store, "a", st)
    assert SU.get_task_status_from_property(store, "a") == st
    assert SU.get_task_status_from_property(store, "b") is None
    store.store_tasks([t])
    assert SU.fetch_task_info(store, status(t)).name == "a"
    with pytest.raises(StateStoreException):
        SU.fetch_task_info(store, status(task("zzz")))


def test_framework_store(persister):
    fs = FrameworkStore(persister)
    assert fs.fetch_framework_id() is None
    fs.store_framework_id(P.FrameworkID(value="fw-1"))
    assert fs.fetch_framework_id().value == "fw-1"
    assert persister.get("FrameworkID") == P.FrameworkID(value="fw-1").SerializeToString()
    fs.clear_framework_id()
    assert fs.fetch_framework_id() is None


class _Cfg:
    def __init__(self, v):
        self.v = v

    def get_bytes(self):
        return self.v.encode()

    def to_json_string(self):
        return self.v


class _Factory:
    def parse(self, data):
        return _Cfg(data.decode())


def test_config_store(persister):
    cs = ConfigStore(_Factory(), persister)
    with pytest.raises(ConfigStoreException) as e:
        cs.get_target_config()
    assert e.value.reason == Reason.NOT_FOUND
    a = cs.store(_Cfg("one"))
    b = cs.store(_Cfg("two"))
    assert sorted(cs.list()) == sorted([a, b])
    assert cs.fetch(a).v == "one"
    cs.set_target_config(b)
    assert cs.get_target_config() == b
    assert persister.get("ConfigTarget") == str(b).encode()
    assert persister.get(f"Configurations/{a}") == b"one"
    cs.clear(a)
    cs.clear(a)
    with pytest.raises(ConfigStoreException):
        cs.fetch(a)
    ns = ConfigStore(_Factory(), persister, "svc")
    c = ns.store(_Cfg("three"))
    assert persister.get(f"Services/svc/Configurations/{c}") == b"three"
