"""StateStore / StateStoreUtils / SchemaVersionStore / FrameworkStore edge cases.

Mirrors the reference's state suites (sdk/scheduler/src/test/java/com/mesosphere/sdk/state/
{StateStoreTest,StateStoreUtilsTest,SchemaVersionStoreTest,FrameworkStoreTest}.java): property
helpers, deploy-completed and uninstalling bits, the ``<task>:task-status`` property, TaskInfo
lookup from a status, TaskID repair at startup, status/TaskID consistency rules, and the
persisted layout of each store.
"""
import pytest

from dcos_commons_amd.mesos import protos as P
from dcos_commons_amd.offer.common_id_utils import to_task_id
from dcos_commons_amd.state import state_store_utils as U
from dcos_commons_amd.state.framework_store import FrameworkStore
from dcos_commons_amd.state.goal_state_override import GoalStateOverride, OverrideProgress, OverrideStatus
from dcos_commons_amd.state.schema_version_store import SchemaVersion, SchemaVersionStore
from dcos_commons_amd.state.state_store import StateStore, StateStoreException
from dcos_commons_amd.storage.mem_persister import MemPersister
from dcos_commons_amd.storage.persister import Reason

SERVICE = "test-service"
TASK = "test-task-name"


@pytest.fixture
def persister():
    return MemPersister()


@pytest.fixture
def store(persister):
    return StateStore(persister)


def info(name=TASK, tid=None):
    t = P.TaskInfo(name=name)
    t.task_id.CopyFrom(tid if tid is not None else to_task_id(SERVICE, name))
    t.agent_id.value = "proto-field-required"
    return t


def status(tid, state=P.TASK_RUNNING):
    s = P.TaskStatus(state=state)
    s.task_id.CopyFrom(tid)
    return s


# ---------------------------------------------------------------------------------------
# StateStoreUtils


def test_property_or_empty(store):
    assert U.fetch_property_or_empty(store, "UNDEFINED") == b""
    store.store_property("DEFINED", b"VALUE")
    assert U.fetch_property_or_empty(store, "UNDEFINED") == b""
    assert U.fetch_property_or_empty(store, "DEFINED") == b"VALUE"


def test_deployment_completed_bit(store, persister):
    assert not U.get_deployment_was_completed(store)
    U.set_deployment_was_completed(store)
    assert U.get_deployment_was_completed(store)
    assert persister.get("Properties/last-completed-update-type") == b"DEPLOY"
    U.set_deployment_was_completed(store)  # idempotent
    assert U.get_deployment_was_completed(store)


def test_task_status_property(store):
    assert U.get_task_status_from_property(store, "test-task") is None
    st = status(info("test-task").task_id, P.TASK_UNKNOWN)
    U.store_task_status_as_property(store, "test-task", st)
    assert U.get_task_status_from_property(store, "not-test-task") is None
    assert U.get_task_status_from_property(store, "test-task") == st
    assert "test-task:task-status" in store.fetch_property_keys()


def test_fetch_task_info_from_status(store):
    t = info("test-task")
    store.store_tasks([t])
    assert U.fetch_task_info(store, status(t.task_id, P.TASK_UNKNOWN)) == t
    with pytest.raises(StateStoreException):
        U.fetch_task_info(StateStore(MemPersister()), status(to_task_id(SERVICE, TASK), P.TASK_UNKNOWN))


def test_fetch_task_info_from_an_unparseable_task_id(store):
    with pytest.raises(StateStoreException):
        U.fetch_task_info(store, status(P.TaskID(value="garbage"), P.TASK_UNKNOWN))


def test_fetch_task_info_is_by_name_embedded_in_the_task_id(store):
    t = info(TASK)
    store.store_tasks([t])
    other = status(to_task_id(SERVICE, "not-" + TASK), P.TASK_UNKNOWN)
    assert t.task_id != other.task_id
    with pytest.raises(StateStoreException):
        U.fetch_task_info(store, other)


def test_repair_nothing_needed(store):
    t = info()
    store.store_tasks([t])
    st = status(t.task_id, P.TASK_UNKNOWN)
    store.store_status(TASK, st)
    U.repair_task_ids(store)
    assert store.fetch_task(TASK) == t and store.fetch_status(TASK) == st


def test_repair_missing_status_is_failed(store):
    t = info()
    store.store_tasks([t])
    U.repair_task_ids(store)
    assert store.fetch_task(TASK) == t
    st = store.fetch_status(TASK)
    assert st.state == P.TASK_FAILED and st.task_id == t.task_id


def test_repair_mismatched_ids_takes_the_status_id_and_fails_it(store):
    store.store_tasks([info()])
    tid = to_task_id(SERVICE, "not-" + TASK)
    store.store_status(TASK, status(tid, P.TASK_UNKNOWN))
    U.repair_task_ids(store)
    assert store.fetch_task(TASK).task_id == tid
    st = store.fetch_status(TASK)
    assert st.state == P.TASK_FAILED and st.task_id == tid


def test_repair_mismatch_with_an_empty_status_id_keeps_the_status(store):
    store.store_tasks([info()])
    empty = P.TaskID(value="")
    store.store_status(TASK, status(empty, P.TASK_UNKNOWN))
    U.repair_task_ids(store)
    assert store.fetch_task(TASK).task_id == empty
    st = store.fetch_status(TASK)
    assert st.state == P.TASK_UNKNOWN and st.task_id == empty


def test_repair_runs_when_a_store_is_opened(persister):
    s1 = StateStore(persister)
    t = info()
    s1.store_tasks([t])
    assert s1.fetch_statuses() == []
    s2 = StateStore(persister)  # a restarted scheduler
    (st,) = s2.fetch_statuses()
    assert st.task_id == t.task_id and st.state == P.TASK_FAILED


def test_repair_of_a_relaunch_recorded_before_its_status(persister):
    """The write-ahead TaskInfo of a relaunch was stored but the scheduler died before anything
    newer than the old task's status: the TaskInfo is reverted to the ID the status knows."""
    s1 = StateStore(persister)
    t = info()
    s1.store_tasks([t])
    s1.store_status(TASK, status(t.task_id))
    relaunch = info(tid=to_task_id(SERVICE, TASK))
    s1.store_tasks([relaunch])
    assert s1.fetch_task(TASK).task_id != t.task_id
    s2 = StateStore(persister)
    assert s2.fetch_task(TASK).task_id == t.task_id
    st = s2.fetch_status(TASK)
    assert st.task_id == t.task_id and st.state == P.TASK_FAILED
    expected = P.TaskInfo()
    expected.CopyFrom(relaunch)
    expected.task_id.CopyFrom(t.task_id)
    assert s2.fetch_task(TASK) == expected


def test_uninstalling_bit(store):
    assert not U.is_uninstalling(store)
    U.set_uninstalling(store)
    assert U.is_uninstalling(store)


@pytest.mark.parametrize("raw,expected", [(b"", False), (b"false", False), (b"true", True)])
def test_boolean_properties(store, raw, expected):
    store.store_property("k", raw)
    assert U._fetch_bool(store, "k") is expected


def test_invalid_boolean_property_raises(store):
    store.store_property("k", b"horses")
    with pytest.raises(StateStoreException):
        U._fetch_bool(store, "k")


# ---------------------------------------------------------------------------------------
# StateStore


def test_task_store_fetch_clear(store):
    assert store.fetch_task(TASK) is None and store.fetch_tasks() == [] and store.fetch_task_names() == []
    t = info()
    store.store_tasks([t])
    store.store_tasks([t])  # repeated store is an overwrite
    assert store.fetch_task(TASK) == t and store.fetch_task_names() == [TASK]
    store.clear_task(TASK)
    assert store.fetch_task(TASK) is None and store.fetch_tasks() == []
    store.clear_task("missing")  # clearing a missing task is a no-op


def test_multiple_tasks_and_statuses(store):
    a, b = info("a"), info("b")
    store.store_tasks([a, b])
    assert store.fetch_task_names() == ["a", "b"] and store.fetch_statuses() == []
    sa = status(a.task_id)
    store.store_status("a", sa)
    assert store.fetch_statuses() == [sa] and len(store.fetch_tasks()) == 2
    sb = status(b.task_id)
    store.store_status("b", sb)
    assert len(store.fetch_statuses()) == 2
    store.clear_task("a")
    assert store.fetch_task_names() == ["b"] and store.fetch_statuses() == [sb]
    store.clear_task("b")
    assert store.fetch_task_names() == [] and store.fetch_statuses() == []


def test_status_id_must_match_unless_a_new_staging(store):
    t = info()
    store.store_tasks([t])
    store.store_status(TASK, status(t.task_id))
    with pytest.raises(StateStoreException) as e:
        store.store_status(TASK, status(to_task_id(SERVICE, TASK)))
    assert e.value.reason == Reason.NOT_FOUND
    staging = status(to_task_id(SERVICE, TASK), P.TASK_STAGING)  # a relaunch's write-ahead status
    store.store_status(TASK, staging)
    assert store.fetch_status(TASK) == staging


def test_status_after_task_id_change_with_new_task_info(store):
    store.store_tasks([info()])
    first = store.fetch_task(TASK)
    store.store_status(TASK, status(first.task_id))
    new = info(tid=to_task_id(SERVICE, TASK))
    store.store_tasks([new])
    store.store_status(TASK, status(new.task_id, P.TASK_STAGING))
    store.store_status(TASK, status(new.task_id))
    assert store.fetch_status(TASK).task_id == new.task_id


@pytest.mark.parametrize("late", [P.TASK_LOST, P.TASK_GONE, P.TASK_DROPPED, P.TASK_UNKNOWN, P.TASK_UNREACHABLE])
def test_terminal_task_is_not_overwritten_by_a_late_lost_like_status(store, late):
    t = info()
    store.store_tasks([t])
    store.store_status(TASK, status(t.task_id, P.TASK_FINISHED))
    with pytest.raises(StateStoreException) as e:
        store.store_status(TASK, status(t.task_id, late))
    assert e.value.reason == Reason.LOGIC_ERROR
    assert store.fetch_status(TASK).state == P.TASK_FINISHED


def test_late_status_of_a_replaced_task_cannot_overwrite_the_relaunch_record():
    """A status of the old task, checked against the old task's status while another thread
    records the relaunch (new TaskInfo + STAGING), must not land on top of that record: the
    check and the write of a status and a launch record's write do not interleave."""
    import threading

    wrote_old = threading.Event()
    release = threading.Event()

    class SlowStatusWrites(MemPersister):
        def set(self, path, data):
            if path.endswith("TaskStatus") and not wrote_old.is_set():
                wrote_old.set()
                release.wait(5)          # the old task's status is checked and about to be written
            super().set(path, data)

    store = StateStore(SlowStatusWrites())
    old = info()
    store.store_tasks([old], [(TASK, status(old.task_id, P.TASK_STAGING))])
    store.persister.set("ready", b"")
    new = info(tid=to_task_id(SERVICE, TASK))
    errors = []

    def late_status():
        try:
            store.store_status(TASK, status(old.task_id, P.TASK_LOST))
        except StateStoreException as e:
            errors.append(e)
    t1 = threading.Thread(target=late_status)
    t1.start()
    assert wrote_old.wait(5)
    t2 = threading.Thread(target=lambda: store.store_tasks([new], [(TASK, status(new.task_id, P.TASK_STAGING))]))
    t2.start()
    t2.join(0.2)                        # the relaunch record waits for the status write in flight
    release.set()
    t1.join(5)
    t2.join(5)
    assert store.fetch_status(TASK).task_id == new.task_id
    assert store.fetch_status(TASK).state == P.TASK_STAGING


def test_terminal_task_accepts_a_new_terminal_state(store):
    t = info()
    store.store_tasks([t])
    store.store_status(TASK, status(t.task_id, P.TASK_FAILED))
    store.store_status(TASK, status(t.task_id, P.TASK_KILLED))
    assert store.fetch_status(TASK).state == P.TASK_KILLED


@pytest.mark.parametrize("key", ["", " ", "a/b", "/"])
@pytest.mark.parametrize("op", ["store", "fetch", "clear"])
def test_invalid_property_keys(store, key, op):
    with pytest.raises(StateStoreException):
        {"store": lambda: store.store_property(key, b"v"), "fetch": lambda: store.fetch_property(key),
         "clear": lambda: store.clear_property(key)}[op]()


def test_property_value_rules(store):
    with pytest.raises(StateStoreException):
        store.store_property("k", None)
    with pytest.raises(StateStoreException):
        store.store_property("k", b"x" * (1000 * 1000 + 1))
    store.store_property("k", b"x" * (1000 * 1000))
    assert store.fetch_property_keys() == ["k"]
    store.clear_property("k")
    store.clear_property("k")  # clearing twice is fine
    assert store.fetch_property_keys() == []
    with pytest.raises(StateStoreException) as e:
        store.fetch_property("k")
    assert e.value.reason == Reason.NOT_FOUND


def test_store_properties_batch(store, persister):
    store.store_properties({"a": b"1", "b": b"2"})
    assert sorted(store.fetch_property_keys()) == ["a", "b"]
    with pytest.raises(StateStoreException):
        store.store_properties({"ok": b"1", "bad/key": b"2"})
    assert "ok" not in store.fetch_property_keys()  # validated before anything is written


def test_goal_override_full_cycle(store, persister):
    assert store.fetch_goal_override_status("hello") == OverrideStatus.INACTIVE
    for target in (GoalStateOverride.PAUSED, GoalStateOverride.NONE):
        for progress in (OverrideProgress.PENDING, OverrideProgress.IN_PROGRESS, OverrideProgress.COMPLETE):
            st = target.new_status(progress)
            store.store_goal_override_status("hello", st)
            assert store.fetch_goal_override_status("hello") == st
    store.store_goal_override_status("hello", OverrideStatus.INACTIVE)
    assert store.fetch_goal_override_status("hello") == OverrideStatus.INACTIVE
    with pytest.raises(Exception):
        persister.get("Tasks/hello/Metadata/goal-state-override")


def test_half_written_override_reads_as_inactive(store, persister):
    persister.set("Tasks/hello/Metadata/goal-state-override", b"PAUSED")
    assert store.fetch_goal_override_status("hello") == OverrideStatus.INACTIVE
    persister.set("Tasks/hello/Metadata/override-status", b"NOT_A_PROGRESS")
    assert store.fetch_goal_override_status("hello") == OverrideStatus.INACTIVE


def test_namespaced_layout_and_delete(persister):
    root = StateStore(persister)
    ns = StateStore(persister, "test-namespace")
    ns2 = StateStore(persister, "test-namespace-two")
    for s in (root, ns, ns2):
        t = info()
        s.store_tasks([t])
        s.store_status(TASK, status(t.task_id))
        s.store_goal_override_status(TASK, GoalStateOverride.PAUSED.new_status(OverrideProgress.PENDING))
        s.store_property("good-key", b"value")
    assert persister.get("Tasks/" + TASK + "/Metadata/override-status") == b"PENDING"
    assert persister.get("Services/test-namespace/Tasks/" + TASK + "/Metadata/goal-state-override") == b"PAUSED"
    assert persister.get("Services/test-namespace/Properties/good-key") == b"value"
    root.delete_all_data_if_namespaced()  # not namespaced: nothing happens
    assert root.fetch_status(TASK) is not None
    ns.delete_all_data_if_namespaced()
    assert ns.fetch_status(TASK) is None and ns.fetch_property_keys() == []
    assert ns2.fetch_status(TASK) is not None and root.fetch_status(TASK) is not None


def test_empty_persisted_task_info_is_a_serialization_error(store, persister):
    persister.set("Tasks/broken/TaskInfo", b"")
    with pytest.raises(StateStoreException) as e:
        store.fetch_task("broken")
    assert e.value.reason == Reason.SERIALIZATION_ERROR


# ---------------------------------------------------------------------------------------
# FrameworkStore / SchemaVersionStore


def test_framework_store_round_trip_and_clear(persister):
    fs = FrameworkStore(persister)
    assert fs.fetch_framework_id() is None
    fs.clear_framework_id()  # clearing a missing ID is fine
    fid = P.FrameworkID(value="test-framework-id")
    fs.store_framework_id(fid)
    assert fs.fetch_framework_id() == fid
    assert P.FrameworkID.FromString(persister.get("FrameworkID")) == fid
    fs.store_framework_id(P.FrameworkID(value="other"))
    assert fs.fetch_framework_id().value == "other"
    fs.clear_framework_id()
    assert fs.fetch_framework_id() is None


def test_schema_version_store(persister):
    sv = SchemaVersionStore(persister)
    sv.check(SchemaVersion.SINGLE_SERVICE)  # an empty store is initialised to the expected version
    assert persister.get("SchemaVersion") == b"1"
    sv.check(SchemaVersion.SINGLE_SERVICE)
    with pytest.raises(Exception):
        sv.check(SchemaVersion.MULTI_SERVICE)  # migrating to multi is an explicit step
    persister.set("SchemaVersion", b"not-a-number")
    with pytest.raises(Exception):
        SchemaVersionStore(persister).check(SchemaVersion.SINGLE_SERVICE)


def test_status_is_stored_even_when_its_property_is_not(store, persister):
    """the ``<task>:task-status`` property rides in the status's transaction, but as in
    the reference (stored after the status, failures only logged) it can never cost the status."""
    t = info()
    store.store_tasks([t])
    st = status(t.task_id)
    # an invalid key or an oversized value: dropped with a warning, the status is stored
    store.store_status(TASK, st, {"bad/key": b"v", TASK + ":task-status": b"x" * (1024 * 1024 + 1)})
    assert store.fetch_status(TASK) == st
    assert store.fetch_property_keys() == []
    # a valid property is written with it
    store.store_status(TASK, st, {TASK + ":task-status": st.SerializeToString()})
    assert store.fetch_property(TASK + ":task-status") == st.SerializeToString()

    # the combined write failing: the status alone is retried
    class Flaky(MemPersister):
        def set_many(self, values):
            from dcos_commons_amd.storage.persister import PersisterException

            if any("Properties" in k for k in values):
                raise PersisterException(Reason.STORAGE_ERROR, "multi failed")
            return super().set_many(values)
    flaky = StateStore(Flaky())
    flaky.store_tasks([t])
    st2 = status(t.task_id, P.TASK_FAILED)
    flaky.store_status(TASK, st2, {TASK + ":task-status": st2.SerializeToString()})
    assert flaky.fetch_status(TASK) == st2


def test_fetch_tasks_shared_reuses_unchanged_tasks(store):
    a, b = info("a"), info("b")
    store.store_tasks([a, b])
    first = {t.name: t for t in store.fetch_tasks_shared()}
    again = {t.name: t for t in store.fetch_tasks_shared()}
    assert first["a"] is again["a"] and first["b"] is again["b"]
    changed = info("a")
    changed.labels.labels.add(key="k", value="v")
    store.store_tasks([changed])
    third = {t.name: t for t in store.fetch_tasks_shared()}
    assert third["a"] is not first["a"] and third["a"] == changed and third["b"] is first["b"]
    store.clear_task("b")
    assert [t.name for t in store.fetch_tasks_shared()] == ["a"] and "b" not in store._shared


def test_fetch_tasks_shared_detects_a_caller_that_modified_a_task(store, monkeypatch):
    from dcos_commons_amd.state import state_store as SS

    monkeypatch.setattr(SS, "_DEBUG_SHARED", True)
    store.store_tasks([info("a")])
    t = store.fetch_tasks_shared()[0]
    t.labels.labels.add(key="oops", value="1")
    with pytest.raises(AssertionError):
        store.fetch_tasks_shared()
