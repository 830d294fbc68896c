"""Launch recorder and schema-version units.

Mirrors sdk/scheduler/src/test/java/com/mesosphere/sdk/state/{PersistentLaunchRecorderTest,
SchemaVersionStoreTest}.java: resources of a launched task are copied onto the stored tasks that
share its resource set (the reference's ``shared-resource-set.yml``: an ONCE ``init`` and a RUNNING
``server`` on one set), tasks outside the spec are left alone, and the schema-version node's
corrupt / empty / failing cases.
"""
import textwrap

import pytest

import testutils as U
from dcos_commons_amd.mesos import protos as P
from dcos_commons_amd.offer.recommendations import LaunchOfferRecommendation, StoreTaskInfoRecommendation
from dcos_commons_amd.offer.taskdata.labels import TaskLabelReader, TaskLabelWriter
from dcos_commons_amd.scheduler.scheduler_config import SchedulerConfig
from dcos_commons_amd.specification.yaml import mappers
from dcos_commons_amd.specification.yaml.raw import RawServiceSpec
from dcos_commons_amd.state.persistent_launch_recorder import PersistentLaunchRecorder
from dcos_commons_amd.state.schema_version_store import SchemaVersion, SchemaVersionStore
from dcos_commons_amd.state.state_store import StateStore, StateStoreException
from dcos_commons_amd.storage.mem_persister import MemPersister
from dcos_commons_amd.storage.persister import Persister, PersisterException, Reason

SHARED = """\
    name: test
    pods:
      pod:
        count: 2
        resource-sets:
          shared-resources:
            cpus: 1.0
        tasks:
          init:
            goal: ONCE
            cmd: ./init
            resource-set: shared-resources
          server:
            goal: RUNNING
            cmd: ./server
            resource-set: shared-resources
    """
SPEC = mappers.ServiceSpecGenerator(RawServiceSpec.from_string(textwrap.dedent(SHARED)), SchedulerConfig.for_testing(),
                                    "/tmp", {}).build()


@pytest.fixture
def env():
    store = StateStore(MemPersister())
    return store, PersistentLaunchRecorder(store, SPEC)


def _cpus(v):
    r = P.Resource(name="cpus", type=P.Value.SCALAR)
    r.scalar.value = v
    return r


def _task(name, type_=None, index=None, resources=(), task_id=None):
    t = P.TaskInfo(name=name)
    t.task_id.CopyFrom(task_id or U.TASK_ID)
    t.agent_id.CopyFrom(U.AGENT_ID)
    w = TaskLabelWriter(t)
    if type_ is not None:
        w.set_type(type_)
    if index is not None:
        w.set_index(index)
    w.apply()
    t.resources.extend(resources)
    return t


def _store(task):
    return StoreTaskInfoRecommendation(U.empty_offer(), task, P.ExecutorInfo())


def test_task_without_a_type_label_is_recorded_without_touching_peers(env):
    store, recorder = env
    assert recorder._pod_instance(_task(U.TASK_NAME)) is None
    recorder.record([_store(_task(U.TASK_NAME))])
    assert store.fetch_task_names() == [U.TASK_NAME]


def test_task_of_an_unknown_pod_type_has_no_pod_instance(env):
    _, recorder = env
    assert recorder._pod_instance(_task(U.TASK_NAME, type_=U.TASK_TYPE, index=0)) is None


def test_lone_task_keeps_its_resources(env):
    store, recorder = env
    init = _task("pod-0-init", "pod", 0, [_cpus(1.0)])
    store.store_tasks([init])
    recorder._update_resource_set_peers(recorder._pod_instance(init), init)
    assert store.fetch_task_names() == ["pod-0-init"]
    assert list(store.fetch_task("pod-0-init").resources) == [_cpus(1.0)]


def test_resources_are_copied_to_tasks_sharing_the_resource_set(env):
    store, recorder = env
    store.store_tasks([_task("pod-0-init", "pod", 0, [_cpus(2.0)]), _task("pod-0-server", "pod", 0, [_cpus(1.0)])])
    server = store.fetch_task("pod-0-server")
    assert store.fetch_task("pod-0-init").resources[0] != server.resources[0]
    recorder._update_resource_set_peers(recorder._pod_instance(server), server)
    assert sorted(store.fetch_task_names()) == ["pod-0-init", "pod-0-server"]
    assert store.fetch_task("pod-0-init").resources[0] == _cpus(1.0)
    assert store.fetch_task("pod-0-server").resources[0] == _cpus(1.0)


def test_other_pod_instances_are_not_touched(env):
    store, recorder = env
    store.store_tasks([_task("pod-1-init", "pod", 1, [_cpus(2.0)])])
    server = _task("pod-0-server", "pod", 0, [_cpus(1.0)])
    recorder.record([_store(server)])
    assert store.fetch_task("pod-1-init").resources[0] == _cpus(2.0)


def test_record_stores_empty_ids_first_and_a_staging_status_for_launches(env):
    store, recorder = env
    launched = _task("pod-0-server", "pod", 0, [_cpus(1.0)], task_id=P.TaskID(value="pod-0-server__id"))
    placeholder = _task("pod-0-init", "pod", 0, [_cpus(1.0)], task_id=P.TaskID(value=""))
    recs = [_store(launched), LaunchOfferRecommendation(U.empty_offer(), launched, P.ExecutorInfo()),
            _store(placeholder)]
    recorder.record(recs)
    assert store.fetch_status("pod-0-server").state == P.TASK_STAGING
    assert store.fetch_status("pod-0-init") is None  # a placeholder is not launched
    assert TaskLabelReader(store.fetch_task("pod-0-server")).is_launch_new_footprint() is False  # no reservation ids


# ---------------------------------------------------------------------------------------
# SchemaVersionStore


def test_schema_version_auto_initializes_and_round_trips():
    p = MemPersister()
    s = SchemaVersionStore(p)
    assert s.get_or_set_version(SchemaVersion.SINGLE_SERVICE) == SchemaVersion.SINGLE_SERVICE
    assert p.get("SchemaVersion") == b"1"
    s.store(SchemaVersion.MULTI_SERVICE)
    assert SchemaVersionStore(p).get_or_set_version(SchemaVersion.SINGLE_SERVICE) == SchemaVersion.MULTI_SERVICE
    with pytest.raises(ValueError, match="version 2 is not supported"):
        SchemaVersionStore(p).check(SchemaVersion.SINGLE_SERVICE)


@pytest.mark.parametrize("raw", [b"hello", b""])
def test_corrupt_or_empty_schema_version(raw):
    p = MemPersister()
    p.set("SchemaVersion", raw)
    with pytest.raises(StateStoreException) as e:
        SchemaVersionStore(p).check(SchemaVersion.UNKNOWN)
    assert e.value.reason == Reason.SERIALIZATION_ERROR


class BrokenPersister(MemPersister):
    def get(self, path):
        raise PersisterException(Reason.LOGIC_ERROR, "hey")

    def set(self, path, data):
        raise PersisterException(Reason.STORAGE_ERROR, "hey")


def test_schema_version_read_failure():
    with pytest.raises(StateStoreException) as e:
        SchemaVersionStore(BrokenPersister()).check(SchemaVersion.UNKNOWN)
    assert e.value.reason == Reason.STORAGE_ERROR


def test_schema_version_store_rejects_unknown_and_reports_write_failures():
    with pytest.raises(ValueError):
        SchemaVersionStore(MemPersister()).store(SchemaVersion.UNKNOWN)
    with pytest.raises(StateStoreException):
        SchemaVersionStore(BrokenPersister()).store(SchemaVersion.MULTI_SERVICE)


# ---------------------------------------------------------------------------------------
# batched recording: the final state of the reference's write-per-task sequence, written once


class CountingPersister(MemPersister):
    def __init__(self):
        super().__init__()
        self.writes = []

    def set(self, path, value):
        self.writes.append(path)
        super().set(path, value)

    def set_many(self, mapping):
        self.writes.extend(mapping)
        super().set_many(mapping)


def _sequential_record(store, recorder, recs):
    """The reference's order (PersistentLaunchRecorder.record): each TaskInfo stored with its
    resource-set peers rewritten from the store, then its STAGING status."""
    stores = sorted((r for r in recs if isinstance(r, StoreTaskInfoRecommendation)),
                    key=lambda r: len(r.task_info.task_id.value))
    for rec in stores:
        info = rec.state_store_task_info()
        pi = recorder._pod_instance(info)
        if pi is not None:
            recorder._update_resource_set_peers(pi, info)
        store.store_tasks([info])
        if info.task_id.value:
            st = P.TaskStatus(state=P.TASK_STAGING)
            st.task_id.CopyFrom(info.task_id)
            store.store_status(info.name, st)


def test_batched_record_matches_the_sequential_final_state():
    new_res = [_cpus(3.0)]
    recs = [_store(_task("pod-0-server", "pod", 0, new_res, task_id=P.TaskID(value="pod-0-server__new"))),
            _store(_task("pod-0-init", "pod", 0, new_res, task_id=P.TaskID(value="")))]
    finals = []
    for batched in (True, False):
        store = StateStore(MemPersister())
        recorder = PersistentLaunchRecorder(store, SPEC)
        store.store_tasks([_task("pod-0-init", "pod", 0, [_cpus(1.0)]), _task("pod-1-init", "pod", 1, [_cpus(2.0)])])
        if batched:
            recorder.record(recs)
        else:
            _sequential_record(store, recorder, recs)
        finals.append({n: (store.fetch_task(n).SerializeToString(deterministic=True),
                           store.fetch_status(n) and store.fetch_status(n).state)
                       for n in store.fetch_task_names()})
    # the launch-footprint label is the batched recorder's own addition: compare without it
    for f in finals:
        for n, (data, st) in list(f.items()):
            t = P.TaskInfo()
            t.ParseFromString(data)
            for label in list(t.labels.labels):
                if label.key == "launch_new_footprint":
                    t.labels.labels.remove(label)
            f[n] = (t.SerializeToString(deterministic=True), st)
    assert finals[0] == finals[1]
    assert finals[0]["pod-1-init"][0] == _task("pod-1-init", "pod", 1, [_cpus(2.0)]).SerializeToString(
        deterministic=True)


def test_record_writes_each_task_once_and_skips_unchanged_peers():
    p = CountingPersister()
    store = StateStore(p)
    recorder = PersistentLaunchRecorder(store, SPEC)
    same = [_cpus(1.0)]
    store.store_tasks([_task("pod-0-init", "pod", 0, same)])
    p.writes.clear()
    recorder.record([_store(_task("pod-0-server", "pod", 0, same, task_id=P.TaskID(value="pod-0-server__x")))])
    task_writes = [w for w in p.writes if w.endswith("/TaskInfo")]
    assert task_writes == ["Tasks/pod-0-server/TaskInfo"]  # the peer already holds these resources
    assert store.fetch_status("pod-0-server").state == P.TASK_STAGING


def test_launch_record_writes_taskinfos_and_staging_statuses_in_one_transaction():
    """A launch's TaskInfos and their STAGING statuses go to the persister in one set_many (one
    ZooKeeper multi); a status the store would reject stops the whole record before any write."""
    from dcos_commons_amd.state.state_store import StateStore, StateStoreException
    from dcos_commons_amd.storage.mem_persister import MemPersister

    class Counting(MemPersister):
        def __init__(self):
            super().__init__()
            self.writes = []

        def set_many(self, m):
            self.writes.append(sorted(m))
            return super().set_many(m)

        def set(self, path, data):
            self.writes.append([path])
            return super().set(path, data)

    p = Counting()
    ss = StateStore(p)
    info = P.TaskInfo(name="pod-0-task")
    info.task_id.value = "svc__pod-0-task__1"
    st = P.TaskStatus(state=P.TASK_STAGING)
    st.task_id.CopyFrom(info.task_id)
    ss.store_tasks([info], [("pod-0-task", st)])
    assert len(p.writes) == 1 and any(w.endswith("TaskStatus") for w in p.writes[0])
    assert ss.fetch_status("pod-0-task").state == P.TASK_STAGING
    # a RUNNING status for another task ID is rejected before anything is written
    p.writes.clear()
    bad = P.TaskStatus(state=P.TASK_RUNNING)
    bad.task_id.value = "svc__pod-0-task__other"
    with pytest.raises(StateStoreException):
        ss.store_tasks([info], [("pod-0-task", bad)])
    assert p.writes == []
