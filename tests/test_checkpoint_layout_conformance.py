"""Checkpoint layout conformance: the persister tree this SDK writes uses the path
names the reference defines, read from the reference's own Java sources.

The reference's scheduler state lives in ZooKeeper under names that are private constants of its
stores (``state/StateStore.java:62-74``, ``ConfigStore.java:38-40``, ``FrameworkStore.java:26``,
``SchemaVersionStore.java:34``, ``StateStoreUtils.java:38-42``, ``storage/PersisterUtils.java:46``,
``curator/CuratorUtils.java:28-34``, ``curator/CuratorLocker.java:20``,
``scheduler/multi/ServiceStore.java:29-34``, ``DisciplineSelectionStore.java:29-32``). A scheduler
built on one can only take over the state of the other if every one of them matches. The test
parses those constants out of the Java files (skipped when the reference checkout is absent),
writes one of everything through this SDK's stores, and compares the resulting tree path by path.
"""
import os
import re
import uuid

import pytest

from dcos_commons_amd.mesos import protos as P
from dcos_commons_amd.scheduler.multi import DisciplineSelectionStore, ServiceStore
from dcos_commons_amd.state import state_store_utils as SSU
from dcos_commons_amd.state.config_store import ConfigStore
from dcos_commons_amd.state.framework_store import FrameworkStore
from dcos_commons_amd.state.goal_state_override import GoalStateOverride, OverrideProgress, OverrideStatus
from dcos_commons_amd.state.schema_version_store import SchemaVersion, SchemaVersionStore
from dcos_commons_amd.state.state_store import StateStore
from dcos_commons_amd.storage import persister_utils as PU
from dcos_commons_amd.storage.mem_persister import MemPersister
from dcos_commons_amd.storage.zk_persister import get_service_root_path

REF = os.environ.get("SDK_REFERENCE_ROOT", "/root/reference")
JAVA = os.path.join(REF, "sdk/scheduler/src/main/java/com/mesosphere/sdk")

pytestmark = pytest.mark.skipif(not os.path.isdir(JAVA), reason="reference sources not available")


def _constants(rel: str) -> dict:
    text = open(os.path.join(JAVA, rel), encoding="utf-8").read()
    return dict(re.findall(r'static final String (\w+) = "([^"]*)";', text))


@pytest.fixture(scope="module")
def ref():
    c = {}
    for rel in ("state/StateStore.java", "state/ConfigStore.java", "state/FrameworkStore.java",
                "state/SchemaVersionStore.java", "state/StateStoreUtils.java", "storage/PersisterUtils.java",
                "curator/CuratorUtils.java", "curator/CuratorLocker.java", "scheduler/multi/ServiceStore.java",
                "scheduler/multi/DisciplineSelectionStore.java"):
        c.update(_constants(rel))
    return c


class _Spec:
    """A config-store payload (the store only needs ``get_bytes``)."""

    def get_bytes(self) -> bytes:
        return b'{"name":"svc"}'


def _write_everything(persister, namespace=None):
    store = StateStore(persister, namespace)
    task = P.TaskInfo(name="hello-0-server")
    task.task_id.value = "svc__hello-0-server__" + str(uuid.uuid4())
    task.agent_id.value = "agent"
    status = P.TaskStatus(state=P.TASK_RUNNING)
    status.task_id.CopyFrom(task.task_id)
    store.store_tasks([task])
    store.store_status("hello-0-server", status)
    store.store_goal_override_status("hello-0-server", OverrideStatus(GoalStateOverride.PAUSED,
                                                                      OverrideProgress.PENDING))
    SSU.set_uninstalling(store)
    SSU.set_deployment_was_completed(store)
    SSU.store_task_status_as_property(store, "hello-0-server", status)
    configs = ConfigStore(None, persister, namespace)
    cid = configs.store(_Spec())
    configs.set_target_config(cid)
    return cid


def test_single_service_tree_uses_the_reference_names(ref):
    p = MemPersister()
    FrameworkStore(p).store_framework_id(P.FrameworkID(value="fw-1"))
    SchemaVersionStore(p).store(SchemaVersion.SINGLE_SERVICE)
    cid = _write_everything(p)
    paths = set(PU.get_all_data(p))
    task = f"{ref['TASKS_ROOT_NAME']}/hello-0-server"
    meta = f"{task}/{ref['TASK_METADATA_PATH_NAME']}"
    expected = {
        ref["FWK_ID_PATH_NAME"],
        ref["SCHEMA_VERSION_NAME"],
        ref["TARGET_ID_PATH_NAME"],
        f"{ref['CONFIGURATIONS_PATH_NAME']}/{cid}",
        f"{task}/{ref['TASK_INFO_PATH_NAME']}",
        f"{task}/{ref['TASK_STATUS_PATH_NAME']}",
        f"{meta}/{ref['TASK_GOAL_OVERRIDE_PATH_NAME']}",
        f"{meta}/{ref['TASK_GOAL_OVERRIDE_STATUS_PATH_NAME']}",
        f"{ref['PROPERTIES_ROOT_NAME']}/{ref['UNINSTALLING_PROPERTY_KEY']}",
        f"{ref['PROPERTIES_ROOT_NAME']}/{ref['LAST_COMPLETED_UPDATE_TYPE_KEY']}",
        f"{ref['PROPERTIES_ROOT_NAME']}/hello-0-server{ref['PROPERTY_TASK_INFO_SUFFIX']}",
    }
    # every leaf written, under exactly the reference's names (leading "/" aside)
    assert {x.strip("/") for x in paths} == expected


def test_multi_service_tree_uses_the_reference_names(ref):
    p = MemPersister()
    SchemaVersionStore(p).store(SchemaVersion.MULTI_SERVICE)
    cid = _write_everything(p, namespace="path/to/svc")
    ServiceStore(p, lambda ctx: type("S", (), {"service_spec": type("X", (), {"name": "/path/to/svc"})()})()) \
        .put(b"context")
    DisciplineSelectionStore(p).store_selected_services({"a", "b"})
    paths = {x.strip("/") for x in PU.get_all_data(p)}
    ns = f"{ref['SERVICE_NAMESPACE_ROOT_NAME']}/path__to__svc"
    assert f"{ns}/{ref['TARGET_ID_PATH_NAME']}" in paths
    assert f"{ns}/{ref['CONFIGURATIONS_PATH_NAME']}/{cid}" in paths
    assert f"{ns}/{ref['TASKS_ROOT_NAME']}/hello-0-server/{ref['TASK_INFO_PATH_NAME']}" in paths
    assert f"{ns}/{ref['PROPERTIES_ROOT_NAME']}/{ref['UNINSTALLING_PROPERTY_KEY']}" in paths
    assert f"{ref['ROOT_PATH_NAME']}/path__to__svc/{ref['CONTEXT_NODE']}" in paths
    assert ref["SELECTED_SERVICES_PATH_NAME"] in paths
    assert p.get(ref["SELECTED_SERVICES_PATH_NAME"]) == ref["SERVICE_NAME_DELIMITER"].join(["a", "b"]).encode()
    assert ref["SCHEMA_VERSION_NAME"] in paths


def test_zookeeper_root_and_lock_names(ref):
    from dcos_commons_amd.storage import zk_persister as ZP

    # CuratorUtils.getServiceRootPath: prefix + SchedulerUtils.withEscapedSlashes(name)
    assert get_service_root_path("/path/to/svc") == ref["SERVICE_ROOT_PATH_PREFIX"] + "path__to__svc"
    assert get_service_root_path("hello-world") == ref["SERVICE_ROOT_PATH_PREFIX"] + "hello-world"
    src = open(ZP.__file__, encoding="utf-8").read()
    assert f'"{ref["SERVICE_NAME_NODE"]}"' in src and f'"{ref["LOCK_PATH_NAME"]}"' in src
