"""StateStore helpers: well-known properties and TaskID repair.

Reference: sdk/.../state/StateStoreUtils.java:38-256.
"""
from __future__ import annotations

import logging
from typing import List, Optional

from dcos_commons_amd.mesos import protos as P
from dcos_commons_amd.offer import common_id_utils
from dcos_commons_amd.storage.persister import Reason

from .serializer import JsonSerializer
from .state_store import StateStore, StateStoreException

LOGGER = logging.getLogger(__name__)
UNINSTALLING_PROPERTY_KEY = "uninstalling"
LAST_COMPLETED_UPDATE_TYPE_KEY = "last-completed-update-type"
PROPERTY_TASK_INFO_SUFFIX = ":task-status"
DEPLOYMENT_TYPE = b"DEPLOY"


def fetch_property_or_empty(store: StateStore, key: str) -> bytes:
    if key in store.fetch_property_keys():
        return store.fetch_property(key) or b""
    return b""


def fetch_pod_tasks(store: StateStore, pod_instance) -> List[P.TaskInfo]:
    out = []
    for t in pod_instance.pod.tasks:
        info = store.fetch_task(f"{pod_instance.name}-{t.name}")
        if info is not None:
            out.append(info)
    return out


def fetch_task_info(store: StateStore, status: P.TaskStatus) -> P.TaskInfo:
    try:
        name = common_id_utils.to_task_name(status.task_id)
    except Exception as e:  # noqa: BLE001
        raise StateStoreException(Reason.SERIALIZATION_ERROR, str(e)) from e
    info = store.fetch_task_shared(name)     # callers read it (and copy before any change)
    if info is None:
        raise StateStoreException(Reason.NOT_FOUND, f"Failed to find a task with TaskID: {status.task_id.value}")
    return info


def repair_task_ids(store: StateStore) -> None:
    """Fix TaskInfo/TaskStatus TaskID mismatches left by a crash between the write-ahead
    TaskInfo record and the launch (StateStoreUtils.repairTaskIDs)."""
    from dcos_commons_amd.offer.task_utils import is_terminal

    repaired_statuses = {}
    repaired_tasks = []
    for task in store.fetch_tasks_shared():     # repairs are made on copies
        status = store.fetch_status(task.name)
        if status is not None:
            if task.task_id.value == "" and is_terminal(status):
                repaired_statuses[task.name] = status
            elif status.task_id.value != task.task_id.value:
                LOGGER.warning("Found StateStore status inconsistency for task %s: task.taskId=%s, status.taskId=%s",
                               task.name, task.task_id.value, status.task_id.value)
                t = P.TaskInfo()
                t.CopyFrom(task)
                t.task_id.CopyFrom(status.task_id)
                repaired_tasks.append(t)
                s = P.TaskStatus()
                s.CopyFrom(status)
                s.state = P.TASK_FAILED
                repaired_statuses[task.name] = s
        else:
            LOGGER.warning("Found StateStore status inconsistency for task %s: no status", task.name)
            s = P.TaskStatus(state=P.TASK_FAILED, message="Assuming failure for inconsistent TaskIDs")
            s.task_id.CopyFrom(task.task_id)
            repaired_statuses[task.name] = s
    if repaired_tasks:
        store.store_tasks(repaired_tasks)
    for name, s in repaired_statuses.items():
        if s.task_id.value != "":
            store.store_status(name, s)


def _fetch_bool(store: StateStore, key: str) -> bool:
    data = fetch_property_or_empty(store, key)
    if not data:
        return False
    try:
        return bool(JsonSerializer().deserialize(data))
    except ValueError as e:
        raise StateStoreException(Reason.SERIALIZATION_ERROR, str(e)) from e


def is_uninstalling(store: StateStore) -> bool:
    return _fetch_bool(store, UNINSTALLING_PROPERTY_KEY)


def set_uninstalling(store: StateStore) -> None:
    store.store_property(UNINSTALLING_PROPERTY_KEY, JsonSerializer().serialize(True))


def store_task_status_as_property(store: StateStore, task_name: str, status: P.TaskStatus) -> None:
    store.store_property(task_name + PROPERTY_TASK_INFO_SUFFIX, status.SerializeToString())


def get_task_status_from_property(store: StateStore, task_name: str) -> Optional[P.TaskStatus]:
    try:
        data = store.fetch_property(task_name + PROPERTY_TASK_INFO_SUFFIX)
        s = P.TaskStatus()
        s.ParseFromString(data or b"")
        return s
    except Exception:  # noqa: BLE001
        LOGGER.error("Unable to decode TaskStatus for taskName=%s", task_name)
        return None


def set_deployment_was_completed(store: StateStore) -> None:
    if not get_deployment_was_completed(store):
        store.store_property(LAST_COMPLETED_UPDATE_TYPE_KEY, DEPLOYMENT_TYPE)


def get_deployment_was_completed(store: StateStore) -> bool:
    return fetch_property_or_empty(store, LAST_COMPLETED_UPDATE_TYPE_KEY) == DEPLOYMENT_TYPE
