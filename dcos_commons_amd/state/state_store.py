"""Persistent task state: TaskInfo / TaskStatus / goal overrides / properties.

Reference: sdk/.../state/StateStore.java:58-688. Layout (per service namespace)::

    Tasks/<pod>-<i>-<task>/TaskInfo                    protobuf TaskInfo bytes
    Tasks/<pod>-<i>-<task>/TaskStatus                  protobuf TaskStatus bytes
    Tasks/<pod>-<i>-<task>/Metadata/goal-state-override
    Tasks/<pod>-<i>-<task>/Metadata/override-status
    Properties/<key>                                   raw bytes (<= 1 MB)

TaskInfo writes are batched into <= 1 MB ``set_many`` transactions (StateStore.java:213).
A status that would move an already-terminal task to LOST/GONE/... is rejected, as is a
status whose TaskID differs from the stored one (other than the synthetic STAGING).
"""
from __future__ import annotations

import functools
import logging
import os
import threading
import weakref
from typing import Collection, Dict, List, Optional, Tuple

from dcos_commons_amd.mesos import protos as P
from dcos_commons_amd.storage.persister import Persister, PersisterException, Reason
from dcos_commons_amd.storage.persister_utils import (
    get_service_namespaced_root,
    get_service_namespaced_root_path,
    join_paths,
)

from .goal_state_override import GoalStateOverride, OverrideProgress, OverrideStatus

MAX_VALUE_LENGTH_BYTES = 1000 * 1000
TASK_INFO_PATH_NAME = "TaskInfo"
TASK_STATUS_PATH_NAME = "TaskStatus"
TASK_METADATA_PATH_NAME = "Metadata"
TASK_GOAL_OVERRIDE_PATH_NAME = "goal-state-override"
TASK_GOAL_OVERRIDE_STATUS_PATH_NAME = "override-status"
PROPERTIES_ROOT_NAME = "Properties"
TASKS_ROOT_NAME = "Tasks"

_NON_TERMINAL_OVERWRITE_STATES = frozenset(
    [P.TASK_LOST, P.TASK_GONE, P.TASK_DROPPED, P.TASK_UNKNOWN, P.TASK_UNREACHABLE])


_UNSET = object()


class StateStoreException(Exception):
    def __init__(self, reason: Reason, message: str = ""):
        super().__init__(f"{reason.value}: {message}")
        self.reason = reason


_DEBUG_SHARED = os.environ.get("SDK_DEBUG_SHARED_TASKS", "") not in ("", "0", "false")
_STATUS_LOCKS: "weakref.WeakKeyDictionary" = weakref.WeakKeyDictionary()
_STATUS_LOCKS_GUARD = threading.Lock()


def _status_lock(persister) -> threading.RLock:
    """One lock per persister for every write that checks or replaces a TaskStatus: the status
    thread's check-then-write (``store_status``) must not interleave with a launch record written
    from another thread (``store_tasks``), or a late status of a replaced task could overwrite the
    new task's STAGING status after passing its check against the old one."""
    with _STATUS_LOCKS_GUARD:
        lock = _STATUS_LOCKS.get(persister)
        if lock is None:
            lock = _STATUS_LOCKS[persister] = threading.RLock()
        return lock


def _status_write(fn):
    @functools.wraps(fn)
    def locked(self, *args, **kwargs):
        with self._status_lock:
            return fn(self, *args, **kwargs)
    return locked


class StateStore:
    def __init__(self, persister: Persister, namespace: Optional[str] = None, repair: bool = True):
        self.persister = persister
        self._status_lock = _status_lock(persister)
        self._shared: Dict[str, tuple] = {}   # task name -> (TaskInfo bytes, parsed TaskInfo)
        self.namespace = namespace or ""
        self.logger = logging.getLogger(__name__ + (f"({self.namespace})" if self.namespace else ""))
        self._tasks_root = get_service_namespaced_root_path(self.namespace, TASKS_ROOT_NAME)
        # task name -> (task, TaskInfo, TaskStatus, goal-override, override-status) paths: every
        # offer cycle and status update reads these for every task
        self._paths: Dict[str, tuple] = {}
        if repair:
            from .state_store_utils import repair_task_ids

            repair_task_ids(self)

    # -- paths ---------------------------------------------------------------------------
    def _task_paths(self, name: str) -> tuple:
        p = self._paths.get(name)
        if p is None:
            task = join_paths(self._tasks_root, name)
            p = (task, join_paths(task, TASK_INFO_PATH_NAME), join_paths(task, TASK_STATUS_PATH_NAME),
                 join_paths(task, TASK_METADATA_PATH_NAME, TASK_GOAL_OVERRIDE_PATH_NAME),
                 join_paths(task, TASK_METADATA_PATH_NAME, TASK_GOAL_OVERRIDE_STATUS_PATH_NAME))
            if len(self._paths) < 100000:      # bounded: task names come from pod specs
                self._paths[name] = p
        return p

    def _task_path(self, task_name: str) -> str:
        return self._task_paths(task_name)[0]

    def _task_info_path(self, name: str) -> str:
        return self._task_paths(name)[1]

    def _task_status_path(self, name: str) -> str:
        return self._task_paths(name)[2]

    def _goal_override_path(self, name: str) -> str:
        return self._task_paths(name)[3]

    def _goal_override_status_path(self, name: str) -> str:
        return self._task_paths(name)[4]

    def _property_path(self, key: str) -> str:
        return join_paths(get_service_namespaced_root_path(self.namespace, PROPERTIES_ROOT_NAME), key)

    @staticmethod
    def _validate_key(key: str) -> None:
        if not key or not key.strip():
            raise StateStoreException(Reason.LOGIC_ERROR, "Key cannot be blank or null")
        if "/" in key:
            raise StateStoreException(Reason.LOGIC_ERROR, "Key cannot contain '/'")

    @staticmethod
    def _validate_value(value: Optional[bytes]) -> None:
        if value is None:
            raise StateStoreException(Reason.LOGIC_ERROR, "Property value must not be null.")
        if len(value) > MAX_VALUE_LENGTH_BYTES:
            raise StateStoreException(
                Reason.LOGIC_ERROR,
                f"Property value length {len(value)} exceeds limit of {MAX_VALUE_LENGTH_BYTES} bytes.")

    # -- tasks ---------------------------------------------------------------------------
    def store_tasks(self, tasks: Collection[P.TaskInfo],
                    statuses: Collection[Tuple[str, P.TaskStatus]] = ()) -> None:
        """Stores TaskInfos in batches under 1 MB (StateStore.storeTasks). ``statuses`` (task
        name, status) are checked as ``store_status`` checks them and, when the TaskInfos fit one
        batch, written in that same transaction (a launch record is one ZooKeeper multi instead of
        one for the TaskInfos and one per status); otherwise they follow, one write each. The
        TaskInfos are serialized before the status lock is taken: it covers only the checks and
        the writes."""
        batches: List[Dict[str, bytes]] = []
        sizes: List[int] = []
        for t in tasks:
            data = t.SerializeToString()
            self._validate_value(data)
            if not batches or len(data) + sizes[-1] >= MAX_VALUE_LENGTH_BYTES:
                batches.append({})
                sizes.append(0)
            batches[-1][self._task_info_path(t.name)] = data
            sizes[-1] += len(data)
        if len(batches) > 1:
            self.logger.warning("Grouped %d TaskInfo writes in to %d batches", len(tasks), len(batches))
        with self._status_lock:
            checked = [(name, st) for name, st in statuses if self._check_status(name, st)]
            if len(batches) <= 1 and checked:
                if not batches:
                    batches.append({})
                for name, st in checked:
                    batches[0][self._task_status_path(name)] = st.SerializeToString()
                checked = []
            for b in batches:
                try:
                    self.persister.set_many(b)
                except PersisterException as e:
                    raise StateStoreException(e.reason, f"Failed to store {len(b)} TaskInfos") from e
            for name, st in checked:
                self.store_status(name, st)

    def _check_status(self, task_name: str, status: P.TaskStatus, current=_UNSET) -> bool:
        """The checks ``store_status`` applies before writing (raises on a rejected status);
        ``current`` is the task's status to check against (default: the stored one)."""
        if current is _UNSET:
            current = self.fetch_status(task_name)
        from dcos_commons_amd.offer.task_utils import is_terminal

        if current is not None and status.state in _NON_TERMINAL_OVERWRITE_STATES and is_terminal(current):
            raise StateStoreException(
                Reason.LOGIC_ERROR,
                f"Skipping task status processing. Ignoring {P.TaskState.Name(status.state)} as task already in a "
                f"terminal state {P.TaskState.Name(current.state)}: {task_name}")
        if (status.state != P.TASK_STAGING and current is not None
                and current.task_id.value != status.task_id.value):
            raise StateStoreException(Reason.NOT_FOUND,
                                      f"Dropping TaskStatus with unknown TaskID: {status.task_id.value}")
        return True

    def store_status(self, task_name: str, status: P.TaskStatus,
                     properties: Optional[Dict[str, bytes]] = None) -> None:
        """Stores ``status`` (StateStore.storeStatus). ``properties`` are written in the same
        persister transaction (one ZooKeeper multi instead of a round trip each), but never at the
        status's expense: the reference stores them after the status in a try/catch that only
        warns (DefaultScheduler.java:541-560, StateStoreUtils.storeTaskStatusAsProperty), so a
        property that fails validation is dropped with a warning, and a combined write that fails
        is retried as the status alone."""
        data = status.SerializeToString()
        valid: Dict[str, bytes] = {}
        for k, v in (properties or {}).items():
            try:
                self._validate_key(k)
                self._validate_value(v)
            except StateStoreException as e:
                self.logger.warning("Not storing property '%s' with the status of %s: %s", k, task_name, e)
                continue
            valid[self._property_path(k)] = v
        with self._status_lock:
            self._check_status(task_name, status)
            try:
                if valid:
                    try:
                        self.persister.set_many(dict(valid, **{self._task_status_path(task_name): data}))
                        return
                    except PersisterException as e:
                        self.logger.warning("Failed to store properties %s with the status of %s (%s); "
                                            "storing the status alone", sorted(valid), task_name, e)
                self.persister.set(self._task_status_path(task_name), data)
            except PersisterException as e:
                raise StateStoreException(e.reason, str(e)) from e

    @_status_write
    def store_statuses(self, items) -> List[Optional[StateStoreException]]:
        """Stores several ``(task_name, status, properties)`` in one persister transaction (a status
        thread that fell behind catches up with one ZooKeeper multi instead of a round trip per
        status). Validation is per item, as in :meth:`store_status`; several statuses of one task
        are checked in order, each against the one before it, and the last one is what ends up
        stored, as storing them one by one would leave it. If the combined write fails, every item
        is stored alone so one bad item cannot take the others with it. Returns each item's error
        (None when stored)."""
        errors: List[Optional[StateStoreException]] = [None] * len(items)
        batch: Dict[str, bytes] = {}
        latest: Dict[str, P.TaskStatus] = {}     # a later status of a task is checked against the earlier
        for i, (name, status, props) in enumerate(items):
            try:
                self._check_status(name, status, latest[name] if name in latest else _UNSET)
            except StateStoreException as e:
                errors[i] = e
                continue
            latest[name] = status
            for k, v in (props or {}).items():
                try:
                    self._validate_key(k)
                    self._validate_value(v)
                except StateStoreException as e:
                    self.logger.warning("Not storing property '%s' with the status of %s: %s", k, name, e)
                    continue
                batch[self._property_path(k)] = v
            batch[self._task_status_path(name)] = status.SerializeToString()
        if not batch:
            return errors
        try:
            self.persister.set_many(batch)
            return errors
        except PersisterException as e:
            self.logger.warning("Failed to store %d statuses together (%s); storing them one at a time",
                                len(items), e)
        for i, (name, status, props) in enumerate(items):
            if errors[i] is None:
                try:
                    self.store_status(name, status, props)
                except StateStoreException as e:
                    errors[i] = e
        return errors

    def clear_task(self, task_name: str) -> None:
        try:
            self.persister.recursive_delete(self._task_path(task_name))
        except PersisterException as e:
            if e.reason == Reason.NOT_FOUND:
                self.logger.warning("Cleared nonexistent Task, continuing silently: %s", task_name)
            else:
                raise StateStoreException(e.reason, str(e)) from e

    def fetch_task_names(self) -> List[str]:
        try:
            return list(self.persister.get_children(self._tasks_root))
        except PersisterException as e:
            if e.reason == Reason.NOT_FOUND:
                return []
            raise StateStoreException(e.reason, str(e)) from e

    def fetch_tasks_bytes(self) -> Dict[str, bytes]:
        """Every task's serialized TaskInfo by name, read in one persister call."""
        names = self.fetch_task_names()
        paths = {self._task_info_path(n): n for n in names}
        try:
            raw = self.persister.get_many(list(paths))
        except PersisterException as e:
            raise StateStoreException(e.reason, "Failed to retrieve tasks") from e
        out = {}
        for path, name in paths.items():
            data = raw.get(path)
            if data is None:
                raise StateStoreException(
                    Reason.NOT_FOUND, f"Expected task named {name} to be present when retrieving all tasks")
            if not data:
                raise StateStoreException(Reason.SERIALIZATION_ERROR, f"Empty TaskInfo for TaskName: {name}")
            out[name] = data
        return out

    def fetch_tasks(self) -> List[P.TaskInfo]:
        out = []
        for name, data in self.fetch_tasks_bytes().items():
            t = P.TaskInfo()
            try:
                t.ParseFromString(data)
            except Exception as e:  # noqa: BLE001
                raise StateStoreException(Reason.SERIALIZATION_ERROR, str(e)) from e
            out.append(t)
        return out

    def fetch_tasks_shared(self) -> List[P.TaskInfo]:
        """``fetch_tasks`` for read-only callers (the offer cycle's task map): a task whose stored
        bytes did not change since the last call is returned as the same parsed object instead of
        being parsed again (a reference hdfs TaskInfo is 16-32 KB: its environment three times
        over). Callers must not modify the returned TaskInfos. With ``SDK_DEBUG_SHARED_TASKS``
        set (the test suite sets it) every call first checks that no cached TaskInfo was
        modified since it was handed out."""
        cache = self._shared
        raw = self.fetch_tasks_bytes()
        out = [self.shared_task(name, data) for name, data in raw.items()]
        if len(cache) > len(raw):
            for gone in set(cache) - set(raw):
                cache.pop(gone, None)       # another reader may have dropped it first
        return out

    def fetch_task_shared(self, task_name: str) -> Optional[P.TaskInfo]:
        """``fetch_task`` for read-only callers, from the same cache as ``fetch_tasks_shared`` (the
        plans built at a scheduler start read the same tasks once per plan that has a step for
        them). Callers must not modify the returned TaskInfo."""
        data = self.fetch_task_bytes(task_name)
        return None if data is None else self.shared_task(task_name, data)

    def shared_task(self, task_name: str, data: bytes) -> P.TaskInfo:
        """The shared parsed TaskInfo of ``task_name`` for its stored bytes ``data`` (as read by
        ``fetch_task_bytes`` / ``fetch_tasks_bytes``): parsed once per distinct bytes, whichever
        reader asks first. Callers must not modify it."""
        hit = self._shared.get(task_name)
        if hit is not None and (hit[0] is data or hit[0] == data):
            if _DEBUG_SHARED and hit[1].SerializeToString() != hit[0]:
                raise AssertionError(f"a caller modified the shared TaskInfo of {task_name}")
            return hit[1]
        if not data:
            raise StateStoreException(Reason.SERIALIZATION_ERROR, f"Empty TaskInfo for TaskName: {task_name}")
        t = P.TaskInfo()
        try:
            t.ParseFromString(data)
        except Exception as e:  # noqa: BLE001
            raise StateStoreException(Reason.SERIALIZATION_ERROR, str(e)) from e
        self._shared[task_name] = (data, t)
        return t

    def fetch_task_bytes(self, task_name: str) -> Optional[bytes]:
        """The serialized TaskInfo as stored (None when absent), for callers that memoize what
        they derive from a task on its exact bytes instead of parsing it on every pass."""
        try:
            return self.persister.get(self._task_info_path(task_name))
        except PersisterException as e:
            if e.reason == Reason.NOT_FOUND:
                return None
            raise StateStoreException(e.reason, f"Failed to retrieve task named {task_name}") from e

    def fetch_task(self, task_name: str) -> Optional[P.TaskInfo]:
        data = self.fetch_task_bytes(task_name)
        if data is None:
            return None
        if not data:
            raise StateStoreException(Reason.SERIALIZATION_ERROR, f"Empty TaskInfo for TaskName: {task_name}")
        t = P.TaskInfo()
        try:
            t.ParseFromString(data)
        except Exception as e:  # noqa: BLE001
            raise StateStoreException(Reason.SERIALIZATION_ERROR, str(e)) from e
        return t

    def fetch_statuses_bytes(self, names: Optional[List[str]] = None) -> Dict[str, bytes]:
        """Serialized TaskStatus by task name, read in one persister call (tasks without one are
        left out), for callers that memoize on the exact bytes."""
        names = self.fetch_task_names() if names is None else names
        paths = {self._task_status_path(n): n for n in names}
        try:
            raw = self.persister.get_many(list(paths))
        except PersisterException as e:
            raise StateStoreException(e.reason, str(e)) from e
        return {n: raw[p] for p, n in paths.items() if raw.get(p) is not None}

    def fetch_statuses(self) -> List[P.TaskStatus]:
        """Every stored TaskStatus, read in one persister call (tasks without one are skipped)."""
        paths = [self._task_status_path(n) for n in self.fetch_task_names()]
        try:
            raw = self.persister.get_many(paths)
        except PersisterException as e:
            raise StateStoreException(e.reason, str(e)) from e
        out = []
        for path in paths:
            data = raw.get(path)
            if data is None:
                continue
            s = P.TaskStatus()
            s.ParseFromString(data)
            out.append(s)
        return out

    def fetch_status(self, task_name: str) -> Optional[P.TaskStatus]:
        try:
            data = self.persister.get(self._task_status_path(task_name))
        except PersisterException as e:
            if e.reason == Reason.NOT_FOUND:
                return None
            raise StateStoreException(e.reason, str(e)) from e
        if not data:
            raise StateStoreException(Reason.SERIALIZATION_ERROR, f"Empty TaskStatus for TaskName: {task_name}")
        s = P.TaskStatus()
        s.ParseFromString(data)
        return s

    # -- properties ----------------------------------------------------------------------
    def store_property(self, key: str, value: bytes) -> None:
        self._validate_key(key)
        self._validate_value(value)
        try:
            self.persister.set(self._property_path(key), value)
        except PersisterException as e:
            raise StateStoreException(e.reason, str(e)) from e

    def store_properties(self, props: Dict[str, bytes]) -> None:
        m = {}
        for k, v in props.items():
            self._validate_key(k)
            self._validate_value(v)
            m[self._property_path(k)] = v
        try:
            self.persister.set_many(m)
        except PersisterException as e:
            raise StateStoreException(e.reason, str(e)) from e

    def fetch_property(self, key: str) -> bytes:
        self._validate_key(key)
        try:
            return self.persister.get(self._property_path(key))
        except PersisterException as e:
            raise StateStoreException(e.reason, str(e)) from e

    def fetch_property_keys(self) -> List[str]:
        try:
            return list(self.persister.get_children(
                get_service_namespaced_root_path(self.namespace, PROPERTIES_ROOT_NAME)))
        except PersisterException as e:
            if e.reason == Reason.NOT_FOUND:
                return []
            raise StateStoreException(e.reason, str(e)) from e

    def clear_property(self, key: str) -> None:
        self._validate_key(key)
        try:
            self.persister.recursive_delete(self._property_path(key))
        except PersisterException as e:
            if e.reason != Reason.NOT_FOUND:
                raise StateStoreException(e.reason, str(e)) from e

    # -- goal overrides ------------------------------------------------------------------
    def store_goal_override_status(self, task_name: str, status: OverrideStatus) -> None:
        try:
            if status == OverrideStatus.INACTIVE:
                self.persister.recursive_delete_many(
                    [self._goal_override_path(task_name), self._goal_override_status_path(task_name)])
            else:
                self.persister.set_many({
                    self._goal_override_path(task_name): status.target.serialized_name.encode(),
                    self._goal_override_status_path(task_name): status.progress.value.encode(),
                })
        except PersisterException as e:
            raise StateStoreException(e.reason, str(e)) from e

    def fetch_goal_override_status(self, task_name: str) -> OverrideStatus:
        p1, p2 = self._goal_override_path(task_name), self._goal_override_status_path(task_name)
        try:
            vals = self.persister.get_many([p1, p2])
        except PersisterException as e:
            raise StateStoreException(e.reason, str(e)) from e
        name_b, prog_b = vals.get(p1), vals.get(p2)
        if name_b is None and prog_b is None:
            return OverrideStatus.INACTIVE
        if name_b is None or prog_b is None:
            self.logger.error("Task %s is missing override name or override status", task_name)
            return OverrideStatus.INACTIVE
        target = GoalStateOverride.from_serialized(name_b.decode())
        if target is None:
            return OverrideStatus.INACTIVE
        try:
            progress = OverrideProgress(prog_b.decode())
        except ValueError:
            return OverrideStatus.INACTIVE
        return OverrideStatus(target, progress)

    def delete_all_data_if_namespaced(self) -> None:
        if not self.namespace:
            return
        try:
            self.persister.recursive_delete(get_service_namespaced_root(self.namespace))
        except PersisterException as e:
            if e.reason != Reason.NOT_FOUND:
                raise StateStoreException(e.reason, str(e)) from e
