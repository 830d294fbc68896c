"""Path helpers, bulk read/delete, namespacing and schema migration.

Reference: sdk/.../storage/PersisterUtils.java:29-323.
"""
from __future__ import annotations

import logging
import time
from typing import Dict, List

from .persister import Persister, PersisterException, Reason

PATH_DELIM = "/"
SERVICE_NAMESPACE_ROOT_NAME = "Services"
LOGGER = logging.getLogger(__name__)


def with_escaped_slashes(name: str) -> str:
    """``/path/to/svc`` -> ``path__to__svc`` (reference SchedulerUtils.withEscapedSlashes:
    one leading slash dropped; names that already contain ``__`` are rejected)."""
    if "__" in name:
        raise ValueError(f"Service names may not contain double underscores: {name}")
    if name.startswith(PATH_DELIM):
        name = name[len(PATH_DELIM):]
    return name.replace(PATH_DELIM, "__")


def join_paths(*paths: str) -> str:
    out = ""
    for second in paths:
        first = out
        if not first or not second:
            out = first + second
        elif first.endswith(PATH_DELIM) and second.startswith(PATH_DELIM):
            out = first[:-1] + second
        elif first.endswith(PATH_DELIM) or second.startswith(PATH_DELIM):
            out = first + second
        else:
            out = first + PATH_DELIM + second
    return out


def get_path_elements(path: str) -> List[str]:
    return [p for p in path.split(PATH_DELIM) if p]


def get_parent_paths(path: str) -> List[str]:
    """All ancestor paths of ``path`` (not itself), shallowest first; a leading slash is kept
    (PersisterUtils.getParentPaths: ``/a/b/c`` -> ``[/a, /a/b]``)."""
    elements = path.split(PATH_DELIM)
    while elements and not elements[-1]:  # a trailing slash names no extra level
        elements.pop()
    out, cur = [], ""
    for i in range(len(elements) - 1):
        if not elements[i]:
            continue
        if i != 0:
            cur += PATH_DELIM
        cur += elements[i]
        out.append(cur)
    return out


def fetch_service_namespaces(persister: Persister):
    try:
        return persister.get_children(SERVICE_NAMESPACE_ROOT_NAME)
    except PersisterException as e:
        if e.reason == Reason.NOT_FOUND:
            return []
        raise


def get_service_namespaced_root(namespace: str) -> str:
    if not namespace:
        raise ValueError("Expected non-empty namespace")
    return join_paths(SERVICE_NAMESPACE_ROOT_NAME, with_escaped_slashes(namespace))


def get_service_namespaced_root_path(namespace: str, path_name: str) -> str:
    return path_name if not namespace else join_paths(get_service_namespaced_root(namespace), path_name)


def get_all_data(persister: Persister) -> Dict[str, bytes]:
    out: Dict[str, bytes] = {}
    _collect(persister, PATH_DELIM, out)
    return dict(sorted(out.items()))


def _collect(persister: Persister, path: str, out: Dict[str, bytes]) -> None:
    for child in persister.get_children(path):
        child_path = join_paths(path, child)
        data = persister.get(child_path)
        if data is not None:
            out[child_path] = data
        _collect(persister, child_path, out)


def get_all_keys(persister: Persister) -> List[str]:
    keys: List[str] = []

    def walk(path: str) -> None:
        for child in persister.get_children(path):
            cp = join_paths(path, child)
            keys.append(cp)
            walk(cp)

    walk(PATH_DELIM)
    return sorted(keys)


def clear_all_data(persister: Persister) -> None:
    try:
        persister.recursive_delete(PATH_DELIM)
    except PersisterException as e:
        if e.reason != Reason.NOT_FOUND:
            raise


def _timestamped(name: str) -> str:
    return "%s-%s" % (name, time.strftime("%Y-%m-%d-%H%M%S"))


def check_and_migrate(framework_name: str, persister: Persister) -> None:
    """Single-service -> multi-service schema migration (PersisterUtils.java:245-314).

    Backs up ``Configurations``, ``ConfigTarget``, ``Properties`` and ``Tasks`` under
    ``backup-<ts>/``, copies them under ``Services/<name>/`` and deletes the originals.
    """
    from dcos_commons_amd.state.schema_version_store import SchemaVersion, SchemaVersionStore

    store = SchemaVersionStore(persister)
    cur = store.get_or_set_version(SchemaVersion.MULTI_SERVICE)
    if cur == SchemaVersion.SINGLE_SERVICE:
        LOGGER.info("Migrating single-service schema to multi-service schema")
        backup_root = _timestamped("backup")
        try:
            persister.recursive_delete(backup_root)
        except PersisterException as e:
            if e.reason != Reason.NOT_FOUND:
                raise
        migrate = ["Configurations", "ConfigTarget", "Properties", "Tasks"]
        present = []
        for path in migrate:
            try:
                persister.get(path)
                present.append(path)
            except PersisterException as e:
                if e.reason != Reason.NOT_FOUND:
                    raise
        for path in present:
            persister.recursive_copy(path, join_paths(backup_root, path))
        for path in present:
            persister.recursive_copy(path, get_service_namespaced_root_path(framework_name, path))
        try:
            for path in present:
                persister.recursive_delete(path)
        except PersisterException:
            LOGGER.exception("Failed to delete single-service schema nodes after migration")
        store.store(SchemaVersion.MULTI_SERVICE)
    elif cur == SchemaVersion.MULTI_SERVICE:
        LOGGER.info("Schema version matches multi-service mode; nothing to migrate.")
    else:
        raise RuntimeError(f"Storage schema version {cur} is not supported")
