"""Versioned configuration storage.

Reference: sdk/.../state/ConfigStore.java:34-277. Configs are stored under
``Configurations/<uuid>`` with the active one pointed to by ``ConfigTarget``.
"""
from __future__ import annotations

import logging
import uuid
from typing import Dict, List, Optional

from dcos_commons_amd.storage.persister import Persister, PersisterException, Reason
from dcos_commons_amd.storage.persister_utils import get_service_namespaced_root_path, join_paths

TARGET_ID_PATH_NAME = "ConfigTarget"
CONFIGURATIONS_PATH_NAME = "Configurations"
LOGGER = logging.getLogger(__name__)


class ConfigStoreException(Exception):
    def __init__(self, reason: Reason, message: str = ""):
        super().__init__(f"{reason.value}: {message}")
        self.reason = reason


class ConfigStore:
    def __init__(self, factory, persister: Persister, namespace: Optional[str] = None):
        self.factory = factory
        self.persister = persister
        self.namespace = namespace or ""
        self._cache: Dict[uuid.UUID, object] = {}

    def _target_path(self) -> str:
        return get_service_namespaced_root_path(self.namespace, TARGET_ID_PATH_NAME)

    def _configs_path(self) -> str:
        return get_service_namespaced_root_path(self.namespace, CONFIGURATIONS_PATH_NAME)

    def _config_path(self, cid: uuid.UUID) -> str:
        return join_paths(self._configs_path(), str(cid))

    def has_key(self, cid: uuid.UUID) -> bool:
        return cid in self._cache or cid in self.list()

    def store(self, config, cid: Optional[uuid.UUID] = None) -> uuid.UUID:
        cid = cid or uuid.uuid4()
        try:
            self.persister.set(self._config_path(cid), config.get_bytes())
        except PersisterException as e:
            raise ConfigStoreException(e.reason, f"Failed to store configuration {cid}") from e
        self._cache[cid] = config
        return cid

    def fetch(self, cid) -> object:
        if not isinstance(cid, uuid.UUID):
            cid = uuid.UUID(str(cid))
        c = self._cache.get(cid)
        if c is not None:
            return c
        path = self._config_path(cid)
        try:
            data = self.persister.get(path)
        except PersisterException as e:
            if e.reason == Reason.NOT_FOUND:
                raise ConfigStoreException(Reason.NOT_FOUND,
                                           f"Configuration '{cid}' was not found at path '{path}'") from e
            raise ConfigStoreException(e.reason, f"Failed to retrieve configuration '{cid}'") from e
        try:
            c = self.factory.parse(data)
        except Exception as e:  # noqa: BLE001
            raise ConfigStoreException(Reason.SERIALIZATION_ERROR, f"Failed to parse configuration {cid}: {e}")
        self._cache[cid] = c
        return c

    def clear(self, cid: uuid.UUID) -> None:
        try:
            self.persister.recursive_delete(self._config_path(cid))
        except PersisterException as e:
            if e.reason == Reason.NOT_FOUND:
                LOGGER.warning("Requested configuration '%s' to be deleted does not exist", cid)
                return
            raise ConfigStoreException(e.reason, str(e)) from e
        self._cache.pop(cid, None)

    def list(self) -> List[uuid.UUID]:
        try:
            names = self.persister.get_children(self._configs_path())
        except PersisterException as e:
            if e.reason == Reason.NOT_FOUND:
                return []
            raise ConfigStoreException(Reason.STORAGE_ERROR, "Failed to retrieve list of configurations") from e
        out = []
        for n in names:
            try:
                out.append(uuid.UUID(n))
            except ValueError:
                raise ConfigStoreException(Reason.SERIALIZATION_ERROR, f"Invalid UUID value: {n}")
        return out

    def get_target_config(self) -> uuid.UUID:
        path = self._target_path()
        try:
            raw = self.persister.get(path)
        except PersisterException as e:
            if e.reason == Reason.NOT_FOUND:
                raise ConfigStoreException(
                    Reason.NOT_FOUND, f"Current target configuration couldn't be found at path '{path}'") from e
            raise ConfigStoreException(e.reason, str(e)) from e
        try:
            return uuid.UUID((raw or b"").decode())
        except ValueError:
            raise ConfigStoreException(Reason.SERIALIZATION_ERROR, f"Failed to parse '{raw}' as a UUID")

    def set_target_config(self, cid: uuid.UUID) -> None:
        try:
            self.persister.set(self._target_path(), str(cid).encode())
        except PersisterException as e:
            raise ConfigStoreException(e.reason, str(e)) from e
