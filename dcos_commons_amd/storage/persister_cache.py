"""Write-through cache in front of a (slow, remote) persister.

Reference: sdk/.../storage/PersisterCache.java:18-173. Reads are served from a full
:class:`MemPersister` mirror; writes go to the backing store first, then to the mirror.
"""
from __future__ import annotations

import logging
from typing import Collection, Dict, Mapping, Optional

from dcos_commons_amd.utils.locks import new_rw_lock

from .mem_persister import MemPersister
from .persister import Persister, PersisterException
from .persister_utils import get_all_data

LOGGER = logging.getLogger(__name__)


class PersisterCache(Persister):
    def __init__(self, persister: Persister):
        self._persister = persister
        rw = new_rw_lock("PersisterCache")
        self._r, self._w = rw.read_lock, rw.write_lock
        self._cache: Optional[MemPersister] = None

    @property
    def backing(self) -> Persister:
        return self._persister

    def _get_cache(self) -> MemPersister:
        if self._cache is None:
            self._cache = MemPersister(locking=False, data=get_all_data(self._persister))
            LOGGER.debug("Loaded data from persister:\n%s", self._cache.debug_string())
        return self._cache

    def get(self, path: str):
        with self._w if self._cache is None else self._r:
            return self._get_cache().get(path)

    def get_children(self, path: str):
        with self._w if self._cache is None else self._r:
            return self._get_cache().get_children(path)

    def get_many(self, paths: Collection[str]) -> Dict[str, Optional[bytes]]:
        with self._w:
            return self._get_cache().get_many(paths)

    def set(self, path: str, data: bytes) -> None:
        with self._w:
            self._persister.set(path, data)
            self._get_cache().set(path, data)

    def set_many(self, path_bytes: Mapping[str, bytes]) -> None:
        with self._w:
            self._persister.set_many(path_bytes)
            self._get_cache().set_many(path_bytes)

    def recursive_copy(self, src: str, dst: str) -> None:
        with self._w:
            self._persister.recursive_copy(src, dst)
            self._get_cache().recursive_copy(src, dst)

    def recursive_delete_many(self, paths: Collection[str]) -> None:
        with self._w:
            self._persister.recursive_delete_many(paths)
            self._get_cache().recursive_delete_many(paths)

    def recursive_delete(self, path: str) -> None:
        with self._w:
            self._persister.recursive_delete(path)
            try:
                self._get_cache().recursive_delete(path)
            except PersisterException:
                LOGGER.error("Didn't find %s in cache to delete, but underlying storage had it", path)

    def close(self) -> None:
        with self._w:
            self._persister.close()
            if self._cache is not None:
                self._cache.close()

    def refresh(self) -> None:
        with self._w:
            if self._cache is not None:
                LOGGER.info("Cache content before refresh:\n%s", self._cache.debug_string())
            self._cache = None
            self._get_cache()
