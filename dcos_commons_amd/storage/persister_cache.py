"""Write-through cache in front of a (slow, remote) persister.

Reference: sdk/.../storage/PersisterCache.java:18-173. Reads are served from a full
:class:`MemPersister` mirror; writes go to the backing store first, then to the mirror.

Unlike the reference, which holds its write lock across the backing store's round trip, writers
here are ordered by a mutex of their own and take the mirror's write lock only to apply a write
that the backing store has already committed. A ZooKeeper write takes a network round trip (and,
in a Python scheduler, the interpreter lock to come back from it); readers on other threads -- the
offer cycle evaluating steps while the status thread stores a TaskStatus -- keep reading the mirror
meanwhile and see the write once it is durable. Writes still reach the mirror in the order they
reached the backing store.
"""
from __future__ import annotations

import logging
import threading
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
        self._writer = threading.RLock()   # orders writes: backing store, then mirror, one at a time
        self._cache: Optional[MemPersister] = None

    @property
    def backing(self) -> Persister:
        return self._persister

    @property
    def remote(self) -> bool:
        return self._persister.remote

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
        with self._w if self._cache is None else self._r:
            return self._get_cache().get_many(paths)

    def _loaded(self) -> MemPersister:
        if self._cache is None:
            with self._w:
                return self._get_cache()
        return self._cache

    def set(self, path: str, data: bytes) -> None:
        with self._writer:
            cache = self._loaded()
            self._persister.set(path, data)
            with self._w:
                cache.set(path, data)

    def set_many(self, path_bytes: Mapping[str, bytes]) -> None:
        with self._writer:
            cache = self._loaded()
            self._persister.set_many(path_bytes)
            with self._w:
                cache.set_many(path_bytes)

    def recursive_copy(self, src: str, dst: str) -> None:
        with self._writer:
            cache = self._loaded()
            self._persister.recursive_copy(src, dst)
            with self._w:
                cache.recursive_copy(src, dst)

    def recursive_delete_many(self, paths: Collection[str]) -> None:
        with self._writer:
            cache = self._loaded()
            self._persister.recursive_delete_many(paths)
            with self._w:
                cache.recursive_delete_many(paths)

    def recursive_delete(self, path: str) -> None:
        with self._writer:
            cache = self._loaded()
            self._persister.recursive_delete(path)
            with self._w:
                try:
                    cache.recursive_delete(path)
                except PersisterException:
                    LOGGER.error("Didn't find %s in cache to delete, but underlying storage had it", path)

    def close(self) -> None:
        with self._writer, self._w:
            self._persister.close()
            if self._cache is not None:
                self._cache.close()

    def refresh(self) -> None:
        with self._writer, self._w:
            if self._cache is not None:
                LOGGER.info("Cache content before refresh:\n%s", self._cache.debug_string())
            self._cache = None
            self._get_cache()
