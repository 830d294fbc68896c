"""The tree-structured key/value persistence contract.

Reference: sdk/.../storage/Persister.java:15-99, StorageError.java, PersisterException.java.
Paths are ``/``-delimited; a node may hold data *and* children (ZooKeeper semantics). ``get`` of
an existing node without data returns ``None``; ``get`` of a missing node raises
``PersisterException(NOT_FOUND)``.
"""
from __future__ import annotations

import enum
from abc import ABC, abstractmethod
from typing import Collection, Dict, Mapping, Optional


class Reason(enum.Enum):
    UNKNOWN = "UNKNOWN"
    NOT_FOUND = "NOT_FOUND"
    STORAGE_ERROR = "STORAGE_ERROR"
    SERIALIZATION_ERROR = "SERIALIZATION_ERROR"
    LOGIC_ERROR = "LOGIC_ERROR"


class PersisterException(Exception):
    def __init__(self, reason: Reason, message: str = "", cause: Optional[BaseException] = None):
        super().__init__(f"{reason.value}: {message}")
        self.reason = reason
        self.message = message
        self.__cause__ = cause


class Persister(ABC):
    @property
    def remote(self) -> bool:
        """Whether a write is a network round trip (ZooKeeper) rather than a local update:
        the scheduler then overlaps its write-ahead launch records with step evaluation."""
        return False

    @abstractmethod
    def get(self, path: str) -> Optional[bytes]:
        ...

    @abstractmethod
    def get_children(self, path: str) -> Collection[str]:
        ...

    @abstractmethod
    def set(self, path: str, data: bytes) -> None:
        ...

    @abstractmethod
    def get_many(self, paths: Collection[str]) -> Dict[str, Optional[bytes]]:
        ...

    @abstractmethod
    def set_many(self, path_bytes: Mapping[str, bytes]) -> None:
        """Atomically sets all values (creating missing parents)."""

    @abstractmethod
    def recursive_copy(self, src: str, dst: str) -> None:
        ...

    @abstractmethod
    def recursive_delete_many(self, paths: Collection[str]) -> None:
        ...

    @abstractmethod
    def recursive_delete(self, path: str) -> None:
        ...

    @abstractmethod
    def close(self) -> None:
        ...
