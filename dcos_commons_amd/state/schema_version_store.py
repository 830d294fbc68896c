"""``SchemaVersion`` node: "1" = single-service, "2" = multi-service.

Reference: sdk/.../state/SchemaVersionStore.java:19-144.
"""
from __future__ import annotations

import enum

from dcos_commons_amd.storage.persister import Persister, PersisterException, Reason

from .state_store import StateStoreException

SCHEMA_VERSION_NAME = "SchemaVersion"


class SchemaVersion(enum.Enum):
    SINGLE_SERVICE = 1
    MULTI_SERVICE = 2
    UNKNOWN = -1

    @staticmethod
    def parse_int(v: int) -> "SchemaVersion":
        return {1: SchemaVersion.SINGLE_SERVICE, 2: SchemaVersion.MULTI_SERVICE}.get(v, SchemaVersion.UNKNOWN)


class SchemaVersionStore:
    def __init__(self, persister: Persister):
        self.persister = persister

    def check(self, expected: SchemaVersion) -> None:
        """ValueError (the reference's IllegalArgumentException) unless the stored version is
        ``expected``; an unknown number is reported as stored."""
        cur = self.get_or_set_version(expected)
        if cur != expected:
            shown = self.persister.get(SCHEMA_VERSION_NAME).decode() if cur == SchemaVersion.UNKNOWN else cur.value
            raise ValueError(
                f"Storage schema version {shown} is not supported by this software (expected: {expected.value})")

    def get_or_set_version(self, expected: SchemaVersion) -> SchemaVersion:
        try:
            data = self.persister.get(SCHEMA_VERSION_NAME)
        except PersisterException as e:
            if e.reason == Reason.NOT_FOUND:
                self.store(expected)
                return expected
            raise StateStoreException(Reason.STORAGE_ERROR, "Storage error when fetching schema storage") from e
        if not data:
            raise StateStoreException(Reason.SERIALIZATION_ERROR, "Invalid data when fetching schema version")
        try:
            return SchemaVersion.parse_int(int(data.decode()))
        except ValueError:
            raise StateStoreException(Reason.SERIALIZATION_ERROR, f"Unable to parse schema version '{data!r}'")

    def store(self, version: SchemaVersion) -> None:
        if version == SchemaVersion.UNKNOWN:
            raise ValueError("Unable to convert UNKNOWN to int")
        try:
            self.persister.set(SCHEMA_VERSION_NAME, str(version.value).encode())
        except Exception as e:  # noqa: BLE001
            raise StateStoreException(Reason.STORAGE_ERROR, f"Storage error when storing schema version {version}") from e
