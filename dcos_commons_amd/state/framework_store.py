"""FrameworkID storage at the persister root (reference sdk/.../state/FrameworkStore.java:22-97).

The absence of a FrameworkID while in uninstall mode means "uninstall already finished".
"""
from __future__ import annotations

import logging
from typing import Optional

from dcos_commons_amd.mesos import protos as P
from dcos_commons_amd.storage.persister import Persister, PersisterException, Reason

from .state_store import StateStoreException

FWK_ID_PATH_NAME = "FrameworkID"
LOGGER = logging.getLogger(__name__)


class FrameworkStore:
    def __init__(self, persister: Persister):
        self.persister = persister

    def store_framework_id(self, fid: P.FrameworkID) -> None:
        try:
            self.persister.set(FWK_ID_PATH_NAME, fid.SerializeToString())
        except PersisterException as e:
            raise StateStoreException(e.reason, "Failed to store FrameworkID") from e

    def clear_framework_id(self) -> None:
        try:
            self.persister.recursive_delete(FWK_ID_PATH_NAME)
        except PersisterException as e:
            if e.reason != Reason.NOT_FOUND:
                raise StateStoreException(e.reason, str(e)) from e

    def fetch_framework_id(self) -> Optional[P.FrameworkID]:
        try:
            data = self.persister.get(FWK_ID_PATH_NAME)
        except PersisterException as e:
            if e.reason == Reason.NOT_FOUND:
                return None
            raise StateStoreException(e.reason, str(e)) from e
        if not data:
            raise StateStoreException(Reason.SERIALIZATION_ERROR, f"Empty FrameworkID in '{FWK_ID_PATH_NAME}'")
        fid = P.FrameworkID()
        fid.ParseFromString(data)
        return fid
