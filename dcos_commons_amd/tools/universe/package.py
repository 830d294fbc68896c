"""Universe package identity: a name plus a (releaseVersion, version) pair.

Reference: tools/universe/package.py. Ordering follows the universe: packages of one name are
ordered by their integer ``releaseVersion`` (the monotonically increasing release counter), never
by the free-form ``version`` string. ``beta-<name>`` packages are the beta channel of ``<name>``.
"""
from __future__ import annotations

import functools
import json
from typing import Mapping


@functools.total_ordering
class Version:
    def __init__(self, release_version, package_version: str):
        self.release_version = int(release_version)
        self.package_version = str(package_version)

    def __eq__(self, other) -> bool:
        return isinstance(other, Version) and self.release_version == other.release_version

    def __lt__(self, other: "Version") -> bool:
        return self.release_version < other.release_version

    def __hash__(self) -> int:
        return hash(self.release_version)

    def __str__(self) -> str:
        return self.package_version

    def __repr__(self) -> str:
        return f"Version({self.release_version}, {self.package_version!r})"

    def to_json(self) -> dict:
        return {"release_version": self.release_version, "package_version": self.package_version}


@functools.total_ordering
class Package:
    BETA_PREFIX = "beta-"

    def __init__(self, name: str, version: Version):
        self._name = name
        self._version = version

    @staticmethod
    def from_json(obj: Mapping) -> "Package":
        return Package(obj["name"], Version(obj.get("releaseVersion", 0), obj["version"]))

    def get_name(self) -> str:
        return self._name

    def get_version(self) -> Version:
        return self._version

    def is_beta(self) -> bool:
        return self._name.startswith(self.BETA_PREFIX)

    def get_non_beta_name(self) -> str:
        return self._name[len(self.BETA_PREFIX):] if self.is_beta() else self._name

    def __eq__(self, other) -> bool:
        return isinstance(other, Package) and (self._name, self._version) == (other._name, other._version)

    def __lt__(self, other: "Package") -> bool:
        if self._name != other._name:
            return self._name < other._name
        return self._version < other._version

    def __hash__(self) -> int:
        return hash((self._name, self._version))

    def __str__(self) -> str:
        return json.dumps({"name": self._name, "version": self._version.package_version,
                           "releaseVersion": self._version.release_version})
