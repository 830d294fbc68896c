"""Universe repositories and the package manager that queries them.

Reference: tools/universe/package_manager.py (asks ``universe.mesosphere.com`` for a package's
releases to find the latest one). There is no public universe to reach from here, so the manager
reads *repositories* the tools in this package write, in any of three forms:

* a stub universe: JSON ``{"packages": [<package definition>, ...]}`` as a file path, ``file://``
  or ``http(s)://`` URL (``build_package`` / ``publish_http`` produce these);
* a ``.dcos`` bundle: a zip holding ``catalog.json`` (a stub universe) and the package's artifacts
  under ``resources/`` (``publish_dcos_file``: everything an air-gapped cluster needs in one file);
* a universe repository tree: ``repo/packages/<L>/<name>/<releaseVersion>/`` holding
  ``package.json``, ``config.json``, ``resource.json`` and ``marathon.json.mustache``
  (``release_builder`` adds releases to one).

A package definition is the universe v4 format: ``package.json`` fields plus ``config`` (the
options schema), ``resource`` and ``marathon.v2AppMustacheTemplate`` (base64 of the Marathon app
template).
"""
from __future__ import annotations

import base64
import collections
import io
import json
import logging
import os
import urllib.parse
import urllib.request
import zipfile
from typing import Dict, Iterable, List, Optional, Sequence, Union

from dcos_commons_amd.tools.universe.package import Package, Version

LOGGER = logging.getLogger(__name__)
CATALOG_NAME = "catalog.json"
RESOURCES_DIR = "resources"
PACKAGE_FILES = ("package.json", "config.json", "resource.json", "marathon.json.mustache")


def _loads(text: Union[str, bytes]) -> dict:
    if isinstance(text, bytes):
        text = text.decode("utf-8")
    return json.loads(text, object_pairs_hook=collections.OrderedDict)


def read_location(location: str, timeout_s: float = 60.0) -> bytes:
    parsed = urllib.parse.urlparse(location)
    if parsed.scheme in ("http", "https"):
        with urllib.request.urlopen(location, timeout=timeout_s) as resp:
            return resp.read()
    path = parsed.path if parsed.scheme == "file" else location
    with open(path, "rb") as f:
        return f.read()


def package_from_files(files: Dict[str, str]) -> dict:
    """The universe v4 definition assembled from a package directory's files."""
    pkg = _loads(files["package.json"])
    if "config.json" in files:
        pkg["config"] = _loads(files["config.json"])
    if "resource.json" in files:
        pkg["resource"] = _loads(files["resource.json"])
    if "marathon.json.mustache" in files:
        pkg["marathon"] = {"v2AppMustacheTemplate":
                           base64.standard_b64encode(files["marathon.json.mustache"].encode("utf-8")).decode()}
    return pkg


def files_from_package(pkg: dict) -> Dict[str, str]:
    """Inverse of ``package_from_files``: the four package files of one definition."""
    body = collections.OrderedDict((k, v) for k, v in pkg.items() if k not in ("config", "resource", "marathon"))
    out = {"package.json": json.dumps(body, indent=2) + "\n"}
    if "config" in pkg:
        out["config.json"] = json.dumps(pkg["config"], indent=2) + "\n"
    if "resource" in pkg:
        out["resource.json"] = json.dumps(pkg["resource"], indent=2) + "\n"
    tmpl = (pkg.get("marathon") or {}).get("v2AppMustacheTemplate")
    if tmpl:
        out["marathon.json.mustache"] = base64.standard_b64decode(tmpl).decode("utf-8")
    return out


def load_repository(location: str) -> List[dict]:
    """Every package definition a repository location holds (see the module docstring)."""
    if os.path.isdir(location):
        return _load_repo_tree(location)
    data = read_location(location)
    if location.endswith(".dcos") or data[:2] == b"PK":
        with zipfile.ZipFile(io.BytesIO(data)) as z:
            return list(_loads(z.read(CATALOG_NAME))["packages"])
    return list(_loads(data)["packages"])


def _load_repo_tree(root: str) -> List[dict]:
    base = os.path.join(root, "repo", "packages") if os.path.isdir(os.path.join(root, "repo")) else root
    out = []
    for dirpath, _dirs, names in sorted(os.walk(base)):
        if "package.json" not in names:
            continue
        files = {}
        for n in PACKAGE_FILES:
            p = os.path.join(dirpath, n)
            if os.path.exists(p):
                with open(p, "r", encoding="utf-8") as f:
                    files[n] = f.read()
        pkg = package_from_files(files)
        rel = os.path.basename(dirpath)
        if "releaseVersion" not in pkg and rel.isdigit():
            pkg["releaseVersion"] = int(rel)
        out.append(pkg)
    return out


def repo_tree_path(root: str, name: str, release_version: int) -> str:
    """Where a release lives in a universe repository tree (``packages/<L>/<name>/<n>``)."""
    return os.path.join(root, "repo", "packages", name[0].upper(), name, str(int(release_version)))


class PackageManager:
    """Finds the releases of a package across repositories (later repositories win on ties)."""

    def __init__(self, repositories: Optional[Sequence[str]] = None, dry_run: bool = False):
        if repositories is None:
            env = os.environ.get("UNIVERSE_REPOSITORIES", "")
            repositories = [r for r in env.split(",") if r]
        self._repositories = list(repositories)
        self._dry_run = dry_run
        self._cache: Optional[List[dict]] = None

    def add_repository(self, location: str) -> None:
        self._repositories.append(location)
        self._cache = None

    def definitions(self) -> List[dict]:
        if self._cache is None:
            defs: List[dict] = []
            for loc in self._repositories:
                try:
                    defs.extend(load_repository(loc))
                except (OSError, ValueError, KeyError, zipfile.BadZipFile) as e:
                    LOGGER.error("Failed to read universe repository %s: %s", loc, e)
            self._cache = defs
        return self._cache

    def get_package_versions(self, package_name: str) -> List[Package]:
        if self._dry_run:
            return [Package(package_name, Version(0, "DRY_RUN_VERSION"))]
        return [Package.from_json(d) for d in self.definitions() if d.get("name") == package_name]

    def get_latest(self, package: Union[str, Package]) -> Optional[Package]:
        name = package.get_name() if isinstance(package, Package) else package
        versions = self.get_package_versions(name)
        return sorted(versions)[-1] if versions else None

    def get_definition(self, package_name: str, version: Optional[str] = None) -> Optional[dict]:
        """The definition of ``version`` (the latest release when None)."""
        matches = [d for d in self.definitions() if d.get("name") == package_name
                   and (version is None or d.get("version") == version)]
        if not matches:
            return None
        return max(matches, key=lambda d: int(d.get("releaseVersion", 0)))

    def names(self) -> Iterable[str]:
        return sorted({d["name"] for d in self.definitions() if "name" in d})
