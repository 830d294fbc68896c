"""Build a stub universe from a framework's ``universe/`` directory.

Reference: tools/universe/package_builder.py. The four package files are read (anything else, or
anything over 1 MiB, is skipped with a warning), build-time template parameters are substituted
(repeatedly, so parameters may nest), and the files are folded into one universe v4 definition
with ``releaseVersion`` 0 and ``lastUpdated``; the result is ``{"packages": [definition]}``.

Build-time parameters (distinct from the ``{{service.*}}`` options Cosmos renders at install):

=================================  ==========================================================
``{{package-name}}``               package name
``{{package-version}}``            version being built (``stub-universe`` for dev builds)
``{{package-build-time-epoch-ms}}`` / ``{{package-build-time-str}}``  build time
``{{upgrades-from}}`` / ``{{downgrades-to}}``  latest known release (``*`` when none)
``{{artifact-dir}}``               URL the artifacts are published under
``{{documentation-path}}`` / ``{{issues-path}}``  docs links
``{{sha256:<file>}}``              SHA-256 of an artifact given on the command line
``{{sha256:<file>@<url>}}``        SHA-256 listed for ``<file>`` in a SHA256SUMS manifest at url
``TEMPLATE_SOME_PARAM`` env        ``{{some-param}}``
=================================  ==========================================================
"""
from __future__ import annotations

import collections
import difflib
import hashlib
import json
import logging
import os
import re
import tempfile
import time
from typing import Dict, Iterable, Mapping, Optional, Sequence, Tuple

from dcos_commons_amd.tools.universe.package import Package
from dcos_commons_amd.tools.universe.package_manager import PACKAGE_FILES, PackageManager, package_from_files, \
    read_location

LOGGER = logging.getLogger(__name__)
MAX_PACKAGE_FILE_BYTES = 1024 * 1024
DOCS_ROOT = os.environ.get("SDK_DOCS_ROOT", "https://docs.mesosphere.com")
_SHA_PARAM = re.compile(r'"{{sha256:(.+?)}}"')
_FILE_AT_URL = re.compile(r"^(.+?)@(.+?)$")


def sha256_of_file(path: str) -> str:
    h = hashlib.sha256()
    with open(path, "rb") as f:
        for block in iter(lambda: f.read(1 << 16), b""):
            h.update(block)
    return h.hexdigest()


def apply_template(content: str, mapping: Mapping[str, str]) -> str:
    """Substitute ``{{key}}`` until a fixed point (a value may itself hold parameters)."""
    prior = None
    while prior != content:
        prior = content
        for key, val in mapping.items():
            content = content.replace("{{%s}}" % key, val)
    return content


class UniversePackageBuilder:
    def __init__(self, package: Package, package_manager: PackageManager, input_dir_path: str,
                 upload_dir_uri: str, artifact_paths: Sequence[str] = (), dry_run: bool = False,
                 now: Optional[float] = None):
        self._package = package
        self._package_manager = package_manager
        self._upload_dir_uri = upload_dir_uri.rstrip("/")
        self._dry_run = dry_run
        self._now = now
        if not os.path.isdir(input_dir_path):
            raise ValueError(f"Provided package path is not a directory: {input_dir_path}")
        if not os.path.isfile(os.path.join(input_dir_path, "package.json")):
            raise ValueError(f"Provided package path does not contain the expected package files: {input_dir_path}")
        self._input_dir_path = input_dir_path
        self._artifacts: Dict[str, str] = {}
        for path in artifact_paths:
            if not os.path.isfile(path):
                raise ValueError(f"Provided artifact path is not a file: {path} (full list: {list(artifact_paths)})")
            base = os.path.basename(path)
            if base in self._artifacts:
                raise ValueError(f'Duplicate filename between "{self._artifacts[base]}" and "{path}". '
                                 "Artifact filenames must be unique.")
            self._artifacts[base] = path

    # -- template parameters -------------------------------------------------------------------
    def _latest_release(self) -> str:
        latest = self._package_manager.get_latest(self._package)
        return "*" if latest is None else str(latest.get_version())

    def documentation_path(self) -> str:
        path = f"{DOCS_ROOT}/service-docs/{self._package.get_name()}/"
        version = str(self._package.get_version())
        return path if version == "stub-universe" else f"{path}{version}/"

    def template_mapping(self, content: str = "") -> Dict[str, str]:
        now = time.time() if self._now is None else self._now
        latest = self._latest_release()
        mapping = {
            "package-name": self._package.get_name(),
            "package-version": str(self._package.get_version()),
            "package-build-time-epoch-ms": str(int(round(now * 1000))),
            "package-build-time-str": time.strftime("%a %b %d %Y %H:%M:%S +0000", time.gmtime(now)),
            "upgrades-from": latest,
            "downgrades-to": latest,
            "artifact-dir": self._upload_dir_uri,
            "documentation-path": self.documentation_path(),
            "issues-path": f"{DOCS_ROOT}/support/",
        }
        for key, val in os.environ.items():
            if key.startswith("TEMPLATE_"):
                mapping[key[len("TEMPLATE_"):].lower().replace("_", "-")] = val
        mapping.update(self._sha_mapping(content, mapping))
        return mapping

    def _sha_mapping(self, content: str, mapping: Mapping[str, str]) -> Dict[str, str]:
        out = {}
        for raw in _SHA_PARAM.findall(content):
            param = apply_template(raw, mapping)
            m = _FILE_AT_URL.match(param)
            if m:
                sha = self._sha_from_manifest(m.group(2), m.group(1))
            else:
                path = self._artifacts.get(param)
                if not path:
                    raise ValueError(f"Missing path for artifact file named '{param}' (to calculate sha256). "
                                     f"Provide the artifact (known: {sorted(self._artifacts)}) or a manifest "
                                     f"URL with '{param}@<manifestURL>'")
                sha = sha256_of_file(path)
            out[f"sha256:{param}"] = sha
            out[f"sha256:{raw}"] = sha
        return out

    def _sha_from_manifest(self, manifest_url: str, filename: str) -> str:
        if self._dry_run:
            return hashlib.sha256((manifest_url + filename).encode("utf-8")).hexdigest()
        text = read_location(manifest_url)[:10240].decode("utf-8").strip()
        for row in text.splitlines():
            cols = row.split()
            if len(cols) == 2 and cols[1] in (filename, f"*{filename}"):   # '*' marks a binary file
                return cols[0]
        raise ValueError(f"No entry found for {filename} in manifest at {manifest_url}:\n{text}")

    # -- build ---------------------------------------------------------------------------------
    def _package_files(self) -> Iterable[Tuple[str, str]]:
        for name in sorted(os.listdir(self._input_dir_path)):
            path = os.path.join(self._input_dir_path, name)
            if os.path.getsize(path) > MAX_PACKAGE_FILE_BYTES:
                LOGGER.warning("Ignoring package file larger than 1MB: %s", path)
                continue
            if name not in PACKAGE_FILES:
                LOGGER.warning("Ignoring unrecognized package file: %s (expected one of: %s)", path,
                               ", ".join(PACKAGE_FILES))
                continue
            with open(path, "r", encoding="utf-8") as f:
                yield name, f.read()

    def build_package_files(self) -> Dict[str, str]:
        out = {}
        for name, content in self._package_files():
            mapping = self.template_mapping(content)
            new = apply_template(content, mapping)
            if new != content:
                LOGGER.debug("Applied templating to %s:\n%s", name, "\n".join(
                    difflib.unified_diff(content.split("\n"), new.split("\n"), lineterm="")))
            out[name] = new
        return out

    def packages_dict(self) -> dict:
        pkg = package_from_files(self.build_package_files())
        pkg["releaseVersion"] = 0
        pkg["lastUpdated"] = round(time.time() if self._now is None else self._now)
        return collections.OrderedDict(packages=[pkg])

    def build_package(self, out_dir: Optional[str] = None) -> str:
        """Write ``stub-universe-<name>.json`` and return its path."""
        out_dir = out_dir or tempfile.mkdtemp(prefix="stub-universe-tmp")
        os.makedirs(out_dir, exist_ok=True)
        path = os.path.join(out_dir, f"stub-universe-{self._package.get_name()}.json")
        with open(path, "w", encoding="utf-8") as f:
            json.dump(self.packages_dict(), f, indent=2)
        return path
