"""Turn a stub universe build into a versioned release.

Reference: tools/release_builder.py (``move`` re-homes a stub universe's artifacts under a release
directory on S3; ``release`` additionally opens a pull request against the public universe repo).
Without S3 or GitHub, both targets are local: the release directory is a filesystem path (or any
URL prefix served from it) and the universe is a repository *tree*
(``repo/packages/<L>/<name>/<releaseVersion>/``) that ``PackageManager``/``LocalCosmos.add_repo``
read. The package edits are the reference's:

* ``package.json``: ``version`` := the release version; ``name`` gains/loses ``beta-``; beta releases
  are never ``selected``; ``upgradesFrom``/``downgradesTo`` := the given list, or the latest release
  of the (renamed) package when the beta bit changed the name;
* ``marathon.json.mustache``: the ``PACKAGE_NAME``/``PACKAGE_VERSION`` env lines;
* ``resource.json``: every URL under the stub universe's directory is rewritten to the release
  directory, and those artifacts are copied there. An existing release directory is never
  overwritten unless ``force``.

Usage: ``python -m dcos_commons_amd.tools.release_builder move|release <version> <stub-universe>
--release-dir DIR [--release-url URL] [--universe-repo DIR] [--beta] [--upgrades-from V ...] [--force]``.
"""
from __future__ import annotations

import argparse
import base64
import collections
import copy
import json
import logging
import os
import re
import sys
from typing import List, Optional, Sequence

from dcos_commons_amd.tools.universe import PackageManager, files_from_package, repo_tree_path
from dcos_commons_amd.tools.universe.package_manager import read_location

LOGGER = logging.getLogger(__name__)
_NAME_LINE = re.compile(r'^ *"PACKAGE_NAME": ?"(.*)",?$')
_VERSION_LINE = re.compile(r'^ *"PACKAGE_VERSION": ?"(.*)",?$')


def left_trim(s: str, prefix: str) -> str:
    return s[len(prefix):] if s.startswith(prefix) else s


def right_trim(s: str, suffix: str) -> str:
    return s[:-len(suffix)] if suffix and s.endswith(suffix) else s


def package_name_from_url(stub_universe_url: str) -> str:
    m = re.match(r".*stub-universe-(.+)\.json$", stub_universe_url)
    if not m:
        raise ValueError('Expected a stub universe file named "stub-universe-<pkgname>.json": ' + stub_universe_url)
    return m.group(1)


def apply_beta_prefix(name: str, beta: bool) -> str:
    base = left_trim(name, "beta-")
    return f"beta-{base}" if beta else base


def apply_beta_version(version: str, beta: bool) -> str:
    base = right_trim(version, "-beta")
    if beta:
        return f"{base}-beta"
    if version.endswith("-beta"):
        raise ValueError(f'Requested package version {version} ends with "-beta", but BETA mode is disabled.')
    return base


class UniverseReleaseBuilder:
    def __init__(self, package_version: str, stub_universe_url: str, release_dir: str,
                 release_url: Optional[str] = None, universe_repo: Optional[str] = None, beta: bool = False,
                 upgrades_from: Sequence[str] = (), force: bool = False,
                 package_manager: Optional[PackageManager] = None):
        if not stub_universe_url.endswith(".json"):
            raise ValueError(f"Expected .json extension for stub universe: {stub_universe_url}")
        self._stub_url = stub_universe_url
        self._stub = json.loads(read_location(stub_universe_url).decode("utf-8"),
                                object_pairs_hook=collections.OrderedDict)
        pkgs = self._stub.get("packages")
        if not isinstance(pkgs, list) or len(pkgs) != 1:
            raise ValueError(f'Expected a single "packages" entry in stub universe JSON: {stub_universe_url}')
        self._stub_pkg_name = pkgs[0].get("name") or package_name_from_url(stub_universe_url)
        self._beta = beta
        self._pkg_name = apply_beta_prefix(os.environ.get("PACKAGE_NAME") or self._stub_pkg_name, beta)
        self._pkg_version = apply_beta_version(package_version, beta)
        # beta-foo's artifacts live under foo/ (with a -beta version)
        self._release_dir = os.path.join(release_dir, left_trim(self._pkg_name, "beta-"), self._pkg_version)
        self._release_url = (release_url.rstrip("/") + f"/{left_trim(self._pkg_name, 'beta-')}/{self._pkg_version}"
                             if release_url else "file://" + self._release_dir)
        self._universe_repo = universe_repo
        self._upgrades_from = list(upgrades_from)
        self._force = force
        self._pkg_manager = package_manager or PackageManager([universe_repo] if universe_repo else [])

    @property
    def release_url(self) -> str:
        return self._release_url

    # -- package edits ---------------------------------------------------------------------------
    def update_package_json(self, pkg: dict) -> None:
        if self._beta:
            pkg["selected"] = False
        pkg["name"] = self._pkg_name
        pkg["version"] = self._pkg_version
        if self._upgrades_from:
            pkg["upgradesFrom"] = list(self._upgrades_from)
            pkg["downgradesTo"] = list(self._upgrades_from)
        elif self._stub_pkg_name != self._pkg_name and (pkg.get("upgradesFrom", ["*"]) != ["*"]
                                                        or pkg.get("downgradesTo", ["*"]) != ["*"]):
            last = self._pkg_manager.get_latest(self._pkg_name)
            versions = [] if last is None else [last.get_version().package_version]
            pkg["upgradesFrom"] = versions
            pkg["downgradesTo"] = list(versions)

    def update_marathon_json(self, pkg: dict) -> None:
        encoded = (pkg.get("marathon") or {}).get("v2AppMustacheTemplate")
        if not encoded:
            return
        lines = []
        for line in base64.standard_b64decode(encoded).decode("utf-8").split("\n"):
            n, v = _NAME_LINE.match(line), _VERSION_LINE.match(line)
            if n:
                line = line.replace(n.group(1), self._pkg_name)
            elif v:
                line = line.replace(v.group(1), self._pkg_version)
            lines.append(line)
        pkg["marathon"]["v2AppMustacheTemplate"] = base64.standard_b64encode("\n".join(lines).encode("utf-8")).decode()

    def update_resource_json(self, pkg: dict) -> List[str]:
        """Rewrite the artifact URLs; returns the original ones (the artifacts to copy)."""
        if "resource" not in pkg:
            return []
        prefix = "/".join(self._stub_url.split("/")[:-1])
        text = json.dumps(pkg["resource"], indent=2)
        originals = re.findall('({}/[^"]+)"'.format(re.escape(prefix)), text)
        pkg["resource"] = json.loads(text.replace(prefix, self._release_url),
                                     object_pairs_hook=collections.OrderedDict)
        return originals

    def _updated_package(self):
        pkg = copy.deepcopy(self._stub["packages"][0])
        self.update_package_json(pkg)
        self.update_marathon_json(pkg)
        return pkg, self.update_resource_json(pkg)

    def _copy_artifacts(self, urls: Sequence[str]) -> None:
        if os.path.isdir(self._release_dir) and os.listdir(self._release_dir) and not self._force:
            raise FileExistsError(f"Release artifact destination already exists: {self._release_dir}. "
                                  "Delete it or pass force=True to overwrite.")
        os.makedirs(self._release_dir, exist_ok=True)
        for i, url in enumerate(urls):
            dest = os.path.join(self._release_dir, os.path.basename(url))
            LOGGER.info("[%d/%d] %s -> %s", i + 1, len(urls), url, dest)
            with open(dest, "wb") as f:
                f.write(read_location(url))

    # -- targets -----------------------------------------------------------------------------------
    def move_package(self) -> str:
        """Copy the artifacts to the release dir and write the re-homed stub universe there."""
        pkg, urls = self._updated_package()
        self._copy_artifacts(urls)
        path = os.path.join(self._release_dir, f"stub-universe-{self._pkg_name}.json")
        with open(path, "w", encoding="utf-8") as f:
            json.dump({"packages": [pkg]}, f, indent=2)
        return path

    def release_package(self) -> str:
        """``move_package`` plus a new release (next ``releaseVersion``) in the universe repo tree."""
        if not self._universe_repo:
            raise ValueError("release needs a universe repository directory")
        pkg, urls = self._updated_package()
        self._copy_artifacts(urls)
        latest = self._pkg_manager.get_latest(self._pkg_name)
        release = 0 if latest is None else latest.get_version().release_version + 1
        pkg["releaseVersion"] = release
        out = repo_tree_path(self._universe_repo, self._pkg_name, release)
        os.makedirs(out, exist_ok=True)
        for name, text in files_from_package(pkg).items():
            if name == "package.json":
                body = json.loads(text, object_pairs_hook=collections.OrderedDict)
                body.pop("releaseVersion", None)     # the directory name carries it
                text = json.dumps(body, indent=2) + "\n"
            with open(os.path.join(out, name), "w", encoding="utf-8") as f:
                f.write(text)
        return out


def main(argv: Optional[Sequence[str]] = None) -> int:
    logging.basicConfig(level=logging.INFO, format="%(message)s")
    ap = argparse.ArgumentParser(description="Move a stub universe build to a release location")
    ap.add_argument("target", choices=["move", "release"])
    ap.add_argument("package_version")
    ap.add_argument("stub_universe")
    ap.add_argument("--release-dir", required=True)
    ap.add_argument("--release-url", default=None)
    ap.add_argument("--universe-repo", default=None)
    ap.add_argument("--beta", action="store_true", default=os.environ.get("BETA", "").lower() == "true")
    ap.add_argument("--upgrades-from", nargs="*", default=[])
    ap.add_argument("--force", action="store_true")
    args = ap.parse_args(argv)
    b = UniverseReleaseBuilder(args.package_version, args.stub_universe, args.release_dir, args.release_url,
                               args.universe_repo, args.beta, args.upgrades_from, args.force)
    print(b.move_package() if args.target == "move" else b.release_package())
    return 0


if __name__ == "__main__":
    sys.exit(main())
