"""Print the version of a package as the cluster's Cosmos describes it, or the git SHA that
version is tagged at (reference: tools/print_package_tag.py).

``python -m dcos_commons_amd.tools.print_package_tag <package> [repo path | repo URL]``. The
version comes from ``describe`` (``dcos package describe`` in the reference; here any callable,
by default the active local cluster's Cosmos); the SHA from the local checkout
(``git rev-parse <tag>^{}``) or the remote (``git ls-remote --tags``, peeled tag first).
"""
from __future__ import annotations

import logging
import os
import subprocess
import sys
from typing import Callable, List, Optional

LOGGER = logging.getLogger(__name__)


def _cluster_describe(package_name: str) -> dict:
    from dcos_commons_amd.testing.cluster import current

    c = current()
    return {"version": c.cosmos.versions(package_name)[-1]}


class PackageVersion:
    def __init__(self, package_name: str, describe: Optional[Callable[[str], dict]] = None):
        self._name = package_name
        self._describe = describe or _cluster_describe

    def get_version(self) -> str:
        try:
            return self._describe(self._name)["version"]
        except Exception:
            LOGGER.error("Failed to get the version of package %s", self._name)
            raise

    def get_version_sha_for_path(self, repo_path: str) -> str:
        tag = self.get_version()
        git_dir = os.path.join(repo_path, ".git")
        return self._run(["git", f"--git-dir={git_dir}", "rev-parse", tag + "^{}"])

    def get_version_sha_for_url(self, repo_url: str) -> str:
        tag = self.get_version()
        rev = self._run(["git", "ls-remote", "--tags", repo_url, f"refs/tags/{tag}^{{}}"])
        if not rev:   # lightweight tag: no peeled entry
            rev = self._run(["git", "ls-remote", "--tags", repo_url, f"refs/tags/{tag}"])
        if not rev:
            raise ValueError(f'No tag "{tag}" in {repo_url}')
        return rev.split()[0]

    @staticmethod
    def _run(argv: List[str]) -> str:
        LOGGER.info("CMD: %s", " ".join(argv))
        return subprocess.check_output(argv).decode("utf-8").strip()


def main(argv: List[str], describe: Optional[Callable[[str], dict]] = None) -> int:
    if len(argv) not in (2, 3):
        LOGGER.error("Syntax: %s <package> [/local/repo/path or git@host.com:remote/repo]", argv[0])
        return 1
    pv = PackageVersion(argv[1], describe)
    if len(argv) == 2:
        print(pv.get_version())
    elif os.path.isdir(argv[2]):
        print(pv.get_version_sha_for_path(argv[2]))
    else:
        print(pv.get_version_sha_for_url(argv[2]))
    return 0


if __name__ == "__main__":
    logging.basicConfig(level=logging.INFO, format="%(message)s")
    sys.exit(main(sys.argv))
