"""The provider-independent half of publishing a built package to an object store: render the
stub universe against the store's HTTP directory, upload it first and the artifacts next to it,
and report the universe URL (reference: the shared flow of tools/publish_aws.py and
tools/publish_azure.py). The providers (``publish_aws``, ``publish_azure``) pick the destination.

``UNIVERSE_URL_PREFIX`` is prepended to the stub universe URL (the reference's
universe-converter), ``UNIVERSE_URL_PATH`` receives the URL, and ``WORKSPACE`` gets the
``<version>.properties`` file for CI.
"""
from __future__ import annotations

import logging
import os
import random
import string
import sys
import time
from typing import List, Sequence

from dcos_commons_amd.tools.universe import Package, PackageManager, UniversePackageBuilder, Version

LOGGER = logging.getLogger(__name__)
UNIVERSE_CONTENT_TYPE = "application/vnd.dcos.universe.repo+json;charset=utf-8"


def unique_dir_name() -> str:
    """``<yyyymmdd-HHMMSS>-<16 random letters/digits>``: concurrent publishes never collide."""
    rand = "".join(random.SystemRandom().choice(string.ascii_letters + string.digits) for _ in range(16))
    return f"{time.strftime('%Y%m%d-%H%M%S')}-{rand}"


class ObjectStorePublisher:
    def __init__(self, package_name: str, package_version: str, input_dir_path: str,
                 artifact_paths: Sequence[str], uploader, dry_run: bool = False):
        if not os.path.isdir(input_dir_path):
            raise ValueError(f"Provided package path is not a directory: {input_dir_path}")
        for p in artifact_paths:
            if not os.path.isfile(p):
                raise ValueError(f"Provided artifact path is not a file: {p} (full list: {list(artifact_paths)})")
        self._name, self._version, self._input_dir = package_name, package_version, input_dir_path
        self._artifacts: List[str] = list(artifact_paths)
        self._uploader = uploader
        self._dry_run = dry_run
        self._url_prefix = os.environ.get("UNIVERSE_URL_PREFIX", "")

    def upload(self, work_dir: str = None) -> str:
        """Uploads the stub universe first, then the artifacts; returns the universe URL."""
        import tempfile

        http_dir = self._uploader.http_directory_url()
        builder = UniversePackageBuilder(Package(self._name, Version(0, self._version)), PackageManager(),
                                         self._input_dir, http_dir, self._artifacts)
        universe_path = builder.build_package(work_dir or tempfile.mkdtemp(prefix="publish-"))
        self._uploader.upload(universe_path, content_type=UNIVERSE_CONTENT_TYPE)
        url = self._url_prefix + http_dir + "/" + os.path.basename(universe_path)
        LOGGER.info("STUB UNIVERSE: %s", url)
        for p in self._artifacts:
            self._uploader.upload(p)
        self._spam_universe_url(url)
        return url

    def _spam_universe_url(self, url: str) -> None:
        ws = os.environ.get("WORKSPACE")
        if ws:
            with open(os.path.join(ws, f"{self._version}.properties"), "w", encoding="utf-8") as f:
                f.write(f"STUB_UNIVERSE_URL={url}\n")
        path = os.environ.get("UNIVERSE_URL_PATH")
        if path:
            with open(path, "w", encoding="utf-8") as f:
                f.write(url + "\n")


def main(argv: Sequence[str], make) -> int:
    """Shared command line of ``publish_aws`` / ``publish_azure``: ``make`` builds the provider's
    publisher for (package name, version, template dir, artifacts)."""
    if len(argv) < 3:
        print("Syntax: {} <package-name> <template-package-dir> [artifact files ...]".format(argv[0]),
              file=sys.stderr)
        return 1
    name, input_dir, artifacts = argv[1], argv[2].rstrip("/"), argv[3:]
    version = os.environ.get("TEMPLATE_PACKAGE_VERSION", "stub-universe")
    print(make(name, version, input_dir, artifacts).upload())
    return 0


