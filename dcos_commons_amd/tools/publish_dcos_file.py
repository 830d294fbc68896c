"""Write a ``.dcos`` bundle: one file holding a package and every artifact it references.

Reference: tools/publish_dcos_file.py (builds the bundle with the DC/OS registry CLI, then uploads
it to S3 for air-gapped installs). Here the bundle is a zip with ``catalog.json`` (a stub universe
whose ``{{artifact-dir}}`` is ``bundle://<package>/<version>``) and the artifacts under
``resources/``. ``LocalCosmos.add_repo("<file>.dcos")`` registers the package and stages the
artifacts into the cluster, where the fetcher resolves them by file name -- no network at all.
"""
from __future__ import annotations

import json
import os
import zipfile
from typing import Optional, Sequence

from dcos_commons_amd.tools.universe import Package, PackageManager, UniversePackageBuilder, Version
from dcos_commons_amd.tools.universe.package_manager import CATALOG_NAME, RESOURCES_DIR


def build_dcos_file(package_name: str, package_version: str, input_dir_path: str, artifact_paths: Sequence[str],
                    out_dir: str, package_manager: Optional[PackageManager] = None) -> str:
    builder = UniversePackageBuilder(Package(package_name, Version(0, package_version)),
                                     package_manager or PackageManager(), input_dir_path,
                                     f"bundle://{package_name}/{package_version}", artifact_paths)
    catalog = builder.packages_dict()
    os.makedirs(out_dir, exist_ok=True)
    path = os.path.join(out_dir, f"{package_name}-{package_version}.dcos")
    with zipfile.ZipFile(path, "w", zipfile.ZIP_DEFLATED) as z:
        z.writestr(CATALOG_NAME, json.dumps(catalog, indent=2))
        for a in artifact_paths:
            z.write(a, f"{RESOURCES_DIR}/{os.path.basename(a)}")
    return path
