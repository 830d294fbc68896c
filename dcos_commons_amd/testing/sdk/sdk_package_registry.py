"""DC/OS package registry for integration tests (reference ``testing/sdk_package_registry.py``).

The reference installs the ``package-registry`` service and uploads ``.dcos`` bundles built from
the stub universes of the packages under test, so an air-gapped cluster can install them. The
stand-in's Cosmos (``testing.cluster.packages.LocalCosmos``) takes ``.dcos`` bundles as
repositories directly; here the registry is a record on the cluster, bundles are built by
``tools.publish_dcos_file``'s format (``catalog.json`` + ``resources/``) and adding one registers
its packages and stages its artifacts.
"""
from __future__ import annotations

import contextlib
import json
import logging
import os
import zipfile
from typing import Dict, Iterable, Iterator, List, Optional, Tuple

from dcos_commons_amd.testing.sdk import sdk_cmd
from dcos_commons_amd.tools.universe import package_manager as pm

LOG = logging.getLogger(__name__)

REGISTRY_APP_ID = "/package-registry"


def install_package_registry(service_secret_path: str) -> Dict[str, str]:
    """Start the registry (a record on the stand-in) under the service account whose secret is at
    ``service_secret_path``; returns its app definition."""
    c = sdk_cmd._cluster()
    app = {"id": REGISTRY_APP_ID, "env": {"DCOS_SERVICE_ACCOUNT_CREDENTIAL": service_secret_path},
           "labels": {"DCOS_PACKAGE_NAME": "package-registry"}}
    c.package_registry = {"app": app, "bundles": []}
    LOG.info("package registry installed (secret %s)", service_secret_path)
    return app


def grant_perms_for_registry_account(service_uid: str) -> None:
    """The reference grants the registry's account read access to the secret store; the stand-in
    keeps no ACLs for it."""
    LOG.info("registry account %s: permissions granted", service_uid)


def build_dcos_file_from_universe_definition(package: dict, dcos_files_path: str,
                                             resources: Optional[Dict[str, str]] = None) -> Tuple[str, str, str]:
    """Write ``<name>-<version>.dcos`` for one universe definition (with ``resources``: artifact
    file name -> local path); returns (name, version, bundle path)."""
    name, version = package["name"], package["version"]
    os.makedirs(dcos_files_path, exist_ok=True)
    path = os.path.join(dcos_files_path, f"{name}-{version}.dcos")
    with zipfile.ZipFile(path, "w", zipfile.ZIP_DEFLATED) as z:
        z.writestr(pm.CATALOG_NAME, json.dumps({"packages": [package]}, indent=2))
        for fname, local in (resources or {}).items():
            z.write(local, f"{pm.RESOURCES_DIR}/{fname}")
    return name, version, path


def build_dcos_files_from_stubs(stub_universe_urls: Iterable[str], dcos_files_path: str) -> List[Tuple[str, str, str]]:
    """One ``.dcos`` bundle per package definition of every stub universe."""
    out = []
    for url in stub_universe_urls:
        for package in pm.load_repository(url):
            out.append(build_dcos_file_from_universe_definition(package, dcos_files_path))
    return out


def add_dcos_files_to_registry(bundles: Iterable[str]) -> List[str]:
    """Upload ``.dcos`` bundles: their packages become installable (``name:version``)."""
    c = sdk_cmd._cluster()
    added = []
    for path in bundles:
        for pv in c.cosmos.add_repo(path, name=os.path.basename(path)):
            added.append(f"{pv.name}:{pv.version}")
        if getattr(c, "package_registry", None) is not None:
            c.package_registry["bundles"].append(path)
    LOG.info("registry: added %s", added)
    return added


@contextlib.contextmanager
def package_registry_session(dcos_files_path: str, stub_universe_urls: Iterable[str] = (),
                             service_secret_path: str = "package-registry/secret") -> Iterator[Dict[str, str]]:
    """Install the registry, add bundles built from ``stub_universe_urls``, and remove both on exit."""
    c = sdk_cmd._cluster()
    app = install_package_registry(service_secret_path)
    names = [os.path.basename(p) for _, _, p in build_dcos_files_from_stubs(stub_universe_urls, dcos_files_path)]
    add_dcos_files_to_registry(os.path.join(dcos_files_path, n) for n in names)
    try:
        yield app
    finally:
        for n in names:
            c.cosmos.remove_repo(n)
        c.package_registry = None
