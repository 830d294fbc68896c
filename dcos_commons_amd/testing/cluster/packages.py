"""Cosmos stand-in: package install / update / uninstall / describe for the local cluster.

A package is a framework's ``universe/`` directory (``config.json`` option schema,
``marathon.json.mustache`` scheduler app, ``resource.json``, ``package.json``). Installing renders
the Marathon app from the option defaults plus the user's options (``testing.cosmos``) and hands
it to ``LocalMarathon``. Several versions of one package can be registered (same or different
directories); the version is rendered into ``PACKAGE_VERSION`` and, for frameworks that force a
rolling update on upgrade, ``TASKCFG_ALL_PACKAGE_VERSION_TO_FORCE_UPDATE``.

``update`` follows ``dcos <svc> update start``: the new options are merged into the ones given at
install time (or replace them with ``replace=True``) and the app is rolled; the scheduler then
runs its config update / ``update`` plan. ``uninstall`` follows the SDK uninstall protocol for apps
labelled ``DCOS_COMMONS_UNINSTALL``: the app is rolled with ``SDK_UNINSTALL=true``, the scheduler
runs its uninstall plan (kill tasks, unreserve, deregister) and the app is destroyed once the plan
is COMPLETE.
"""
from __future__ import annotations

import copy
import json
import logging
import os
import time
import urllib.error
import urllib.request
from dataclasses import dataclass, field
from typing import Dict, List, Mapping, Optional

from dcos_commons_amd.testing import cosmos
from dcos_commons_amd.testing.cluster.marathon import REPO_ROOT, normalize_app_id

LOGGER = logging.getLogger(__name__)
DEFAULT_VERSION = "1.0.0-local"
PREVIOUS_VERSION = "0.9.0-local"


def flatten_options(options: Mapping, prefix: str = "") -> Dict[str, str]:
    """``{"service": {"name": "x"}}`` -> ``{"service.name": "x"}`` (values kept as Python types)."""
    out: Dict[str, object] = {}
    for k, v in (options or {}).items():
        key = f"{prefix}.{k}" if prefix else str(k)
        if isinstance(v, Mapping):
            out.update(flatten_options(v, key))
        else:
            out[key] = v
    return out


def merge_options(base: Mapping, update: Mapping) -> dict:
    out = copy.deepcopy(dict(base or {}))
    for k, v in (update or {}).items():
        if isinstance(v, Mapping) and isinstance(out.get(k), Mapping):
            out[k] = merge_options(out[k], v)
        else:
            out[k] = copy.deepcopy(v)
    return out


@dataclass
class PackageVersion:
    name: str
    version: str
    universe_dir: str

    def package_json(self) -> dict:
        path = os.path.join(self.universe_dir, "package.json")
        if not os.path.exists(path):
            return {"name": self.name, "version": self.version}
        with open(path, "r", encoding="utf-8") as f:
            text = f.read()
        return json.loads(text.replace("{{package-version}}", self.version))


@dataclass
class InstalledService:
    service_name: str
    package: PackageVersion
    user_options: dict
    history: List[str] = field(default_factory=list)


def default_packages() -> Dict[str, str]:
    """Package name -> universe directory for the frameworks in this repo."""
    base = os.path.join(REPO_ROOT, "frameworks")
    out = {}
    for fw in sorted(os.listdir(base)):
        udir = os.path.join(base, fw, "universe")
        pj = os.path.join(udir, "package.json")
        if os.path.exists(pj):
            with open(pj, "r", encoding="utf-8") as f:
                name = json.loads(f.read().replace("{{package-version}}", DEFAULT_VERSION))["name"]
            out[name] = udir
    return out


class LocalCosmos:
    def __init__(self, cluster, packages: Optional[Mapping[str, str]] = None):
        self.cluster = cluster
        self._versions: Dict[str, List[PackageVersion]] = {}
        for name, udir in (packages if packages is not None else default_packages()).items():
            # a "released" version and the one built from this tree (the stub universe): upgrade
            # tests roll every task from one to the other (the version is in the task env)
            self.register(name, udir, PREVIOUS_VERSION)
            self.register(name, udir)
        self.installed: Dict[str, InstalledService] = {}
        self.repositories: List[dict] = []

    # -- repositories -------------------------------------------------------------------------
    def add_repo(self, location: str, name: Optional[str] = None) -> List[PackageVersion]:
        """``dcos package repo add``: register every release a universe repository holds (a stub
        universe JSON file/URL, a ``.dcos`` bundle or a repository tree; see
        ``tools.universe.package_manager``). Releases register in ``releaseVersion`` order, so the
        newest one is what an install without ``--package-version`` gets. A ``.dcos`` bundle's
        artifacts are staged into the cluster's artifact store, where the fetcher finds them by
        file name (the air-gapped path: nothing is downloaded)."""
        from dcos_commons_amd.tools.universe import package_manager as pm

        definitions = sorted(pm.load_repository(location), key=lambda d: int(d.get("releaseVersion", 0)))
        base = os.path.join(self.cluster.work_dir, "universe")
        added = []
        for d in definitions:
            pdir = os.path.join(base, d["name"], str(d.get("releaseVersion", 0)) + "-" + d["version"])
            os.makedirs(pdir, exist_ok=True)
            for fname, text in pm.files_from_package(d).items():
                with open(os.path.join(pdir, fname), "w", encoding="utf-8") as f:
                    f.write(text)
            added.append(self.register(d["name"], pdir, d["version"]))
        if location.endswith(".dcos"):
            self._stage_bundle_resources(location, os.path.join(base, "resources"))
        self.repositories.append({"name": name or f"repo-{len(self.repositories)}", "uri": location,
                                  "packages": [f"{p.name}:{p.version}" for p in added]})
        return added

    def _stage_bundle_resources(self, bundle: str, out_dir: str) -> None:
        import zipfile

        from dcos_commons_amd.tools.universe.package_manager import RESOURCES_DIR

        with zipfile.ZipFile(bundle) as z:
            for member in z.namelist():
                if not member.startswith(RESOURCES_DIR + "/") or member.endswith("/"):
                    continue
                base = os.path.basename(member)
                dest = os.path.join(out_dir, base)
                os.makedirs(out_dir, exist_ok=True)
                with z.open(member) as src, open(dest, "wb") as dst:
                    dst.write(src.read())
                self.cluster.register_artifact(base, dest)

    def remove_repo(self, name: str) -> None:
        self.repositories = [r for r in self.repositories if r["name"] != name]

    # -- registry -------------------------------------------------------------------------
    def register(self, name: str, universe_dir: str, version: str = DEFAULT_VERSION) -> PackageVersion:
        pv = PackageVersion(name, version, universe_dir)
        versions = [v for v in self._versions.get(name, []) if v.version != version]
        versions.append(pv)
        self._versions[name] = versions
        return pv

    def versions(self, name: str) -> List[str]:
        return [v.version for v in self._versions.get(name, [])]

    def package(self, name: str, version: Optional[str] = None) -> PackageVersion:
        versions = self._versions.get(name)
        if not versions:
            raise KeyError(f"Package [{name}] not found")
        if version is None:
            return versions[-1]
        for v in versions:
            if v.version == version:
                return v
        raise KeyError(f"Version [{version}] of package [{name}] not found")

    # -- rendering ------------------------------------------------------------------------
    def render(self, pv: PackageVersion, options: Mapping) -> dict:
        flat = {k: v for k, v in flatten_options(options).items()}
        app = cosmos.render_marathon_app(pv.universe_dir, flat, {},
                                         {"package-name": pv.name, "package-version": pv.version})
        labels = app.setdefault("labels", {})
        labels.setdefault("DCOS_PACKAGE_NAME", pv.name)
        labels["DCOS_PACKAGE_VERSION"] = pv.version
        labels["DCOS_PACKAGE_OPTIONS"] = json.dumps(options, sort_keys=True)
        return app

    def resolved_options(self, pv: PackageVersion, options: Mapping) -> dict:
        flat = cosmos.option_defaults(pv.universe_dir)
        flat.update({k: cosmos._scalar(v) for k, v in flatten_options(options).items()})
        out: dict = {}
        for key, val in sorted(flat.items()):
            node = out
            parts = key.split(".")
            for p in parts[:-1]:
                node = node.setdefault(p, {})
            node[parts[-1]] = val
        return out

    @staticmethod
    def service_name_of(app: dict) -> str:
        return app.get("labels", {}).get("DCOS_SERVICE_NAME") or app["id"].lstrip("/")

    # -- package operations ------------------------------------------------------------------
    def install(self, package: str, service_name: Optional[str] = None, options: Optional[Mapping] = None,
                version: Optional[str] = None, wait: bool = True) -> dict:
        pv = self.package(package, version)
        options = copy.deepcopy(dict(options or {}))
        if service_name:
            options = merge_options(options, {"service": {"name": service_name}})
        app = self.render(pv, options)
        name = normalize_app_id(app["id"]).lstrip("/")
        if name in self.installed:
            raise ValueError(f"A service named [{name}] is already installed")
        self.installed[name] = InstalledService(name, pv, options, [pv.version])
        self.cluster.marathon.install_app(app, wait=wait)
        return app

    def update(self, service_name: str, options: Optional[Mapping] = None, version: Optional[str] = None,
               replace: bool = False, wait: bool = True) -> dict:
        svc = self._installed(service_name)
        pv = self.package(svc.package.name, version) if version else svc.package
        merged = copy.deepcopy(dict(options or {})) if replace else merge_options(svc.user_options, options or {})
        # the service name is fixed at install time
        name = svc.user_options.get("service", {}).get("name")
        if name is not None:
            merged = merge_options(merged, {"service": {"name": name}})
        app = self.render(pv, merged)
        svc.package, svc.user_options = pv, merged
        svc.history.append(pv.version)
        self.cluster.marathon.update_app(app, wait=wait)
        return app

    def describe(self, service_name: str) -> dict:
        svc = self._installed(service_name)
        pv = svc.package
        vs = self.versions(pv.name)
        return {"package": pv.package_json(), "upgradesTo": [v for v in vs if v != pv.version],
                "downgradesTo": [v for v in vs if v != pv.version], "userProvidedOptions": svc.user_options,
                "resolvedOptions": self.resolved_options(pv, svc.user_options)}

    def list(self) -> List[dict]:
        return [{"name": s.package.name, "version": s.package.version, "appId": "/" + n}
                for n, s in sorted(self.installed.items())]

    def uninstall(self, service_name: str, timeout_s: float = 120.0) -> None:
        svc = self._installed(service_name)
        marathon = self.cluster.marathon
        app_id = "/" + svc.service_name
        app = marathon.get_app(app_id)
        sdk_uninstall = app.get("labels", {}).get("DCOS_COMMONS_UNINSTALL", "").lower() == "true"
        if sdk_uninstall:
            definition = {k: v for k, v in app.items() if k not in ("tasks", "tasksRunning", "deployments", "version")}
            definition.setdefault("env", {})["SDK_UNINSTALL"] = "true"
            marathon.update_app(definition, wait=True)
            self._wait_uninstalled(app_id, timeout_s)
        marathon.destroy_app(app_id)
        del self.installed[svc.service_name]

    def _wait_uninstalled(self, app_id: str, timeout_s: float) -> None:
        url = self.cluster.marathon.scheduler_url(app_id) + "/v1/plans/deploy"
        deadline = time.time() + timeout_s
        while time.time() < deadline:
            try:
                with urllib.request.urlopen(url, timeout=5) as r:
                    if r.status == 200:
                        return
            except urllib.error.HTTPError:
                pass
            except (urllib.error.URLError, OSError):
                pass
            time.sleep(0.1)
        raise TimeoutError(f"Uninstall of {app_id} did not complete in {timeout_s}s:\n"
                           f"{self.cluster.marathon.log_tail(app_id)}")

    def _installed(self, service_name: str) -> InstalledService:
        name = service_name.strip("/")
        svc = self.installed.get(name)
        if svc is None:
            raise KeyError(f"Service [{name}] is not installed")
        return svc
