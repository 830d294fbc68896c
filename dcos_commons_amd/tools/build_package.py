"""Build a framework's universe package and its artifacts, then optionally publish them.

Reference: tools/build_package.sh (+ the framework ``build.sh`` scripts that call it). Usage::

    python -m dcos_commons_amd.tools.build_package <package-name> <framework-dir>
        [-a ARTIFACT ...] [--out DIR] [local|.dcos|dir] [PACKAGE_VERSION]

Artifacts are built from this tree (no Gradle/Go): ``bootstrap.zip`` holds the native
``sdk-bootstrap`` as ``bootstrap``; ``<package>-scheduler.zip`` holds the scheduler (the
``dcos_commons_amd`` package, the framework's specs and ``bin/<package>`` launcher); and
``sdk-cli-linux`` is the native service CLI. Extra ``-a`` artifacts are added as given.

Publish methods: ``local`` serves the stub universe and artifacts over HTTP (``publish_http``),
``.dcos`` writes one air-gap bundle (``publish_dcos_file``), ``dir`` writes the stub universe next
to the artifacts with ``file://`` URLs; with none the stub universe is only built. Like the
reference, every framework except hello-world is run through the air-gap linter first.
"""
from __future__ import annotations

import argparse
import logging
import os
import shutil
import stat
import sys
import tempfile
import zipfile
from typing import List, Optional, Sequence

from dcos_commons_amd.tools import airgap_linter
from dcos_commons_amd.tools.universe import Package, PackageManager, UniversePackageBuilder, Version

LOGGER = logging.getLogger(__name__)
REPO_ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
NATIVE_BUILD = os.path.join(REPO_ROOT, "native", "build")
_SKIP_DIRS = {"__pycache__", ".pytest_cache"}


def _zip_tree(z: zipfile.ZipFile, src: str, arc_root: str) -> None:
    for dirpath, dirs, files in os.walk(src):
        dirs[:] = sorted(d for d in dirs if d not in _SKIP_DIRS)
        for f in sorted(files):
            if f.endswith(".pyc"):
                continue
            full = os.path.join(dirpath, f)
            z.write(full, os.path.join(arc_root, os.path.relpath(full, src)))


def _add_executable(z: zipfile.ZipFile, arcname: str, data: bytes) -> None:
    info = zipfile.ZipInfo(arcname)
    info.external_attr = (stat.S_IFREG | 0o755) << 16
    info.compress_type = zipfile.ZIP_DEFLATED
    z.writestr(info, data)


def build_bootstrap_zip(out_dir: str) -> str:
    src = os.path.join(NATIVE_BUILD, "sdk-bootstrap")
    if not os.path.exists(src):
        raise FileNotFoundError(f"{src} is missing: build the native tree first (cmake/ninja in native/build)")
    path = os.path.join(out_dir, "bootstrap.zip")
    with zipfile.ZipFile(path, "w", zipfile.ZIP_DEFLATED) as z, open(src, "rb") as f:
        _add_executable(z, "bootstrap", f.read())
    return path


def model_module(framework_dir: str) -> str:
    """``frameworks/helloworld`` -> ``helloworld`` (the ``dcos_commons_amd.models`` entry point)."""
    return os.path.basename(os.path.normpath(framework_dir)).replace("-", "")


def build_scheduler_zip(package_name: str, framework_dir: str, out_dir: str) -> str:
    root = f"{package_name}-scheduler"
    path = os.path.join(out_dir, f"{package_name}-scheduler.zip")
    launcher = ("#!/bin/sh\n"
                'HERE="$(cd "$(dirname "$0")/.." && pwd)"\n'
                'export PYTHONPATH="$HERE/lib${PYTHONPATH:+:$PYTHONPATH}"\n'
                f'export {package_name.upper().replace("-", "_")}_SPEC_DIR="$HERE/specs"\n'
                f'exec python3 -m dcos_commons_amd.models.{model_module(framework_dir)} "$@"\n')
    with zipfile.ZipFile(path, "w", zipfile.ZIP_DEFLATED) as z:
        _zip_tree(z, os.path.join(REPO_ROOT, "dcos_commons_amd"), f"{root}/lib/dcos_commons_amd")
        specs = os.path.join(framework_dir, "specs")
        if os.path.isdir(specs):
            _zip_tree(z, specs, f"{root}/specs")
        _add_executable(z, f"{root}/bin/{package_name}", launcher.encode("utf-8"))
    return path


def build_cli(out_dir: str) -> str:
    src = os.path.join(NATIVE_BUILD, "sdk-cli")
    if not os.path.exists(src):
        raise FileNotFoundError(f"{src} is missing: build the native tree first (cmake/ninja in native/build)")
    dest = os.path.join(out_dir, "sdk-cli-linux")
    shutil.copy2(src, dest)
    os.chmod(dest, 0o755)
    return dest


def build_artifacts(package_name: str, framework_dir: str, out_dir: str, extra: Sequence[str] = ()) -> List[str]:
    os.makedirs(out_dir, exist_ok=True)
    paths = [build_bootstrap_zip(out_dir), build_scheduler_zip(package_name, framework_dir, out_dir),
             build_cli(out_dir)]
    for a in extra:
        dest = os.path.join(out_dir, os.path.basename(a))
        if os.path.abspath(a) != os.path.abspath(dest):
            shutil.copy2(a, dest)
        paths.append(dest)
    return paths


def build_stub_universe(package_name: str, framework_dir: str, artifact_dir_uri: str, artifacts: Sequence[str],
                        version: str = "stub-universe", out_dir: Optional[str] = None,
                        package_manager: Optional[PackageManager] = None) -> str:
    universe_dir = os.environ.get("UNIVERSE_DIR") or os.path.join(framework_dir, "universe")
    builder = UniversePackageBuilder(Package(package_name, Version(0, version)),
                                     package_manager or PackageManager(), universe_dir, artifact_dir_uri, artifacts)
    return builder.build_package(out_dir)


def main(argv: Optional[Sequence[str]] = None) -> int:
    logging.basicConfig(level=logging.INFO, format="%(message)s")
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("package_name")
    ap.add_argument("framework_dir")
    ap.add_argument("-a", dest="artifacts", action="append", default=[], help="extra artifact file")
    ap.add_argument("--out", default=None, help="output directory (default: a temp dir)")
    ap.add_argument("publish", nargs="?", default="", choices=["", "local", ".dcos", "dir"])
    ap.add_argument("version", nargs="?", default="stub-universe")
    args = ap.parse_intermixed_args(argv)

    fw = os.path.abspath(args.framework_dir)
    LOGGER.info("Building %s package in %s (publish: %s)", args.package_name, fw, args.publish or "no")
    if args.package_name != "hello-world" and not airgap_linter.check(fw):
        return 1
    out = args.out or tempfile.mkdtemp(prefix=f"build-{args.package_name}-")
    artifacts = build_artifacts(args.package_name, fw, os.path.join(out, "artifacts"), args.artifacts)
    if args.publish == "local":
        from dcos_commons_amd.tools.publish_http import HTTPPublisher

        pub = HTTPPublisher(args.package_name, args.version, os.path.join(fw, "universe"), artifacts,
                            http_dir=os.path.join(out, "http"))
        url = pub.start()
        print(url, flush=True)
        pub.serve_forever()
        return 0
    if args.publish == ".dcos":
        from dcos_commons_amd.tools.publish_dcos_file import build_dcos_file

        print(build_dcos_file(args.package_name, args.version, os.path.join(fw, "universe"), artifacts, out))
        return 0
    uri = "file://" + os.path.join(out, "artifacts") if args.publish == "dir" else "https://artifacts.invalid"
    print(build_stub_universe(args.package_name, fw, uri, artifacts, args.version, out))
    return 0


if __name__ == "__main__":
    sys.exit(main())
