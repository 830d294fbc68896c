"""Check that a framework can run on an air-gapped cluster.

Reference: tools/airgap_linter.py. Two rules, over the package files (``universe/config.json``,
``marathon.json.mustache``, ``resource.json``, ``package.json``) and every file of the scheduler's
distribution (the reference's ``src/main/dist``; here the framework's ``specs/``):

* no plain ``http://`` URI outside the cluster: a URI is allowed only when it names a cluster-internal
  host (``.thisdcos``, ``.mesos``, or a task/scheduler address variable); everything else must
  be exported through ``resource.json`` (which an air-gap bundle rewrites to local copies);
* no container image named directly: ``image:`` must be a ``{{TEMPLATED}}`` reference.

Comment lines (``#``, ``//``, ``*``) and ``"id":`` lines are ignored. Usage:
``python -m dcos_commons_amd.tools.airgap_linter <framework-dir>`` (exit 1 on any violation).
"""
from __future__ import annotations

import os
import re
import sys
from typing import List, Sequence, Tuple

_URI = re.compile(r".*http?://([^?\s]*)", re.IGNORECASE)
_IMAGE = re.compile(r"image:\s?(.*)$", re.IGNORECASE)
_TEMPLATED = re.compile(r'["]?\{\{[A-Z0-9_]*\}\}["]?')
CLUSTER_INTERNAL = (".thisdcos", ".mesos:", ".mesos/", "$MESOS_CONTAINER_IP", "${MESOS_CONTAINER_IP}",
                    "$LIBPROCESS_IP", "${LIBPROCESS_IP}", "{{LIBPROCESS_IP}}", "{{FRAMEWORK_HOST}}",
                    "$FRAMEWORK_HOST", "${FRAMEWORK_HOST}", "{{SCHEDULER_API_HOSTNAME}}",
                    "${SCHEDULER_API_HOSTNAME}", "$SCHEDULER_API_HOSTNAME")
PACKAGE_FILES = ("config.json", "marathon.json.mustache", "resource.json", "package.json")


def _lines(path: str) -> List[str]:
    try:
        with open(path, "r", encoding="utf-8") as f:
            return f.readlines()
    except UnicodeDecodeError:
        print(f"Skipping binary file {path}")
        return []
    except FileNotFoundError:
        return []


def extract_uris(path: str) -> List[str]:
    out = []
    for line in _lines(path):
        line = line.strip()
        if line.startswith(("*", "#", "//")) or '"id":' in line:
            continue
        m = _URI.match(line)
        if m:
            out.append(m.group(1))
    return out


def is_bad_uri(uri: str) -> bool:
    return not any(marker in uri for marker in CLUSTER_INTERNAL)


def files_to_check(framework_dir: str) -> List[str]:
    files = [os.path.join(framework_dir, "universe", n) for n in PACKAGE_FILES]
    for dist in ("specs", os.path.join("src", "main", "dist")):
        for dirpath, dirs, names in os.walk(os.path.join(framework_dir, dist)):
            dirs.sort()
            files.extend(os.path.join(dirpath, n) for n in sorted(names))
    return files


def bad_uris(framework_dir: str) -> List[Tuple[str, str]]:
    return [(path, uri) for path in files_to_check(framework_dir) for uri in extract_uris(path) if is_bad_uri(uri)]


def bad_images(framework_dir: str) -> List[Tuple[str, str]]:
    out = []
    for path in files_to_check(framework_dir):
        for line in _lines(path):
            line = line.strip()
            if "image:" not in line:
                continue
            m = _IMAGE.match(line)
            if m and not _TEMPLATED.match(m.group(1)):
                out.append((path, m.group(1)))
    return out


def check(framework_dir: str) -> bool:
    ok = True
    for path, uri in bad_uris(framework_dir):
        print(f"Found a bad URI: {uri} in: {path} Export URIs to resource.json to allow packaging for "
              "airgapped clusters.")
        ok = False
    for path, image in bad_images(framework_dir):
        print(f"Bad image found in {path}. It is a direct reference instead of a templated reference: {image} "
              "Export images to resource.json to allow packaging for airgapped clusters.")
        ok = False
    if ok:
        print("Airgap check complete: no external URIs or direct image references found.")
    else:
        print("Airgap check FAILED: the package references non-https or external resources; move them to "
              "resource.json (or, for cluster-internal URLs, into the service YAML).")
    return ok


def main(argv: Sequence[str] = None) -> int:
    argv = list(sys.argv if argv is None else argv)
    if len(argv) < 2:
        print(__doc__)
        return 0
    if not os.path.isdir(argv[1]):
        print(f"Supplied framework directory {argv[1]} does not exist or is not a directory.")
        return 1
    return 0 if check(argv[1]) else 1


if __name__ == "__main__":
    sys.exit(main())
