"""Host a freshly built package (stub universe + artifacts) from a local HTTP server.

Reference: tools/publish_http.py. The artifacts are copied into ``HTTP_DIR`` (default
``/tmp/dcos-http-<package>/``), the stub universe is built with ``{{artifact-dir}}`` pointing at
the server, and the directory is served (``HTTP_HOST`` default 127.0.0.1, ``HTTP_PORT`` default
0 = ephemeral). ``.json`` is served as ``application/json`` and everything else as
``application/octet-stream``. The URL printed/returned is what ``dcos package repo add`` takes;
in this repo ``LocalCosmos.add_repo`` / ``sdk_cmd.run_cli("package repo add ...")`` install from
it and the local cluster's fetcher downloads the artifacts from the same server.

Differences from the reference: the server runs in-process (a ``ThreadingHTTPServer`` on a
daemon thread, ``stop()`` ends it) instead of a detached ``python -m http.server``, and the
Jenkins ``.properties`` side output is written only when ``WORKSPACE`` is set.
"""
from __future__ import annotations

import http.server
import json
import logging
import os
import shutil
import threading
from functools import partial
from typing import List, Optional, Sequence

from dcos_commons_amd.tools.universe import Package, PackageManager, UniversePackageBuilder, Version

LOGGER = logging.getLogger(__name__)


class _Handler(http.server.SimpleHTTPRequestHandler):
    def guess_type(self, path):
        return "application/json" if str(path).endswith(".json") else "application/octet-stream"

    def log_message(self, fmt, *args):
        LOGGER.debug("http: " + fmt, *args)


class HTTPPublisher:
    def __init__(self, package_name: str, package_version: str, input_dir_path: str, artifact_paths: Sequence[str],
                 http_dir: Optional[str] = None, http_host: Optional[str] = None, http_port: Optional[int] = None,
                 package_manager: Optional[PackageManager] = None):
        if not os.path.isdir(input_dir_path):
            raise ValueError(f"Provided package path is not a directory: {input_dir_path}")
        for p in artifact_paths:
            if not os.path.isfile(p):
                raise ValueError(f"Provided artifact path is not a file: {p} (full list: {list(artifact_paths)})")
        self._pkg_name = package_name
        self._pkg_version = package_version
        self._input_dir = input_dir_path
        self._artifacts = list(artifact_paths)
        self._http_dir = http_dir or os.environ.get("HTTP_DIR") or f"/tmp/dcos-http-{package_name}/"
        self._http_host = http_host or os.environ.get("HTTP_HOST", "127.0.0.1")
        self._http_port = int(http_port if http_port is not None else os.environ.get("HTTP_PORT", "0"))
        self._package_manager = package_manager or PackageManager()
        self._server: Optional[http.server.ThreadingHTTPServer] = None
        self._thread: Optional[threading.Thread] = None
        self.universe_url: Optional[str] = None

    def build(self, http_url_root: str) -> str:
        """Copy the artifacts and write the stub universe into the HTTP dir; returns its URL."""
        if os.path.isdir(self._http_dir):
            shutil.rmtree(self._http_dir)
        os.makedirs(self._http_dir)
        copied: List[str] = []
        for p in self._artifacts:
            dest = os.path.join(self._http_dir, os.path.basename(p))
            shutil.copyfile(p, dest)
            copied.append(dest)
        builder = UniversePackageBuilder(Package(self._pkg_name, Version(0, self._pkg_version)),
                                         self._package_manager, self._input_dir, http_url_root, copied)
        path = builder.build_package(self._http_dir)
        url = f"{http_url_root}/{os.path.basename(path)}"
        self._write_properties(url)
        return url

    def _write_properties(self, url: str) -> None:
        ws = os.environ.get("WORKSPACE")
        if ws:
            with open(os.path.join(ws, f"{self._pkg_version}.properties"), "w", encoding="utf-8") as f:
                f.write(f"STUB_UNIVERSE_URL={url}\n")

    def start(self) -> str:
        """Bind, build against the bound port, serve on a daemon thread; returns the universe URL."""
        handler = partial(_Handler, directory=self._http_dir)
        os.makedirs(self._http_dir, exist_ok=True)
        self._server = http.server.ThreadingHTTPServer((self._http_host, self._http_port), handler)
        host, port = self._server.server_address[:2]
        self.universe_url = self.build(f"http://{host}:{port}")
        self._thread = threading.Thread(target=self._server.serve_forever, name="publish-http", daemon=True)
        self._thread.start()
        LOGGER.info("Serving %s at %s", self._http_dir, self.universe_url)
        return self.universe_url

    def serve_forever(self) -> None:
        if self._thread is not None:
            self._thread.join()

    def stop(self) -> None:
        if self._server is not None:
            self._server.shutdown()
            self._server.server_close()
            self._server = None

    def describe(self) -> str:
        return json.dumps({"package": self._pkg_name, "version": self._pkg_version, "url": self.universe_url})
