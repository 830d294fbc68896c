"""Object-store uploaders for published packages (reference: tools/universe/s3_uploader.py,
tools/universe/azure_uploader.py).

There is no network here, so the stores are emulated by ``LocalObjectStore``: a bucket
(``s3://<bucket>/<dir>``) or container (``https://<account>.blob.core.windows.net/<container>/<dir>``)
is a directory under ``SDK_OBJECT_STORE_ROOT`` and its objects are served read-only over HTTP
from 127.0.0.1, the way a public-read S3 bucket or Azure container serves them. Uploads keep the
reference's contract: ``upload(path, content_type=None)`` puts the file at ``<dir>/<basename>`` and
records its content type; ``DRY_RUN`` logs instead of writing.
"""
from __future__ import annotations

import http.server
import json
import logging
import os
import shutil
import threading
import urllib.parse
from functools import partial
from typing import Dict, Optional, Tuple

LOGGER = logging.getLogger(__name__)
_META = ".content-types.json"


class LocalObjectStore:
    """Directory-backed buckets served over HTTP; one process-wide instance per root."""

    _instances: Dict[str, "LocalObjectStore"] = {}
    _lock = threading.Lock()

    def __init__(self, root: str):
        self.root = os.path.abspath(root)
        os.makedirs(self.root, exist_ok=True)
        self._server: Optional[http.server.ThreadingHTTPServer] = None

    @classmethod
    def get(cls, root: Optional[str] = None) -> "LocalObjectStore":
        root = os.path.abspath(root or os.environ.get("SDK_OBJECT_STORE_ROOT") or "/tmp/sdk-object-store")
        with cls._lock:
            if root not in cls._instances:
                cls._instances[root] = LocalObjectStore(root)
            return cls._instances[root]

    def put(self, bucket: str, key: str, src: str, content_type: Optional[str]) -> str:
        dest = os.path.join(self.root, bucket, key)
        os.makedirs(os.path.dirname(dest), exist_ok=True)
        shutil.copyfile(src, dest)
        meta_path = os.path.join(os.path.dirname(dest), _META)
        meta = json.load(open(meta_path)) if os.path.exists(meta_path) else {}
        meta[os.path.basename(dest)] = content_type or "application/octet-stream"
        with open(meta_path, "w", encoding="utf-8") as f:
            json.dump(meta, f)
        return dest

    def http_root(self) -> str:
        with self._lock:
            if self._server is None:
                store = self

                class Handler(http.server.SimpleHTTPRequestHandler):
                    def guess_type(self, path):
                        meta_path = os.path.join(os.path.dirname(path), _META)
                        try:
                            return json.load(open(meta_path)).get(os.path.basename(path), "application/octet-stream")
                        except (OSError, ValueError):
                            return "application/octet-stream"

                    def log_message(self, fmt, *args):
                        LOGGER.debug("object store: " + fmt, *args)

                self._server = http.server.ThreadingHTTPServer(("127.0.0.1", 0),
                                                               partial(Handler, directory=store.root))
                threading.Thread(target=self._server.serve_forever, name="object-store", daemon=True).start()
            host, port = self._server.server_address[:2]
            return f"http://{host}:{port}"

    def stop(self) -> None:
        with self._lock:
            if self._server is not None:
                self._server.shutdown()
                self._server.server_close()
                self._server = None


def parse_s3_url(url: str) -> Tuple[str, str]:
    p = urllib.parse.urlparse(url)
    if p.scheme != "s3" or not p.netloc:
        raise ValueError(f"Expected s3://<bucket>/<dir>, got {url}")
    return p.netloc, p.path.strip("/")


def parse_azure_url(url: str) -> Tuple[str, str]:
    """``https://<account>.blob.core.windows.net/<container>/<dir>`` -> ("<account>/<container>", dir)."""
    p = urllib.parse.urlparse(url)
    parts = p.path.strip("/").split("/", 1)
    if not p.netloc.endswith(".blob.core.windows.net") or not parts[0]:
        raise ValueError(f"Expected https://<account>.blob.core.windows.net/<container>/<dir>, got {url}")
    account = p.netloc.split(".", 1)[0]
    return f"{account}/{parts[0]}", parts[1] if len(parts) > 1 else ""


class _Uploader:
    def __init__(self, bucket: str, directory: str, dry_run: bool = False, store: Optional[LocalObjectStore] = None):
        self.bucket, self.directory, self.dry_run = bucket, directory.strip("/"), bool(dry_run)
        self.store = store or LocalObjectStore.get()

    def upload(self, filepath: str, content_type: Optional[str] = None) -> str:
        key = "/".join(p for p in (self.directory, os.path.basename(filepath)) if p)
        if self.dry_run:
            LOGGER.info("[DRY RUN] upload %s -> %s/%s (%s)", filepath, self.bucket, key, content_type)
            return key
        LOGGER.info("Uploading %s -> %s/%s", filepath, self.bucket, key)
        self.store.put(self.bucket, key, filepath, content_type)
        return key

    def http_directory_url(self) -> str:
        return "/".join(p for p in (self.store.http_root(), self.bucket, self.directory) if p)


class S3Uploader(_Uploader):
    def __init__(self, s3_directory: str, dry_run: bool = False, store: Optional[LocalObjectStore] = None):
        bucket, directory = parse_s3_url(s3_directory)
        super().__init__(bucket, directory, dry_run, store)
        self._s3_directory = s3_directory

    def get_s3_directory(self) -> str:
        return self._s3_directory


class AzureUploader(_Uploader):
    def __init__(self, azure_directory: str, dry_run: bool = False, store: Optional[LocalObjectStore] = None):
        bucket, directory = parse_azure_url(azure_directory)
        super().__init__(bucket, directory, dry_run, store)
