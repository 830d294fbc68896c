"""Durable persister backed by a local directory tree.

Each persister node is a directory; node data lives in a ``.data`` file inside it, so a node can
hold data and children at once (ZooKeeper semantics, as in the reference's CuratorPersister,
sdk/.../curator/CuratorPersister.java:43). Node names are percent-encoded on disk.

Atomicity: ``set_many`` / ``recursive_delete_many`` are made crash-atomic with a write-ahead
journal (``.journal``): the whole batch is written and fsync'd first, then applied, then the
journal is removed. A journal found at open time is replayed, so a crash mid-batch never leaves
half a batch visible -- the equivalent of the reference's single ZK ``multi`` transaction
(CuratorPersister.setMany, :229).
"""
from __future__ import annotations

import base64
import json
import os
import shutil
import tempfile
import threading
from typing import Collection, Dict, List, Mapping, Optional
from urllib.parse import quote, unquote

from .persister import Persister, PersisterException, Reason
from .persister_utils import get_path_elements

_DATA = ".data"
_JOURNAL = ".journal"


def _enc(name: str) -> str:
    q = quote(name, safe="-_:~@+=,")
    if q.startswith("."):
        q = "%2E" + q[1:]
    return q


class FilePersister(Persister):
    def __init__(self, root_dir: str, fsync: bool = True):
        self._root = os.path.abspath(root_dir)
        self._fsync = fsync
        self._lock = threading.RLock()
        os.makedirs(self._root, exist_ok=True)
        self._replay_journal()

    # -- paths ---------------------------------------------------------------------------
    def _dir(self, path: str) -> str:
        elems = get_path_elements(path)
        return os.path.join(self._root, *[_enc(e) for e in elems]) if elems else self._root

    def _write_file(self, fname: str, data: bytes) -> None:
        d = os.path.dirname(fname)
        os.makedirs(d, exist_ok=True)
        fd, tmp = tempfile.mkstemp(dir=d, prefix=".tmp")
        try:
            with os.fdopen(fd, "wb") as f:
                f.write(data)
                if self._fsync:
                    f.flush()
                    os.fsync(f.fileno())
            os.replace(tmp, fname)
        except BaseException:
            try:
                os.unlink(tmp)
            except OSError:
                pass
            raise

    # -- journal -------------------------------------------------------------------------
    def _journal_path(self) -> str:
        return os.path.join(self._root, _JOURNAL)

    def _write_journal(self, ops: List[dict]) -> None:
        self._write_file(self._journal_path(), json.dumps(ops).encode())

    def _apply(self, ops: List[dict]) -> None:
        for op in ops:
            if op["op"] == "set":
                self._write_file(os.path.join(self._dir(op["path"]), _DATA), base64.b64decode(op["data"]))
            elif op["op"] == "del":
                self._rm(op["path"])

    def _replay_journal(self) -> None:
        jp = self._journal_path()
        if os.path.exists(jp):
            try:
                with open(jp, "rb") as f:
                    ops = json.loads(f.read().decode())
            except ValueError:
                ops = []  # torn journal write: the batch never started applying
            self._apply(ops)
            os.unlink(jp)

    def _batch(self, ops: List[dict]) -> None:
        if len(ops) == 1:
            self._apply(ops)
            return
        self._write_journal(ops)
        self._apply(ops)
        os.unlink(self._journal_path())

    def _rm(self, path: str) -> bool:
        elems = get_path_elements(path)
        if not elems:
            existed = False
            for n in os.listdir(self._root):
                if n == _JOURNAL:
                    continue
                p = os.path.join(self._root, n)
                existed = True
                if os.path.isdir(p):
                    shutil.rmtree(p)
                else:
                    os.unlink(p)
            return True
        d = self._dir(path)
        if not os.path.isdir(d):
            return False
        shutil.rmtree(d)
        return True

    # -- Persister -----------------------------------------------------------------------
    def get(self, path: str) -> Optional[bytes]:
        with self._lock:
            d = self._dir(path)
            if not os.path.isdir(d):
                raise PersisterException(Reason.NOT_FOUND, path)
            f = os.path.join(d, _DATA)
            if not os.path.exists(f):
                return None
            with open(f, "rb") as fh:
                return fh.read()

    def get_children(self, path: str) -> List[str]:
        with self._lock:
            d = self._dir(path)
            if not os.path.isdir(d):
                raise PersisterException(Reason.NOT_FOUND, path)
            return sorted(
                unquote(n) for n in os.listdir(d)
                if not n.startswith(".") and os.path.isdir(os.path.join(d, n))
            )

    def set(self, path: str, data: bytes) -> None:
        with self._lock:
            self._write_file(os.path.join(self._dir(path), _DATA), bytes(data))

    def set_many(self, path_bytes: Mapping[str, bytes]) -> None:
        if not path_bytes:
            return
        with self._lock:
            self._batch([
                {"op": "set", "path": p, "data": base64.b64encode(bytes(v)).decode()}
                for p, v in path_bytes.items()
            ])

    def get_many(self, paths: Collection[str]) -> Dict[str, Optional[bytes]]:
        out = {}
        with self._lock:
            for p in sorted(paths):
                try:
                    out[p] = self.get(p)
                except PersisterException:
                    out[p] = None
        return out

    def recursive_copy(self, src: str, dst: str) -> None:
        with self._lock:
            s, d = self._dir(src), self._dir(dst)
            if not os.path.isdir(s):
                raise PersisterException(Reason.NOT_FOUND, "Source path not found: " + src)
            if os.path.isdir(d):
                raise PersisterException(Reason.LOGIC_ERROR, "Destination path already exists: " + dst)
            shutil.copytree(s, d)

    def recursive_delete_many(self, paths: Collection[str]) -> None:
        with self._lock:
            self._batch([{"op": "del", "path": p} for p in paths])

    def recursive_delete(self, path: str) -> None:
        with self._lock:
            if not self._rm(path):
                raise PersisterException(Reason.NOT_FOUND, path)

    def close(self) -> None:
        pass
