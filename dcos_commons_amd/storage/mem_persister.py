"""In-memory tree persister mirroring the ZooKeeper semantics.

Reference: sdk/.../storage/MemPersister.java:26-380 (TreeMap nodes, optional RW lock with
deadlock detection, ``getDebugString``).
"""
from __future__ import annotations

from collections import deque
from typing import Collection, Dict, List, Mapping, Optional

from dcos_commons_amd.utils.locks import new_rw_lock

from .persister import Persister, PersisterException, Reason
from .persister_utils import get_path_elements, join_paths

_NO_DATA = object()


class _Node:
    __slots__ = ("children", "data")

    def __init__(self):
        self.children: Dict[str, "_Node"] = {}
        self.data = _NO_DATA


class _NullLock:
    def __enter__(self):
        return self

    def __exit__(self, *exc):
        return False


_NULL = _NullLock()


_SPLIT: Dict[str, List[str]] = {}   # path -> its elements (never mutated by callers)
_SPLIT_MAX = 65536


class MemPersister(Persister):
    def __init__(self, locking: bool = True, data: Optional[Mapping[str, bytes]] = None):
        self._root = _Node()
        for path, value in (data or {}).items():
            self._node(path, create=True).data = value
        if locking:
            rw = new_rw_lock("MemPersister")
            self._r, self._w = rw.read_lock, rw.write_lock
        else:
            self._r = self._w = _NULL

    # -- internals -----------------------------------------------------------------------
    def _node(self, path, create: bool) -> Optional[_Node]:
        if isinstance(path, list):
            elems = path
        else:
            # the state store asks for the same few hundred paths over and over (every task's
            # TaskInfo/TaskStatus on each plan query): split each path string once
            elems = _SPLIT.get(path)
            if elems is None:
                elems = get_path_elements(path)
                if len(_SPLIT) >= _SPLIT_MAX:
                    _SPLIT.clear()
                _SPLIT[path] = elems
        cur = self._root
        for e in elems:
            nxt = cur.children.get(e)
            if nxt is None:
                if not create:
                    return None
                nxt = _Node()
                cur.children[e] = nxt
            cur = nxt
        return cur

    def _delete(self, path: str) -> bool:
        elems = get_path_elements(path)
        if not elems:
            self._root.children.clear()
            self._root.data = _NO_DATA
            return True
        parent = self._node(elems[:-1], create=False)
        if parent is None:
            return False
        return parent.children.pop(elems[-1], None) is not None

    # -- Persister -----------------------------------------------------------------------
    def get(self, path: str) -> Optional[bytes]:
        with self._r:
            node = self._node(path, create=False)
            if node is None:
                raise PersisterException(Reason.NOT_FOUND, path)
            return None if node.data is _NO_DATA else node.data

    def get_children(self, path: str) -> List[str]:
        with self._r:
            node = self._node(path, create=False)
            if node is None:
                raise PersisterException(Reason.NOT_FOUND, path)
            return sorted(node.children)

    def set(self, path: str, data: bytes) -> None:
        with self._w:
            self._node(path, create=True).data = bytes(data)

    def set_many(self, path_bytes: Mapping[str, bytes]) -> None:
        if not path_bytes:
            return
        with self._w:
            for path, data in path_bytes.items():
                self._node(path, create=True).data = bytes(data)

    def get_many(self, paths: Collection[str]) -> Dict[str, Optional[bytes]]:
        with self._r:
            out = {}
            for path in sorted(paths):
                node = self._node(path, create=False)
                out[path] = None if node is None or node.data is _NO_DATA else node.data
            return out

    def recursive_copy(self, src: str, dst: str) -> None:
        with self._w:
            src_node = self._node(src, create=False)
            if src_node is None:
                raise PersisterException(Reason.NOT_FOUND, "Source path not found: " + src)
            if self._node(dst, create=False) is not None:
                raise PersisterException(Reason.LOGIC_ERROR, "Destination path already exists: " + dst)
            queue = deque([(dst, src_node)])
            while queue:
                path, node = queue.popleft()
                self._node(path, create=True).data = node.data
                for name, child in node.children.items():
                    queue.append((join_paths(path, name), child))

    def recursive_delete_many(self, paths: Collection[str]) -> None:
        with self._w:
            for p in paths:
                self._delete(p)

    def recursive_delete(self, path: str) -> None:
        with self._w:
            if not self._delete(path):
                raise PersisterException(Reason.NOT_FOUND, path)

    def close(self) -> None:
        with self._w:
            self._root.children.clear()
            self._root.data = _NO_DATA

    def debug_string(self) -> str:
        lines: List[str] = []

        def info(d) -> str:
            if d is _NO_DATA:
                return "NULL"
            return "1 byte" if len(d) == 1 else f"{len(d)} bytes"

        def walk(name: str, node: _Node, level: int) -> None:
            lines.append("  " * level + f"{name}: {info(node.data)}")
            for n, c in node.children.items():
                walk(n, c, level + 1)

        with self._r:
            walk("ROOT", self._root, 1)
        return "\n".join(lines)
