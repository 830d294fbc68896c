"""ZooKeeper-backed ``Persister`` plus the single-scheduler lock.

Reference parity:
* ``ZooKeeperPersister`` <- sdk/.../curator/CuratorPersister.java: every path lives under
  ``/dcos-service-<name with / -> __>`` (CuratorUtils.java:53); ``set_many`` and
  ``recursive_delete_many`` are single ZK transactions prefixed by a ``check`` of the root and
  creating missing parents / deleting children first, retried ``ATOMIC_WRITE_ATTEMPTS = 3`` times
  (:51, :229, :288); deleting the root wipes its children except ``lock`` and then nulls the root
  data (:300-345); the root reads as empty when missing (:146, :166); ``recursive_copy`` refuses
  the root and the lock node (:214); digest credentials give CREATOR_ALL + READ ACLs (:486-505).
* ``ZkLocker`` <- curator/CuratorLocker.java: an exclusive lease under ``<root>/lock`` acquired in
  ``LOCK_ATTEMPTS = 3`` tries of ``wait_s`` each (:20, :59-110), released at shutdown; on failure
  the process exits with ``LOCK_UNAVAILABLE``. The lease is an ephemeral-sequential node under
  ``<root>/lock/leases``: the lowest sequence number holds the lock, so a crashed scheduler's lease
  disappears with its session.
* ``init_service_name`` <- CuratorUtils.initServiceName: the ``servicename`` node detects
  collisions between e.g. ``/team/db`` and ``team.db``.
"""
from __future__ import annotations

import atexit
import logging
import threading
from typing import Collection, Dict, List, Mapping, Optional, Set

from . import zookeeper as Z
from .persister import Persister, PersisterException, Reason
from .persister_utils import get_parent_paths, join_paths, with_escaped_slashes

LOGGER = logging.getLogger(__name__)

ATOMIC_WRITE_ATTEMPTS = 3
LOCK_PATH_NAME = "lock"
LOCK_ATTEMPTS = 3
SERVICE_NAME_NODE = "servicename"
SERVICE_ROOT_PATH_PREFIX = "/dcos-service-"


def get_service_root_path(framework_name: str) -> str:
    return SERVICE_ROOT_PATH_PREFIX + with_escaped_slashes(framework_name)


def _acls_for(username: str, password: str) -> Optional[List[Z.ACL]]:
    if username and password:
        return list(Z.CREATOR_ALL_ACL) + list(Z.READ_ACL_UNSAFE)
    if username or password:
        raise ValueError("username and password must both be provided, or both must be empty.")
    return None


def new_client(connect: str, username: str = "", password: str = "", session_timeout_ms: int = 10000) -> Z.ZkClient:
    acls = _acls_for(username, password)
    auth = [("digest", f"{username}:{password}".encode("utf-8"))] if acls else None
    return Z.ZkClient(connect, session_timeout_ms=session_timeout_ms, auth=auth, default_acl=acls).start()


class ZooKeeperPersister(Persister):
    def __init__(self, connect: str, service_name_or_root: str, username: str = "", password: str = "",
                 client: Optional[Z.ZkClient] = None, session_timeout_ms: int = 10000):
        root = service_name_or_root
        self.root = root if root.startswith(SERVICE_ROOT_PATH_PREFIX) else get_service_root_path(root)
        self.client = client or new_client(connect, username, password, session_timeout_ms)

    # -- helpers ------------------------------------------------------------------------
    @property
    def remote(self) -> bool:
        return True

    def _p(self, path: str) -> str:
        p = join_paths(self.root, path or "")
        while len(p) > 1 and p.endswith("/"):
            p = p[:-1]
        return p

    def _storage_error(self, msg: str, e: BaseException) -> PersisterException:
        return PersisterException(Reason.STORAGE_ERROR, f"{msg}: {e}", e)

    # -- reads --------------------------------------------------------------------------
    def get(self, path: str) -> Optional[bytes]:
        p = self._p(path)
        try:
            return self.client.get(p)[0]
        except Z.NoNodeError as e:
            if p == self.root:
                return None
            raise PersisterException(Reason.NOT_FOUND, f"Path to get does not exist: {p}", e)
        except Z.ZkError as e:
            raise self._storage_error(f"Unable to retrieve data from {p}", e)

    def get_children(self, path: str) -> Collection[str]:
        p = self._p(path)
        try:
            return sorted(self.client.get_children(p))
        except Z.NoNodeError as e:
            if p == self.root:
                return []
            raise PersisterException(Reason.NOT_FOUND, f"Path to list does not exist: {p}", e)
        except Z.ZkError as e:
            raise self._storage_error(f"Unable to get children of {p}", e)

    def get_many(self, paths: Collection[str]) -> Dict[str, Optional[bytes]]:
        out: Dict[str, Optional[bytes]] = {}
        for path in paths:
            try:
                out[path] = self.client.get(self._p(path))[0]
            except Z.NoNodeError:
                out[path] = None
            except Z.ZkError as e:
                raise self._storage_error(f"Unable to retrieve data from {self._p(path)}", e)
        return out

    # -- writes -------------------------------------------------------------------------
    def set(self, path: str, data: Optional[bytes]) -> None:
        """setData on the node, creating it (and its parents) when it does not exist yet
        (CuratorPersister.set). The common case, an existing node, is one round trip: the write
        is tried first and the creation path only runs on NoNode."""
        p = self._p(path)
        try:
            try:
                self.client.set(p, data)
                return
            except Z.NoNodeError:
                pass
            for parent in get_parent_paths(p):
                if self.client.exists(parent) is None:
                    try:
                        self.client.create(parent)
                    except Z.NodeExistsError:
                        pass
            try:
                self.client.create(p, data)
            except Z.NodeExistsError:
                self.client.set(p, data)  # created concurrently since the failed setData
        except Z.ZkError as e:
            raise self._storage_error(f"Unable to set {len(data or b'')} bytes in {p}", e)

    def _run_transaction(self, build) -> None:
        for attempt in range(1, ATOMIC_WRITE_ATTEMPTS + 1):
            try:
                ops = build()
                self.client.multi(ops)
                return
            except Z.ZkError as e:
                if attempt == ATOMIC_WRITE_ATTEMPTS:
                    raise PersisterException(Reason.STORAGE_ERROR, str(e), e)
                LOGGER.error("Failed to complete transaction attempt %d/%d: %s", attempt, ATOMIC_WRITE_ATTEMPTS, e)

    def _ensure_root(self) -> None:
        if self.client.exists(self.root) is None:
            self.client.ensure_path(self.root)

    def set_many(self, path_bytes: Mapping[str, Optional[bytes]]) -> None:
        """One transaction (CuratorPersister.setMany): setData on existing nodes, creates for
        missing ones and their parents. It is first tried as setData only, which is one round
        trip when every node exists (status updates, relaunches); a transaction that fails on a
        missing node is rebuilt with existence checks, as the reference always does."""
        if not path_bytes:
            return
        prefixed = {self._p(k): v for k, v in sorted(path_bytes.items())}
        try:
            self.client.multi([Z.Check(self.root)] + [Z.SetData(p, d) for p, d in prefixed.items()])
            return
        except Z.TransactionError as e:
            if not isinstance(e.failed, Z.NoNodeError):
                LOGGER.info("Optimistic setData transaction failed (%s): rebuilding it", e)
        except Z.ZkError as e:
            LOGGER.info("Optimistic setData transaction failed (%s): rebuilding it", e)
        try:
            self._ensure_root()
        except Z.ZkError as e:
            raise self._storage_error("Unable to create service root", e)

        def build():
            existing: Set[str] = set()
            ops: List = [Z.Check(self.root)]
            for path, data in prefixed.items():
                if path not in existing and self.client.exists(path) is None:
                    for parent in get_parent_paths(path):
                        if parent not in existing and self.client.exists(parent) is None:
                            ops.append(Z.Create(parent, None, list(self.client.default_acl)))
                        existing.add(parent)
                    ops.append(Z.Create(path, data, list(self.client.default_acl)))
                    existing.add(path)
                else:
                    ops.append(Z.SetData(path, data))
            return ops
        self._run_transaction(build)

    def _delete_children_ops(self, path: str, ops: List, pending: Set[str]) -> None:
        if path in pending:
            return
        for child in self.client.get_children(path):
            cp = join_paths(path, child)
            self._delete_children_ops(cp, ops, pending)
            if cp not in pending:
                ops.append(Z.Delete(cp))
                pending.add(cp)

    def recursive_delete(self, path: str) -> None:
        p = self._p(path)
        if p == self.root:
            # The root node itself cannot be deleted (DC/OS ZK ACLs): wipe everything but the lock.
            try:
                if self.client.exists(self.root) is not None:
                    ops: List = [Z.Check(self.root)]
                    pending: Set[str] = set()
                    for child in self.client.get_children(self.root):
                        if child == LOCK_PATH_NAME:
                            continue
                        cp = join_paths(self.root, child)
                        self._delete_children_ops(cp, ops, pending)
                        ops.append(Z.Delete(cp))
                    self.client.multi(ops)
            except Z.ZkError as e:
                raise self._storage_error(f"Unable to delete children of root {p}", e)
            self.set(path, None)
            return
        try:
            self.client.delete(p, recursive=True)
        except Z.NoNodeError as e:
            raise PersisterException(Reason.NOT_FOUND, f"Path to delete does not exist: {p}", e)
        except Z.ZkError as e:
            raise self._storage_error(f"Unable to delete {p}", e)

    def recursive_delete_many(self, paths: Collection[str]) -> None:
        if not paths:
            return
        prefixed = [self._p(x) for x in paths]

        def build():
            ops: List = [Z.Check(self.root)]
            pending: Set[str] = set()
            for path in prefixed:
                if path not in pending and self.client.exists(path) is not None:
                    self._delete_children_ops(path, ops, pending)
                    ops.append(Z.Delete(path))
                    pending.add(path)
            return ops
        self._run_transaction(build)

    def recursive_copy(self, src: str, dst: str) -> None:
        for x in (self.root, LOCK_PATH_NAME):
            if x in (src, dst):
                raise ValueError(f"Cannot copy from {src} to {dst}")
        try:
            if self.client.exists(self._p(src)) is None:
                raise PersisterException(Reason.NOT_FOUND, f"Source node does not exist: {src}")
            if self.client.exists(self._p(dst)) is not None:
                raise PersisterException(Reason.LOGIC_ERROR, f"Destination exists: {dst}")
        except Z.ZkError as e:
            raise self._storage_error(f"Failed to copy {src} to {dst}", e)
        to_walk = [src]
        to_add: Dict[str, Optional[bytes]] = {}
        while to_walk:
            cur = to_walk.pop(0)
            to_add[dst + cur[len(src):]] = self.get(cur)
            to_walk.extend(join_paths(cur, c) for c in self.get_children(cur))
        self.set_many(to_add)

    def close(self) -> None:
        self.client.close()


def init_service_name(persister: Persister, service_name: str) -> None:
    try:
        data = persister.get(SERVICE_NAME_NODE)
        if not data:
            raise ValueError(f"Invalid data when fetching service name in '{SERVICE_NAME_NODE}'")
        current = data.decode("utf-8")
        if current != service_name:
            raise ValueError(f"Collision between similar service names: Expected name '{service_name}', "
                             f"but stored name is '{current}'.")
    except PersisterException as e:
        if e.reason != Reason.NOT_FOUND:
            raise RuntimeError("Failed to fetch prior service name for validation") from e
        persister.set(SERVICE_NAME_NODE, service_name.encode("utf-8"))


class ZkLocker:
    """Exclusive per-service lease; one instance per process (``lock()``/``unlock()``)."""
    _instance: Optional["ZkLocker"] = None
    # re-entrant: ``unlock`` runs as a shutdown hook, possibly from a SIGTERM handler on a thread
    # that is already inside ``lock``
    _instance_lock = threading.RLock()
    _hooks_registered = False
    enabled = True

    def __init__(self, service_name: str, connect: str, username: str = "", password: str = "",
                 wait_s: float = 10.0, session_timeout_ms: int = 10000):
        self.service_name = service_name
        self.connect = connect
        self.username, self.password = username, password
        self.wait_s = wait_s
        self.session_timeout_ms = session_timeout_ms
        self.lock_path = join_paths(get_service_root_path(service_name), LOCK_PATH_NAME)
        self.client: Optional[Z.ZkClient] = None
        self.lease: Optional[str] = None

    @classmethod
    def lock(cls, service_name: str, connect: str, **kw) -> Optional["ZkLocker"]:
        from dcos_commons_amd.framework.process_exit import ProcessExit, add_shutdown_hook

        with cls._instance_lock:
            if not cls.enabled:
                return None
            if cls._instance is not None:
                raise RuntimeError("Already locked")
            inst = cls(service_name, connect, **kw)
            acquired = inst.lock_internal()
            if acquired:
                cls._instance = inst
                if not cls._hooks_registered:  # once per process, however often lock() runs
                    cls._hooks_registered = True
                    atexit.register(cls.unlock)
                    add_shutdown_hook(cls.unlock)
        if not acquired:
            # outside _instance_lock: the exit runs the shutdown hooks, and ``unlock`` needs that lock
            ProcessExit.exit(ProcessExit.LOCK_UNAVAILABLE)
            return None
        return inst

    @classmethod
    def unlock(cls) -> None:
        with cls._instance_lock:
            if cls._instance is not None:
                cls._instance.unlock_internal()
                cls._instance = None

    def _try_acquire(self, wait_s: float) -> bool:
        leases = self.lock_path + "/leases"
        if self.lease is None:
            self.client.ensure_path(leases)
            self.lease = self.client.create(leases + "/lease-", None, ephemeral=True, sequence=True)
        mine = self.lease.rsplit("/", 1)[1]
        deadline_event = threading.Event()
        timer = threading.Timer(wait_s, deadline_event.set)
        timer.daemon = True
        timer.start()
        try:
            while not deadline_event.is_set():
                children = sorted(self.client.get_children(leases))
                if mine not in children:  # our session expired and the lease went with it
                    self.lease = None
                    return False
                idx = children.index(mine)
                if idx == 0:
                    return True
                changed = threading.Event()
                if self.client.exists(leases + "/" + children[idx - 1], watch=lambda ev: changed.set()) is None:
                    continue
                while not changed.is_set() and not deadline_event.is_set():
                    changed.wait(0.05)
            return False
        finally:
            timer.cancel()

    def lock_internal(self) -> bool:
        if self.client is not None:
            raise RuntimeError("Already locked")
        self.client = new_client(self.connect, self.username, self.password, self.session_timeout_ms)
        LOGGER.info("Acquiring ZK lock on %s...", self.lock_path)
        msg = (f"Failed to acquire ZK lock on {self.lock_path}. Duplicate service named '{self.service_name}', "
               f"or recently restarted instance of '{self.service_name}'?")
        try:
            for attempt in range(1, LOCK_ATTEMPTS + 1):
                if self._try_acquire(self.wait_s):
                    LOGGER.info("%d/%d Lock acquired.", attempt, LOCK_ATTEMPTS)
                    return True
                if attempt < LOCK_ATTEMPTS:
                    LOGGER.error("%d/%d %s Retrying lock...", attempt, LOCK_ATTEMPTS, msg)
            LOGGER.error("%s Restarting scheduler process to try again.", msg)
        except Z.ZkError as e:
            LOGGER.error("Error acquiring ZK lock on path: %s: %s", self.lock_path, e)
        self._release()
        return False

    def _release(self) -> None:
        if self.client is None:
            return
        if self.lease is not None:
            try:
                self.client.delete(self.lease)
            except Z.ZkError as e:
                LOGGER.error("Error releasing ZK lock: %s", e)
        self.client.close()
        self.client = None
        self.lease = None

    def unlock_internal(self) -> None:
        if self.client is None:
            raise RuntimeError("Already unlocked")
        self._release()
