"""Persister selection for a service.

Reference: sdk/.../curator/CuratorPersister.java:64-93 (``/dcos-service-<name>`` ZooKeeper root,
wrapped in PersisterCache unless DISABLE_STATE_CACHE) and SchedulerBuilder.java:189-193.

Backends here (``SDK_PERSISTER``):
* ``file`` (default) -- crash-safe WAL-journaled tree under ``SDK_STATE_DIR`` (default
  ``./state``) at ``dcos-service-<name>``; the same node layout the reference keeps in ZK;
* ``mem`` -- in-memory, for tests and benchmarks;
* ``zk`` -- ZooKeeper at the spec's ``scheduler.zookeeper`` / ``FRAMEWORK_ZOOKEEPER``
  (``storage.zk_persister``), optional digest credentials ``SDK_ZK_USERNAME``/``SDK_ZK_PASSWORD``.
  ``SDK_ZOOKEEPER`` replaces the connect string where the spec's default (``master.mesos:2181``)
  does not resolve, e.g. the local cluster of ``dcos_commons_amd.testing.cluster``.
  ``SDK_LOCK_WAIT_S`` (default 10) is how long each of the 3 attempts waits for the service lock;
  ``SDK_ZK_SESSION_TIMEOUT_MS`` (default 10000) bounds how long a crashed scheduler's lock outlives it.

Like ``CuratorPersister.Builder.build`` (:480-520) the durable backends first take the
single-scheduler lock (``ZkLocker`` / ``FileLocker``; ``SDK_DISABLE_LOCK=true`` skips it, for tests)
and then check the ``servicename`` node for folder-name collisions.
"""
from __future__ import annotations

import fcntl
import logging
import os
import time
from typing import Optional

from .mem_persister import MemPersister
from .persister import Persister
from .persister_cache import PersisterCache


def service_root_name(service_name: str) -> str:
    # Curator root: "/dcos-service-" + name with '/' replaced by "__" (CuratorUtils.getServiceRootPath)
    return "dcos-service-" + service_name.lstrip("/").replace("/", "__")


LOGGER = logging.getLogger(__name__)


class FileLocker:
    """``flock`` on ``<state root>.lock``: one live scheduler per service for the file backend
    (same contract as CuratorLocker: 3 attempts, then ``ProcessExit.LOCK_UNAVAILABLE``)."""
    _held = {}

    def __init__(self, root: str, wait_s: float = 10.0, attempts: int = 3):
        self.path = root.rstrip("/") + ".lock"
        self.wait_s = wait_s
        self.attempts = attempts
        self.fd: Optional[int] = None

    def lock(self) -> bool:
        os.makedirs(os.path.dirname(os.path.abspath(self.path)), exist_ok=True)
        fd = os.open(self.path, os.O_RDWR | os.O_CREAT, 0o644)
        for attempt in range(1, self.attempts + 1):
            deadline = time.monotonic() + self.wait_s
            while True:
                try:
                    fcntl.flock(fd, fcntl.LOCK_EX | fcntl.LOCK_NB)
                    os.ftruncate(fd, 0)
                    os.write(fd, str(os.getpid()).encode())
                    self.fd = fd
                    FileLocker._held[self.path] = self
                    return True
                except BlockingIOError:
                    if time.monotonic() >= deadline:
                        break
                    time.sleep(0.05)
            LOGGER.error("%d/%d Failed to acquire lock %s: another scheduler for this service is running?",
                         attempt, self.attempts, self.path)
        os.close(fd)
        return False

    def unlock(self) -> None:
        if self.fd is not None:
            fcntl.flock(self.fd, fcntl.LOCK_UN)
            os.close(self.fd)
            self.fd = None
            FileLocker._held.pop(self.path, None)


def _lock_or_exit(locker) -> None:
    if not locker.lock():
        from dcos_commons_amd.framework.process_exit import ProcessExit

        ProcessExit.exit(ProcessExit.LOCK_UNAVAILABLE)


def persister_for_service(service_spec, scheduler_config) -> Persister:
    env = scheduler_config.env
    kind = env.get_optional("SDK_PERSISTER", "file")
    lock_enabled = not env.get_optional_boolean("SDK_DISABLE_LOCK", False)
    if kind == "mem":
        base: Persister = MemPersister()
    elif kind == "file":
        from .file_persister import FilePersister

        root = os.path.join(env.get_optional("SDK_STATE_DIR", "state"), service_root_name(service_spec.name))
        if lock_enabled and root.rstrip("/") + ".lock" not in FileLocker._held:
            _lock_or_exit(FileLocker(root))
        base = FilePersister(root)
    elif kind == "zk":
        from .zk_persister import ZkLocker, ZooKeeperPersister, init_service_name

        connect = (env.get_optional("SDK_ZOOKEEPER", "") or service_spec.zookeeper_connection
                   or "127.0.0.1:2181")
        user, pw = env.get_optional("SDK_ZK_USERNAME", ""), env.get_optional("SDK_ZK_PASSWORD", "")
        session_ms = env.get_optional_int("SDK_ZK_SESSION_TIMEOUT_MS", 10000)
        if lock_enabled and ZkLocker._instance is None:
            ZkLocker.lock(service_spec.name, connect, username=user, password=pw,
                          wait_s=env.get_optional_double("SDK_LOCK_WAIT_S", 10.0), session_timeout_ms=session_ms)
        base = ZooKeeperPersister(connect, service_spec.name, username=user, password=pw,
                                  session_timeout_ms=session_ms)
        init_service_name(base, service_spec.name)
    else:
        raise ValueError(f"Unknown SDK_PERSISTER '{kind}' (expected file, mem or zk)")
    from dcos_commons_amd import trace

    if trace.enabled():
        base = trace.TracingPersister(base)
    if scheduler_config.is_state_cache_enabled() and kind != "mem":
        return PersisterCache(base)
    return base
