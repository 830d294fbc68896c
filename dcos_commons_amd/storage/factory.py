"""Persister selection for a service.

Reference: sdk/.../curator/CuratorPersister.java:64-93 (``/dcos-service-<name>`` ZooKeeper root,
wrapped in PersisterCache unless DISABLE_STATE_CACHE) and SchedulerBuilder.java:189-193.

Backends here (``SDK_PERSISTER``):
* ``file`` (default) -- crash-safe WAL-journaled tree under ``SDK_STATE_DIR`` (default
  ``./state``) at ``dcos-service-<name>``; the same node layout the reference keeps in ZK;
* ``mem`` -- in-memory, for tests and benchmarks;
* ``zk`` -- ZooKeeper at ``FRAMEWORK_ZOOKEEPER`` (``storage.zk_persister``).
"""
from __future__ import annotations

import os

from .mem_persister import MemPersister
from .persister import Persister
from .persister_cache import PersisterCache


def service_root_name(service_name: str) -> str:
    # Curator root: "/dcos-service-" + name with '/' replaced by "__" (CuratorUtils.getServiceRootPath)
    return "dcos-service-" + service_name.lstrip("/").replace("/", "__")


def persister_for_service(service_spec, scheduler_config) -> Persister:
    env = scheduler_config.env
    kind = env.get_optional("SDK_PERSISTER", "file")
    if kind == "mem":
        base: Persister = MemPersister()
    elif kind == "file":
        from .file_persister import FilePersister

        root = os.path.join(env.get_optional("SDK_STATE_DIR", "state"), service_root_name(service_spec.name))
        base = FilePersister(root)
    elif kind == "zk":
        from .zk_persister import ZooKeeperPersister

        base = ZooKeeperPersister(service_spec.zookeeper_connection or "127.0.0.1:2181",
                                  "/" + service_root_name(service_spec.name))
    else:
        raise ValueError(f"Unknown SDK_PERSISTER '{kind}' (expected file, mem or zk)")
    if scheduler_config.is_state_cache_enabled() and kind != "mem":
        return PersisterCache(base)
    return base
