"""Give the agents of a cluster MOUNT volumes for the volume tests (reference:
tools/create_testing_volumes.py, which creates loopback-backed ``/dcos/volume<N>`` filesystems
over SSH and restarts each agent so it re-registers with them).

On the local DC/OS stand-in the agents re-register in place: ``create_testing_volumes(cluster,
count, size_mb, profile)`` attaches ``/dcos/volume<N>`` disks (optionally of a CSI profile such as
``xfs``) to every agent; running tasks are untouched.
"""
from __future__ import annotations

from typing import List, Optional, Sequence


def create_testing_volumes(cluster=None, count: int = 2, size_mb: float = 10240.0, profile: Optional[str] = None,
                           hosts: Optional[Sequence[str]] = None) -> List[str]:
    if cluster is None:
        from dcos_commons_amd.testing.cluster import current

        cluster = current()
    return cluster.create_testing_volumes(count, size_mb, profile, hosts)
