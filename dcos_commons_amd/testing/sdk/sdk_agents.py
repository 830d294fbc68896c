"""Agent listing and fault injection (reference: testing/sdk_agents.py).

On DC/OS these SSH into agents (``iptables`` partitions, ``shutdown``); here they drive the local
master: a partitioned agent goes unreachable and keeps its tasks, a shut-down agent never comes
back, a decommissioned agent is marked GONE by the operator.
"""
from __future__ import annotations

import logging
from typing import Any, Dict, List

LOG = logging.getLogger(__name__)


def _cluster():
    from dcos_commons_amd.testing.cluster import current

    return current()


def get_agents() -> List[Dict[str, Any]]:
    return _cluster().agents()


def get_private_agents() -> List[Dict[str, Any]]:
    return [a for a in get_agents() if a["attributes"].get("public_ip") != "true"]


def get_public_agents() -> List[Dict[str, Any]]:
    return [a for a in get_agents() if a["attributes"].get("public_ip") == "true"]


def partition_agent(agent_host: str) -> None:
    LOG.info("Partitioning agent %s", agent_host)
    _cluster().partition_agent(agent_host)


def reconnect_agent(agent_host: str) -> None:
    LOG.info("Reconnecting agent %s", agent_host)
    _cluster().reconnect_agent(agent_host)


def shutdown_agent(agent_host: str) -> None:
    """The agent goes away for good (its tasks become unreachable and it never re-registers)."""
    LOG.info("Shutting down agent %s", agent_host)
    _cluster().partition_agent(agent_host)


def decommission_agent(agent_host: str) -> None:
    LOG.info("Decommissioning agent %s", agent_host)
    _cluster().decommission_agent(agent_host)
