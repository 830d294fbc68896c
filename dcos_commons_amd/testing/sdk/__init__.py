"""Integration-test helpers for the local DC/OS stand-in (``testing.cluster``).

Module and function names follow the reference's ``testing/sdk_*.py`` so framework integration
tests read the same: ``sdk_install``, ``sdk_plan``, ``sdk_tasks``, ``sdk_cmd``, ``sdk_marathon``,
``sdk_agents``, ``sdk_recovery``, ``sdk_metrics``, ``sdk_hosts``, ``sdk_networks``,
``sdk_upgrade``, ``sdk_service``, ``sdk_fault_domain``, ``sdk_diag``, ``sdk_utils``.
They act on ``testing.cluster.current()``.
"""
