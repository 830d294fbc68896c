"""Options update of a running service (reference: testing/sdk_service.py)."""
from __future__ import annotations

from typing import Any, Dict

from dcos_commons_amd.testing.sdk import sdk_upgrade


def update_configuration(package_name: str, service_name: str, configuration: Dict[str, Any],
                         expected_task_count: int, wait_for_deployment: bool = True,
                         timeout_seconds: int = 120) -> None:
    sdk_upgrade.update_or_upgrade_or_downgrade(package_name, service_name, None, configuration,
                                               expected_task_count, wait_for_deployment, timeout_seconds)
