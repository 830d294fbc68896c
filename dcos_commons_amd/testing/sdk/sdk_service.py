"""Options update of a running service (reference: testing/sdk_service.py)."""
from __future__ import annotations

from typing import Any, Dict

from dcos_commons_amd.testing.sdk import sdk_upgrade


DEFAULT_TIMEOUT_SECONDS = 10 * 60   # testing/sdk_service.py: a rolling options update can take minutes


def update_configuration(package_name: str, service_name: str, configuration: Dict[str, Any],
                         expected_task_count: int, wait_for_deployment: bool = True,
                         timeout_seconds: int = DEFAULT_TIMEOUT_SECONDS) -> None:
    """Applies ``configuration`` as the service's new options (no version change) and, with
    ``wait_for_deployment``, waits for the rollout and ``expected_task_count`` running tasks."""
    sdk_upgrade.update_or_upgrade_or_downgrade(package_name, service_name, None, configuration,
                                               expected_task_count, wait_for_deployment, timeout_seconds)
