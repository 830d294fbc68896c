"""Logger construction (reference: sdk/scheduler/.../offer/LoggingUtils.java:12-60 and
src/main/resources/log4j2.xml).

``get_logger(__name__, namespace)`` tags a module logger with the service it manages, the way the
reference prefixes ``(<namespace>)`` in multi-service mode. The tagged logger stays a child of the
module's package (``pkg.module(svc-a)``), so levels configured on ``dcos_commons_amd`` still apply.
``configure(env)`` sets the process-wide level from ``FRAMEWORK_LOG_LEVEL`` (default INFO).
"""
from __future__ import annotations

import logging
import os
from typing import Mapping, Optional

FORMAT = "%(asctime)s %(levelname)-5s [%(threadName)s] %(name)s: %(message)s"


def get_logger(name: str, namespace: Optional[str] = None) -> logging.Logger:
    if namespace is None or not str(namespace).strip():
        return logging.getLogger(name)
    return logging.getLogger(f"{name}({namespace})")


def configure(env: Optional[Mapping[str, str]] = None) -> int:
    """Root logging for a scheduler process; returns the level applied. Unknown level names fall
    back to INFO with a warning instead of failing the scheduler start."""
    env = os.environ if env is None else env
    name = str(env.get("FRAMEWORK_LOG_LEVEL", "INFO")).strip().upper()
    level = logging.getLevelName(name)
    bad = not isinstance(level, int)
    if bad:
        level = logging.INFO
    logging.basicConfig(level=level, format=FORMAT)
    logging.getLogger().setLevel(level)
    if bad:
        logging.getLogger(__name__).warning("Unknown FRAMEWORK_LOG_LEVEL %r, using INFO", name)
    return level
