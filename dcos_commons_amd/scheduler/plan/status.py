"""Plan element status (reference sdk/.../scheduler/plan/Status.java:22-92)."""
from __future__ import annotations

import enum


class Status(enum.Enum):
    ERROR = "ERROR"
    WAITING = "WAITING"
    PENDING = "PENDING"
    PREPARED = "PREPARED"
    STARTING = "STARTING"
    STARTED = "STARTED"
    COMPLETE = "COMPLETE"
    IN_PROGRESS = "IN_PROGRESS"
    DELAYED = "DELAYED"

    def is_running(self) -> bool:
        return self in (Status.PREPARED, Status.STARTING, Status.STARTED, Status.IN_PROGRESS)

    def __str__(self):
        return self.value
