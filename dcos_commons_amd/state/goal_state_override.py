"""Goal-state overrides: pause/resume and decommission.

Reference: sdk/.../state/GoalStateOverride.java:17-205. A PAUSED task is relaunched with its
command replaced by a sleep loop and its readiness check replaced by ``exit 1``.
"""
from __future__ import annotations

import enum
from typing import Optional

LONG_DECLINE_SECONDS = 3600
PAUSE_COMMAND = ("echo This task is PAUSED, sleeping ... && ./bootstrap --resolve=false && "
                 f"while true; do sleep {LONG_DECLINE_SECONDS}; done")
PAUSE_READINESS_COMMAND = "exit 1"


class GoalStateOverride(enum.Enum):
    NONE = ("NONE", "STARTING")
    PAUSED = ("PAUSED", "PAUSING")
    DECOMMISSIONED = ("DECOMMISSIONED", "DECOMMISSIONING")

    @property
    def serialized_name(self) -> str:
        return self.value[0]

    @property
    def transitioning_name(self) -> str:
        return self.value[1]

    @staticmethod
    def from_serialized(name: str) -> Optional["GoalStateOverride"]:
        for o in GoalStateOverride:
            if o.serialized_name == name:
                return o
        return GoalStateOverride.NONE

    def new_status(self, progress: "OverrideProgress") -> "OverrideStatus":
        return OverrideStatus(self, progress)


class OverrideProgress(enum.Enum):
    PENDING = "PENDING"
    IN_PROGRESS = "IN_PROGRESS"
    COMPLETE = "COMPLETE"


class OverrideStatus:
    __slots__ = ("target", "progress")

    def __init__(self, target: GoalStateOverride, progress: OverrideProgress):
        self.target = target
        self.progress = progress

    @staticmethod
    def translate_status(plan_status) -> OverrideProgress:
        from dcos_commons_amd.scheduler.plan.status import Status

        if plan_status == Status.PENDING:
            return OverrideProgress.PENDING
        if plan_status in (Status.STARTED, Status.COMPLETE):
            return OverrideProgress.COMPLETE
        return OverrideProgress.IN_PROGRESS

    def __eq__(self, other):
        return isinstance(other, OverrideStatus) and self.target == other.target and self.progress == other.progress

    def __hash__(self):
        return hash((self.target, self.progress))

    def __repr__(self):
        return f"{self.target.name}/{self.progress.name}"


OverrideStatus.INACTIVE = OverrideStatus(GoalStateOverride.NONE, OverrideProgress.COMPLETE)
