"""The unit of work a step asks the offer evaluator to satisfy.

Reference: sdk/.../scheduler/plan/PodInstanceRequirement.java:17-147 and
scheduler/recovery/RecoveryType.java:7. Two requirements *conflict* when they target the same
pod instance and share at least one task -- the basis of the dirty-asset mutual exclusion
between deploy, recovery and custom plans.
"""
from __future__ import annotations

import enum
from typing import Dict, Iterable, List, Optional

from dcos_commons_amd.specification.specs import PodInstance


class RecoveryType(enum.Enum):
    NONE = "NONE"
    TRANSIENT = "TRANSIENT"
    PERMANENT = "PERMANENT"

    def __str__(self):
        return self.value


class PodInstanceRequirement:
    __slots__ = ("pod_instance", "tasks_to_launch", "environment", "recovery_type")

    def __init__(self, pod_instance: PodInstance, tasks_to_launch: Iterable[str],
                 environment: Optional[Dict[str, str]] = None, recovery_type: RecoveryType = RecoveryType.NONE):
        self.pod_instance = pod_instance
        self.tasks_to_launch: List[str] = list(tasks_to_launch)
        self.environment: Dict[str, str] = dict(environment or {})
        self.recovery_type = recovery_type

    def with_environment(self, env: Dict[str, str]) -> "PodInstanceRequirement":
        return PodInstanceRequirement(self.pod_instance, self.tasks_to_launch, env, self.recovery_type)

    def with_recovery_type(self, rt: RecoveryType) -> "PodInstanceRequirement":
        return PodInstanceRequirement(self.pod_instance, self.tasks_to_launch, self.environment, rt)

    @property
    def name(self) -> str:
        return f"{self.pod_instance.name}:[{', '.join(self.tasks_to_launch)}]"

    def conflicts_with(self, other: "PodInstanceRequirement") -> bool:
        if not other.pod_instance.conflicts_with(self.pod_instance):
            return False
        return any(t in other.tasks_to_launch for t in self.tasks_to_launch)

    def _key(self):
        return (self.pod_instance.name, tuple(self.tasks_to_launch), tuple(sorted(self.environment.items())),
                self.recovery_type)

    def __eq__(self, other):
        return isinstance(other, PodInstanceRequirement) and self._key() == other._key()

    def __hash__(self):
        return hash(self._key())

    def __repr__(self):
        return f"{self.name}({self.recovery_type})"
