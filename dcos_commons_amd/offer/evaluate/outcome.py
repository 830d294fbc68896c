"""Pass/fail tree produced by every evaluation stage and placement rule.

Reference: sdk/.../offer/evaluate/EvaluationOutcome.java:17-216.
"""
from __future__ import annotations

from typing import Any, List, Optional


class EvaluationOutcome:
    __slots__ = ("passing", "source", "reason", "children", "recommendations", "mesos_resource")

    def __init__(self, passing: bool, source: Any, reason: str, recommendations=None, children=None,
                 mesos_resource=None):
        self.passing = passing
        self.source = source if isinstance(source, str) else type(source).__name__
        self.reason = reason
        self.recommendations = list(recommendations or [])
        self.children: List["EvaluationOutcome"] = list(children or [])
        self.mesos_resource = mesos_resource

    @staticmethod
    def pass_(source, reason: str, *args, recommendations=None, children=None, mesos_resource=None):
        return EvaluationOutcome(True, source, reason % args if args else reason, recommendations, children,
                                 mesos_resource)

    @staticmethod
    def fail(source, reason: str, *args, children=None):
        return EvaluationOutcome(False, source, reason % args if args else reason, None, children)

    def is_passing(self) -> bool:
        return self.passing

    def get_offer_recommendations(self) -> list:
        recs = list(self.recommendations)
        for c in self.children:
            recs.extend(c.get_offer_recommendations())
        return recs

    def to_dict(self) -> dict:
        return {"type": "PASS" if self.passing else "FAIL", "source": self.source, "reason": self.reason,
                "children": [c.to_dict() for c in self.children]}

    def __str__(self):
        return f"{'PASS' if self.passing else 'FAIL'}({self.source}): {self.reason}"

    __repr__ = __str__

    def tree_lines(self, indent: int = 0) -> List[str]:
        lines = ["  " * indent + str(self)]
        for c in self.children:
            lines.extend(c.tree_lines(indent + 1))
        return lines
