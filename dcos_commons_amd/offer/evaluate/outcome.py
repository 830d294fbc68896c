"""Pass/fail tree produced by every evaluation stage and placement rule.

Reference: sdk/.../offer/evaluate/EvaluationOutcome.java:17-216.
"""
from __future__ import annotations

from typing import Any, List


class EvaluationOutcome:
    """``reason`` is rendered lazily: the format arguments (specs, protobufs) are only turned into
    text when a log line, debug tracker or failure report reads it. Evaluating a pod produces dozens
    of passing outcomes per offer, and formatting them eagerly cost about a third of
    ``OfferEvaluator.evaluate``."""

    __slots__ = ("passing", "source", "_fmt", "_args", "children", "recommendations", "mesos_resource")

    def __init__(self, passing: bool, source: Any, reason: str, recommendations=None, children=None,
                 mesos_resource=None, args: tuple = ()):
        self.passing = passing
        self.source = source if isinstance(source, str) else type(source).__name__
        self._fmt = reason
        self._args = args
        self.recommendations = list(recommendations or [])
        self.children: List["EvaluationOutcome"] = list(children or [])
        self.mesos_resource = mesos_resource

    @property
    def reason(self) -> str:
        if self._args:
            self._fmt, self._args = self._fmt % self._args, ()
        return self._fmt

    @staticmethod
    def pass_(source, reason: str, *args, recommendations=None, children=None, mesos_resource=None):
        return EvaluationOutcome(True, source, reason, recommendations, children, mesos_resource, args)

    @staticmethod
    def fail(source, reason: str, *args, children=None):
        return EvaluationOutcome(False, source, reason, None, children, None, args)

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
