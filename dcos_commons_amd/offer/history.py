"""Offer evaluation history for the debug endpoints.

Reference: sdk/.../offer/history/OfferOutcomeTracker.java (ring of 100, ``/v1/debug/offers``) and
sdk/.../debug/OfferOutcomeTrackerV2.java (aggregated failure reasons/agents, ``/v2/debug/offers``).
"""
from __future__ import annotations

import collections
import html
import threading
import time
from typing import Dict

from dcos_commons_amd.mesos import protos as P

DEFAULT_CAPACITY = 100


class OfferOutcome:
    """``details`` may be given as a zero-argument callable: it is rendered (once) when a debug
    endpoint reads it, not on the offer-evaluation path."""

    __slots__ = ("timestamp", "pod_instance_name", "passed", "offer", "_details")

    def __init__(self, pod_instance_name: str, passed: bool, offer: P.Offer, details):
        self.timestamp = int(time.time() * 1000)
        self.pod_instance_name = pod_instance_name
        self.passed = passed
        self.offer = offer
        self._details = details

    @property
    def details(self):
        if callable(self._details):
            self._details = self._details()
        return self._details


class OfferOutcomeTracker:
    def __init__(self, capacity: int = DEFAULT_CAPACITY):
        self.outcomes = collections.deque(maxlen=capacity)
        self._lock = threading.Lock()

    def track(self, outcome: OfferOutcome) -> None:
        with self._lock:
            self.outcomes.append(outcome)

    def to_json(self) -> dict:
        with self._lock:
            items = list(self.outcomes)
        items.reverse()
        return {"outcomes": [{
            "timestamp": o.timestamp,
            "pod-instance-name": o.pod_instance_name,
            "outcome": "pass" if o.passed else "fail",
            "explanation": o.details,
            "offer": P.to_text(o.offer),
        } for o in items]}

    def to_html(self) -> str:
        rows = []
        for o in self.to_json()["outcomes"]:
            expl = "".join(f"<div>{html.escape(line)}</div><br>" for line in str(o["explanation"]).split("\n"))
            rows.append(
                f"<tr><td style=\"white-space: nowrap\">{time.ctime(o['timestamp'] / 1000)}</td>"
                f"<td style=\"white-space: nowrap\">{html.escape(o['pod-instance-name'])}</td>"
                f"<td>{o['outcome'].upper()}</td><td style=\"width: 500px\">{expl}</td>"
                f"<td style=\"width: 500px\">{html.escape(o['offer'])}</td></tr>")
        return ("<html><style>table, th, td { border: 1px solid black; }\n"
                "tbody tr:nth-child(odd) { background-color: #E8E8E8 }\nth, td { padding: 10px }</style><body>"
                "<table style=\"border: 1px solid black\"><tr><th>Time</th><th>Pod Instance</th><th>Outcome</th>"
                "<th>Explanation</th><th>Offer</th></tr>" + "".join(rows) + "</table></body></html>")


class OfferOutcomeSummary:
    def __init__(self, capacity: int = DEFAULT_CAPACITY):
        self.accepted_count = 0
        self.rejected_count = 0
        self.outcomes = collections.deque(maxlen=capacity)
        self.failure_reasons: Dict[str, int] = {}
        self.rejected_agents: Dict[str, int] = {}
        self._lock = threading.Lock()

    def add_offer(self, outcome: OfferOutcome) -> None:
        with self._lock:
            self.outcomes.append(outcome)
            if outcome.passed:
                self.accepted_count += 1
            else:
                self.rejected_count += 1

    def add_failure_reason(self, reason: str) -> None:
        with self._lock:
            self.failure_reasons[reason] = self.failure_reasons.get(reason, 0) + 1

    def add_failure_agent(self, agent_id: str) -> None:
        with self._lock:
            self.rejected_agents[agent_id] = self.rejected_agents.get(agent_id, 0) + 1

    def to_json(self) -> dict:
        with self._lock:
            offers = [{
                "timestamp": o.timestamp,
                "pod-instance-name": o.pod_instance_name,
                "outcome": "pass" if o.passed else "fail",
                "explanation": o.details,
                "offer": P.to_text(o.offer),
            } for o in self.outcomes]
            return {"acceptedCount": self.accepted_count, "rejectedCount": self.rejected_count,
                    "failureReasons": dict(self.failure_reasons), "rejectedAgents": dict(self.rejected_agents),
                    "offers": offers}


class OfferOutcomeTrackerV2:
    def __init__(self):
        self.summary = OfferOutcomeSummary()

    def to_json(self) -> dict:
        return self.summary.to_json()
