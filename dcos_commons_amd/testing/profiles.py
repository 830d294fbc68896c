"""Scheduler flag profiles the test suites run under.

The scheduler defaults (``mi355x``) differ from the reference's behaviour in a dozen flags
(README "Scheduler flags that differ from the reference"). The suites that exercise whole
deployments -- simulation (``ServiceTestRunner``), fault injection (live scheduler on
``LocalMaster``) and the cassandra / hdfs framework suites -- run under both profiles, so a change
that only works with the deviations on (or off) is caught.

``reference`` switches every deviation off, exactly as ``deploy_bench.PROFILES["reference"]``
does, but keeps its waits short: the offer-queue wait and the revive spacing are 0.2 s instead of
the reference's 5 s (``OfferProcessor.java:46``, ``TokenBucket.java:18-24``). Those two constants
set how long the reference takes, not what it does; the bench's ``reference`` profile keeps the
real 5 s values to measure the cadence.
"""
from __future__ import annotations

from typing import Dict

REFERENCE_SEMANTICS: Dict[str, str] = {
    "SDK_EVENT_DRIVEN": "false",
    "SDK_OFFER_HOLD_S": "0",
    "SDK_OFFER_WAIT_S": "0.2",
    "SDK_REVIVE_INTERVAL_S": "0.2",
    "SDK_REVIVE_BURST_INTERVAL_S": "0.2",
    "SDK_RESERVATION_GC_ALL_OFFERS": "false",
    "SDK_FAST_UNSUPPRESS": "false",
    "SDK_MERGE_AGENT_OFFERS": "false",
    "SDK_LAUNCH_RECONCILE_S": "0",
    "SDK_UNKNOWN_AS_LOST": "false",
    "SDK_STREAM_LAUNCHES": "false",
    "SDK_REVIVE_ONLY_UNMATCHED": "false",
    "SDK_GC_GEN0_THRESHOLD": "0",
    "SDK_STATUS_CYCLE_WAIT_MS": "0",
}

PROFILES: Dict[str, Dict[str, str]] = {"mi355x": {}, "reference": REFERENCE_SEMANTICS}

# the profile ServiceTestRunner and the live-scheduler test fixtures apply under their own defaults
# and under every flag a test sets explicitly (set by the suites' parametrized fixture)
ACTIVE: Dict[str, str] = {}


def use(name: str) -> Dict[str, str]:
    """Makes ``name`` the active profile; returns the previous one's flags."""
    global ACTIVE
    prev, ACTIVE = ACTIVE, dict(PROFILES[name])
    return prev
