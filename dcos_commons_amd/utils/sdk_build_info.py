"""The SDK's own build stamp (reference: the generated ``SDKBuildInfo`` class that
SchedulerConfig.getBuildInfo reports, SchedulerConfig.java:655-665).

``__graft_entry__.build()`` writes ``_build_info.json`` next to this module (git SHA of the tree and
the build time); without it the SHA is read from the checkout's ``.git`` if there is one, else
``UNKNOWN``, and the build time falls back to the newest mtime of the package's sources.
"""
from __future__ import annotations

import datetime
import json
import os
from typing import Optional

NAME = "dcos-commons-amd"
VERSION = "0.58.0-mi355x"

_HERE = os.path.dirname(os.path.abspath(__file__))
_PKG = os.path.dirname(_HERE)
_ROOT = os.path.dirname(_PKG)
STAMP_FILE = os.path.join(_HERE, "_build_info.json")


def _stamp() -> dict:
    try:
        with open(STAMP_FILE, "r", encoding="utf-8") as f:
            d = json.load(f)
        return d if isinstance(d, dict) else {}
    except (OSError, ValueError):
        return {}


def _git_head(root: str) -> Optional[str]:
    head = os.path.join(root, ".git", "HEAD")
    try:
        with open(head, "r", encoding="utf-8") as f:
            ref = f.read().strip()
    except OSError:
        return None
    if not ref.startswith("ref: "):
        return ref or None
    name = ref[5:]
    try:
        with open(os.path.join(root, ".git", name), "r", encoding="utf-8") as f:
            return f.read().strip() or None
    except OSError:
        pass
    try:  # packed refs
        with open(os.path.join(root, ".git", "packed-refs"), "r", encoding="utf-8") as f:
            for line in f:
                parts = line.strip().split(" ")
                if len(parts) == 2 and parts[1] == name:
                    return parts[0]
    except OSError:
        pass
    return None


def git_sha() -> str:
    return str(_stamp().get("git_sha") or _git_head(_ROOT) or "UNKNOWN")


def build_time_ms() -> int:
    t = _stamp().get("built_at_ms")
    if isinstance(t, int):
        return t
    newest = 0.0
    for d, _, files in os.walk(_PKG):
        for f in files:
            if f.endswith(".py"):
                try:
                    newest = max(newest, os.path.getmtime(os.path.join(d, f)))
                except OSError:
                    pass
    return int(newest * 1000)


def iso_instant(epoch_ms: int) -> str:
    """``java.time.Instant.toString()`` of an epoch-millis value: ISO-8601 UTC, ``Z`` suffix,
    fractional seconds only when non-zero (``1970-01-01T00:00:00Z``, ``...T00:00:00.123Z``)."""
    dt = datetime.datetime.fromtimestamp(epoch_ms // 1000, tz=datetime.timezone.utc)
    base = dt.strftime("%Y-%m-%dT%H:%M:%S")
    ms = epoch_ms % 1000
    return f"{base}.{ms:03d}Z" if ms else f"{base}Z"


def write_stamp(git_sha_value: Optional[str] = None, built_at_ms: Optional[int] = None) -> str:
    import time

    data = {"git_sha": git_sha_value or _git_head(_ROOT) or "UNKNOWN",
            "built_at_ms": int(time.time() * 1000) if built_at_ms is None else int(built_at_ms)}
    with open(STAMP_FILE, "w", encoding="utf-8") as f:
        json.dump(data, f)
    return STAMP_FILE
