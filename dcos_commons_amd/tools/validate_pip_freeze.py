"""Check that the installed Python modules match a pinned requirements file (reference:
tools/validate_pip_freeze.py, run in the test container's CI).

Every requirement must be pinned (``name==version``), appear once, and be installed at exactly
that version; ``git+http...#egg=...`` lines use the ``validator-hint: name=<n> version=<v>`` in
their fragment. Installed versions come from ``importlib.metadata`` (no ``pip freeze`` subprocess).
"""
from __future__ import annotations

import logging
import os
import re
import sys
import urllib.parse
from importlib import metadata
from typing import Dict, List, Optional, Tuple

LOGGER = logging.getLogger(__name__)
_HINT_RE = re.compile(r".*validator-hint:( +name=(?P<name>[\w.-]+))?( +version=(?P<version>[\w.+-]+))? *$")
_REQ_RE = re.compile(r"^(?P<name>[A-Za-z0-9][\w.-]*)\s*(?P<op>===|==)\s*(?P<version>[\w.+!-]+)\s*$")


def _normalize(name: str) -> str:
    return re.sub(r"[-_.]+", "-", name).lower()


def _process_line(line: str) -> Optional[str]:
    line = line.split(" #", 1)[0].strip()
    if not line or line.startswith("#"):
        return None
    if not line.startswith("git+http"):
        return line
    parsed = urllib.parse.urlparse(line)
    name = os.path.splitext(os.path.basename(parsed.path))[0]
    m = _HINT_RE.match(parsed.fragment)
    if m and m.group("name"):
        name = m.group("name")
    if m and m.group("version"):
        return f"{name}==={m.group('version')}" if m.group("version") == "SNAPSHOT" else f"{name}=={m.group('version')}"
    return name


def parse_requirements(text: str) -> Tuple[Dict[str, str], List[str]]:
    """(normalized name -> pinned version, problems)."""
    pins: Dict[str, str] = {}
    problems: List[str] = []
    for raw in text.splitlines():
        line = _process_line(raw)
        if line is None:
            continue
        m = _REQ_RE.match(line)
        if m is None:
            problems.append(f"not pinned to an exact version: {line}")
            continue
        name = _normalize(m.group("name"))
        if name in pins:
            problems.append(f"duplicate requirement: {name}")
        pins[name] = m.group("version")
    return pins, problems


def installed_versions() -> Dict[str, str]:
    return {_normalize(d.metadata["Name"]): d.version for d in metadata.distributions() if d.metadata["Name"]}


def validate(requirements_text: str, installed: Optional[Dict[str, str]] = None) -> List[str]:
    pins, problems = parse_requirements(requirements_text)
    have = installed if installed is not None else installed_versions()
    for name, version in sorted(pins.items()):
        if version == "SNAPSHOT":
            if name not in have:
                problems.append(f"{name} is not installed")
        elif name not in have:
            problems.append(f"{name}=={version} is not installed")
        elif have[name] != version:
            problems.append(f"{name}: requirements pin {version}, installed {have[name]}")
    return problems


def main(argv: List[str]) -> int:
    if len(argv) != 2:
        LOGGER.error("Syntax: %s <requirements.txt>", argv[0])
        return 1
    with open(argv[1], "r", encoding="utf-8") as f:
        problems = validate(f.read())
    for p in problems:
        LOGGER.critical(p)
    return 1 if problems else 0


if __name__ == "__main__":
    logging.basicConfig(level=logging.INFO, format="%(message)s")
    sys.exit(main(sys.argv))
