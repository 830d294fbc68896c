"""Universe repositories of the cluster's Cosmos (reference: testing/sdk_repository.py).

``STUB_UNIVERSE_URL`` (comma/space separated) names stub universes -- JSON files or URLs, ``.dcos``
bundles or repository trees built by ``tools.universe`` -- that are added in front of the
default repository for a test session and removed afterwards.
"""
from __future__ import annotations

import contextlib
import logging
import os
import re
from typing import Dict, Iterator, List, Optional, Tuple

LOG = logging.getLogger(__name__)


def _cosmos():
    from dcos_commons_amd.testing.cluster import current

    return current().cosmos


def parse_stub_universe_url_string(stub_universe_url: str) -> List[str]:
    """Split on commas and whitespace; duplicates dropped, order kept."""
    out: List[str] = []
    for u in re.split(r"[,\s]+", stub_universe_url or ""):
        if u and u not in out:
            out.append(u)
    return out


def get_repos() -> List[dict]:
    return [{"name": r["name"], "uri": r["uri"]} for r in _cosmos().repositories]


def remove_repo(repo_name: str) -> bool:
    before = len(_cosmos().repositories)
    _cosmos().remove_repo(repo_name)
    return len(_cosmos().repositories) < before


def add_repo(repo_name: str, repo_url: str, index: Optional[int] = None) -> bool:
    added = _cosmos().add_repo(repo_url, repo_name)
    LOG.info("Added repo %s (%s): %s", repo_name, repo_url, [f"{p.name}:{p.version}" for p in added])
    return bool(added)


def add_stub_universe_urls(stub_universe_urls: List[str]) -> Dict[str, str]:
    """Adds each stub universe as repo ``testpkg-<n>``; returns name -> URL for the cleanup."""
    stub_urls: Dict[str, str] = {}
    for i, url in enumerate(stub_universe_urls):
        name = f"testpkg-{i}"
        remove_repo(name)
        add_repo(name, url, index=0)
        stub_urls[name] = url
    return stub_urls


def remove_stub_universe_urls(stub_universe_urls: List[str]) -> None:
    for r in list(_cosmos().repositories):
        if r["uri"] in stub_universe_urls:
            remove_repo(r["name"])


def remove_universe_repos(stub_urls: Dict[str, str]) -> None:
    for name in stub_urls:
        remove_repo(name)


def get_package_versions(package_name: str) -> List[str]:
    return _cosmos().versions(package_name)


def move_universe_repo(package_name: str, universe_repo_index: Optional[int] = None) -> Tuple[str, str]:
    """(previous newest version, newest version) of a package once its repos are in place."""
    versions = get_package_versions(package_name)
    return (versions[-2] if len(versions) > 1 else versions[-1]), versions[-1]


@contextlib.contextmanager
def universe_session() -> Iterator[None]:
    """Stub universes from ``STUB_UNIVERSE_URL`` are added for the session, then removed."""
    stub_urls: Dict[str, str] = {}
    try:
        stub_urls = add_stub_universe_urls(parse_stub_universe_url_string(os.environ.get("STUB_UNIVERSE_URL", "")))
        yield
    finally:
        remove_universe_repos(stub_urls)
