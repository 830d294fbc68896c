"""Publish a release into a universe repository checkout as a reviewable git branch.

Reference: ``tools/universe/package_publisher.py`` (clones mesosphere/universe from GitHub, commits
the release on a new branch and opens a pull request). Without network access the repository is a
local git checkout (``RELEASE_UNIVERSE_REPO``: a path or anything ``git clone`` takes) and the
"pull request" is the pushed branch plus its description file; everything else follows the same
rules:

* the package's releases live in ``repo/packages/<L>/<name>/<releaseVersion>/``;
* a GA release takes the next multiple of 100 above the newest release, a beta release the next
  integer (so betas can follow a GA, and the next GA leaves room); ``RELEASE_INDEX`` pins it and
  must be free;
* the commit message lists the files added, removed and changed (as unified diffs) against the
  nearest earlier release.

    python -m dcos_commons_amd.tools.universe.package_publisher <name> <version> <package dir> [--beta]
"""
from __future__ import annotations

import argparse
import difflib
import os
import secrets
import shutil
import subprocess
import sys
import tempfile
from typing import List, Optional, Sequence, Tuple

GA_INDEX_MULTIPLIER = 100
BETA_INDEX_MULTIPLIER = 1


def release_indexes(repo_pkg_base: str, beta: bool, requested: int = -1) -> Tuple[int, int]:
    """(prior release index or -1, this release's index)."""
    existing = sorted(int(d) for d in (os.listdir(repo_pkg_base) if os.path.isdir(repo_pkg_base) else [])
                      if d.isdigit() and os.path.isdir(os.path.join(repo_pkg_base, d)))
    if requested >= 0:
        if requested in existing:
            raise ValueError(f"release index {requested} is already taken in {repo_pkg_base}: {existing}")
        prior = [i for i in existing if i < requested]
        return (prior[-1] if prior else -1), requested
    if not existing:
        return -1, 0
    last = existing[-1]
    step = BETA_INDEX_MULTIPLIER if beta else GA_INDEX_MULTIPLIER
    return last, step * (last // step + 1)


def describe_changes(last_dir: str, this_dir: str, last_index: int, this_index: int,
                     commit_desc: str = "") -> List[str]:
    """The commit message body: file lists and unified diffs between two release directories."""
    this_files = set(os.listdir(this_dir))
    last_files = set(os.listdir(last_dir)) if os.path.isdir(last_dir) else set()
    diffs = {}
    for name in sorted(this_files & last_files):
        with open(os.path.join(last_dir, name), encoding="utf-8") as a, \
                open(os.path.join(this_dir, name), encoding="utf-8") as b:
            d = "".join(difflib.unified_diff(a.readlines(), b.readlines(), fromfile=f"{last_index}/{name}",
                                             tofile=f"{this_index}/{name}"))
        if d:
            diffs[name] = d
    added, removed = sorted(this_files - last_files), sorted(last_files - this_files)
    lines = [f"Changes between revisions {last_index} => {this_index}:\n",
             f"{len(added)} files added: [{', '.join(added)}]\n",
             f"{len(removed)} files removed: [{', '.join(removed)}]\n",
             f"{len(diffs)} files changed:\n\n"]
    if commit_desc:
        lines.append(f"Description:\n{commit_desc}\n\n")
    for name in sorted(diffs):
        lines.append(f"```\n{diffs[name]}```\n\n")
    return lines


class UniversePackagePublisher:
    def __init__(self, package_name: str, package_version: str, commit_desc: str = "", beta_release: bool = False,
                 dry_run: bool = False, universe_repo: Optional[str] = None, release_branch: Optional[str] = None,
                 release_index: Optional[int] = None):
        self.name = package_name
        self.version = package_version
        self.commit_desc = commit_desc
        self.beta = beta_release
        self.dry_run = dry_run
        self.universe_repo = universe_repo or os.environ.get("RELEASE_UNIVERSE_REPO", "")
        self.release_branch = release_branch or os.environ.get("RELEASE_BRANCH", "version-3.x")
        self.release_index = release_index if release_index is not None else int(os.environ.get("RELEASE_INDEX", -1))
        self.title = f"Release {self.name} {self.version} (automated commit)\n\n"

    @staticmethod
    def _git(cwd: str, *args: str) -> str:
        return subprocess.run(["git", *args], cwd=cwd, check=True, capture_output=True, text=True).stdout

    def publish(self, scratchdir: str, pkgdir: str) -> Tuple[str, str]:
        """Clone the universe repository into ``scratchdir``, add ``pkgdir`` as the next release on
        a new branch, commit, and push the branch back (not in a dry run). Returns (branch, path of
        the commit message / pull-request description)."""
        if not self.universe_repo:
            raise ValueError("RELEASE_UNIVERSE_REPO (a universe repository to clone) is not set")
        checkout = os.path.join(scratchdir, "universe")
        subprocess.run(["git", "clone", "-q", "--branch", self.release_branch, self.universe_repo, checkout],
                       check=True, capture_output=True)
        branch = f"automated/release_{self.name}_{self.version}_{secrets.token_hex(3)}"
        self._git(checkout, "config", "--local", "user.email", "release@localhost")
        self._git(checkout, "config", "--local", "user.name", "package_publisher")
        self._git(checkout, "checkout", "-q", "-b", branch)
        base = os.path.join(checkout, "repo", "packages", self.name[0].upper(), self.name)
        os.makedirs(base, exist_ok=True)
        last, this = release_indexes(base, self.beta, self.release_index)
        shutil.copytree(pkgdir, os.path.join(base, str(this)))
        msg = os.path.join(scratchdir, "commitmsg.txt")
        with open(msg, "w", encoding="utf-8") as f:
            f.write(self.title)
            f.writelines(describe_changes(os.path.join(base, str(last)), os.path.join(base, str(this)), last, this,
                                          self.commit_desc))
        self._git(checkout, "add", ".")
        self._git(checkout, "commit", "-q", "-F", msg)
        if not self.dry_run:
            self._git(checkout, "push", "-q", "origin", branch)
        return branch, msg


def main(argv: Optional[Sequence[str]] = None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("name")
    ap.add_argument("version")
    ap.add_argument("pkgdir")
    ap.add_argument("--beta", action="store_true")
    ap.add_argument("--dry-run", action="store_true")
    ap.add_argument("--description", default="")
    args = ap.parse_args(argv)
    with tempfile.TemporaryDirectory(prefix="universe-publish-") as scratch:
        branch, msg = UniversePackagePublisher(args.name, args.version, args.description, args.beta,
                                               args.dry_run).publish(scratch, args.pkgdir)
        with open(msg, encoding="utf-8") as f:
            sys.stdout.write(f"branch {branch}\n{f.read()}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
