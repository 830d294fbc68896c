"""Universe release publishing into a local git repository (``tools.universe.package_publisher``;
reference ``tools/universe/package_publisher.py``)."""
import os
import subprocess

import pytest

from dcos_commons_amd.tools.universe import package_publisher as pp


def _mkdirs(base, *names):
    for n in names:
        os.makedirs(os.path.join(base, str(n)))


@pytest.mark.parametrize("existing,beta,requested,expected", [
    ((), False, -1, (-1, 0)),
    ((0,), False, -1, (0, 100)),
    ((0, 100), True, -1, (100, 101)),
    ((0, 100, 101), False, -1, (101, 200)),
    ((0, 100), False, 50, (0, 50)),
])
def test_release_indexes(tmp_path, existing, beta, requested, expected):
    _mkdirs(tmp_path, *existing)
    assert pp.release_indexes(str(tmp_path), beta, requested) == expected


def test_requested_index_must_be_free(tmp_path):
    _mkdirs(tmp_path, 0, 100)
    with pytest.raises(ValueError):
        pp.release_indexes(str(tmp_path), False, 100)


def _git(cwd, *args):
    subprocess.run(["git", "-c", "user.email=t@t", "-c", "user.name=t", *args], cwd=cwd, check=True,
                   capture_output=True)


def test_publish_commits_the_release_on_a_branch(tmp_path):
    origin = tmp_path / "universe-origin"
    rel0 = origin / "repo" / "packages" / "H" / "hello-world" / "0"
    rel0.mkdir(parents=True)
    (rel0 / "package.json").write_text('{"name": "hello-world", "version": "1.0.0"}\n')
    (rel0 / "config.json").write_text("{}\n")
    _git(origin, "init", "-q", "-b", "version-3.x")
    _git(origin, "add", ".")
    _git(origin, "commit", "-q", "-m", "initial")
    _git(origin, "config", "receive.denyCurrentBranch", "ignore")
    pkg = tmp_path / "pkg"
    pkg.mkdir()
    (pkg / "package.json").write_text('{"name": "hello-world", "version": "1.1.0"}\n')
    (pkg / "resource.json").write_text("{}\n")
    scratch = tmp_path / "scratch"
    scratch.mkdir()
    publisher = pp.UniversePackagePublisher("hello-world", "1.1.0", "new features", universe_repo=str(origin))
    branch, msg = publisher.publish(str(scratch), str(pkg))
    assert branch.startswith("automated/release_hello-world_1.1.0_")
    text = open(msg, encoding="utf-8").read()
    assert text.startswith("Release hello-world 1.1.0 (automated commit)")
    assert "Changes between revisions 0 => 100" in text and "1 files added: [resource.json]" in text
    assert "1 files removed: [config.json]" in text and '+{"name": "hello-world", "version": "1.1.0"}' in text
    # the branch reached the origin with release 100
    out = subprocess.run(["git", "ls-tree", "-r", "--name-only", branch], cwd=origin, check=True,
                         capture_output=True, text=True).stdout
    assert "repo/packages/H/hello-world/100/package.json" in out
