"""Packaging / release tooling (reference: tools/universe/*, tools/release_builder.py,
tools/publish_http.py, tools/airgap_linter.py, tools/standardize_config_json.py)."""
import base64
import hashlib
import json
import os
import shutil
import urllib.request
import zipfile

import pytest

from dcos_commons_amd.tools import airgap_linter, build_package, standardize_config_json
from dcos_commons_amd.tools.publish_dcos_file import build_dcos_file
from dcos_commons_amd.tools.publish_http import HTTPPublisher
from dcos_commons_amd.tools.release_builder import UniverseReleaseBuilder, apply_beta_version
from dcos_commons_amd.tools.universe import (Package, PackageManager, UniversePackageBuilder, Version,
                                             files_from_package, load_repository, package_from_files)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HELLO_UNIVERSE = os.path.join(ROOT, "frameworks", "helloworld", "universe")
NATIVE_READY = os.path.exists(os.path.join(ROOT, "native", "build", "sdk-cli")) and \
    os.path.exists(os.path.join(ROOT, "native", "build", "sdk-bootstrap"))
needs_native = pytest.mark.skipif(not NATIVE_READY, reason="native tree not built")


def _artifact(tmp_path, name="sdk-cli-linux", data=b"cli-bytes"):
    p = tmp_path / name
    p.write_bytes(data)
    return str(p)


def _builder(tmp_path, version="stub-universe", repos=(), artifacts=None, uri="https://example.invalid/art"):
    arts = artifacts if artifacts is not None else [_artifact(tmp_path)]
    return UniversePackageBuilder(Package("hello-world", Version(0, version)), PackageManager(list(repos)),
                                  HELLO_UNIVERSE, uri, arts, now=1_700_000_000)


def test_versions_order_by_release_version_not_by_string():
    a, b = Package("x", Version(2, "1.0")), Package("x", Version(10, "0.9"))
    assert a < b and sorted([b, a])[-1] is b
    assert Package("beta-x", Version(0, "1")).get_non_beta_name() == "x"
    assert json.loads(str(a)) == {"name": "x", "version": "1.0", "releaseVersion": 2}


def test_builder_substitutes_build_parameters(tmp_path, monkeypatch):
    monkeypatch.setenv("TEMPLATE_EXTRA_PARAM", "unused")
    cli = _artifact(tmp_path)
    pkg = _builder(tmp_path, "1.2.3", artifacts=[cli]).packages_dict()["packages"][0]
    assert pkg["version"] == "1.2.3" and pkg["releaseVersion"] == 0 and pkg["lastUpdated"] == 1_700_000_000
    linux = pkg["resource"]["cli"]["binaries"]["linux"]["x86-64"]
    assert linux["url"] == "https://example.invalid/art/sdk-cli-linux"
    assert linux["contentHash"][0]["value"] == hashlib.sha256(b"cli-bytes").hexdigest()
    assert pkg["resource"]["assets"]["uris"]["bootstrap-zip"] == "https://example.invalid/art/bootstrap.zip"
    tmpl = base64.standard_b64decode(pkg["marathon"]["v2AppMustacheTemplate"]).decode()
    assert '"PACKAGE_VERSION": "1.2.3"' in tmpl and "{{service.name}}" in tmpl   # install-time params stay
    assert pkg["config"]["properties"]["service"]["properties"]["name"]["default"] == "hello-world"


def test_builder_requires_artifacts_for_sha_params(tmp_path):
    with pytest.raises(ValueError, match="sdk-cli-linux"):
        _builder(tmp_path, artifacts=[]).packages_dict()
    with pytest.raises(ValueError, match="Duplicate"):
        d = tmp_path / "d"
        d.mkdir()
        _builder(tmp_path, artifacts=[_artifact(tmp_path), _artifact(d)])


def test_upgrades_from_uses_the_latest_known_release(tmp_path):
    repo = tmp_path / "repo.json"
    repo.write_text(json.dumps({"packages": [{"name": "hello-world", "version": "1.0", "releaseVersion": 3},
                                             {"name": "hello-world", "version": "1.1", "releaseVersion": 7}]}))
    b = _builder(tmp_path, repos=[str(repo)])
    m = b.template_mapping()
    assert m["upgrades-from"] == "1.1" and m["downgrades-to"] == "1.1"
    assert b.documentation_path().endswith("/service-docs/hello-world/")
    assert _builder(tmp_path).template_mapping()["upgrades-from"] == "*"


def test_package_files_round_trip():
    files = {}
    for n in ("package.json", "config.json", "resource.json", "marathon.json.mustache"):
        with open(os.path.join(HELLO_UNIVERSE, n), "r", encoding="utf-8") as f:
            files[n] = f.read()
    back = files_from_package(package_from_files(files))
    assert back["marathon.json.mustache"] == files["marathon.json.mustache"]
    assert json.loads(back["config.json"]) == json.loads(files["config.json"])


def test_airgap_linter(tmp_path):
    fw = tmp_path / "fw"
    (fw / "universe").mkdir(parents=True)
    (fw / "specs").mkdir()
    (fw / "universe" / "package.json").write_text('{"name": "x"}\n')
    (fw / "specs" / "svc.yml").write_text("cmd: curl http://$MESOS_CONTAINER_IP:80/x\n"
                                          "# http://comment.example.com\n"
                                          "image: {{IMAGE}}\n")
    assert airgap_linter.check(str(fw))
    (fw / "specs" / "svc.yml").write_text("cmd: curl http://downloads.example.com/x.tgz\nimage: nginx:1.0\n")
    assert airgap_linter.bad_uris(str(fw)) == [(str(fw / "specs" / "svc.yml"), "downloads.example.com/x.tgz")]
    assert airgap_linter.bad_images(str(fw))[0][1] == "nginx:1.0"
    assert airgap_linter.main(["lint", str(fw)]) == 1
    for name in ("cassandra", "hdfs"):   # build_package lints every framework but hello-world
        assert airgap_linter.check(os.path.join(ROOT, "frameworks", name))


def test_standardize_config_json(tmp_path):
    cfg = {"type": "object", "properties": {"service": {"type": "object", "properties": {
        "security": {"type": "object"}, "zeta": {"default": 1, "type": "integer", "description": "z"},
        "log_level": {"type": "string"}, "name": {"default": "n", "description": "d", "type": "string"}}},
        "node": {"properties": {"b": {"type": "integer"}, "a": {"type": "integer"}}}}}
    out = standardize_config_json.standardize(cfg, {"sections": {"node": {"head": ["b"], "tail": []}}})
    svc = out["properties"]["service"]["properties"]
    assert list(svc) == ["name", "log_level", "zeta", "security"]
    assert list(svc["zeta"]) == ["description", "type", "default"]
    assert list(out["properties"]["node"]["properties"]) == ["b", "a"]
    path = tmp_path / "config.json"
    path.write_text(json.dumps(cfg))
    assert standardize_config_json.main(["--service-config-json", str(path), "--check"]) == 1
    assert standardize_config_json.main(["--service-config-json", str(path)]) == 0
    assert standardize_config_json.main(["--service-config-json", str(path), "--check"]) == 0
    for name in ("helloworld", "cassandra", "hdfs"):   # the shipped packages are already standard
        assert standardize_config_json.main(["--service-config-json", os.path.join(
            ROOT, "frameworks", name, "universe", "config.json"), "--check"]) == 0


def _stub_in_dir(tmp_path):
    art_dir = tmp_path / "build"
    art_dir.mkdir()
    arts = [_artifact(art_dir), _artifact(art_dir, "bootstrap.zip", b"zip"),
            _artifact(art_dir, "hello-world-scheduler.zip", b"sched")]
    b = UniversePackageBuilder(Package("hello-world", Version(0, "stub-universe")), PackageManager([]),
                               HELLO_UNIVERSE, "file://" + str(art_dir), arts)
    return b.build_package(str(art_dir))


def test_release_builder_moves_and_releases(tmp_path):
    stub = "file://" + _stub_in_dir(tmp_path)
    rel, repo = tmp_path / "releases", tmp_path / "universe"
    b = UniverseReleaseBuilder("2.0.0", stub, str(rel), universe_repo=str(repo))
    moved = json.load(open(b.move_package()))["packages"][0]
    assert moved["version"] == "2.0.0"
    assert moved["resource"]["assets"]["uris"]["bootstrap-zip"] == f"file://{rel}/hello-world/2.0.0/bootstrap.zip"
    assert (rel / "hello-world" / "2.0.0" / "sdk-cli-linux").read_bytes() == b"cli-bytes"
    tmpl = base64.standard_b64decode(moved["marathon"]["v2AppMustacheTemplate"]).decode()
    assert '"PACKAGE_VERSION": "2.0.0"' in tmpl
    with pytest.raises(FileExistsError):            # never stomps an existing release
        UniverseReleaseBuilder("2.0.0", stub, str(rel), universe_repo=str(repo)).release_package()
    first = UniverseReleaseBuilder("2.0.0", stub, str(rel), universe_repo=str(repo), force=True).release_package()
    second = UniverseReleaseBuilder("2.1.0", stub, str(rel), universe_repo=str(repo)).release_package()
    assert first.endswith("/H/hello-world/0") and second.endswith("/H/hello-world/1")
    latest = PackageManager([str(repo)]).get_latest("hello-world")
    assert latest.get_version().release_version == 1 and str(latest.get_version()) == "2.1.0"
    beta = UniverseReleaseBuilder("3.0.0", stub, str(rel), universe_repo=str(repo), beta=True)
    pkg = json.load(open(beta.move_package()))["packages"][0]
    assert pkg["name"] == "beta-hello-world" and pkg["version"] == "3.0.0-beta" and pkg["selected"] is False
    with pytest.raises(ValueError):
        apply_beta_version("1.0-beta", False)


def test_publish_http_serves_universe_and_artifacts(tmp_path):
    cli = _artifact(tmp_path)
    pub = HTTPPublisher("hello-world", "stub-universe", HELLO_UNIVERSE, [cli], http_dir=str(tmp_path / "http"))
    try:
        url = pub.start()
        assert url.startswith("http://127.0.0.1:") and url.endswith("/stub-universe-hello-world.json")
        pkgs = load_repository(url)
        link = pkgs[0]["resource"]["cli"]["binaries"]["linux"]["x86-64"]["url"]
        with urllib.request.urlopen(link, timeout=5) as r:
            assert r.read() == b"cli-bytes"
    finally:
        pub.stop()


def test_dcos_bundle_carries_catalog_and_artifacts(tmp_path):
    cli = _artifact(tmp_path)
    path = build_dcos_file("hello-world", "1.0.0", HELLO_UNIVERSE, [cli], str(tmp_path / "out"))
    assert path.endswith("hello-world-1.0.0.dcos")
    with zipfile.ZipFile(path) as z:
        assert z.read("resources/sdk-cli-linux") == b"cli-bytes"
    (pkg,) = load_repository(path)
    assert pkg["version"] == "1.0.0"
    assert pkg["resource"]["assets"]["uris"]["bootstrap-zip"] == "bundle://hello-world/1.0.0/bootstrap.zip"


@needs_native
def test_build_package_builds_artifacts_and_stub_universe(tmp_path):
    out = tmp_path / "out"
    assert build_package.main(["hello-world", os.path.join(ROOT, "frameworks", "helloworld"), "--out", str(out),
                               "dir", "4.5.6"]) == 0
    stub = json.load(open(out / "stub-universe-hello-world.json"))["packages"][0]
    assert stub["version"] == "4.5.6"
    with zipfile.ZipFile(out / "artifacts" / "hello-world-scheduler.zip") as z:
        names = set(z.namelist())
        assert "hello-world-scheduler/bin/hello-world" in names
        assert "hello-world-scheduler/specs/svc.yml" in names
        assert "hello-world-scheduler/lib/dcos_commons_amd/models/helloworld.py" in names
        assert not any(n.endswith(".pyc") for n in names)
    with zipfile.ZipFile(out / "artifacts" / "bootstrap.zip") as z:
        assert z.getinfo("bootstrap").external_attr >> 16 & 0o111
    sha = stub["resource"]["cli"]["binaries"]["linux"]["x86-64"]["contentHash"][0]["value"]
    assert sha == hashlib.sha256((out / "artifacts" / "sdk-cli-linux").read_bytes()).hexdigest()


@needs_native
def test_scheduler_zip_launcher_runs_from_the_unpacked_artifact(tmp_path):
    """The scheduler artifact is self-contained: its launcher finds the SDK and specs it carries."""
    import subprocess

    path = build_package.build_scheduler_zip("hello-world", os.path.join(ROOT, "frameworks", "helloworld"),
                                             str(tmp_path))
    shutil.unpack_archive(path, str(tmp_path / "x"))
    launcher = tmp_path / "x" / "hello-world-scheduler" / "bin" / "hello-world"
    os.chmod(launcher, 0o755)
    env = {k: v for k, v in os.environ.items() if k != "PYTHONPATH"}
    code = ("import dcos_commons_amd, os; from dcos_commons_amd.models import helloworld as h; "
            "print(dcos_commons_amd.__file__); print(h.SPEC_DIR)")
    script = launcher.read_text().replace('exec python3 -m dcos_commons_amd.models.helloworld "$@"',
                                          f'exec python3 -c "{code}"')
    launcher.write_text(script)
    out = subprocess.run([str(launcher)], env=env, cwd=str(tmp_path), capture_output=True, text=True, timeout=60)
    assert out.returncode == 0, out.stderr
    lib, specs = out.stdout.split()
    assert lib.startswith(str(tmp_path / "x")) and specs == str(tmp_path / "x" / "hello-world-scheduler" / "specs")


def test_print_package_tag_version_and_sha(tmp_path, capsys):
    """tools/print_package_tag.py: the described version, then the SHA it is tagged at in a
    local checkout and through ``git ls-remote``."""
    import subprocess

    from dcos_commons_amd.tools import print_package_tag as ppt

    repo = tmp_path / "repo"
    repo.mkdir()
    git = ["git", "-C", str(repo), "-c", "user.email=ci@example.com", "-c", "user.name=ci"]
    subprocess.run(["git", "init", "-q", str(repo)], check=True)
    (repo / "f").write_text("x")
    subprocess.run(git + ["add", "f"], check=True)
    subprocess.run(git + ["commit", "-qm", "c"], check=True)
    subprocess.run(git + ["tag", "-a", "2.3.0-1.0", "-m", "release"], check=True)
    sha = subprocess.check_output(["git", "-C", str(repo), "rev-parse", "HEAD"]).decode().strip()

    def describe(name):
        return {"version": "2.3.0-1.0"}
    assert ppt.main(["ppt", "hello-world"], describe) == 0
    assert capsys.readouterr().out.strip() == "2.3.0-1.0"
    assert ppt.main(["ppt", "hello-world", str(repo)], describe) == 0
    assert capsys.readouterr().out.strip() == sha
    assert ppt.PackageVersion("hello-world", describe).get_version_sha_for_url(str(repo)) == sha
    assert ppt.main(["ppt"], describe) == 1


def test_save_properties_uploads_to_the_object_store(tmp_path, monkeypatch):
    from dcos_commons_amd.tools import save_properties

    monkeypatch.setenv("WORKSPACE", str(tmp_path))
    monkeypatch.setenv("SDK_OBJECT_STORE_ROOT", str(tmp_path / "store"))
    (tmp_path / "stub-universe.properties").write_text("STUB_UNIVERSE_URL=http://x/stub.json\n")
    assert save_properties.main(["save", "s3://bucket/ci/run-1"]) == 0
    assert (tmp_path / "store" / "bucket" / "ci" / "run-1" / "stub-universe.properties").read_text() == \
        "STUB_UNIVERSE_URL=http://x/stub.json\n"
    monkeypatch.setenv("WORKSPACE", str(tmp_path / "missing"))
    with pytest.raises(FileNotFoundError):
        save_properties.upload_to_s3("s3://bucket/ci")


@needs_native
def test_dcos_login_user_and_service_account(tmp_path, monkeypatch):
    """tools/dcos_login.py against the fake IAM: user/password and service-account logins, the
    attached cluster config carries a token the cluster accepts."""
    from dcos_commons_amd.testing.dcos_fakes import FakeDcosCluster
    from dcos_commons_amd.tools import dcos_login

    cluster = FakeDcosCluster().start()
    try:
        cluster.add_user("bootstrapuser", "deleteme")
        monkeypatch.setenv("CLUSTER_URL", cluster.url)
        monkeypatch.setenv("DCOS_DIR", str(tmp_path / "dcos"))
        path = dcos_login.login_session()
        text = open(path).read()
        token = text.split('dcos_acs_token = "')[1].split('"')[0]
        assert cluster.authorized(f"token={token}") and f'dcos_url = "{cluster.url}"' in text
        assert os.path.exists(os.path.join(os.path.dirname(path), "attached"))
        with pytest.raises(Exception):
            dcos_login.login(cluster.url, "bootstrapuser", "wrong")
        cred = cluster.add_service_account("ci-account")
        token = dcos_login.login(cluster.url, service_account_credential=cred)
        assert cluster.authorized(f"token={token}")
    finally:
        cluster.stop()


def test_validate_pip_freeze():
    from dcos_commons_amd.tools import validate_pip_freeze as v

    installed = {"pyyaml": "6.0.1", "requests": "2.31.0", "sdk-testing": "0.1"}
    good = "PyYAML==6.0.1\n# comment\nrequests==2.31.0  # pinned\n" \
           "git+https://github.com/acme/sdk-testing.git@abc#egg=x&validator-hint: name=sdk-testing version=SNAPSHOT\n"
    assert v.validate(good, installed) == []
    bad = "PyYAML>=6\nrequests==2.30.0\nsdk-testing==0.1\nsdk_testing==0.1\nmissing==1.0\n"
    problems = v.validate(bad, installed)
    assert any("not pinned" in p for p in problems) and any("duplicate" in p for p in problems)
    assert any("missing==1.0 is not installed" in p for p in problems)
    assert any("requests: requirements pin" in p for p in problems)
    # this interpreter's own packages validate against themselves
    import yaml

    assert v.validate(f"PyYAML=={yaml.__version__}\n") == []


def test_publish_aws_destination_from_env(monkeypatch):
    """tools/publish_aws.py ``s3_urls_from_env``: bucket / dir path / dir name defaults and the
    ``S3_URL`` / ``ARTIFACT_DIR`` overrides."""
    from dcos_commons_amd.tools import publish_aws as A

    for k in ("S3_BUCKET", "S3_DIR_PATH", "S3_DIR_NAME", "S3_URL", "ARTIFACT_DIR"):
        monkeypatch.delenv(k, raising=False)
    s3, http = A.s3_urls_from_env("hello-world")
    assert s3.startswith("s3://infinity-artifacts/autodelete7d/hello-world/") and http == ""
    name = s3.rsplit("/", 1)[1]
    assert len(name.split("-")) == 3 and len(name.split("-")[2]) == 16   # <date>-<time>-<16 random>
    monkeypatch.setenv("S3_BUCKET", "b")
    monkeypatch.setenv("S3_DIR_PATH", "/nightly/")
    monkeypatch.setenv("S3_DIR_NAME", "run-7")
    assert A.s3_urls_from_env("pkg") == ("s3://b/nightly/pkg/run-7", "")
    monkeypatch.setenv("S3_URL", "s3://other/x/y/")
    monkeypatch.setenv("ARTIFACT_DIR", "https://cdn.example.com/x/y/")
    assert A.s3_urls_from_env("pkg") == ("s3://other/x/y", "https://cdn.example.com/x/y")
    monkeypatch.setenv("S3_URL", "https://not-s3")
    with pytest.raises(ValueError):
        A.s3_urls_from_env("pkg")


def test_publish_azure_requires_account_and_container(monkeypatch, tmp_path):
    from dcos_commons_amd.tools import publish_azure as Z

    monkeypatch.delenv("AZURE_STORAGE_ACCOUNT", raising=False)
    monkeypatch.setenv("AZURE_CONTAINER_NAME", "c")
    with pytest.raises(ValueError, match="AZURE_STORAGE_ACCOUNT"):
        Z.azure_publisher("pkg", "1.0", str(tmp_path), [])
    monkeypatch.setenv("AZURE_STORAGE_ACCOUNT", "acct")
    monkeypatch.delenv("AZURE_DIR_PATH", raising=False)
    assert Z.azure_directory_from_env() == "https://acct.blob.core.windows.net/c"
    monkeypatch.setenv("AZURE_DIR_PATH", "/nested/dir/")
    assert Z.azure_directory_from_env() == "https://acct.blob.core.windows.net/c/nested/dir"
