"""Build -> publish -> install on the local cluster, through the packaging tools.

Reference flow: ``tools/build_package.sh <fw> <dir> local`` hosts a stub universe over HTTP,
``dcos package repo add`` registers it and ``dcos package install --package-version=...``
deploys it (frameworks/*/tests run against exactly such stub universes); ``.dcos`` files carry a
package and its artifacts into air-gapped clusters (tools/publish_dcos_file.py). Here the same
steps use ``tools.publish_http`` / ``tools.publish_dcos_file`` and the local Cosmos.
"""
import os

import pytest

from dcos_commons_amd.testing.sdk import sdk_cmd, sdk_install, sdk_marathon, sdk_plan, sdk_tasks
from dcos_commons_amd.tools import build_package
from dcos_commons_amd.tools.publish_dcos_file import build_dcos_file
from dcos_commons_amd.tools.publish_http import HTTPPublisher
from tests.integration import hw_config as config
from tests.integration.conftest import make_cluster
from tests.test_tools import needs_native

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
HELLO_DIR = os.path.join(ROOT, "frameworks", "helloworld")
SVC = "hello-world-packaged"

pytestmark = needs_native


@pytest.fixture(scope="module")
def built(tmp_path_factory):
    out = tmp_path_factory.mktemp("build")
    artifacts = build_package.build_artifacts(config.PACKAGE_NAME, HELLO_DIR, str(out / "artifacts"))
    c = make_cluster()
    pub = HTTPPublisher(config.PACKAGE_NAME, "2.0.0-http", os.path.join(HELLO_DIR, "universe"), artifacts,
                        http_dir=str(out / "http"))
    url = pub.start()
    yield c, url, artifacts, out
    pub.stop()
    c.shutdown()


def test_install_from_published_stub_universe(built):
    c, url, _, _ = built
    rc, out, _ = sdk_cmd.run_cli(f"package repo add local-http {url}")
    assert rc == 0 and "hello-world 2.0.0-http" in out
    assert "local-http" in sdk_cmd.run_cli("package repo list")[1]
    sdk_install.install(config.PACKAGE_NAME, SVC, config.DEFAULT_TASK_COUNT, package_version="2.0.0-http")
    env = sdk_marathon.get_config(SVC)["env"]
    assert env["PACKAGE_VERSION"] == "2.0.0-http"
    assert env["BOOTSTRAP_URI"] == url.rsplit("/", 1)[0] + "/bootstrap.zip"
    # the world tasks ran their real commands in their sandboxes
    task = sdk_tasks.get_service_tasks(SVC, "world-0-server")[0]
    assert os.path.exists(os.path.join(c.behavior.sandbox_of(task.id), "world-a", "out"))


def test_upgrade_to_an_airgap_bundle(built):
    c, _, artifacts, out = built
    bundle = build_dcos_file(config.PACKAGE_NAME, "2.1.0-airgap", os.path.join(HELLO_DIR, "universe"), artifacts,
                             str(out / "bundle"))
    sdk_cmd.run_cli(f"package repo add airgap {bundle}", check=True)
    # the bundle's artifacts are staged in the cluster: found by name, nothing is downloaded
    assert c.resolve_artifact("bundle://hello-world/2.1.0-airgap/sdk-cli-linux").endswith("sdk-cli-linux")
    ids = sdk_tasks.get_task_ids(SVC, "")
    c.cosmos.update(SVC, version="2.1.0-airgap")
    sdk_tasks.check_tasks_updated(SVC, "", ids)      # the version is in every task's env
    sdk_plan.wait_for_completed_deployment(SVC)
    config.check_running(SVC)
    assert sdk_marathon.get_config(SVC)["env"]["PACKAGE_VERSION"] == "2.1.0-airgap"


def test_uninstall_packaged_service(built):
    sdk_install.uninstall(config.PACKAGE_NAME, SVC)
    assert not sdk_marathon.app_exists(SVC)


@pytest.mark.parametrize("store", ["aws", "azure"])
def test_install_from_object_store(built, store, tmp_path, monkeypatch):
    """tools/publish_aws.py / publish_azure.py: artifacts and the stub universe go to a bucket
    (container) under a unique directory; the repo URL is the bucket's HTTP address."""
    from dcos_commons_amd.tools.publish_aws import aws_publisher
    from dcos_commons_amd.tools.publish_azure import azure_publisher
    from dcos_commons_amd.tools.universe.uploaders import LocalObjectStore

    c, _, artifacts, _ = built
    monkeypatch.setenv("SDK_OBJECT_STORE_ROOT", str(tmp_path / "store"))
    monkeypatch.setenv("AZURE_STORAGE_ACCOUNT", "infinityartifacts")
    monkeypatch.setenv("AZURE_CONTAINER_NAME", "artifacts")
    monkeypatch.setenv("UNIVERSE_URL_PATH", str(tmp_path / "url.txt"))
    version = f"3.0.0-{store}"
    make = aws_publisher if store == "aws" else azure_publisher
    url = make(config.PACKAGE_NAME, version, os.path.join(HELLO_DIR, "universe"), artifacts).upload(str(tmp_path / "w"))
    try:
        assert open(tmp_path / "url.txt").read().strip() == url
        assert ("/infinity-artifacts/autodelete7d/" if store == "aws" else "/infinityartifacts/artifacts/") in url
        bucket_dir = os.path.dirname(url.split("/", 3)[3])
        for a in artifacts:   # every artifact landed next to the stub universe
            assert os.path.exists(os.path.join(str(tmp_path / "store"), bucket_dir, os.path.basename(a)))
        rc, out, _ = sdk_cmd.run_cli(f"package repo add {store}-repo {url}")
        assert rc == 0 and f"hello-world {version}" in out
        svc = f"{SVC}-{store}"
        sdk_install.install(config.PACKAGE_NAME, svc, config.DEFAULT_TASK_COUNT, package_version=version)
        try:
            env = sdk_marathon.get_config(svc)["env"]
            assert env["PACKAGE_VERSION"] == version and env["BOOTSTRAP_URI"].startswith(url.rsplit("/", 1)[0])
            sdk_plan.wait_for_completed_deployment(svc)
        finally:
            sdk_install.uninstall(config.PACKAGE_NAME, svc)
        sdk_cmd.run_cli(f"package repo remove {store}-repo")
    finally:
        LocalObjectStore.get(str(tmp_path / "store")).stop()
