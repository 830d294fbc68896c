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
