"""HDFS with transport encryption on a strict-mode local cluster (synthetic task payloads).

Reference: frameworks/hdfs/tests/test_tls.py, on one TLS service: it is healthy; every journal,
name and data node gets keystore artifacts signed by the cluster CA and ``hdfs-site.xml`` switches
to ``HTTPS_ONLY`` with the HTTPS addresses (the reference writes and reads data through a TLS
client); each node type has its HTTPS port reserved and advertised (the reference curls it); every
pod replaced in turn comes back with fresh TLS artifacts and nothing else relaunches.
"""
import pytest

from dcos_commons_amd.testing.sdk import sdk_install, sdk_networks, sdk_plan, sdk_recovery, sdk_security, sdk_tasks
from tests.integration.test_hdfs import DEFAULT_TASK_COUNT, PACKAGE
from tests.integration.test_hdfs_features import ACCOUNT, ACCOUNT_SECRET, SVC, _info, _opts, local_cluster  # noqa: F401

HTTPS_PORTS = {"journal": 8481, "name": 9006, "data": 9007}   # the package defaults


@pytest.fixture(scope="module", autouse=True)
def hdfs_service(local_cluster):  # noqa: F811
    sdk_install.install(PACKAGE, SVC, DEFAULT_TASK_COUNT, additional_options=_opts({
        "service": {"service_account": ACCOUNT, "service_account_secret": ACCOUNT_SECRET,
                    "security": {"transport_encryption": {"enabled": True}}}}))
    yield {"package_name": PACKAGE, "service": {"name": SVC}}
    sdk_install.uninstall(PACKAGE, SVC)
    assert not [n for n in sdk_security.list_secrets(SVC) if n.endswith(("keystore", "truststore"))]


def check_healthy():
    sdk_plan.wait_for_completed_deployment(SVC)
    sdk_plan.wait_for_completed_recovery(SVC)
    sdk_tasks.check_running(SVC, DEFAULT_TASK_COUNT)


def _secret_volumes(task):
    return [v["containerPath"] for v in _info(task).get("container", {}).get("volumes", [])
            if v.get("source", {}).get("type") == "SECRET"]


def test_healthy():
    check_healthy()


def test_tls_artifacts_and_https_only():
    site = sdk_networks.get_endpoint_string(PACKAGE, SVC, "hdfs-site.xml")
    assert "HTTPS_ONLY" in site and "dfs.namenode.https-address" in site
    for task in ("journal-0-node", "name-0-node", "name-1-node", "data-0-node"):
        vols = _secret_volumes(task)
        assert any(v.endswith(".keystore") for v in vols) and any(v.endswith(".truststore") for v in vols), \
            (task, vols)
    # one signed certificate per TLS-enabled task, stored under the service's secret namespace
    names = sdk_security.list_secrets(SVC)
    assert sum(1 for n in names if n.endswith("keystore")) >= 6, names
    assert len(sdk_install._cluster().dcos.signed) >= 6


@pytest.mark.parametrize("node_type,port", sorted(HTTPS_PORTS.items()))
def test_verify_https_ports(node_type, port):
    """The node's HTTPS port is reserved for it and advertised under its name."""
    info = _info(f"{node_type}-0-node")
    ports = {p["name"]: p["number"] for p in info["discovery"]["ports"]["ports"]}
    assert ports[f"{node_type}-https"] == port, ports
    ranges = [(int(r["begin"]), int(r["end"])) for res in info["resources"] if res["name"] == "ports"
              for r in res["ranges"]["range"]]
    assert any(b <= port <= e for b, e in ranges), ranges


def test_tls_recovery():
    for pod in ("name-0", "name-1", "data-0", "data-1", "data-2", "journal-0", "journal-1", "journal-2"):
        sdk_recovery.check_permanent_recovery(PACKAGE, SVC, pod, recovery_timeout_s=300)
        vols = _secret_volumes(f"{pod}-node")
        assert any(v.endswith(".keystore") for v in vols), (pod, vols)
    check_healthy()
