"""HDFS features on a strict-mode local cluster (synthetic task payloads).

Reference: frameworks/hdfs/tests/{test_overlay.py, test_racks.py, test_upgrade.py}; test_tls.py is
test_hdfs_tls.py.
Every node type joins the overlay network (container addresses, no host ports) while the
``hdfs-site.xml`` / ``core-site.xml`` endpoints keep being served; zone placement makes data nodes rack-aware
(each sees its zone); the package upgrades to the newest published version and back.
"""
import pytest

from dcos_commons_amd.testing.sdk import (sdk_agents, sdk_cmd, sdk_install, sdk_networks, sdk_plan, sdk_security,
                                          sdk_tasks, sdk_upgrade)
from tests.integration.conftest import make_cluster
from tests.integration.test_hdfs import DEFAULT_TASK_COUNT, FINISH_TASKS, PACKAGE

SVC = "hdfs"
ACCOUNT, ACCOUNT_SECRET = "hdfs-principal", "hdfs-secret"
# data nodes pass their first readiness check after 1 s instead of the default 10 s
FAST = {"data_node": {"readiness_check": {"delay": 1, "interval": 1}}}


def _opts(extra):
    from dcos_commons_amd.testing.sdk.sdk_utils import merge_dictionaries

    return merge_dictionaries(FAST, extra)


@pytest.fixture(scope="module")
def local_cluster():
    c = make_cluster(executor="synthetic", finish_tasks=FINISH_TASKS, dcos_security=True, honor_check_delays=False)
    sdk_security.create_service_account(ACCOUNT, ACCOUNT_SECRET)
    yield c
    c.shutdown()


pytestmark = pytest.mark.usefixtures("local_cluster")


def _info(task):
    pod = task.rsplit("-", 1)[0]
    return next(t["info"] for t in sdk_cmd.service_request("GET", SVC, f"/v1/pod/{pod}/info").json()
                if t["info"]["name"] == task)


def test_tasks_and_endpoints_on_overlay():
    sdk_install.install(PACKAGE, SVC, DEFAULT_TASK_COUNT,
                        additional_options=_opts(sdk_networks.ENABLE_VIRTUAL_NETWORKS_OPTIONS))
    try:
        tasks = sdk_tasks.get_service_tasks(SVC)
        assert len(tasks) == DEFAULT_TASK_COUNT
        for t in tasks:
            sdk_networks.check_task_network(t.name)
            assert sdk_networks.get_task_ip(SVC, t.name).startswith("9."), t.name
            assert "ports" not in t.resources, t.name
        assert set(sdk_networks.get_endpoint_names(PACKAGE, SVC)) >= {"hdfs-site.xml", "core-site.xml"}
        assert "dfs.namenode.rpc-address" in sdk_networks.get_endpoint_string(PACKAGE, SVC, "hdfs-site.xml")
    finally:
        sdk_install.uninstall(PACKAGE, SVC)


def test_detect_racks():
    sdk_install.install(PACKAGE, SVC, DEFAULT_TASK_COUNT, additional_options=_opts({
        "data_node": {"placement": '[["@zone", "GROUP_BY", "3"]]'}}))
    try:
        zones = {a["hostname"]: a["zone"] for a in sdk_agents.get_agents()}
        data = [t for t in sdk_tasks.get_service_tasks(SVC) if t.name.startswith("data-")]
        assert len(data) == 3
        assert len({zones[t.host] for t in data}) == 3                 # spread over the 3 zones
        for t in data:
            env = {v["name"]: v.get("value") for v in _info(t.name)["command"]["environment"]["variables"]}
            assert env["PLACEMENT_REFERENCED_ZONE"] == "true" and env["ZONE"] == zones[t.host]
    finally:
        sdk_install.uninstall(PACKAGE, SVC)


def test_upgrade_and_downgrade():
    sdk_upgrade.test_upgrade(PACKAGE, SVC, DEFAULT_TASK_COUNT, from_options=FAST, to_options=FAST)
    try:
        sdk_plan.wait_for_completed_deployment(SVC)
        sdk_tasks.check_running(SVC, DEFAULT_TASK_COUNT)
        sdk_upgrade.test_downgrade(PACKAGE, SVC, DEFAULT_TASK_COUNT)
        sdk_plan.wait_for_completed_deployment(SVC)
    finally:
        sdk_install.uninstall(PACKAGE, SVC)


def test_kerberos_tls_and_metrics_together():
    """Kerberos (keytab from the secret store, krb5.conf), HTTPS (ssl-server/ssl-client from the
    provisioned TLS artifacts) and the metrics2 StatsD sinks, all on: every node gets the templates
    and the flags that use them."""
    c = sdk_install._cluster()
    c.secrets["__dcos_base64__hdfs_keytab"] = b"not-a-real-keytab"
    sdk_install.install(PACKAGE, SVC, DEFAULT_TASK_COUNT, additional_options=_opts({
        "service": {"service_account": ACCOUNT, "service_account_secret": ACCOUNT_SECRET,
                    "security": {"transport_encryption": {"enabled": True},
                                 "kerberos": {"enabled": True, "realm": "EXAMPLE.COM",
                                              "kdc": {"hostname": "kdc.example.com", "port": 88}}}},
        "hdfs": {"metrics_enabled": True}}))
    try:
        for task in ("journal-0-node", "name-0-node", "name-1-node", "data-0-node"):
            info = _info(task)
            env = {v["name"]: v.get("value", "") for v in info["command"]["environment"]["variables"]}
            for cfg in ("KRB5", "SSL_SERVER", "SSL_CLIENT", "HADOOP_METRICS2"):
                assert f"CONFIG_TEMPLATE_{cfg}" in env, (task, cfg)
            assert env["SECURITY_KERBEROS_KDC_HOSTNAME"] == "kdc.example.com"
            assert env["SECURITY_KERBEROS_REALM"] == "EXAMPLE.COM"
            assert "-Djava.security.krb5.conf=" in info["command"]["value"]
        site = sdk_networks.get_endpoint_string(PACKAGE, SVC, "hdfs-site.xml")
        assert "HTTPS_ONLY" in site and "ssl-server.xml" in site
    finally:
        sdk_install.uninstall(PACKAGE, SVC)
