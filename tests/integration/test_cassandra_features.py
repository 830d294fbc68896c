"""Cassandra features on a strict-mode local cluster (synthetic task payloads).

Reference: frameworks/cassandra/tests/{test_racks.py, test_overlay.py, test_custom_domain.py,
test_tls.py, test_backup_and_restore.py, test_auth.py, test_sanity.py}; test_toggle_tls.py is
test_cassandra_toggle_tls.py. Without Cassandra
binaries the checks stop at what the scheduler hands the nodes, rendered the way bootstrap renders
it inside the task: ``cassandra-rackdc.properties`` names the node's zone as its rack when the
placement references zones and the configured rack otherwise; the overlay network gives nodes
container addresses and no host ports; a custom domain replaces the autoip endpoint domain;
turning transport encryption on (with and without plaintext) and off again rolls every node,
mounting keystore artifacts from the secret store only while it is on; backup and restore plans
run their phases in order; authentication settings reach ``cassandra.yaml``.
"""
import json
import urllib.parse

import pytest

from dcos_commons_amd.specification.yaml.template_utils import render_mustache
from dcos_commons_amd.testing.sdk import (sdk_agents, sdk_cmd, sdk_install, sdk_networks, sdk_plan, sdk_recovery,
                                          sdk_security, sdk_tasks, sdk_upgrade)
from tests.integration.conftest import make_cluster
from tests.integration.test_cassandra import ONCE_TASKS, PACKAGE

SVC = "cassandra"
ACCOUNT, ACCOUNT_SECRET = "cassandra-principal", "cassandra-secret"


@pytest.fixture(scope="module")
def local_cluster():
    c = make_cluster(executor="synthetic", finish_tasks=ONCE_TASKS, dcos_security=True)
    sdk_security.create_service_account(ACCOUNT, ACCOUNT_SECRET)
    yield c
    c.shutdown()


pytestmark = pytest.mark.usefixtures("local_cluster")
ACCOUNT_OPTIONS = {"service": {"service_account": ACCOUNT, "service_account_secret": ACCOUNT_SECRET}}


def _server_info(node):
    return next(t["info"] for t in sdk_cmd.service_request("GET", SVC, f"/v1/pod/node-{node}/info").json()
                if t["info"]["name"] == f"node-{node}-server")


def _rendered(node, config):
    """A node's config file as bootstrap renders it: the template the scheduler serves under
    ``CONFIG_TEMPLATE_<name>``, rendered against the task's environment."""
    info = _server_info(node)
    env = {v["name"]: v.get("value", "") for v in info["command"]["environment"]["variables"]}
    sandbox_path = env[f"CONFIG_TEMPLATE_{config.upper().replace('-', '_')}"].split(",")[0]   # "<fetched template>,<dest>"
    url = next(u["value"] for u in info["command"]["uris"] if u.get("outputFile") == sandbox_path)
    template = sdk_cmd.service_request("GET", SVC, urllib.parse.urlparse(url).path, retry=False).text
    return render_mustache(config, template, env, [])


def _rack(node):
    return next(l.split("=", 1)[1] for l in _rendered(node, "rackdc").splitlines() if l.startswith("rack="))


def _agent_zones():
    return {a["hostname"]: a["zone"] for a in sdk_agents.get_agents()}


def test_rack_follows_zone_placement():
    sdk_install.install(PACKAGE, SVC, 3, additional_options={
        "nodes": {"placement_constraint": '[["@zone", "GROUP_BY", "1"]]'}})
    try:
        zones = _agent_zones()
        tasks = {t.name: t for t in sdk_tasks.get_service_tasks(SVC)}
        for i in range(3):
            rack = _rack(i)
            assert rack != "rack1" and rack == zones[tasks[f"node-{i}-server"].host], rack
    finally:
        sdk_install.uninstall(PACKAGE, SVC)


def test_custom_rack_without_zone_placement():
    sdk_install.install(PACKAGE, SVC, 3, additional_options={"service": {"rack": "not-rack1"}})
    try:
        assert {_rack(i) for i in range(3)} == {"not-rack1"}
    finally:
        sdk_install.uninstall(PACKAGE, SVC)


def test_overlay_network():
    sdk_install.install(PACKAGE, SVC, 3, additional_options=sdk_networks.ENABLE_VIRTUAL_NETWORKS_OPTIONS)
    try:
        for t in sdk_tasks.get_service_tasks(SVC):
            sdk_networks.check_task_network(t.name)
            assert "ports" not in t.resources
        assert sdk_networks.get_endpoint_names(PACKAGE, SVC) == ["native-client"]
        sdk_networks.check_endpoint_on_overlay(PACKAGE, SVC, "native-client", 3)
        # seeds are the nodes' autoip names, which resolve to their overlay addresses
        seeds = sdk_cmd.service_request("GET", SVC, "/v1/seeds").json()["seeds"]
        assert seeds == [f"node-{i}-server.{SVC}.autoip.dcos.thisdcos.directory" for i in range(2)], seeds
    finally:
        sdk_install.uninstall(PACKAGE, SVC)


def test_custom_domain():
    domain = "custom.example.tld"
    sdk_install.install(PACKAGE, SVC, 3, additional_options={"service": {"security": {"custom_domain": domain}}})
    try:
        assert sdk_networks.get_endpoint_names(PACKAGE, SVC) == ["native-client"]
        ep = sdk_networks.get_endpoint(PACKAGE, SVC, "native-client")
        assert set(ep) == {"address", "dns"} and len(ep["address"]) == 3 and len(ep["dns"]) == 3
        assert all(len(a.split(":")) == 2 for a in ep["address"])
        assert all(domain in d for d in ep["dns"]), ep["dns"]
    finally:
        sdk_install.uninstall(PACKAGE, SVC)


def _keystore_volumes(node):
    info = _server_info(node)
    return sorted(v["containerPath"] for v in info.get("container", {}).get("volumes", [])
                  if v.get("source", {}).get("type") == "SECRET")


def _toggle(enabled, allow_plaintext):
    ids = sdk_tasks.get_task_ids(SVC, "node")
    sdk_upgrade.update_or_upgrade_or_downgrade(
        PACKAGE, SVC, to_version=None, expected_running_tasks=3,
        to_options={"service": {"security": {"transport_encryption": {"enabled": enabled,
                                                                        "allow_plaintext": allow_plaintext}}}})
    sdk_tasks.check_tasks_updated(SVC, "node", ids)
    sdk_plan.wait_for_completed_deployment(SVC)


def test_custom_jmx_port():
    """cassandra.jmx_port rolls every node onto the new JMX port (reference test_sanity.py
    ``test_custom_jmx_port``; there ``lsof`` sees Cassandra listen on it)."""
    sdk_install.install(PACKAGE, SVC, 3)
    try:
        ids = sdk_tasks.get_task_ids(SVC, "node")
        sdk_upgrade.update_or_upgrade_or_downgrade(PACKAGE, SVC, to_version=None, expected_running_tasks=3,
                                                   to_options={"cassandra": {"jmx_port": 7200}})
        sdk_tasks.check_tasks_updated(SVC, "node", ids)
        sdk_plan.wait_for_completed_deployment(SVC)
        for i in range(3):
            env = {v["name"]: v.get("value", "") for v in _server_info(i)["command"]["environment"]["variables"]}
            assert env["JMX_PORT"] == "7200"
    finally:
        sdk_install.uninstall(PACKAGE, SVC)


def test_tls_recovery():
    """Every node of a TLS service replaced in turn: each replacement gets its TLS artifacts
    mounted again and only the seed-list restarts touch other pods (reference test_tls.py
    ``test_tls_recovery``)."""
    sdk_install.install(PACKAGE, SVC, 3, additional_options=dict(
        ACCOUNT_OPTIONS, service=dict(ACCOUNT_OPTIONS["service"],
                                      security={"transport_encryption": {"enabled": True}})))
    try:
        rc, out, _ = sdk_cmd.svc_cli(PACKAGE, SVC, "pod list")
        pods = json.loads(out)
        for pod in pods:
            i = int(pod.split("-")[1])
            # replacing a seed (the first two nodes) restarts the others with the new seed list
            sdk_recovery.check_permanent_recovery(PACKAGE, SVC, pod, recovery_timeout_s=300,
                                                  pods_with_updated_tasks=pods if i < 2 else None)
            vols = _keystore_volumes(i)
            assert any(v.endswith("node.keystore") for v in vols) and any(v.endswith("node.truststore") for v in vols)
    finally:
        sdk_install.uninstall(PACKAGE, SVC)


def test_backup_and_restore_plans():
    sdk_install.install(PACKAGE, SVC, 3)
    try:
        params = {"SNAPSHOT_NAME": "snap", "CASSANDRA_KEYSPACES": "testspace1 testspace2",
                  "S3_BUCKET_NAME": "bucket", "AWS_ACCESS_KEY_ID": "key", "AWS_SECRET_ACCESS_KEY": "secret",
                  "AWS_REGION": "us-west-2"}
        sdk_plan.start_plan(SVC, "backup-s3", parameters=params)
        plan = sdk_plan.wait_for_completed_plan(SVC, "backup-s3")
        assert [p["name"] for p in plan["phases"]] == ["backup-schema", "create-snapshots", "upload-backups",
                                                        "cleanup-snapshots"]
        sdk_plan.start_plan(SVC, "restore-s3", parameters=params)
        plan = sdk_plan.wait_for_completed_plan(SVC, "restore-s3")
        assert [p["name"] for p in plan["phases"]][0] == "fetch-s3"
        assert all(p["status"] == "COMPLETE" for p in plan["phases"])
        # the parameters reached the one-shot tasks of the plan
        info = next(t["info"] for t in sdk_cmd.service_request("GET", SVC, "/v1/pod/node-0/info").json()
                    if t["info"]["name"] == "node-0-fetch-s3")
        env = {v["name"]: v.get("value") for v in info["command"]["environment"]["variables"]}
        assert env["S3_BUCKET_NAME"] == "bucket" and env["SNAPSHOT_NAME"] == "snap"
        # the servers kept running through both plans
        sdk_tasks.check_running(SVC, 3)
    finally:
        sdk_install.uninstall(PACKAGE, SVC)


def test_authentication_settings():
    """PasswordAuthenticator with the superuser's password from the secret store and
    CassandraAuthorizer, then authorization switched off by an update that rolls every node
    (reference cassandra config.json ``service.security.authentication/authorization``)."""
    c = sdk_install._cluster()
    c.secrets[f"{SVC.strip('/')}/superuser-pw"] = b"s3cret"
    sdk_install.install(PACKAGE, SVC, 3, additional_options={"service": {"security": {
        "authentication": {"enabled": True, "superuser": {"name": "admin",
                                                           "password_secret_path": f"{SVC.strip('/')}/superuser-pw"}},
        "authorization": {"enabled": True, "roles_validity_in_ms": 5000}}}})
    try:
        for i in range(3):
            cfg = _rendered(i, "cassandra")
            assert "authenticator: PasswordAuthenticator" in cfg and "authorizer: CassandraAuthorizer" in cfg
            assert "roles_validity_in_ms: 5000" in cfg
            assert _keystore_volumes(i) == ["superuser/password"]
        init = next(t["info"] for t in sdk_cmd.service_request("GET", SVC, "/v1/pod/node-0/info").json()
                    if t["info"]["name"] == "node-0-init_system_keyspaces")
        assert "CREATE ROLE" in init["command"]["value"]
        ids = sdk_tasks.get_task_ids(SVC, "node")
        sdk_upgrade.update_or_upgrade_or_downgrade(
            PACKAGE, SVC, to_version=None, expected_running_tasks=3,
            to_options={"service": {"security": {"authorization": {"enabled": False}}}})
        sdk_tasks.check_tasks_updated(SVC, "node", ids)
        sdk_plan.wait_for_completed_deployment(SVC)
        cfg = _rendered(0, "cassandra")
        assert "authenticator: PasswordAuthenticator" in cfg and "authorizer: AllowAllAuthorizer" in cfg
    finally:
        sdk_install.uninstall(PACKAGE, SVC)


def test_secure_jmx_g1_and_metrics_toggle():
    """Secure JMX (its credentials from the cluster's secret store), the G1 collector and the
    metrics reporter, set at install and then changed by a package update that rolls every node."""
    c = sdk_install._cluster()
    for name, data in (("jmx/password", b"admin secret\n"), ("jmx/access", b"admin readwrite\n"),
                       ("jmx/keystore", b"KS"), ("jmx/keystore-pass", b"changeit\n")):
        c.secrets[f"{SVC.strip('/')}/{name}"] = data
    jmx = {"enabled": True, "password_file": f"{SVC.strip('/')}/jmx/password",
           "access_file": f"{SVC.strip('/')}/jmx/access", "key_store": f"{SVC.strip('/')}/jmx/keystore",
           "key_store_password_file": f"{SVC.strip('/')}/jmx/keystore-pass"}
    sdk_install.install(PACKAGE, SVC, 3, additional_options={"service": {"jmx": jmx},
                                                             "nodes": {"heap": {"gc": "G1"}}})
    try:
        for i in range(3):
            info = _server_info(i)
            secret_files = sorted(v["containerPath"] for v in info.get("container", {}).get("volumes", [])
                                  if v.get("source", {}).get("type") == "SECRET")
            assert secret_files == ["jmx/access_file", "jmx/key_store", "jmx/key_store_password_file",
                                    "jmx/password_file"], secret_files
            assert "bash ./jmx-ssl-setup.sh" in info["command"]["value"]
            assert "metricsReporterConfigFile" in info["command"]["value"]
        assert "-XX:+UseG1GC" in _rendered(0, "jvm")
        assert "rmi.port=7198" in _rendered(0, "jmx-ssl-setup")

        ids = sdk_tasks.get_task_ids(SVC, "node")
        sdk_upgrade.update_or_upgrade_or_downgrade(
            PACKAGE, SVC, to_version=None, expected_running_tasks=3,
            to_options={"cassandra": {"metrics_enabled": False}, "nodes": {"heap": {"gc": "CMS"}}})
        sdk_tasks.check_tasks_updated(SVC, "node", ids)
        sdk_plan.wait_for_completed_deployment(SVC)
        assert "metricsReporterConfigFile" not in _server_info(0)["command"]["value"]
        assert "-XX:+UseConcMarkSweepGC" in _rendered(0, "jvm")
    finally:
        sdk_install.uninstall(PACKAGE, SVC)
