"""helloworld transport encryption on a strict-mode local cluster.

Reference: frameworks/helloworld/tests/test_tls.py. The cluster runs the DC/OS IAM, secrets and CA
services; the scheduler logs in with its service account, has a certificate signed for every
``transport-encryption`` entry, stores the artifacts in the secret store and mounts them into the
tasks: PEM certificate / key / CA files for ``TLS``, PKCS#12 keystore and truststore for
``KEYSTORE``. The end-entity certificate names the task's autoip host, chains to the cluster CA
and its truststore holds that CA; changing a task's discovery prefix rolls it with a certificate
for the new name; uninstalling removes every artifact from the secret store.
"""
import base64

import pytest

from dcos_commons_amd.offer.evaluate.security import native
from dcos_commons_amd.testing.sdk import (sdk_cmd, sdk_hosts, sdk_install, sdk_marathon, sdk_plan, sdk_security,
                                          sdk_utils)
from tests.integration import hw_config as config
from tests.integration.conftest import make_cluster

DISCOVERY_TASK_PREFIX = "discovery-prefix"
ACCOUNT, ACCOUNT_SECRET = config.SERVICE_NAME, config.SERVICE_NAME + "-secret"
ARTIFACT_SUFFIXES = ("certificate", "private-key", "root-ca-certificate", "keystore", "truststore")


@pytest.fixture(scope="module")
def local_cluster():
    c = make_cluster(dcos_security=True)
    yield c
    c.shutdown()


@pytest.fixture(scope="module", autouse=True)
def tls_service(local_cluster):
    sdk_security.create_service_account(ACCOUNT, ACCOUNT_SECRET)
    sdk_install.install(config.PACKAGE_NAME, config.SERVICE_NAME, 7, additional_options={
        "service": {"yaml": "tls", "service_account": ACCOUNT, "service_account_secret": ACCOUNT_SECRET},
        "hello": {"count": 2}, "tls": {"discovery_task_prefix": DISCOVERY_TASK_PREFIX}})
    sdk_plan.wait_for_completed_deployment(config.SERVICE_NAME)
    yield
    sdk_install.uninstall(config.PACKAGE_NAME, config.SERVICE_NAME)
    sdk_security.delete_service_account(ACCOUNT, ACCOUNT_SECRET)
    # every TLS artifact left the secret store
    leftovers = [s for s in sdk_security.list_secrets(config.SERVICE_NAME)
                 if any(s.endswith(x) for x in ARTIFACT_SUFFIXES)]
    assert not leftovers, leftovers


def _task_file(task, path):
    @sdk_utils.retry(timeout_s=30, interval_s=0.5)
    def read():
        rc, out, _ = sdk_cmd.service_task_exec(config.SERVICE_NAME, task, f"cat {path}")
        assert rc == 0 and out, (task, path)
        return out
    return read()


def _task_bytes(task, path):
    rc, out, _ = sdk_cmd.service_task_exec(config.SERVICE_NAME, task, f"base64 -w0 {path}")
    assert rc == 0, (task, path)
    return base64.b64decode(out.strip())


def _ca_bundle():
    c = sdk_install._cluster()
    return c.dcos.root_cert


def test_tls_basic_artifacts():
    n = native()
    cert = _task_file("artifacts-0-node", "artifacts.crt")
    key = _task_file("artifacts-0-node", "artifacts.key")
    ca = _task_file("artifacts-0-node", "artifacts.ca")
    info = n.cert_info(cert)
    assert info["subject"].startswith("CN=") or "CN=" in info["subject"]
    cn = [p for p in info["subject"].split(",") if p.startswith("CN=")][0][3:]
    assert cn in sdk_hosts.autoip_host(config.SERVICE_NAME, "artifacts-0-node")
    assert info["dns"] == [sdk_hosts.autoip_host(config.SERVICE_NAME, "artifacts-0-node")]
    assert "BEGIN PRIVATE KEY" in key
    # the chain (end entity + intermediate) verifies against the cluster's root CA
    assert ca.strip() == _ca_bundle().strip()
    assert n.verify_chain(cert, _ca_bundle(), cert[cert.find("-----END CERTIFICATE-----") + 25:] or None)
    # every pod instance got its own certificate
    other = n.cert_info(_task_file("artifacts-1-node", "artifacts.crt"))
    assert other["dns"] == [sdk_hosts.autoip_host(config.SERVICE_NAME, "artifacts-1-node")]


def test_java_keystore_and_truststore():
    n = native()
    keystore = _task_bytes("artifacts-0-node", "store.keystore")
    truststore = _task_bytes("artifacts-0-node", "store.truststore")
    # the keystore holds the private key and the task's certificate chain, the truststore only
    # the cluster's root CA (reference alias "dcos-root")
    n_certs, has_key = n.pkcs12_inspect(keystore, "notsecure")
    assert has_key and n_certs >= 2
    n_certs, has_key = n.pkcs12_inspect(truststore, "notsecure")
    assert not has_key and n_certs == 1
    import subprocess

    dump = subprocess.run(["openssl", "pkcs12", "-nokeys", "-passin", "pass:notsecure"], input=truststore,
                          capture_output=True)
    if dump.returncode == 0:
        assert b"dcos-root" in dump.stdout and b"DC/OS Root CA" in dump.stdout
    # a KEYSTORE-only task gets no PEM files
    rc, _, _ = sdk_cmd.service_task_exec(config.SERVICE_NAME, "gateway-0-server", "ls gateway.crt")
    assert rc != 0
    assert _task_bytes("gateway-0-server", "gateway.keystore")


def test_tls_nginx():
    """The webserver task serves HTTPS with its mounted PEM certificate and key; a client in
    another task, trusting only the cluster CA it was given, verifies the chain and the
    certificate's name (the task's autoip host) and gets 200 (reference test_tls.py: NGINX and the
    keystore app's ``truststoretest``)."""
    info = next(t["info"] for t in sdk_cmd.service_request("GET", config.SERVICE_NAME,
                                                             "/v1/pod/webserver-0/info").json())
    port = next(p["number"] for p in info["discovery"]["ports"]["ports"] if p["name"] == "web-https")
    host = sdk_hosts.autoip_host(config.SERVICE_NAME, "webserver-0-https")

    @sdk_utils.retry(timeout_s=30, interval_s=0.5)
    def fetch():
        rc, out, err = sdk_cmd.service_task_exec(
            config.SERVICE_NAME, "artifacts-0-node",
            f"python3 -m dcos_commons_amd.testing.tls_probe get --ca artifacts.ca --host {host} "
            f"--connect 127.0.0.1:{port}")
        assert rc == 0 and "status=200" in out, (out, err)
    fetch()
    # a name the certificate does not carry is refused
    rc, out, err = sdk_cmd.service_task_exec(
        config.SERVICE_NAME, "artifacts-0-node",
        f"python3 -m dcos_commons_amd.testing.tls_probe get --ca artifacts.ca --host not-the-task.example "
        f"--connect 127.0.0.1:{port}")
    assert rc != 0 and "status=200" not in out


def test_tls_secrets_in_store():
    names = sdk_security.list_secrets(config.SERVICE_NAME)
    for suffix in ARTIFACT_SUFFIXES:
        assert any(s.endswith(suffix) for s in names), (suffix, names)
    # the scheduler authenticated with its service account against IAM
    assert sdk_install._cluster().dcos.logins >= 1


def test_changing_discovery_replaces_certificate_sans():
    n = native()
    sans = n.cert_info(_task_file("discovery-0-node", "server.crt"))["dns"]
    assert f"{DISCOVERY_TASK_PREFIX}-0.{config.SERVICE_NAME}.autoip.dcos.thisdcos.directory" in sans

    cfg = sdk_marathon.get_config(config.SERVICE_NAME)
    cfg["env"]["DISCOVERY_TASK_PREFIX"] = DISCOVERY_TASK_PREFIX + "-new"
    sdk_marathon.update_app(cfg)
    sdk_plan.wait_for_completed_deployment(config.SERVICE_NAME)

    @sdk_utils.retry(timeout_s=60, interval_s=0.5)
    def renewed():
        sans = n.cert_info(_task_file("discovery-0-node", "server.crt"))["dns"]
        assert f"{DISCOVERY_TASK_PREFIX}-new-0.{config.SERVICE_NAME}.autoip.dcos.thisdcos.directory" in sans, sans
    renewed()
