"""The integration tier's security and packaging helpers against the stand-in (reference
``testing/security/*``, ``testing/sdk_auth.py``, ``testing/sdk_package_registry.py``): TLS service
accounts and CA-signed client artifacts, the Kerberos environment's keytab secret and krb5.conf,
and ``.dcos`` bundles added through the package registry."""
import json
import os
import ssl

import pytest

from dcos_commons_amd.testing import keytab as kt
from dcos_commons_amd.testing.sdk import sdk_auth, sdk_cmd, sdk_install, sdk_package_registry
from dcos_commons_amd.testing.security import kerberos, transport_encryption
from dcos_commons_amd.tools.universe import package_manager as pm
from tests.integration import hw_config as config
from tests.integration.conftest import make_cluster

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


@pytest.fixture(scope="module")
def local_cluster():
    c = make_cluster(dcos_security=True)
    sdk_install.install(config.PACKAGE_NAME, config.SERVICE_NAME, config.DEFAULT_TASK_COUNT)
    yield c
    sdk_install.uninstall(config.PACKAGE_NAME, config.SERVICE_NAME)
    c.shutdown()


pytestmark = pytest.mark.usefixtures("local_cluster")


def test_tls_service_account():
    info = transport_encryption.setup_service_account("hello-world")
    assert info["name"] == "hello-world-service-account" and info["secret"] == "hello-world-secret"
    assert {p["rid"] for p in info["permissions"]} >= {"dcos:secrets:default:/hello-world/*",
                                                        "dcos:adminrouter:ops:ca:rw"}
    assert info["service"]["service_account"] == "hello-world-service-account"
    transport_encryption.cleanup_service_account("hello-world", info)


def test_ca_signed_client_artifacts(local_cluster, tmp_path):
    ca = transport_encryption.fetch_dcos_ca_bundle_contents()
    assert ca.startswith(b"-----BEGIN CERTIFICATE-----")
    dn = transport_encryption.create_tls_artifacts("client", config.SERVICE_NAME)
    assert dn.startswith("CN=client,")
    sandbox = sdk_cmd.marathon_task_sandbox(config.SERVICE_NAME)
    names = set(os.listdir(sandbox))
    assert {"client_pub.crt", "client_priv.key", "client_chain.crt", "client_keystore.p12", "client_truststore.p12",
            "dcos-ca.crt"} <= names
    # the key matches the certificate, and the certificate chains to the cluster CA
    ctx = ssl.SSLContext(ssl.PROTOCOL_TLS_SERVER)
    ctx.load_cert_chain(os.path.join(sandbox, "client_pub.crt"), os.path.join(sandbox, "client_priv.key"))
    cert = ssl._ssl._test_decode_cert(os.path.join(sandbox, "client_pub.crt"))
    root = ssl._ssl._test_decode_cert(os.path.join(sandbox, "dcos-ca.crt"))
    with open(os.path.join(sandbox, "client_chain.crt"), encoding="utf-8") as f:
        pems = ["-----BEGIN CERTIFICATE-----" + p for p in f.read().split("-----BEGIN CERTIFICATE-----")[1:]]
    inter = tmp_path / "intermediate.crt"
    inter.write_text(pems[-1])
    issuer = ssl._ssl._test_decode_cert(str(inter))
    # leaf <- the stand-in's intermediate CA <- the cluster root
    assert cert["issuer"] == issuer["subject"] and issuer["issuer"] == root["subject"]
    assert ("commonName", "client") in [x[0] for x in cert["subject"]]
    from dcos_commons_amd.offer.evaluate.security import native

    with open(os.path.join(sandbox, "client_keystore.p12"), "rb") as f:
        assert native().pkcs12_inspect(f.read(), transport_encryption.STORE_PASSWORD)


def test_kerberos_environment_keytab_and_krb5_conf(local_cluster):
    krb5 = sdk_auth.KerberosEnvironment()
    principals = kerberos.generate_principal_list(["hdfs", "HTTP"], ["name-0-node.hdfs.autoip.dcos.thisdcos.directory"],
                                                  krb5.get_realm())
    krb5.add_principals(principals + ["client"])
    krb5.finalize()
    assert krb5.list_principals("hdfs/*") == [principals[0]]
    keytab = kt.decode(local_cluster.resolve_secret(krb5.get_keytab_path()))
    got = sorted("/".join(e.components) + "@" + e.realm for e in keytab.entries)
    assert got == sorted(principals + ["client@LOCAL"])
    assert kerberos.genererate_principal("hdfs", None, "local") == "hdfs@LOCAL"
    kerberos.write_krb5_config_file(config.SERVICE_NAME, "krb5.conf", krb5)
    sandbox = sdk_cmd.marathon_task_sandbox(config.SERVICE_NAME)
    with open(os.path.join(sandbox, "krb5.conf"), encoding="utf-8") as f:
        text = f.read()
    assert "default_realm = LOCAL" in text and f"kdc = {krb5.get_kdc_address()}" in text
    sdk_auth.kinit(config.SERVICE_NAME, "hdfs.keytab", principals[0])
    assert os.path.exists(os.path.join(sandbox, "krb5cc"))
    sdk_auth.kdestroy(config.SERVICE_NAME)
    assert not os.path.exists(os.path.join(sandbox, "krb5cc"))
    krb5.cleanup()
    assert local_cluster.resolve_secret(krb5.get_keytab_path()) is None


def test_package_registry_bundles(local_cluster, tmp_path):
    udir = os.path.join(ROOT, "frameworks", "helloworld", "universe")
    files = {}
    for n in pm.PACKAGE_FILES:
        p = os.path.join(udir, n)
        if os.path.exists(p):
            with open(p, encoding="utf-8") as f:
                files[n] = f.read()
    pkg = pm.package_from_files(files)
    pkg["version"], pkg["releaseVersion"] = "9.9.9-registry", 99
    stub = tmp_path / "stub-universe.json"
    stub.write_text(json.dumps({"packages": [pkg]}))
    with sdk_package_registry.package_registry_session(str(tmp_path / "dcos-files"), [str(stub)]) as app:
        assert app["id"] == sdk_package_registry.REGISTRY_APP_ID
        assert "9.9.9-registry" in local_cluster.cosmos.versions("hello-world")
        assert local_cluster.package_registry["bundles"][0].endswith("hello-world-9.9.9-registry.dcos")
    assert local_cluster.package_registry is None
