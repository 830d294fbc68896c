"""TLS set-up for integration tests (reference ``testing/security/transport_encryption.py``): a
service account allowed to provision certificates, the cluster CA bundle, and a client
certificate + key / keystore / truststore signed by the cluster CA in a Marathon task's sandbox.

The stand-in's CA is ``testing.dcos_fakes.FakeDcosCluster`` (``LocalCluster(dcos_security=True)``);
keys, CSRs and PKCS#12 stores come from the SDK's own TLS code (``offer.evaluate.security.native``)
instead of ``openssl``/``keytool`` inside the task, and the stores are PKCS#12, which Java 9+ reads
as its default keystore type."""
from __future__ import annotations

import json
import logging
import os
from typing import Any, Dict, Optional

from dcos_commons_amd.testing.sdk import sdk_cmd, sdk_security

LOG = logging.getLogger(__name__)

TLS_ACLS = ("dcos:secrets:default:/{svc}/*", "dcos:secrets:list:default:/{svc}", "dcos:adminrouter:ops:ca:rw",
            "dcos:adminrouter:ops:ca:ro")
STORE_PASSWORD = "changeit"


def setup_service_account(service_name: str, service_account_secret: Optional[str] = None) -> Dict[str, Any]:
    """Create ``<service>-service-account`` with its secret and the permissions TLS provisioning
    needs (the service's secrets and the CA); an existing account of that name is replaced."""
    secret = service_account_secret or service_name + "-secret"
    account = "{}-service-account".format(service_name.replace("/", ""))
    info = sdk_security.setup_security(service_name, service_account=account, service_account_secret=secret)
    svc = service_name.strip("/")
    info = dict(info or {}, name=account, secret=secret,
                permissions=[{"rid": rid.format(svc=svc), "action": "full" if "list" not in rid else "read"}
                             for rid in TLS_ACLS])
    LOG.info("TLS service account %s: %s", account, info["permissions"])
    return info


def cleanup_service_account(service_name: str, service_account_info) -> None:
    if isinstance(service_account_info, str):
        service_account_info = {"name": service_account_info}
    sdk_security.cleanup_security(service_name, service_account=service_account_info.get("name", ""),
                                  service_account_secret=service_account_info.get("secret", ""))


def fetch_dcos_ca_bundle_contents() -> bytes:
    """The cluster CA's root certificate (``GET /ca/dcos-ca.crt``)."""
    cert = sdk_cmd.cluster_request("GET", "/ca/dcos-ca.crt").content
    if not cert:
        raise RuntimeError("empty DC/OS CA bundle")
    return cert


def fetch_dcos_ca_bundle(marathon_task: str) -> str:
    """Write the CA bundle into the task's sandbox as ``dcos-ca.crt``; returns the file name."""
    _write(marathon_task, "dcos-ca.crt", fetch_dcos_ca_bundle_contents())
    return "dcos-ca.crt"


def _sandbox(marathon_task: str) -> str:
    return sdk_cmd.marathon_task_sandbox(marathon_task)


def _write(marathon_task: str, name: str, data: bytes) -> None:
    with open(os.path.join(_sandbox(marathon_task), name), "wb") as f:
        f.write(data)


def create_tls_artifacts(cn: str, marathon_task: str) -> str:
    """A key and a certificate for ``cn`` signed by the cluster CA (``POST /ca/api/v2/sign``),
    written into the task's sandbox as ``<cn>_priv.key`` / ``<cn>_pub.crt`` (and ``<cn>_chain.crt``:
    the leaf with any intermediate CA) together with ``<cn>_keystore.p12`` (key + chain) and ``<cn>_truststore.p12`` (the CA), both protected by
    ``changeit``. Returns the certificate's subject DN."""
    from dcos_commons_amd.offer.evaluate.security import native

    n = native()
    subject = f"CN={cn},OU=Mesosphere,O=Mesosphere,L=SF,ST=CA,C=US"
    key = n.generate_rsa_key(2048)
    csr = n.make_csr(key, subject, [cn])
    resp = sdk_cmd.cluster_request("POST", "/ca/api/v2/sign", json={"certificate_request": csr})
    cert = json.loads(resp.text)["result"]["certificate"]
    # the leaf plus any intermediate CA, as the CA's bundle endpoint chains it
    bundle = json.loads(sdk_cmd.cluster_request("POST", "/ca/api/v2/bundle", json={"certificate": cert}).text)
    chain = bundle["result"]["bundle"]
    ca = fetch_dcos_ca_bundle_contents().decode("utf-8")
    _write(marathon_task, f"{cn}_priv.key", key.encode("utf-8"))
    _write(marathon_task, f"{cn}_pub.crt", cert.encode("utf-8"))
    _write(marathon_task, f"{cn}_chain.crt", chain.encode("utf-8"))
    _write(marathon_task, "dcos-ca.crt", ca.encode("utf-8"))
    _write(marathon_task, f"{cn}_keystore.p12", n.pkcs12(key, chain + ca, "keypair", STORE_PASSWORD))
    _write(marathon_task, f"{cn}_truststore.p12", n.pkcs12(None, ca, "root", STORE_PASSWORD))
    return subject
