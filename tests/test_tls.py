"""TLS provisioning: native crypto (libsdktls), artifact naming, DC/OS IAM/secrets/CA clients and
the TLSEvaluationStage end-to-end (reference: offer/evaluate/TLSEvaluationStageTest.java,
security/{TLSArtifactsGeneratorTest,TLSArtifactsUpdaterTest,CertificateNamesGeneratorTest,
TLSArtifactPathsTest}.java, dcos/clients/*Test.java, dcos/auth/CachedTokenProviderTest.java)."""
import base64
import json
import os
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def tls():
    from dcos_commons_amd.ops import build

    try:
        build.build_cpp_tools()
    except Exception as e:  # noqa: BLE001
        pytest.skip(f"native toolchain unavailable: {e}")
    from dcos_commons_amd.offer.evaluate import security

    return security.native()


@pytest.fixture
def dcos(tls, monkeypatch):
    from dcos_commons_amd.testing.dcos_fakes import FakeDcosCluster

    cluster = FakeDcosCluster(intermediate_ca=True).start()
    monkeypatch.setenv("SDK_DCOS_MASTER_URI", cluster.url)
    yield cluster
    cluster.stop()


def test_native_key_csr_sign_verify(tls):
    ca_key = tls.generate_rsa_key()
    ca = tls.self_signed_ca(ca_key, "CN=Test Root,O=Acme\\, Inc")
    assert tls.cert_info(ca)["is_ca"]
    key = tls.generate_rsa_key()
    assert "BEGIN PRIVATE KEY" in key  # PKCS#8
    csr = tls.make_csr(key, "CN=pod-0-node.svc,O=Mesosphere\\, Inc,C=US", ["a.example", "b.example"])
    cert = tls.sign_csr(ca_key, ca, csr, days=30, serial=77)
    info = tls.cert_info(cert)
    assert info["dns"] == ["a.example", "b.example"]
    assert info["eku"] == ["clientAuth", "serverAuth"]
    assert "CN=pod-0-node.svc" in info["subject"] and "O=Mesosphere\\, Inc" in info["subject"]
    assert info["serial"] == "4D" and not info["is_ca"]
    assert 29 * 86400 < info["not_after"] - time.time() < 31 * 86400
    assert tls.verify_chain(cert, ca)
    other = tls.self_signed_ca(tls.generate_rsa_key(), "CN=Other")
    assert not tls.verify_chain(cert, other)
    with pytest.raises(Exception):
        tls.sign_csr(ca_key, ca, csr.replace("A", "B", 5))  # tampered CSR does not verify


def test_native_pkcs12_and_jwt(tls):
    ca_key = tls.generate_rsa_key()
    ca = tls.self_signed_ca(ca_key, "CN=Root")
    key = tls.generate_rsa_key()
    cert = tls.sign_csr(ca_key, ca, tls.make_csr(key, "CN=x", ["x"]))
    ks = tls.pkcs12(key, cert + ca, "default", "notsecure")
    assert tls.pkcs12_inspect(ks, "notsecure") == (2, True)
    ts = tls.pkcs12(None, ca, "dcos-root", "notsecure")
    assert tls.pkcs12_inspect(ts, "notsecure") == (1, False)
    with pytest.raises(Exception):
        tls.pkcs12_inspect(ks, "wrong")
    token = tls.jwt_rs256(key, {"uid": "svc", "exp": 123})
    pub = tls.public_key_pem(key)
    assert tls.verify_jwt(pub, token) == {"uid": "svc", "exp": 123}
    h, p, s = token.split(".")
    forged = h + "." + base64.urlsafe_b64encode(b'{"uid":"root","exp":123}').decode().rstrip("=") + "." + s
    assert tls.verify_jwt(pub, forged) is None
    assert tls.verify_jwt(tls.public_key_pem(ca_key), token) is None


def test_artifact_names_and_paths():
    from dcos_commons_amd.offer.evaluate.security import TLSArtifact, TLSArtifactPaths, known_tls_artifacts

    paths = TLSArtifactPaths("ns", "pod-0-task", "abc")
    assert paths.get_all_names("exposed") == [
        "abc__pod-0-task__exposed__certificate", "abc__pod-0-task__exposed__private-key",
        "abc__pod-0-task__exposed__root-ca-certificate", "__dcos_base64__abc__pod-0-task__exposed__keystore",
        "__dcos_base64__abc__pod-0-task__exposed__truststore"]
    tls_entries = paths.get_paths_for_type("TLS", "exposed")
    assert [e.mount_path for e in tls_entries] == ["exposed.crt", "exposed.key", "exposed.ca"]
    assert tls_entries[0].secret_store_path == "ns/abc__pod-0-task__exposed__certificate"
    assert [e.mount_path for e in paths.get_paths_for_type("KEYSTORE", "k")] == ["k.keystore", "k.truststore"]
    assert TLSArtifact.KEYSTORE.secret_store_name("", "t", "n") == "__dcos_base64__t__n__keystore"
    assert known_tls_artifacts(["a__b__certificate", "a__b__keystore", "random", "certificate",
                                "x__private-key"]) == ["a__b__certificate", "a__b__keystore", "x__private-key"]


def _pod(spec_file, env, pod_type, index=0):
    from dcos_commons_amd.scheduler.scheduler_config import SchedulerConfig
    from dcos_commons_amd.specification.specs import PodInstance
    from dcos_commons_amd.specification.yaml.mappers import ServiceSpecGenerator
    from dcos_commons_amd.specification.yaml.raw import RawServiceSpec

    specs = os.path.join(ROOT, "frameworks", "helloworld", "specs")
    cfg = SchedulerConfig.for_testing()
    raw = RawServiceSpec.new_builder(os.path.join(specs, spec_file)).set_env(env).build()
    spec = ServiceSpecGenerator(raw, cfg, specs, env).build()
    pod = next(p for p in spec.pods if p.type == pod_type)
    return spec, cfg, PodInstance(pod, index)


TLS_ENV = dict(FRAMEWORK_NAME="/folder/tls-svc", FRAMEWORK_PRINCIPAL="p", HELLO_COUNT="2", SLEEP_DURATION="1000",
               DISCOVERY_TASK_PREFIX="custom")


def test_certificate_names():
    from dcos_commons_amd.offer.evaluate.security import CertificateNamesGenerator

    spec, cfg, pi = _pod("tls.yml", TLS_ENV, "gateway", 1)
    names = CertificateNamesGenerator(spec.name, pi.pod.tasks[0], pi, cfg)
    assert names.subject() == "CN=gateway-1-server.foldertls-svc,O=Mesosphere\\, Inc,L=San Francisco,ST=CA,C=US"
    assert names.sans() == ["gateway-1-server.foldertls-svc.autoip.dcos.thisdcos.directory",
                            "gateway-https.foldertls-svc.l4lb.thisdcos.directory"]
    import hashlib

    assert names.sans_hash() == hashlib.sha1(";".join(names.sans()).encode()).hexdigest()
    spec, cfg, pi = _pod("tls.yml", TLS_ENV, "discovery", 0)
    d = CertificateNamesGenerator(spec.name, pi.pod.tasks[0], pi, cfg)
    assert d.sans() == ["custom-0.foldertls-svc.autoip.dcos.thisdcos.directory"]
    long_env = dict(TLS_ENV, FRAMEWORK_NAME="a" * 80)
    spec, cfg, pi = _pod("tls.yml", long_env, "artifacts", 0)
    cn = CertificateNamesGenerator(spec.name, pi.pod.tasks[0], pi, cfg).subject().split(",")[0][3:]
    assert len(cn) == 64 and cn.endswith("a" * 10)


def test_iam_token_login_and_cache(dcos):
    from dcos_commons_amd.dcos import clients as C

    cred = dcos.add_service_account("svc-acct")
    provider = C.token_provider_from_service_account(cred, refresh_threshold_s=30)
    t1 = provider.get_token()
    assert t1.expires_at > time.time() + 200 and dcos.logins == 1
    assert provider.get_token() is t1 and dcos.logins == 1  # cached
    dcos.token_lifetime_s = 10  # next token expires inside the 30 s refresh threshold
    provider._token = None
    provider.get_token()
    provider.get_token()
    assert dcos.logins == 3  # refreshed every time it is within threshold of expiry
    from dcos_commons_amd.offer.evaluate.security import native

    bad = json.loads(cred)
    bad["private_key"] = native().generate_rsa_key()  # not the registered key
    with pytest.raises(C.DcosHttpError) as e:
        C.token_provider_from_service_account(json.dumps(bad)).get_token()
    assert e.value.status == 401


def test_secrets_and_ca_clients(dcos):
    from dcos_commons_amd.dcos import clients as C
    from dcos_commons_amd.offer.evaluate.security import native

    unauth = C.SecretsClient(C.DcosHttpExecutor())
    with pytest.raises(C.DcosHttpError) as e:
        unauth.list("ns")
    assert e.value.status == 401
    ex = C.DcosHttpExecutor(C.token_provider_from_service_account(dcos.add_service_account("sa")))
    s = C.SecretsClient(ex)
    s.create("ns/a", C.SecretPayload("me", "v1", "d"))
    s.create("ns/sub/b", C.SecretPayload("me", "v2", "d"))
    with pytest.raises(C.DcosHttpError):
        s.create("ns/a", C.SecretPayload("me", "v1", "d"))
    assert s.list("ns") == ["a", "sub/b"]
    s.update("ns/a", C.SecretPayload("me", "v3", "d"))
    assert dcos.secrets["ns/a"]["value"] == "v3"
    s.delete("ns/a")
    with pytest.raises(C.DcosHttpError):
        s.delete("ns/a")
    ca = C.CertificateAuthorityClient(ex)
    key = native().generate_rsa_key()
    cert = ca.sign(native().make_csr(key, "CN=t", ["t.example"]))
    chain = ca.chain_with_root_cert(cert)
    assert chain == [dcos.int_cert, dcos.root_cert]
    assert native().verify_chain(cert, dcos.root_cert, dcos.int_cert)
    with pytest.raises(C.DcosHttpError):
        ca.sign("not a csr")
    assert C.DcosVersionClient(ex).get_version() == "1.13.0"


def test_artifacts_updater_generates_once_and_on_san_change(dcos):
    from dcos_commons_amd.dcos import clients as C
    from dcos_commons_amd.offer.evaluate.security import (CertificateNamesGenerator, TLSArtifactPaths,
                                                          TLSArtifactsGenerator, TLSArtifactsUpdater, native)

    ex = C.DcosHttpExecutor(C.token_provider_from_service_account(dcos.add_service_account("sa")))
    updater = TLSArtifactsUpdater("svc", C.SecretsClient(ex), TLSArtifactsGenerator(C.CertificateAuthorityClient(ex)))
    spec, cfg, pi = _pod("tls.yml", TLS_ENV, "artifacts", 0)
    names = CertificateNamesGenerator(spec.name, pi.pod.tasks[0], pi, cfg)
    paths = TLSArtifactPaths("ns", "artifacts-0-node", names.sans_hash())
    updater.update(paths, names, "artifacts")
    assert len(dcos.secrets) == 5 and len(dcos.signed) == 1
    updater.update(paths, names, "artifacts")
    assert len(dcos.signed) == 1  # everything present: nothing regenerated
    # one secret goes missing -> regenerate all five
    from dcos_commons_amd.offer.evaluate.security import TLSArtifact

    del dcos.secrets[paths.get_secret_store_path(TLSArtifact.CERTIFICATE, "artifacts")]
    updater.update(paths, names, "artifacts")
    assert len(dcos.signed) == 2 and len(dcos.secrets) == 5
    vals = {k.split("__")[-1]: v["value"] for k, v in dcos.secrets.items()}
    n = native()
    certs = vals["certificate"]
    assert certs.count("BEGIN CERTIFICATE") == 2  # end-entity + intermediate, root excluded
    assert vals["root-ca-certificate"] == dcos.root_cert
    assert n.verify_chain(certs.split("-----END CERTIFICATE-----")[0] + "-----END CERTIFICATE-----\n",
                          dcos.root_cert, dcos.int_cert)
    assert n.pkcs12_inspect(base64.b64decode(vals["keystore"]), "notsecure") == (3, True)
    assert n.pkcs12_inspect(base64.b64decode(vals["truststore"]), "notsecure") == (1, False)
    assert all(v["author"] == "svc" for v in dcos.secrets.values())


def test_tls_service_deploys_with_secret_volumes_and_uninstall_cleans_up(dcos):
    from dcos_commons_amd.dcos import clients as C
    from dcos_commons_amd.mesos import protos as P
    from dcos_commons_amd.scheduler.uninstall import TLSCleanupStep
    from test_e2e_helloworld import Cluster

    cred = dcos.add_service_account("tls-svc")
    env = dict(TLS_ENV)
    with Cluster(spec_file="tls.yml", env=env, agents=3, DCOS_SERVICE_ACCOUNT_CREDENTIAL=cred,
                 DCOS_SPACE="/folder/tls-svc") as c:
        c.wait_plan("deploy", timeout=60)
        states = c.master.task_states()
        assert len(states) == 8 and set(states.values()) == {P.TASK_RUNNING}
        # 5 artifacts per transport-encryption entry per task instance:
        # artifacts 2x2, gateway 2x1, discovery 1, webserver 1, multi 2 -> 10 entries
        ns = "folder/tls-svc"
        assert len([k for k in dcos.secrets if k.startswith(ns + "/")]) == 50
        tasks = {t.name: t for t in c.master.tasks_by_name().values()}
        vols = {v.container_path: v for v in tasks["artifacts-0-node"].container.volumes}
        assert {"artifacts.crt", "artifacts.key", "artifacts.ca", "store.keystore", "store.truststore"} <= set(vols)
        v = vols["store.keystore"]
        assert v.mode == P.Volume.RO and v.source.type == P.Volume.Source.SECRET
        assert v.source.secret.reference.name.startswith(ns + "/__dcos_base64__")
        gw = {v.container_path for v in tasks["gateway-0-server"].container.volumes}
        assert gw >= {"gateway.keystore", "gateway.truststore"} and "gateway.crt" not in gw
        # the gateway certificate carries its VIP name
        from dcos_commons_amd.offer.evaluate.security import native

        gw_cert = next(s["value"] for k, s in dcos.secrets.items() if "gateway-0-server__gateway__certificate" in k)
        assert "gateway-https.foldertls-svc.l4lb.thisdcos.directory" in native().cert_info(gw_cert)["dns"]
        # restart: artifacts are reused (nothing new is signed)
        signed = len(dcos.signed)
        old = c.store.fetch_task("artifacts-0-node").task_id.value
        c.master.fail_task(old)
        c.wait(lambda: c.store.fetch_status("artifacts-0-node").task_id.value != old and
               c.store.fetch_status("artifacts-0-node").state == P.TASK_RUNNING, timeout=30)
        assert len(dcos.signed) == signed
        # uninstall's tls-cleanup phase removes exactly the TLS artifacts
        ex = C.DcosHttpExecutor(C.token_provider_from_service_account(cred))
        secrets = C.SecretsClient(ex)
        secrets.create(ns + "/unrelated", C.SecretPayload("x", "y", "z"))
        step = TLSCleanupStep(secrets, ns)
        step.start()
        assert [k for k in dcos.secrets if k.startswith(ns + "/")] == [ns + "/unrelated"]


def test_tls_requires_service_account():
    from dcos_commons_amd.config.validate import TLSRequiresServiceAccount
    from dcos_commons_amd.scheduler.scheduler_config import SchedulerConfig

    spec, _, _ = _pod("tls.yml", TLS_ENV, "artifacts")
    errs = TLSRequiresServiceAccount(SchedulerConfig.for_testing()).validate(None, spec)
    assert errs and "service account" in str(errs[0])
    bad = SchedulerConfig.for_testing(DCOS_SERVICE_ACCOUNT_CREDENTIAL="{}")  # no uid / private_key
    assert TLSRequiresServiceAccount(bad).validate(None, spec)
    ok = SchedulerConfig.for_testing(DCOS_SERVICE_ACCOUNT_CREDENTIAL='{"uid": "sa", "private_key": "k"}')
    assert TLSRequiresServiceAccount(ok).validate(None, spec) == []
