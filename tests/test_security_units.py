"""TLS naming units: certificate subject and SANs, secret-store paths of each artifact, and the
artifacts updater's list / delete / create protocol against the secrets service.

Mirrors sdk/scheduler/src/test/java/com/mesosphere/sdk/offer/evaluate/security/
{CertificateNamesGeneratorTest,TLSArtifactPathsTest,TLSArtifactsUpdaterTest}.java. The artifact
generator itself (key, CSR, CA signing, PKCS#12 stores) runs against the native TLS library in
``test_tls``.
"""
import hashlib
import types
import uuid

import pytest

import testutils as U
from dcos_commons_amd.dcos.clients import SecretPayload
from dcos_commons_amd.offer.evaluate.security import (CertificateNamesGenerator, TLSArtifact, TLSArtifactPaths,
                                                      TLSArtifactsUpdater, known_tls_artifacts)
from dcos_commons_amd.scheduler.scheduler_config import SchedulerConfig
from dcos_commons_amd.specification.specs import NamedVIPSpec, ranges_value

CFG = SchedulerConfig.for_testing()
POD_NAME = "some-pod"


def _pod_instance():
    return types.SimpleNamespace(name=POD_NAME, index=0)


def _task(name=U.TASK_NAME, prefix=None, resources=()):
    discovery = types.SimpleNamespace(prefix=prefix) if prefix else None
    return types.SimpleNamespace(name=name, discovery=discovery,
                                 resource_set=types.SimpleNamespace(resources=tuple(resources)))


def _names(service=U.SERVICE_NAME, task=None):
    return CertificateNamesGenerator(service, task or _task(), _pod_instance(), CFG)


def _cn(subject):
    return [kv.split("=", 1)[1] for kv in subject.split(",") if kv.startswith("CN=")]


def _sha1(s):
    return hashlib.sha1(s.encode("utf-8")).hexdigest()


def _task_dns(task, service, pod=POD_NAME):
    return f"{pod}-{task}.{service}.{CFG.autoip_tld()}"


def _vip_dns(vip, service):
    return f"{vip}.{service}.{CFG.vip_tld()}"


def test_subject():
    assert _cn(_names().subject()) == [f"{POD_NAME}-{U.TASK_NAME}.{U.SERVICE_NAME}"]


def test_long_cn_is_truncated_to_64():
    cn = _cn(_names(str(uuid.uuid4()), _task(str(uuid.uuid4()))).subject())
    assert len(cn) == 1 and len(cn[0]) == 64


def test_sans():
    n = _names()
    assert n.sans() == [_task_dns(U.TASK_NAME, U.SERVICE_NAME)]
    assert _task_dns("*", U.SERVICE_NAME) not in n.sans()
    assert n.sans_hash() == _sha1(f"some-pod-test-task-name.service-name.{CFG.autoip_tld()}")


def test_slashes_in_service_name():
    n = _names("service/name/with/slashes")
    assert _cn(n.subject()) == [f"{POD_NAME}-{U.TASK_NAME}.servicenamewithslashes"]
    assert n.sans() == [_task_dns(U.TASK_NAME, "servicenamewithslashes")]
    assert n.sans_hash() == _sha1(f"some-pod-test-task-name.servicenamewithslashes.{CFG.autoip_tld()}")


def test_discovery_name_is_the_san():
    n = _names(task=_task(prefix="custom-name"))
    assert n.sans() == [_task_dns("name-0", U.SERVICE_NAME, pod="custom")]
    assert n.sans_hash() == _sha1(f"custom-name-0.service-name.{CFG.autoip_tld()}")


def test_vips_are_added_as_sans():
    vip = NamedVIPSpec(name="ports", value=ranges_value([(8000, 8000)]), role=U.ROLE, principal=U.PRINCIPAL,
                       port_name="p", vip_name="test-vip", vip_port=80)
    n = _names(task=_task(resources=[vip]))
    assert n.sans() == [_task_dns(U.TASK_NAME, U.SERVICE_NAME), _vip_dns("test-vip", U.SERVICE_NAME)]
    assert n.sans_hash() == _sha1(f"some-pod-test-task-name.service-name.{CFG.autoip_tld()};"
                                  f"test-vip.service-name.{CFG.vip_tld()}")


# ---------------------------------------------------------------------------------------
# TLSArtifactPaths


SANS_HASH = "a-test-hash"
SPEC = "exposed"
NAME_PREFIX = f"{SANS_HASH}__pod-0-task__{SPEC}__"
PATH_PREFIX = f"namespace/{NAME_PREFIX}"
KS_NAME_PREFIX = f"__dcos_base64__{SANS_HASH}__pod-0-task__{SPEC}__"
KS_PATH_PREFIX = f"namespace/{KS_NAME_PREFIX}"
PATHS = TLSArtifactPaths("namespace", "pod-0-task", SANS_HASH)


@pytest.mark.parametrize("artifact,expected", [
    (TLSArtifact.CERTIFICATE, PATH_PREFIX + "certificate"),
    (TLSArtifact.PRIVATE_KEY, PATH_PREFIX + "private-key"),
    (TLSArtifact.CA_CERTIFICATE, PATH_PREFIX + "root-ca-certificate"),
    (TLSArtifact.KEYSTORE, KS_PATH_PREFIX + "keystore"),
    (TLSArtifact.TRUSTSTORE, KS_PATH_PREFIX + "truststore"),
])
def test_secret_store_path(artifact, expected):
    assert PATHS.get_secret_store_path(artifact, SPEC) == expected


def test_all_names():
    assert sorted(PATHS.get_all_names(SPEC)) == sorted([
        NAME_PREFIX + "certificate", NAME_PREFIX + "private-key", NAME_PREFIX + "root-ca-certificate",
        KS_NAME_PREFIX + "keystore", KS_NAME_PREFIX + "truststore"])


def test_paths_for_tls():
    assert [(e.mount_path, e.secret_store_path) for e in PATHS.get_paths_for_type("TLS", SPEC)] == [
        ("exposed.crt", PATH_PREFIX + "certificate"), ("exposed.key", PATH_PREFIX + "private-key"),
        ("exposed.ca", PATH_PREFIX + "root-ca-certificate")]


def test_paths_for_keystore():
    assert [(e.mount_path, e.secret_store_path) for e in PATHS.get_paths_for_type("KEYSTORE", SPEC)] == [
        ("exposed.keystore", KS_PATH_PREFIX + "keystore"), ("exposed.truststore", KS_PATH_PREFIX + "truststore")]


def test_known_artifacts_filter():
    names = PATHS.get_all_names(SPEC) + ["unrelated-secret", "x__not-an-artifact"]
    assert sorted(known_tls_artifacts(names)) == sorted(PATHS.get_all_names(SPEC))


# ---------------------------------------------------------------------------------------
# TLSArtifactsUpdater


SPEC_NAME = "spec-name"
GENERATED = {TLSArtifact.CERTIFICATE: "cert", TLSArtifact.CA_CERTIFICATE: "ca-cert",
             TLSArtifact.TRUSTSTORE: "truststore"}


class FakePaths:
    secrets_namespace = U.SERVICE_NAME
    task_instance_name = "pod-0-task"

    def get_all_names(self, tls_name):
        assert tls_name == SPEC_NAME
        return ["secret1", "secret2", "secret3"]

    def get_secret_store_path(self, artifact, tls_name):
        assert tls_name == SPEC_NAME
        return "a-secret-path"


class FakeSecrets:
    def __init__(self, listing):
        self.listing = listing
        self.calls = []

    def list(self, path):
        self.calls.append(("list", path))
        return list(self.listing)

    def delete(self, path):
        self.calls.append(("delete", path))

    def create(self, path, payload):
        self.calls.append(("create", path, payload))


class FakeGenerator:
    def __init__(self):
        self.calls = 0

    def generate(self, names):
        self.calls += 1
        return dict(GENERATED)


def _update(listing):
    secrets, gen = FakeSecrets(listing), FakeGenerator()
    TLSArtifactsUpdater(U.SERVICE_NAME, secrets, gen).update(FakePaths(), object(), SPEC_NAME)
    return secrets.calls, gen.calls


CREATES = sorted((SecretPayload(U.SERVICE_NAME, v, a.description) for a, v in GENERATED.items()), key=repr)


def _sorted_creates(calls):
    assert all(c[1] == "a-secret-path" for c in calls if c[0] == "create")
    return sorted((c[2] for c in calls if c[0] == "create"), key=repr)


@pytest.mark.parametrize("listing", [["secret1", "secret2", "secret3"],
                                     ["secret1", "secret2", "secret3", "secret4", "secret5"]])
def test_nothing_missing_lists_only(listing):
    calls, generated = _update(listing)
    assert calls == [("list", U.SERVICE_NAME)] and generated == 0


@pytest.mark.parametrize("listing,deletes", [
    (["secret2"], ["secret2"]),                 # some missing: stale present ones are replaced
    ([], []),                                   # all missing
    (["secret4", "secret5"], []),               # only unrecognized secrets: left alone
    (["secret2", "secret4"], ["secret2"]),      # mixed
])
def test_missing_secrets_regenerate_everything(listing, deletes):
    calls, generated = _update(listing)
    assert generated == 1
    assert calls[0] == ("list", U.SERVICE_NAME)
    assert [c for c in calls if c[0] == "delete"] == [("delete", f"{U.SERVICE_NAME}/{d}") for d in deletes]
    assert _sorted_creates(calls) == CREATES
    assert len(calls) == 1 + len(deletes) + len(GENERATED)
