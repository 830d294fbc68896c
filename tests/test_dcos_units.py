"""DC/OS integration units: version-gated capabilities, the version document, token caching and
the secrets / CA / version clients over a recording HTTP executor.

Mirrors sdk/scheduler/src/test/java/com/mesosphere/sdk/dcos/{CapabilitiesTest,DcosVersionTest}.java,
dcos/auth/{CachedTokenProviderTest,ConstantTokenProviderTest}.java and dcos/clients/
{SecretsClientTest,CertificateAuthorityClientTest,DcosVersionClientTest}.java. The CA responses are
the reference's own fixtures (sdk/scheduler/src/test/resources/response-ca-*.json). ``test_tls``
runs the same clients against a live fake of the DC/OS services.
"""
import base64
import json
import os
import time

import pytest

from conftest import reference_path
from dcos_commons_amd.dcos import clients as C
from dcos_commons_amd.dcos.capabilities import Capabilities, DcosVariant, DcosVersion

RESOURCES = reference_path("sdk", "scheduler", "src", "test", "resources")


# ---------------------------------------------------------------------------------------
# Capabilities by DC/OS version


def _gates(c):
    return {
        "vips": c.supports_named_vips, "rlimits": c.supports_rlimits, "gpu": c.supports_gpu_resource,
        "directive": c.supports_env_based_secrets_directive_label, "env_proto": c.supports_env_based_secrets,
        "file": c.supports_file_based_secrets, "v1": c.supports_v1_api_by_default, "domains": c.supports_domains,
    }


@pytest.mark.parametrize("version,expected", [
    ("0.9.0", dict(vips=False, rlimits=False, domains=False)),
    ("1.7.0", dict(vips=False, rlimits=False, domains=False)),
    ("1.7-dev", dict(vips=False, rlimits=False, domains=False)),
    ("1.8.0", dict(vips=True, rlimits=False, directive=True, domains=False)),
    ("1.8-dev", dict(vips=True, rlimits=False, directive=True, domains=False)),
    ("1.9.0", dict(vips=True, gpu=True, rlimits=True, directive=True, env_proto=False, file=False, domains=False)),
    ("1.9-dev", dict(vips=True, gpu=True, rlimits=True, directive=True, env_proto=False, file=False, domains=False)),
    ("1.10.0", dict(vips=True, gpu=True, rlimits=True, directive=True, env_proto=True, file=True, v1=False,
                    domains=False)),
    ("1.10-dev", dict(vips=True, gpu=True, rlimits=True, directive=True, env_proto=True, file=True, v1=False,
                      domains=False)),
    ("1.11.0", dict(vips=True, gpu=True, rlimits=True, directive=True, env_proto=True, file=True, v1=True,
                    domains=True)),
    ("1.11-dev", dict(vips=True, gpu=True, rlimits=True, directive=True, env_proto=True, file=True, v1=True,
                      domains=True)),
    ("2.0.0", dict(vips=True, gpu=True, rlimits=True, directive=True, env_proto=True, file=True, domains=True)),
    ("2.0-dev", dict(vips=True, gpu=True, rlimits=True, directive=True, env_proto=True, file=True, domains=True)),
])
def test_capabilities_by_version(version, expected):
    gates = _gates(Capabilities.for_version(version))
    for k, v in expected.items():
        assert gates[k] is v, (version, k)


def test_later_gates():
    assert not Capabilities.for_version("1.11").supports_profile_mount_volumes
    assert Capabilities.for_version("1.12").supports_profile_mount_volumes
    assert not Capabilities.for_version("1.12").supports_seccomp
    assert Capabilities.for_version("1.13").supports_seccomp and not Capabilities.for_version("1.13").supports_shm
    assert Capabilities.for_version("1.14").supports_shm


def test_unparseable_version_closes_every_gate():
    c = Capabilities.for_version("test-version")
    assert not any(_gates(c).values())


def test_default_capabilities_are_a_current_cluster():
    c = Capabilities()
    assert all(_gates(c).values()) and c.supports_shm and c.supports_seccomp
    assert c.supports_cni_port_mapping is c.supports_cni_networking
    assert not c.with_overrides(supports_cni_port_mapping=False).supports_cni_networking


# ---------------------------------------------------------------------------------------
# DcosVersion


def test_version_construction():
    v = DcosVersion("test-version", DcosVariant.UNKNOWN)
    assert v.version == "test-version" and v.variant == DcosVariant.UNKNOWN


@pytest.mark.parametrize("variant,expected", [
    (None, DcosVariant.UNKNOWN), ("open", DcosVariant.OPEN), ("enterprise", DcosVariant.ENTERPRISE),
    ("UNKNOWN", DcosVariant.UNKNOWN), ("DC/OS Enterprise", DcosVariant.UNKNOWN),
])
def test_version_variant_from_json(variant, expected):
    doc = {"version": "test-version"}
    if variant is not None:
        doc["dcos-variant"] = variant
    assert DcosVersion.from_json(doc).variant == expected


# ---------------------------------------------------------------------------------------
# recording HTTP executor


class Executor:
    def __init__(self, status=200, body=b""):
        self.status = status
        self.body = body
        self.calls = []

    def execute(self, method, url, body=None, content_type="application/json"):
        self.calls.append((method, url, body))
        return self.status, self.body


def _version_doc(version):
    return json.dumps({"version": version, "dcos-image-commit": "test-dcos-image-commit",
                       "bootstrap-id": "test-bootstrap-id"}).encode()


def test_version_client():
    ex = Executor(body=_version_doc("1.9-dev"))
    v = C.DcosVersionClient(ex, "http://master").get_dcos_version()
    assert ex.calls == [("GET", "http://master/dcos-metadata/dcos-version.json", None)]
    assert v.version == "1.9-dev" and (v.first_element(), v.second_element()) == (1, 9)


@pytest.mark.parametrize("version,first", [("5", 5), ("0.", 0), ("0.hello", 0), ("0.5-hey", 0)])
def test_bad_second_element(version, first):
    v = C.DcosVersionClient(Executor(body=_version_doc(version)), "http://m").get_dcos_version()
    assert v.version == version and v.first_element() == first
    with pytest.raises(ValueError):
        v.second_element()


def test_bad_first_element():
    v = C.DcosVersionClient(Executor(body=_version_doc(".")), "http://m").get_dcos_version()
    with pytest.raises(ValueError):
        v.first_element()


# ---------------------------------------------------------------------------------------
# tokens


def _jwt(exp):
    payload = base64.urlsafe_b64encode(json.dumps({"uid": "svc", "exp": exp}).encode()).rstrip(b"=").decode()
    return f"eyJhbGciOiJSUzI1NiJ9.{payload}.sig"


class CountingProvider(C.TokenProvider):
    def __init__(self, exp):
        self.exp = exp
        self.calls = 0

    def get_token(self):
        self.calls += 1
        return C.Token.decode(_jwt(self.exp))


def test_cached_token_is_fetched_once():
    inner = CountingProvider(time.time() + 60)
    p = C.CachedTokenProvider(inner, 30)
    t = p.get_token()
    assert p.get_token() is t
    assert inner.calls == 1


def test_expired_token_is_refreshed():
    inner = CountingProvider(time.time() - 60)
    p = C.CachedTokenProvider(inner, 30)
    p.get_token()
    p.get_token()
    assert inner.calls == 2


def test_token_inside_the_refresh_threshold_is_refreshed():
    inner = CountingProvider(time.time() + 10)
    p = C.CachedTokenProvider(inner, 30)
    p.get_token()
    p.get_token()
    assert inner.calls == 2


def test_constant_token_provider():
    raw = _jwt(1234)
    t = C.ConstantTokenProvider(raw).get_token()
    assert t.value == raw and t.expires_at == 1234
    assert C.Token.decode("not-a-jwt").expires_at == 0


# ---------------------------------------------------------------------------------------
# SecretsClient


PAYLOAD = C.SecretPayload("scheduler-name", "secret-value", "description")
BASE = "http://master/secrets/v1/secret/default/"


def _secrets(status=200, body=b""):
    ex = Executor(status, body)
    return C.SecretsClient(ex, BASE), ex


def test_list():
    client, ex = _secrets(body=b'{"array":["one","two"]}')
    assert sorted(client.list("test")) == ["one", "two"]
    assert ex.calls == [("GET", BASE + "test?list=true", None)]


@pytest.mark.parametrize("status", [403, 404])
def test_list_errors(status):
    client, _ = _secrets(status)
    with pytest.raises(IOError, match=f"code={status}"):
        client.list("test")


def _sent_payload(ex):
    return json.loads(ex.calls[0][2])


def test_create():
    client, ex = _secrets(201)
    client.create("scheduler-name/secret-name", PAYLOAD)
    method, url, _ = ex.calls[0]
    assert (method, url) == ("PUT", BASE + "scheduler-name/secret-name")
    assert _sent_payload(ex) == {"value": "secret-value", "author": "scheduler-name", "description": "description"}


@pytest.mark.parametrize("status", [403, 409])
def test_create_errors(status):
    client, _ = _secrets(status)
    with pytest.raises(IOError, match=f"code={status}"):
        client.create("scheduler-name/secret-name", PAYLOAD)


def test_update():
    client, ex = _secrets(204)
    client.update("scheduler-name/secret-name", PAYLOAD)
    method, url, _ = ex.calls[0]
    assert (method, url) == ("PATCH", BASE + "scheduler-name/secret-name")
    assert _sent_payload(ex)["value"] == "secret-value"


@pytest.mark.parametrize("status", [403, 404])
def test_update_errors(status):
    client, _ = _secrets(status)
    with pytest.raises(IOError):
        client.update("scheduler-name/secret-name", PAYLOAD)


def test_delete():
    client, ex = _secrets(204)
    client.delete("scheduler-name/secret-name")
    assert ex.calls == [("DELETE", BASE + "scheduler-name/secret-name", None)]


# ---------------------------------------------------------------------------------------
# CertificateAuthorityClient


needs_resources = pytest.mark.skipif(RESOURCES is None, reason="reference fixtures not present")


def _resource(name):
    with open(os.path.join(RESOURCES, name), "rb") as f:
        return f.read()


def _ca(status=200, body=b""):
    return C.CertificateAuthorityClient(Executor(status, body), "http://master/ca/api/v2/")


@needs_resources
def test_sign_with_a_valid_response():
    from dcos_commons_amd.offer.evaluate.security import native

    cert = _ca(body=_resource("response-ca-sign-valid.json")).sign("csr")
    assert int(native().cert_info(cert)["serial"], 16) == 232536721977418639703314578745637408882101009293


@needs_resources
def test_sign_with_an_error_in_the_response():
    with pytest.raises(IOError, match=r"\[1234\] Test error"):
        _ca(body=_resource("response-ca-sign-with-error.json")).sign("csr")


def test_sign_with_a_non_200_response():
    with pytest.raises(IOError, match="400 - error from CA"):
        _ca(400).sign("csr")


@needs_resources
def test_chain_with_root_cert():
    chain = _ca(body=_resource("response-ca-bundle-valid.json")).chain_with_root_cert("cert")
    assert len(chain) > 0 and all(c.startswith("-----BEGIN CERTIFICATE-----") for c in chain)


@needs_resources
def test_chain_with_an_error_in_the_response():
    with pytest.raises(IOError, match=r"\[1234\] Test message"):
        _ca(body=_resource("response-ca-bundle-with-error.json")).chain_with_root_cert("cert")


def test_chain_with_a_non_200_response():
    with pytest.raises(IOError, match="400 - error from CA"):
        _ca(400).chain_with_root_cert("cert")
