"""TLS artifact provisioning for tasks with ``transport-encryption``.

Reference: sdk/.../offer/evaluate/security/{TLSArtifact,TLSArtifactPaths,CertificateNamesGenerator,
TLSArtifactsGenerator,TLSArtifactsUpdater,PEMUtils}.java.

* ``TLSArtifact`` -- certificate / private-key / root-ca-certificate (type TLS: ``.crt``/``.key``/
  ``.ca``) and keystore / truststore (type KEYSTORE, stored with the ``__dcos_base64__`` prefix so
  the Mesos secrets module decodes them); secret names ``<sansHash>__<pod-i-task>__<tls name>__<artifact>``.
* ``CertificateNamesGenerator`` -- subject ``CN=<task instance>.<service>`` (dots -> dashes, no
  slashes, last 64 chars) + fixed O/L/ST/C; SANs = the task's autoip hostname (discovery prefix
  aware) + every named-VIP hostname; ``sans_hash`` = sha1 hex of the ';'-joined SANs, so a SAN
  change invalidates the stored secrets.
* ``TLSArtifactsGenerator`` -- RSA key + CSR (native ``libsdktls``), CA sign + bundle, PEM
  certificate chain (end-entity + intermediates), PKCS#12 keystore (``default`` alias, full chain)
  and truststore (``dcos-root``), password ``notsecure`` as in the reference.
* ``TLSArtifactsUpdater`` -- if any expected secret is missing: generate first, then delete the
  stale ones and create all new ones (never leaves a half-provisioned task).

The crypto runs in ``native/tls/sdk_tls.cpp`` (OpenSSL libcrypto), loaded through ctypes; there is
no Python fallback -- a missing library raises ``TLSUnavailable``.
"""
from __future__ import annotations

import base64
import ctypes
import enum
import hashlib
import json
import logging
import os
import re
import threading
from dataclasses import dataclass
from typing import Collection, Dict, List, Optional

LOGGER = logging.getLogger(__name__)

KEYSTORE_PASSWORD = "notsecure"
KEYSTORE_PRIVATE_KEY_ALIAS = "default"
KEYSTORE_ROOT_CA_CERT_ALIAS = "dcos-root"
SECRET_STORE_NAME_DELIMITER = "__"
CN_MAX_LENGTH = 64

_ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))))
_LIB_PATHS = [os.path.join(_ROOT, "native", "build", "libsdktls.so")]


class TLSUnavailable(RuntimeError):
    pass


class TLSError(RuntimeError):
    pass


class NativeTLS:
    def __init__(self, path: str):
        lib = ctypes.CDLL(path)
        c, u8p, i = ctypes.c_char_p, ctypes.POINTER(ctypes.c_void_p), ctypes.c_int
        lib.sdktls_last_error.restype = c
        lib.sdktls_free.argtypes = [ctypes.c_void_p]
        sigs = {
            "sdktls_generate_rsa_key": [i, ctypes.POINTER(ctypes.c_void_p)],
            "sdktls_public_key_pem": [c, ctypes.POINTER(ctypes.c_void_p)],
            "sdktls_make_csr": [c, c, c, ctypes.POINTER(ctypes.c_void_p)],
            "sdktls_self_signed_ca": [c, c, i, ctypes.POINTER(ctypes.c_void_p)],
            "sdktls_sign_csr_ex": [c, c, c, i, ctypes.c_long, i, ctypes.POINTER(ctypes.c_void_p)],
            "sdktls_verify_chain": [c, c, c],
            "sdktls_cert_info": [c, ctypes.POINTER(ctypes.c_void_p)],
            "sdktls_pkcs12": [c, c, c, c, u8p, ctypes.POINTER(i)],
            "sdktls_pkcs12_inspect": [ctypes.c_char_p, i, c, ctypes.POINTER(i)],
            "sdktls_rs256_sign": [c, ctypes.c_char_p, i, u8p, ctypes.POINTER(i)],
            "sdktls_rs256_verify": [c, ctypes.c_char_p, i, ctypes.c_char_p, i],
            "sdktls_jwt_rs256": [c, c, ctypes.POINTER(ctypes.c_void_p)],
        }
        for name, args in sigs.items():
            fn = getattr(lib, name)
            fn.argtypes = args
            fn.restype = i
        self.lib = lib

    def _err(self, what: str) -> TLSError:
        return TLSError(f"{what}: {self.lib.sdktls_last_error().decode('utf-8', 'replace')}")

    def _str_out(self, fn, *args) -> str:
        out = ctypes.c_void_p()
        if fn(*args, ctypes.byref(out)) != 0:
            raise self._err(fn.__name__)
        try:
            return ctypes.string_at(out.value).decode("utf-8")
        finally:
            self.lib.sdktls_free(out)

    def _bytes_out(self, fn, *args) -> bytes:
        out, n = ctypes.c_void_p(), ctypes.c_int()
        if fn(*args, ctypes.byref(out), ctypes.byref(n)) != 0:
            raise self._err(fn.__name__)
        try:
            return ctypes.string_at(out.value, n.value)
        finally:
            self.lib.sdktls_free(out)

    @staticmethod
    def _b(s: Optional[str]) -> Optional[bytes]:
        return None if s is None else s.encode("utf-8")

    def generate_rsa_key(self, bits: int = 2048) -> str:
        return self._str_out(self.lib.sdktls_generate_rsa_key, bits)

    def public_key_pem(self, key_pem: str) -> str:
        return self._str_out(self.lib.sdktls_public_key_pem, self._b(key_pem))

    def make_csr(self, key_pem: str, subject: str, dns_sans: List[str]) -> str:
        sans = ",".join("DNS:" + s for s in dns_sans)
        return self._str_out(self.lib.sdktls_make_csr, self._b(key_pem), self._b(subject), self._b(sans))

    def self_signed_ca(self, key_pem: str, subject: str, days: int = 3650) -> str:
        return self._str_out(self.lib.sdktls_self_signed_ca, self._b(key_pem), self._b(subject), days)

    def sign_csr(self, ca_key_pem: str, ca_cert_pem: str, csr_pem: str, days: int = 365, serial: int = 0,
                 as_ca: bool = False) -> str:
        return self._str_out(self.lib.sdktls_sign_csr_ex, self._b(ca_key_pem), self._b(ca_cert_pem),
                             self._b(csr_pem), days, serial, 1 if as_ca else 0)

    def verify_chain(self, cert_pem: str, trusted_pem: str, untrusted_pem: Optional[str] = None) -> bool:
        r = self.lib.sdktls_verify_chain(self._b(cert_pem), self._b(trusted_pem), self._b(untrusted_pem))
        if r < 0:
            raise self._err("verify_chain")
        return r == 1

    def cert_info(self, cert_pem: str) -> Dict:
        return json.loads(self._str_out(self.lib.sdktls_cert_info, self._b(cert_pem)))

    def pkcs12(self, key_pem: Optional[str], chain_pem: str, alias: str, password: str) -> bytes:
        return self._bytes_out(self.lib.sdktls_pkcs12, self._b(key_pem or ""), self._b(chain_pem), self._b(alias),
                               self._b(password))

    def pkcs12_inspect(self, der: bytes, password: str):
        has_key = ctypes.c_int()
        n = self.lib.sdktls_pkcs12_inspect(der, len(der), self._b(password), ctypes.byref(has_key))
        if n < 0:
            raise self._err("pkcs12_inspect")
        return n, bool(has_key.value)

    def rs256_sign(self, key_pem: str, msg: bytes) -> bytes:
        return self._bytes_out(self.lib.sdktls_rs256_sign, self._b(key_pem), msg, len(msg))

    def rs256_verify(self, pub_pem: str, msg: bytes, sig: bytes) -> bool:
        r = self.lib.sdktls_rs256_verify(self._b(pub_pem), msg, len(msg), sig, len(sig))
        if r < 0:
            raise self._err("rs256_verify")
        return r == 1

    def jwt_rs256(self, key_pem: str, claims: Dict) -> str:
        return self._str_out(self.lib.sdktls_jwt_rs256, self._b(key_pem),
                             self._b(json.dumps(claims, separators=(",", ":"))))

    def verify_jwt(self, pub_pem: str, token: str) -> Optional[Dict]:
        try:
            h, p, s = token.split(".")
            sig = base64.urlsafe_b64decode(s + "=" * (-len(s) % 4))
        except ValueError:
            return None
        if not self.rs256_verify(pub_pem, f"{h}.{p}".encode("ascii"), sig):
            return None
        return json.loads(base64.urlsafe_b64decode(p + "=" * (-len(p) % 4)))


_native: Optional[NativeTLS] = None
_native_lock = threading.Lock()


def native() -> NativeTLS:
    global _native
    with _native_lock:
        if _native is None:
            for path in _LIB_PATHS:
                if os.path.exists(path):
                    _native = NativeTLS(path)
                    break
            else:
                raise TLSUnavailable(f"libsdktls.so not built (looked in {_LIB_PATHS}); run __graft_entry__.build()")
        return _native


# -- artifacts ----------------------------------------------------------------------------
class TLSArtifact(enum.Enum):
    CERTIFICATE = ("TLS", "certificate", "crt", "PEM encoded certificate")
    PRIVATE_KEY = ("TLS", "private-key", "key", "PEM encoded private key")
    CA_CERTIFICATE = ("TLS", "root-ca-certificate", "ca", "PEM encoded root CA certificate")
    KEYSTORE = ("KEYSTORE", "keystore", "keystore", "Base64 encoded java keystore")
    TRUSTSTORE = ("KEYSTORE", "truststore", "truststore", "Base64 encoded java trust store")

    @property
    def type(self) -> str:
        return self.value[0]

    @property
    def artifact_name(self) -> str:
        return self.value[1]

    @property
    def extension(self) -> str:
        return self.value[2]

    @property
    def description(self) -> str:
        return self.value[3]

    def secret_store_name(self, sans_hash: str, task_instance_name: str, tls_name: str) -> str:
        full = SECRET_STORE_NAME_DELIMITER.join(
            x for x in (sans_hash, task_instance_name, tls_name, self.artifact_name) if x and x.strip())
        if self.type == "KEYSTORE":
            full = "__dcos_base64__" + full
        return full

    def mount_path(self, tls_name: str) -> str:
        return f"{tls_name}.{self.extension}"


_KNOWN = re.compile("^.+%s(?:%s)$" % (SECRET_STORE_NAME_DELIMITER, "|".join(a.artifact_name for a in TLSArtifact)))


def known_tls_artifacts(secret_store_paths: Collection[str]) -> List[str]:
    return [p for p in secret_store_paths if _KNOWN.match(p)]


@dataclass(frozen=True)
class ArtifactPathEntry:
    secret_store_path: str
    mount_path: str


class TLSArtifactPaths:
    def __init__(self, secrets_namespace: str, task_instance_name: str, sans_hash: str):
        self.secrets_namespace = secrets_namespace
        self.task_instance_name = task_instance_name
        self.sans_hash = sans_hash

    def get_all_names(self, tls_name: str) -> List[str]:
        return [self._name(a, tls_name) for a in TLSArtifact]

    def get_paths_for_type(self, tls_type: str, tls_name: str) -> List[ArtifactPathEntry]:
        return [ArtifactPathEntry(self.get_secret_store_path(a, tls_name), a.mount_path(tls_name))
                for a in TLSArtifact if a.type == tls_type]

    def get_secret_store_path(self, artifact: TLSArtifact, tls_name: str) -> str:
        return f"{self.secrets_namespace}/{self._name(artifact, tls_name)}"

    def _name(self, artifact: TLSArtifact, tls_name: str) -> str:
        return artifact.secret_store_name(self.sans_hash, self.task_instance_name, tls_name)


class CertificateNamesGenerator:
    def __init__(self, service_name: str, task_spec, pod_instance, scheduler_config):
        from dcos_commons_amd.http import endpoint_utils as E
        from dcos_commons_amd.offer.common_id_utils import get_task_instance_name
        from dcos_commons_amd.specification.specs import NamedVIPSpec

        self.service_name = service_name
        self.task_instance_name = get_task_instance_name(pod_instance, task_spec)
        discovery = getattr(task_spec, "discovery", None)
        prefix = getattr(discovery, "prefix", None) if discovery is not None else None
        if prefix:
            self.auto_ip_hostname = E.to_auto_ip_hostname(service_name, f"{prefix}-{pod_instance.index}",
                                                          scheduler_config)
        else:
            self.auto_ip_hostname = E.to_auto_ip_hostname(service_name, self.task_instance_name, scheduler_config)
        self.vip_hostnames = [E.to_vip_hostname(service_name, scheduler_config, r.vip_name)
                              for r in task_spec.resource_set.resources if isinstance(r, NamedVIPSpec)]
        self._E = E

    def subject(self) -> str:
        E = self._E
        cn = (f"{E.remove_slashes(E.replace_dots_with_dashes(self.task_instance_name))}."
              f"{E.remove_slashes(E.replace_dots_with_dashes(self.service_name))}")
        if len(cn) > CN_MAX_LENGTH:
            cn = cn[-CN_MAX_LENGTH:]
        esc = lambda v: v.replace("\\", "\\\\").replace(",", "\\,")  # noqa: E731
        return ",".join(f"{k}={esc(v)}" for k, v in (("CN", cn), ("O", "Mesosphere, Inc"), ("L", "San Francisco"),
                                                     ("ST", "CA"), ("C", "US")))

    def sans(self) -> List[str]:
        return [self.auto_ip_hostname] + self.vip_hostnames

    def sans_hash(self) -> str:
        return hashlib.sha1(";".join(self.sans()).encode("utf-8")).hexdigest()


class TLSArtifactsGenerator:
    def __init__(self, ca_client, key_bits: int = 2048):
        self.ca_client = ca_client
        self.key_bits = key_bits

    def generate(self, names: CertificateNamesGenerator) -> Dict[TLSArtifact, str]:
        n = native()
        key = n.generate_rsa_key(self.key_bits)
        csr = n.make_csr(key, names.subject(), names.sans())
        cert = self.ca_client.sign(csr)
        chain = list(self.ca_client.chain_with_root_cert(cert))  # intermediates..., root
        root = chain[-1]
        end_entity_with_chain = [cert] + chain[:-1]
        keystore = n.pkcs12(key, "".join([cert] + chain), KEYSTORE_PRIVATE_KEY_ALIAS, KEYSTORE_PASSWORD)
        truststore = n.pkcs12(None, root, KEYSTORE_ROOT_CA_CERT_ALIAS, KEYSTORE_PASSWORD)
        return {
            TLSArtifact.CERTIFICATE: "".join(end_entity_with_chain),
            TLSArtifact.PRIVATE_KEY: key,
            TLSArtifact.CA_CERTIFICATE: root,
            TLSArtifact.KEYSTORE: base64.b64encode(keystore).decode("ascii"),
            TLSArtifact.TRUSTSTORE: base64.b64encode(truststore).decode("ascii"),
        }


class TLSArtifactsUpdater:
    def __init__(self, service_name: str, secrets_client, generator: TLSArtifactsGenerator):
        self.service_name = service_name
        self.secrets_client = secrets_client
        self.generator = generator

    def update(self, paths: TLSArtifactPaths, names: CertificateNamesGenerator, tls_name: str) -> None:
        from dcos_commons_amd.dcos.clients import SecretPayload

        namespace = paths.secrets_namespace
        current = list(self.secrets_client.list(namespace))
        expected = set(paths.get_all_names(tls_name))
        missing = sorted(expected - set(current))
        if not missing:
            LOGGER.info("Task '%s' already has all %d expected secrets for TLS config '%s' in namespace '%s'",
                        paths.task_instance_name, len(expected), tls_name, namespace)
            return
        LOGGER.info("Task '%s' is missing %d/%d expected secrets for TLS config '%s' in namespace '%s': %s",
                    paths.task_instance_name, len(missing), len(expected), tls_name, namespace, missing)
        values = self.generator.generate(names)  # generate BEFORE deleting anything
        for name in [c for c in current if c in expected]:
            LOGGER.info("Deleting secret: %s/%s", namespace, name)
            self.secrets_client.delete(f"{namespace}/{name}")
        for artifact, value in values.items():
            path = paths.get_secret_store_path(artifact, tls_name)
            LOGGER.info("Creating new secret: %s", path)
            self.secrets_client.create(path, SecretPayload(self.service_name, value, artifact.description))
