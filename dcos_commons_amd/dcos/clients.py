"""DC/OS cluster service clients: IAM tokens, secrets store, certificate authority, version.

Reference: sdk/.../dcos/{DcosHttpExecutor,DcosHttpClientBuilder}.java, dcos/auth/
{TokenProvider,ConstantTokenProvider,CachedTokenProvider}.java, dcos/clients/{SecretsClient,
CertificateAuthorityClient,ServiceAccountIAMTokenClient,DcosVersionClient}.java.

* ``DcosHttpExecutor`` -- stdlib HTTP with ``Authorization: token=<jwt>`` from a token provider and
  lax redirects (PUT/PATCH/DELETE are re-issued to the ``Location``, as the reference's
  ``LaxRedirectStrategy`` override does for PUT);
* ``ServiceAccountIAMTokenClient`` -- signs a 120 s RS256 login JWT ``{"uid", "exp"}`` with the
  service account key (native ``libsdktls``) and exchanges it at ``/acs/api/v1/auth/login``;
* ``CachedTokenProvider`` -- reuses the token until ``ttl`` before its ``exp``;
* ``SecretsClient`` -- list (``?list=true`` -> ``{"array": [...]}``) / create (PUT, 201) / update
  (PATCH, 204) / delete (DELETE, 204) under ``/secrets/v1/secret/default/``;
* ``CertificateAuthorityClient`` -- ``/ca/api/v2/sign`` and ``/bundle`` (CFSSL-style JSON with
  ``success``/``errors``/``result``).

The cluster base URI defaults to ``http://master.mesos`` and can be pointed elsewhere with
``SDK_DCOS_MASTER_URI`` (tests run a local stand-in, ``testing.dcos_fakes``).
"""
from __future__ import annotations

import base64
import json
import logging
import os
import threading
import time
import urllib.error
import urllib.parse
import urllib.request
from dataclasses import dataclass
from typing import Dict, List, Optional, Tuple

from . import constants as C

LOGGER = logging.getLogger(__name__)


def master_uri() -> str:
    return os.environ.get("SDK_DCOS_MASTER_URI", C.MESOS_MASTER_URI).rstrip("/")


class DcosHttpError(IOError):
    def __init__(self, status: int, reason: str, body: str = ""):
        # "<code> - <reason>" and "code=<code>" as the reference's clients word it
        super().__init__(f"{status} - {reason} (code={status})" + (f": {body[:200]}" if body else ""))
        self.status = status
        self.reason = reason
        self.body = body


# -- tokens --------------------------------------------------------------------------------
@dataclass
class Token:
    value: str
    expires_at: float  # epoch seconds

    @staticmethod
    def decode(jwt: str) -> "Token":
        """Reads ``exp`` from a JWT payload (no signature check; the issuer is trusted)."""
        try:
            payload = jwt.split(".")[1]
            claims = json.loads(base64.urlsafe_b64decode(payload + "=" * (-len(payload) % 4)))
            exp = float(claims.get("exp", 0))
        except (IndexError, ValueError):
            exp = 0.0
        return Token(jwt, exp)


class TokenProvider:
    def get_token(self) -> Token:
        raise NotImplementedError


class ConstantTokenProvider(TokenProvider):
    def __init__(self, token: str):
        self.token = Token.decode(token)

    def get_token(self) -> Token:
        return self.token


class CachedTokenProvider(TokenProvider):
    def __init__(self, provider: TokenProvider, ttl_s: float):
        self.provider = provider
        self.ttl_s = ttl_s
        self._lock = threading.Lock()
        self._token: Optional[Token] = None

    def get_token(self) -> Token:
        with self._lock:
            t = self._token
            if t is not None and t.expires_at - self.ttl_s > time.time():
                return t
            self._token = self.provider.get_token()
            return self._token


class _LaxRedirect(urllib.request.HTTPRedirectHandler):
    def redirect_request(self, req, fp, code, msg, headers, newurl):
        if req.get_method() in ("PUT", "PATCH", "DELETE", "POST") and code in (301, 302, 303, 307, 308):
            new = urllib.request.Request(newurl, data=req.data, headers=dict(req.header_items()),
                                         method=req.get_method())
            return new
        return super().redirect_request(req, fp, code, msg, headers, newurl)


class DcosHttpExecutor:
    def __init__(self, token_provider: Optional[TokenProvider] = None, timeout_s: float = 30.0):
        self.token_provider = token_provider
        self.timeout_s = timeout_s
        self._opener = urllib.request.build_opener(_LaxRedirect())

    def execute(self, method: str, url: str, body: Optional[bytes] = None,
                content_type: str = "application/json") -> Tuple[int, bytes]:
        req = urllib.request.Request(url, data=body, method=method)
        if body is not None:
            req.add_header("Content-Type", content_type)
        if self.token_provider is not None:
            req.add_header("Authorization", "token=" + self.token_provider.get_token().value)
        try:
            with self._opener.open(req, timeout=self.timeout_s) as resp:
                return resp.status, resp.read()
        except urllib.error.HTTPError as e:
            return e.code, e.read() or b""


class ServiceAccountIAMTokenClient(TokenProvider):
    def __init__(self, executor: DcosHttpExecutor, uid: str, private_key_pem: str, login_url: Optional[str] = None):
        self.executor = executor
        self.uid = uid
        self.private_key_pem = private_key_pem
        self.login_url = login_url or master_uri() + "/acs/api/v1/auth/login"

    def get_token(self) -> Token:
        from dcos_commons_amd.offer.evaluate.security import native

        login = native().jwt_rs256(self.private_key_pem, {"uid": self.uid, "exp": int(time.time()) + 120})
        status, body = self.executor.execute("POST", self.login_url,
                                             json.dumps({"uid": self.uid, "token": login}).encode())
        if status != 200:
            raise DcosHttpError(status, "IAM login failed", body.decode("utf-8", "replace"))
        return Token.decode(json.loads(body)["token"])


def token_provider_from_service_account(credential: str, refresh_threshold_s: float = 30.0) -> TokenProvider:
    """``DCOS_SERVICE_ACCOUNT_CREDENTIAL`` is a file path or inline JSON with ``uid`` and ``private_key``
    (SchedulerConfig.getDcosAuthTokenProvider / loadFileOrEnvSecret, :484-536)."""
    if os.path.isfile(credential):
        with open(credential, "r", encoding="utf-8") as f:
            obj = json.load(f)
    else:
        obj = json.loads(credential)
    client = ServiceAccountIAMTokenClient(DcosHttpExecutor(timeout_s=30.0), obj["uid"], obj["private_key"],
                                          obj.get("login_endpoint"))
    return CachedTokenProvider(client, refresh_threshold_s)


# -- secrets -------------------------------------------------------------------------------
@dataclass
class SecretPayload:
    author: str
    value: str
    description: str

    def to_json(self) -> bytes:
        return json.dumps({"author": self.author, "value": self.value, "description": self.description}).encode()


class SecretsClient:
    def __init__(self, executor: DcosHttpExecutor, base_uri: Optional[str] = None):
        self.executor = executor
        self.base = base_uri or master_uri() + "/secrets/v1/secret/default/"

    def _query(self, op: str, path: str, method: str, ok: int, body: Optional[bytes] = None,
               suffix: str = "") -> bytes:
        url = self.base + urllib.parse.quote(path) + suffix
        status, data = self.executor.execute(method, url, body)
        if status != ok:
            raise DcosHttpError(status, f"Unable to {op} secret at '{path}'", data.decode("utf-8", "replace"))
        return data

    def list(self, path: str) -> List[str]:
        data = self._query("list", path, "GET", 200, suffix="?list=true")
        return list(json.loads(data).get("array") or [])

    def create(self, path: str, secret: SecretPayload) -> None:
        self._query("create", path, "PUT", 201, secret.to_json())

    def update(self, path: str, secret: SecretPayload) -> None:
        self._query("update", path, "PATCH", 204, secret.to_json())

    def delete(self, path: str) -> None:
        self._query("delete", path, "DELETE", 204)


# -- certificate authority -----------------------------------------------------------------
class CertificateAuthorityClient:
    def __init__(self, executor: DcosHttpExecutor, base_uri: Optional[str] = None):
        self.executor = executor
        self.base = base_uri or master_uri() + "/ca/api/v2/"

    def _post(self, path: str, data: Dict) -> Dict:
        status, body = self.executor.execute("POST", self.base + path, json.dumps(data).encode())
        if status != 200:
            raise DcosHttpError(status, "error from CA", body.decode("utf-8", "replace"))
        out = json.loads(body)
        if not out.get("success"):
            raise DcosHttpError(status, "CA request failed", "\n".join(
                f"[{e.get('code')}] {e.get('message')}" for e in out.get("errors") or []))
        return out["result"]

    def sign(self, csr_pem: str) -> str:
        return self._post("sign", {"certificate_request": csr_pem, "profile": ""})["certificate"]

    def chain_with_root_cert(self, cert_pem: str) -> List[str]:
        """Intermediates (without the submitted certificate) followed by the root CA certificate."""
        result = self._post("bundle", {"certificate": cert_pem})
        chain = split_pem(result.get("bundle") or "")
        if chain:
            chain = chain[1:]  # the bundle starts with the submitted certificate
        root = result.get("root") or ""
        if not root:
            raise DcosHttpError(200, "Failed to retrieve Root CA certificate")
        return chain + [root]


def split_pem(bundle: str) -> List[str]:
    out, cur = [], []
    for line in bundle.splitlines(keepends=True):
        if line.startswith("-----BEGIN"):
            cur = [line]
        elif line.startswith("-----END"):
            cur.append(line if line.endswith("\n") else line + "\n")
            out.append("".join(cur))
            cur = []
        elif cur:
            cur.append(line)
    return out


class DcosVersionClient:
    """``GET /dcos-metadata/dcos-version.json`` -> ``{"version": ...}`` (DcosVersionClient.java)."""

    def __init__(self, executor: DcosHttpExecutor, base_uri: Optional[str] = None):
        self.executor = executor
        self.url = (base_uri or master_uri()) + "/dcos-metadata/dcos-version.json"

    def get_version(self) -> str:
        return self.get_dcos_version().version

    def get_dcos_version(self):
        """The version document as a ``DcosVersion`` (version string + variant)."""
        from dcos_commons_amd.dcos.capabilities import DcosVersion

        status, body = self.executor.execute("GET", self.url)
        if status != 200:
            raise DcosHttpError(status, "version lookup failed")
        return DcosVersion.from_json(body)
