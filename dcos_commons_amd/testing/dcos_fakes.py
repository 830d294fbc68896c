"""Local stand-ins for the DC/OS cluster services the scheduler talks to ("DC/OS CA /
Secrets / IAM (HTTPS) -> pluggable interfaces with in-memory fakes").

``FakeDcosCluster`` serves, on 127.0.0.1:
* ``POST /acs/api/v1/auth/login`` -- verifies the service account's RS256 login JWT against the
  registered public key and issues a signed session token with an ``exp`` claim;
* ``/secrets/v1/secret/default/<path>`` -- GET (value, or ``?list=true`` -> ``{"array": [...]}``),
  PUT (201 / 409 exists), PATCH (204 / 404), DELETE (204 / 404); requires a valid token when
  ``require_auth``;
* ``POST /ca/api/v2/sign`` and ``/bundle`` -- a real CA (root, optionally an intermediate) that
  signs CSRs with ``libsdktls`` and answers in the CFSSL JSON shape the reference parses;
* ``GET /dcos-metadata/dcos-version.json``.
Set ``SDK_DCOS_MASTER_URI`` to ``cluster.url`` to point the clients at it.
"""
from __future__ import annotations

import json
import threading
import time
import urllib.parse
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer
from typing import Dict, List, Optional

from dcos_commons_amd.offer.evaluate.security import native

SECRETS_PREFIX = "/secrets/v1/secret/default/"


class FakeDcosCluster:
    def __init__(self, require_auth: bool = True, token_lifetime_s: float = 300.0, intermediate_ca: bool = False,
                 version: str = "1.13.0"):
        n = native()
        self.require_auth = require_auth
        self.token_lifetime_s = token_lifetime_s
        self.version = version
        self.secrets: Dict[str, dict] = {}
        self.service_accounts: Dict[str, str] = {}  # uid -> public key PEM
        self.users: Dict[str, str] = {}             # uid -> password
        self.cluster_id = "local-" + "%08x" % (id(self) & 0xffffffff)
        self.cluster_name = "local-dcos"
        self.issued: Dict[str, float] = {}
        self.logins = 0
        self.signed: List[str] = []
        self.requests: List[tuple] = []
        self._lock = threading.Lock()
        self._iam_key = n.generate_rsa_key()
        self.root_key = n.generate_rsa_key()
        self.root_cert = n.self_signed_ca(self.root_key, "CN=DC/OS Root CA,O=Mesosphere\\, Inc")
        if intermediate_ca:
            self.int_key = n.generate_rsa_key()
            csr = n.make_csr(self.int_key, "CN=DC/OS Intermediate CA", [])
            self.int_cert = n.sign_csr(self.root_key, self.root_cert, csr, 3650, as_ca=True)
        else:
            self.int_key = self.int_cert = None
        owner = self

        class Handler(_Handler):
            cluster = owner

        self.httpd = ThreadingHTTPServer(("127.0.0.1", 0), Handler)
        self.httpd.daemon_threads = True
        self._thread: Optional[threading.Thread] = None

    @property
    def url(self) -> str:
        return f"http://127.0.0.1:{self.httpd.server_address[1]}"

    def start(self) -> "FakeDcosCluster":
        self._thread = threading.Thread(target=self.httpd.serve_forever, name="fake-dcos", daemon=True)
        self._thread.start()
        return self

    def stop(self) -> None:
        self.httpd.shutdown()
        self.httpd.server_close()

    def add_service_account(self, uid: str) -> str:
        """Registers a service account and returns its credential JSON (uid + private_key)."""
        n = native()
        key = n.generate_rsa_key()
        self.service_accounts[uid] = n.public_key_pem(key)
        return json.dumps({"uid": uid, "private_key": key, "scheme": "RS256",
                           "login_endpoint": self.url + "/acs/api/v1/auth/login"})

    # -- handlers -------------------------------------------------------------------------
    def add_user(self, uid: str, password: str) -> None:
        """A local user account (``dcos auth login --username/--password``)."""
        self.users[uid] = password

    def login(self, body: dict):
        uid, token = body.get("uid"), body.get("token")
        if uid in self.users and "password" in body:
            if body["password"] != self.users[uid]:
                return 401, {"title": "Invalid authentication credentials"}
            exp = int(time.time() + self.token_lifetime_s)
            session = native().jwt_rs256(self._iam_key, {"uid": uid, "exp": exp})
            with self._lock:
                self.issued[session] = exp
                self.logins += 1
            return 200, {"token": session}
        pub = self.service_accounts.get(uid)
        claims = native().verify_jwt(pub, token) if pub and token else None
        if claims is None or claims.get("uid") != uid or claims.get("exp", 0) < time.time():
            return 401, {"title": "Invalid authentication credentials"}
        exp = int(time.time() + self.token_lifetime_s)
        session = native().jwt_rs256(self._iam_key, {"uid": uid, "exp": exp})
        with self._lock:
            self.issued[session] = exp
            self.logins += 1
        return 200, {"token": session}

    def authorized(self, header: Optional[str]) -> bool:
        if not self.require_auth:
            return True
        if not header or not header.startswith("token="):
            return False
        exp = self.issued.get(header[len("token="):])
        return exp is not None and exp > time.time()

    def sign(self, body: dict):
        csr = body.get("certificate_request") or ""
        try:
            if self.int_cert is not None:
                cert = native().sign_csr(self.int_key, self.int_cert, csr, 365)
            else:
                cert = native().sign_csr(self.root_key, self.root_cert, csr, 365)
        except Exception as e:  # noqa: BLE001
            return 200, {"success": False, "errors": [{"code": 1000, "message": str(e)}], "result": None}
        with self._lock:
            self.signed.append(cert)
        return 200, {"success": True, "errors": [], "result": {"certificate": cert}}

    def bundle(self, body: dict):
        cert = body.get("certificate") or ""
        chain = cert + (self.int_cert or "")
        return 200, {"success": True, "errors": [], "result": {"bundle": chain, "root": self.root_cert}}

    def secret_op(self, method: str, path: str, query: Dict[str, str], body: Optional[dict]):
        with self._lock:
            if method == "GET" and query.get("list") == "true":
                prefix = path.rstrip("/") + "/" if path else ""
                names = sorted(k[len(prefix):] for k in self.secrets if k.startswith(prefix))
                return 200, {"array": names}
            if method == "GET":
                s = self.secrets.get(path)
                return (200, s) if s is not None else (404, {"message": "not found"})
            if method == "PUT":
                if path in self.secrets:
                    return 409, {"message": "exists"}
                self.secrets[path] = dict(body or {})
                return 201, None
            if method == "PATCH":
                if path not in self.secrets:
                    return 404, {"message": "not found"}
                self.secrets[path].update(body or {})
                return 204, None
            if method == "DELETE":
                if self.secrets.pop(path, None) is None:
                    return 404, {"message": "not found"}
                return 204, None
        return 405, None


class _Handler(BaseHTTPRequestHandler):
    protocol_version = "HTTP/1.1"
    cluster: FakeDcosCluster = None

    def log_message(self, fmt, *args):
        pass

    def _reply(self, status: int, body=None) -> None:
        data = b"" if body is None else json.dumps(body).encode()
        self.send_response(status)
        self.send_header("Content-Type", "application/json")
        self.send_header("Content-Length", str(len(data)))
        self.end_headers()
        if data:
            self.wfile.write(data)

    def _handle(self, method: str) -> None:
        c = self.cluster
        u = urllib.parse.urlsplit(self.path)
        query = {k: v[-1] for k, v in urllib.parse.parse_qs(u.query).items()}
        n = int(self.headers.get("Content-Length") or 0)
        raw = self.rfile.read(n) if n else b""
        try:
            body = json.loads(raw) if raw else None
        except ValueError:
            self._reply(400, {"message": "bad json"})
            return
        c.requests.append((method, u.path))
        if u.path == "/acs/api/v1/auth/login" and method == "POST":
            self._reply(*c.login(body or {}))
            return
        if u.path == "/dcos-metadata/dcos-version.json" and method == "GET":
            self._reply(200, {"version": c.version, "dcos-variant": "enterprise"})
            return
        if not c.authorized(self.headers.get("Authorization")):
            self._reply(401, {"title": "Unauthorized"})
            return
        if u.path == "/metadata" and method == "GET":
            self._reply(200, {"CLUSTER_ID": c.cluster_id, "PUBLIC_IPV4": "127.0.0.1"})
        elif u.path == "/mesos/state-summary" and method == "GET":
            self._reply(200, {"cluster": c.cluster_name, "slaves": [], "frameworks": []})
        elif u.path == "/ca/api/v2/sign" and method == "POST":
            self._reply(*c.sign(body or {}))
        elif u.path == "/ca/api/v2/bundle" and method == "POST":
            self._reply(*c.bundle(body or {}))
        elif u.path.startswith(SECRETS_PREFIX):
            path = urllib.parse.unquote(u.path[len(SECRETS_PREFIX):])
            self._reply(*c.secret_op(method, path, query, body))
        else:
            self._reply(404, {"message": "no such endpoint"})

    def do_GET(self):  # noqa: N802
        self._handle("GET")

    def do_POST(self):  # noqa: N802
        self._handle("POST")

    def do_PUT(self):  # noqa: N802
        self._handle("PUT")

    def do_PATCH(self):  # noqa: N802
        self._handle("PATCH")

    def do_DELETE(self):  # noqa: N802
        self._handle("DELETE")
