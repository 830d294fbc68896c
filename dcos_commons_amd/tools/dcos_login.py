"""Log in to a DC/OS cluster and set up the CLI's cluster config (reference: tools/dcos_login.py).

``python -m dcos_commons_amd.tools.dcos_login`` with ``CLUSTER_URL`` (required) and either
``DCOS_ACS_TOKEN`` (used as is), a service account (``DCOS_SERVICE_ACCOUNT_CREDENTIAL``: the
``{"uid", "private_key"}`` JSON, logged in with an RS256 JWT) or ``DCOS_LOGIN_USERNAME`` /
``DCOS_LOGIN_PASSWORD`` (default ``bootstrapuser`` / ``deleteme``). The token lands in
``$DCOS_DIR/clusters/<cluster id>/dcos.toml`` (``DCOS_DIR`` default ``~/.dcos``), which becomes
the attached cluster.
"""
from __future__ import annotations

import json
import logging
import os
import sys
import time
import urllib.request
from typing import Optional

LOGGER = logging.getLogger(__name__)
DEFAULT_USERNAME, DEFAULT_PASSWORD = "bootstrapuser", "deleteme"
TOML_TEMPLATE = """[cluster]
name = "{name}"
[core]
dcos_acs_token = "{token}"
dcos_url = "{url}"
ssl_verify = "false"
"""


def http_request(method: str, url: str, path: str, token: Optional[str] = None, body: Optional[dict] = None) -> dict:
    data = json.dumps(body).encode() if body is not None else None
    req = urllib.request.Request(url.rstrip("/") + path, data=data, method=method)
    req.add_header("Content-Type", "application/json")
    if token:
        req.add_header("Authorization", f"token={token}")
    with urllib.request.urlopen(req, timeout=30) as r:
        return json.loads(r.read() or b"null")


def login(dcos_url: str, username: str = DEFAULT_USERNAME, password: str = DEFAULT_PASSWORD,
          service_account_credential: Optional[str] = None) -> str:
    """A session token for the user, or for the service account when its credential is given."""
    if service_account_credential:
        from dcos_commons_amd.offer.evaluate.security import native

        cred = json.loads(service_account_credential)
        jwt = native().jwt_rs256(cred["private_key"], {"uid": cred["uid"], "exp": int(time.time()) + 300})
        body = {"uid": cred["uid"], "token": jwt}
    else:
        body = {"uid": username, "password": password}
    LOGGER.info("Logging into %s as %s", dcos_url, body["uid"])
    return http_request("POST", dcos_url, "/acs/api/v1/auth/login", body=body)["token"]


def configure_cli(dcos_url: str, token: str, dcos_dir: Optional[str] = None) -> str:
    """Writes the cluster config and attaches it; returns the config path."""
    cluster_id = http_request("GET", dcos_url, "/metadata", token)["CLUSTER_ID"]
    name = http_request("GET", dcos_url, "/mesos/state-summary", token)["cluster"]
    base = dcos_dir or os.environ.get("DCOS_DIR") or os.path.expanduser("~/.dcos")
    cluster_dir = os.path.join(base, "clusters", cluster_id)
    os.makedirs(cluster_dir, exist_ok=True)
    path = os.path.join(cluster_dir, "dcos.toml")
    with open(path, "w", encoding="utf-8") as f:
        f.write(TOML_TEMPLATE.format(name=name, token=token, url=dcos_url))
    os.chmod(path, 0o600)
    for other in os.listdir(os.path.join(base, "clusters")):   # attach: exactly one cluster marked
        marker = os.path.join(base, "clusters", other, "attached")
        if other != cluster_id and os.path.exists(marker):
            os.remove(marker)
    open(os.path.join(cluster_dir, "attached"), "w").close()
    return path


def login_session() -> str:
    url = os.environ.get("CLUSTER_URL")
    if not url:
        raise ValueError("CLUSTER_URL must be set")
    token = os.environ.get("DCOS_ACS_TOKEN") or login(
        url, os.environ.get("DCOS_LOGIN_USERNAME") or DEFAULT_USERNAME,
        os.environ.get("DCOS_LOGIN_PASSWORD") or DEFAULT_PASSWORD,
        os.environ.get("DCOS_SERVICE_ACCOUNT_CREDENTIAL"))
    return configure_cli(url, token)


if __name__ == "__main__":
    logging.basicConfig(level=logging.INFO, format="%(message)s")
    print(login_session())
    sys.exit(0)
