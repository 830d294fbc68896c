"""Service accounts and strict-mode setup (reference: testing/sdk_security.py).

On a cluster started with ``dcos_security=True`` the IAM service registers the account's public
key and the credential (uid + private key) is stored in the secret store under
``service_account_secret``, where Marathon hands it to the scheduler as
``DCOS_SERVICE_ACCOUNT_CREDENTIAL``.
"""
from __future__ import annotations

import logging
from typing import Any, Dict

LOG = logging.getLogger(__name__)


def _cluster():
    from dcos_commons_amd.testing.cluster import current

    return current()


def create_service_account(service_account_name: str, service_account_secret: str) -> None:
    c = _cluster()
    if c.dcos is None:
        raise RuntimeError("the local cluster runs without DC/OS security services (dcos_security=False)")
    LOG.info("Creating service account %s with credential secret %s", service_account_name, service_account_secret)
    credential = c.dcos.add_service_account(service_account_name)
    c.secrets[service_account_secret.strip("/")] = credential.encode("utf-8")


def delete_service_account(service_account_name: str, service_account_secret: str) -> None:
    c = _cluster()
    if c.dcos is not None:
        c.dcos.service_accounts.pop(service_account_name, None)
    c.secrets.pop(service_account_secret.strip("/"), None)


def setup_security(service_name: str, service_account: str = "", service_account_secret: str = "") -> Dict[str, Any]:
    """Creates the service's account; returns the package options that make the scheduler use it."""
    account = service_account or f"{service_name.strip('/').replace('/', '__')}-service-account"
    secret = service_account_secret or f"{service_name.strip('/')}/service-account-secret"
    create_service_account(account, secret)
    return {"service": {"service_account": account, "service_account_secret": secret}}


def cleanup_security(service_name: str, service_account: str = "", service_account_secret: str = "") -> None:
    account = service_account or f"{service_name.strip('/').replace('/', '__')}-service-account"
    secret = service_account_secret or f"{service_name.strip('/')}/service-account-secret"
    delete_service_account(account, secret)


def list_secrets(prefix: str = "") -> list:
    """Every secret under ``prefix`` in the store (CLI-created and scheduler-written)."""
    c = _cluster()
    names = set(c.secrets)
    if c.dcos is not None:
        with c.dcos._lock:
            names |= set(c.dcos.secrets)
    p = prefix.strip("/")
    return sorted(n for n in names if not p or n == p or n.startswith(p + "/"))
