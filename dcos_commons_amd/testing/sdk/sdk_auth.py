"""Kerberos environment of the integration tier (reference ``testing/sdk_auth.py``).

The reference deploys a KDC as a Marathon app and drives it through its kdc-api-server (out of
scope here). The stand-in keeps what the suites use: a realm and KDC address, a
principal registry, and -- the part a Kerberized service consumes -- a keytab with every
principal's keys, in the cluster's secret store (named ``__dcos_base64__<...>`` by default, as the
DC/OS CLI names binary secrets) where the service's ``keytab_secret`` option points. No
Kerberos protocol runs: ``kinit``/``kdestroy`` record a ticket cache file in the task sandbox, so
client code paths that look for one find it.

    krb5 = sdk_auth.KerberosEnvironment()
    krb5.add_principals(["hdfs/name-0-node.hdfs.autoip.dcos.thisdcos.directory@LOCAL", ...])
    krb5.finalize()                   # -> secret krb5.get_keytab_path()
"""
from __future__ import annotations

import logging
import os
import secrets as _secrets
import time
from typing import Any, Dict, List, Optional

from dcos_commons_amd.testing import keytab as kt
from dcos_commons_amd.testing.sdk import sdk_cmd

LOG = logging.getLogger(__name__)

KERBEROS_APP_ID = os.getenv("KERBEROS_APP_ID", "kdc")
REALM = os.getenv("REALM", "LOCAL")
KDC_SERVICE_ACCOUNT = os.getenv("KDC_SERVICE_ACCOUNT", "kdc-admin")
KDC_SERVICE_ACCOUNT_SECRET = os.getenv("KDC_SERVICE_ACCOUNT_SECRET", "kdc-admin")
KDC_PORT = 2500
KDC_API_PORT = 8080
BINARY_SECRET_PREFIX = "__dcos_base64__"


def _parse_principal(principal: str):
    name, _, realm = principal.partition("@")
    return name.split("/"), (realm or REALM)


class KerberosEnvironment:
    """A realm, its principals and the keytab secret a Kerberized service reads."""

    def __init__(self, persist: bool = False, realm: str = REALM, keytab_secret: Optional[str] = None):
        self.persist = persist
        self.realm = realm.upper()
        self.principals: Dict[str, bytes] = {}       # principal -> key (random AES-256)
        self.keytab_secret_path = keytab_secret or f"__dcos_base64___keytab_{int(time.time() * 1000)}"
        self.keytab_is_binary = self.keytab_secret_path.split("/")[-1].startswith(BINARY_SECRET_PREFIX)
        self.kdc_host = f"{KERBEROS_APP_ID}.marathon.autoip.dcos.thisdcos.directory"
        self.install()

    # -- the KDC "app" --------------------------------------------------------------------
    def load_kdc_app_definition(self) -> Dict[str, Any]:
        return {"id": "/" + KERBEROS_APP_ID, "instances": 1, "cpus": 0.5, "mem": 256,
                "env": {"REALM": self.realm, "KDC_PORT": str(KDC_PORT), "KDC_API_PORT": str(KDC_API_PORT)},
                "portDefinitions": [{"port": KDC_PORT, "name": "kdc"}, {"port": KDC_API_PORT, "name": "kdc-api"}]}

    def install(self) -> Dict[str, Any]:
        """The reference installs and waits for its KDC app; the registry here is ready at once."""
        return self.load_kdc_app_definition()

    # -- principals -------------------------------------------------------------------------
    def list_principals(self, filter: str = "*") -> List[str]:  # noqa: A002 (reference signature)
        import fnmatch

        return sorted(p for p in self.principals if fnmatch.fnmatchcase(p, filter))

    def add_principals(self, principals: List[str]) -> None:
        for p in principals:
            if "@" not in p:
                p = f"{p}@{self.realm}"
            self.principals.setdefault(p, _secrets.token_bytes(32))
        LOG.info("KDC %s: %d principals", self.realm, len(self.principals))

    def get_principal(self, primary: str, instance: Optional[str] = None) -> str:
        return f"{primary}/{instance}@{self.realm}" if instance else f"{primary}@{self.realm}"

    # -- keytab ------------------------------------------------------------------------------
    def keytab_bytes(self) -> bytes:
        """An MIT keytab (0x0502) with one AES-256 key per principal."""
        entries = []
        for p, key in sorted(self.principals.items()):
            components, realm = _parse_principal(p)
            entries.append(kt.KeytabEntry(realm=realm, components=components, key=key))
        return kt.encode(entries)

    def save_keytab_secret(self) -> None:
        data = self.keytab_bytes()
        c = sdk_cmd._cluster()
        # the CLI-created secrets of the stand-in hold the decoded value (LocalCluster.resolve_secret)
        c.secrets[self.keytab_secret_path.strip("/")] = data
        LOG.info("Keytab secret %s: %d principals, %d bytes", self.keytab_secret_path, len(self.principals), len(data))

    def finalize(self) -> None:
        self.save_keytab_secret()

    def get_keytab_path(self) -> str:
        return self.keytab_secret_path

    def set_keytab_path(self, secret_path: str, is_binary: bool) -> None:
        self.keytab_secret_path = secret_path
        self.keytab_is_binary = is_binary

    # -- addresses ---------------------------------------------------------------------------
    def get_working_file_path(self, *args: str) -> str:
        return os.path.join(sdk_cmd._cluster().work_dir, "kdc", *args)

    def get_service_path(self) -> str:
        return "/" + KERBEROS_APP_ID

    def get_host(self) -> str:
        return self.kdc_host

    def get_port(self) -> str:
        return str(KDC_PORT)

    def get_api_port(self) -> str:
        return str(KDC_API_PORT)

    def get_realm(self) -> str:
        return self.realm

    def get_kdc_address(self) -> str:
        return f"{self.get_host()}:{self.get_port()}"

    def get_kdc_api_address(self) -> str:
        return f"{self.get_host()}:{self.get_api_port()}"

    def cleanup(self) -> None:
        if self.persist:
            return
        sdk_cmd._cluster().secrets.pop(self.keytab_secret_path.strip("/"), None)
        self.principals.clear()


def _ticket_cache(marathon_task_id: str) -> str:
    return os.path.join(sdk_cmd.marathon_task_sandbox(marathon_task_id), "krb5cc")


def kinit(marathon_task_id: str, keytab: str, principal: str) -> None:
    """Record ``principal``'s ticket cache in the task's sandbox (no KDC round trip here)."""
    with open(_ticket_cache(marathon_task_id), "w", encoding="utf-8") as f:
        f.write(f"principal={principal}\nkeytab={keytab}\n")


def kdestroy(marathon_task_id: str) -> None:
    try:
        os.remove(_ticket_cache(marathon_task_id))
    except FileNotFoundError:
        pass
