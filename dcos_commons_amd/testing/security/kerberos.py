"""Kerberos principal names and krb5.conf for test clients (reference
``testing/security/kerberos.py``). The KDC side is ``testing.sdk.sdk_auth.KerberosEnvironment``."""
from __future__ import annotations

import itertools
import logging
from typing import Iterable, List, Optional

from dcos_commons_amd.testing.sdk import sdk_cmd

LOG = logging.getLogger(__name__)


def generate_principal(primary: str, instance: Optional[str], realm: str) -> str:
    """``primary[/instance]@REALM`` (realms are upper case)."""
    name = f"{primary}/{instance}" if instance else primary
    return f"{name}@{realm.upper()}"


# the reference's spelling, kept so that suites written against it import unchanged
genererate_principal = generate_principal


def generate_principal_list(primaries: Iterable[str], instances: Iterable[str], realm: str) -> List[str]:
    """Every primary on every instance."""
    return [generate_principal(p, i, realm) for p, i in itertools.product(list(primaries), list(instances))]


def krb5_config_lines(realm: str, kdc_address: str) -> List[str]:
    return ["[libdefaults]", f"default_realm = {realm}", "", "[realms]", f"  {realm} = {{",
            f"    kdc = {kdc_address}", "  }"]


def write_krb5_config_file(task: str, filename: str, krb5) -> str:
    """Write a client krb5.conf for ``krb5``'s realm and KDC into the sandbox of the Marathon task
    ``task``; returns the file name."""
    lines = krb5_config_lines(krb5.get_realm(), krb5.get_kdc_address())
    LOG.info("Writing %s to %s: %s", filename, task, lines)
    if not sdk_cmd.create_task_text_file(task, filename, lines):
        raise RuntimeError(f"could not write {filename} in task {task}")
    return filename
