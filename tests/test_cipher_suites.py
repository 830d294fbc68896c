"""OpenSSL <-> IANA cipher-suite names (``testing.security.cipher_suites``; reference
``testing/security/cipher_suites.py``)."""
import ast
import os

import pytest

from dcos_commons_amd.testing.security import cipher_suites as cs

KNOWN = {
    "ECDHE-RSA-AES128-GCM-SHA256": "TLS_ECDHE_RSA_WITH_AES_128_GCM_SHA256",
    "ECDHE-ECDSA-AES256-GCM-SHA384": "TLS_ECDHE_ECDSA_WITH_AES_256_GCM_SHA384",
    "ECDHE-ECDSA-CHACHA20-POLY1305": "TLS_ECDHE_ECDSA_WITH_CHACHA20_POLY1305_SHA256",
    "DHE-RSA-AES256-SHA256": "TLS_DHE_RSA_WITH_AES_256_CBC_SHA256",
    "AES128-SHA": "TLS_RSA_WITH_AES_128_CBC_SHA",
    "DES-CBC3-SHA": "TLS_RSA_WITH_3DES_EDE_CBC_SHA",
    "EDH-RSA-DES-CBC3-SHA": "TLS_DHE_RSA_WITH_3DES_EDE_CBC_SHA",
    "ADH-AES128-SHA": "TLS_DH_anon_WITH_AES_128_CBC_SHA",
    "AECDH-AES256-SHA": "TLS_ECDH_anon_WITH_AES_256_CBC_SHA",
    "RC4-MD5": "TLS_RSA_WITH_RC4_128_MD5",
    "PSK-AES128-CBC-SHA": "TLS_PSK_WITH_AES_128_CBC_SHA",
    "ECDHE-ECDSA-AES128-CCM8": "TLS_ECDHE_ECDSA_WITH_AES_128_CCM_8",
    "EXP-EDH-RSA-DES-CBC-SHA": "TLS_DHE_RSA_EXPORT_WITH_DES40_CBC_SHA",
    "TLS_AES_128_GCM_SHA256": "TLS_AES_128_GCM_SHA256",
    "TLS_FALLBACK_SCSV": "TLS_FALLBACK_SCSV",
}


@pytest.mark.parametrize("ossl,rfc", sorted(KNOWN.items()))
def test_known_suites_both_ways(ossl, rfc):
    assert cs.rfc_name(ossl) == rfc
    assert cs.openssl_name(rfc) == ossl


def test_unknown_names_and_missing():
    assert cs.rfc_name("NOT-A-CIPHER") is None and cs.openssl_name("NOT_A_SUITE") is None
    assert cs.missing_openssl_ciphers({"AES128-SHA", "NOT-A-CIPHER"}) == {"NOT-A-CIPHER"}


def test_every_modern_local_openssl_suite_translates():
    names = cs.local_openssl_ciphers()
    modern = {n: r for n, r in names.items() if n.startswith(("ECDHE-", "DHE-", "AES", "TLS_"))
              and "ARIA" not in n and "PSK" not in n}
    assert modern and all(modern.values()), {n for n, r in modern.items() if r is None}
    for n, r in modern.items():
        assert cs.openssl_name(r) == n


REF = "/root/reference/testing/security/cipher_suites.py"


@pytest.mark.skipif(not os.path.exists(REF), reason="no reference tree")
def test_rules_reproduce_the_reference_table():
    """Every pair of the reference's literal table (read as data, never imported): the rules give
    the same names, ignoring the ``TLS_`` prefix the table drops from most entries; the reverse
    direction lands on one of OpenSSL's aliases of the suite (the table has EDH-/DHE- twins)."""
    with open(REF, encoding="utf-8") as f:
        tree = ast.parse(f.read())
    table = next(ast.literal_eval(n.value) for n in tree.body
                 if isinstance(n, ast.Assign) and getattr(n.targets[0], "id", "") == "OPENSSL_TO_RFC_NAMES")

    def norm(x):
        return x[4:] if x and x.startswith("TLS_") else x

    assert len(table) > 200
    assert [k for k, v in table.items() if norm(cs.rfc_name(k)) != norm(v)] == []
    for k, v in table.items():
        full = v if v.startswith(("TLS_", "SSL_")) else "TLS_" + v
        back = cs.openssl_name(full)
        assert back is not None and norm(cs.rfc_name(back)) == norm(v), (k, v, back)
