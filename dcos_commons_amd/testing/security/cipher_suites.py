"""OpenSSL <-> IANA/RFC TLS cipher-suite names (reference ``testing/security/cipher_suites.py``,
which holds a literal table).

Here the names are translated by rule from their parts -- key exchange, authentication, bulk
cipher and MAC -- so any suite OpenSSL can name (``ssl.SSLContext.get_ciphers``) converts, not just
those of a fixed list: ``ECDHE-RSA-AES128-GCM-SHA256`` <-> ``TLS_ECDHE_RSA_WITH_AES_128_GCM_SHA256``,
``DES-CBC3-SHA`` <-> ``TLS_RSA_WITH_3DES_EDE_CBC_SHA``, ``ADH-AES128-SHA`` <->
``TLS_DH_anon_WITH_AES_128_CBC_SHA``. TLS 1.3 suites (``TLS_AES_128_GCM_SHA256``) carry the same
name in both; SSLv2 suites keep their ``SSL_CK_*`` names. ``tests/test_cipher_suites.py`` checks the
rules against the reference's table when the reference tree is present (that table drops the
``TLS_`` prefix from most entries; the comparison ignores it).
"""
from __future__ import annotations

import re
from typing import Dict, Optional, Set, Tuple

# OpenSSL key-exchange/auth prefixes -> RFC "<kx>_<auth>" (longest match first)
_KX_PREFIXES = [
    ("ECDHE-ECDSA-", "ECDHE_ECDSA"), ("ECDHE-RSA-", "ECDHE_RSA"), ("ECDHE-PSK-", "ECDHE_PSK"),
    ("ECDH-ECDSA-", "ECDH_ECDSA"), ("ECDH-RSA-", "ECDH_RSA"), ("AECDH-", "ECDH_anon"),
    ("DHE-RSA-", "DHE_RSA"), ("DHE-DSS-", "DHE_DSS"), ("DHE-PSK-", "DHE_PSK"),
    ("EDH-RSA-", "DHE_RSA"), ("EDH-DSS-", "DHE_DSS"),
    ("DH-RSA-", "DH_RSA"), ("DH-DSS-", "DH_DSS"), ("ADH-", "DH_anon"),
    ("RSA-PSK-", "RSA_PSK"), ("PSK-", "PSK"),
    ("SRP-RSA-", "SRP_SHA_RSA"), ("SRP-DSS-", "SRP_SHA_DSS"), ("SRP-", "SRP_SHA"), ("KRB5-", "KRB5"),
]
# OpenSSL bulk-cipher spellings -> RFC (mode included); "+" marks an AEAD whose RFC name carries the PRF hash
_CIPHERS = [
    ("AES128-CBC", "AES_128_CBC"), ("AES256-CBC", "AES_256_CBC"),         # newer spellings (PSK/SRP suites)
    ("AES-128-CBC", "AES_128_CBC"), ("AES-256-CBC", "AES_256_CBC"), ("3DES-EDE-CBC", "3DES_EDE_CBC"),
    ("AES128-GCM", "AES_128_GCM"), ("AES256-GCM", "AES_256_GCM"),
    ("AES128-CCM8", "AES_128_CCM_8"), ("AES256-CCM8", "AES_256_CCM_8"),
    ("AES128-CCM", "AES_128_CCM"), ("AES256-CCM", "AES_256_CCM"),
    ("AES128", "AES_128_CBC"), ("AES256", "AES_256_CBC"),
    ("CAMELLIA128", "CAMELLIA_128_CBC"), ("CAMELLIA256", "CAMELLIA_256_CBC"),
    ("ARIA128-GCM", "ARIA_128_GCM"), ("ARIA256-GCM", "ARIA_256_GCM"),
    ("CHACHA20-POLY1305", "CHACHA20_POLY1305"),
    ("DES-CBC3", "3DES_EDE_CBC"), ("DES-CBC", "DES_CBC"), ("RC4", "RC4_128"),
    ("SEED", "SEED_CBC"), ("IDEA-CBC", "IDEA_CBC"), ("IDEA", "IDEA_CBC"), ("NULL", "NULL"),
]
# export-grade suites (obsolete, kept for parity): "EXP-" / "EXP1024-" + the usual parts
_EXPORT_CIPHERS = {"EXP": [("DES-CBC", "DES40_CBC"), ("RC4", "RC4_40"), ("RC2-CBC", "RC2_CBC_40")],
                   "EXP1024": [("DES-CBC", "DES_CBC"), ("RC4", "RC4_56")]}
_MACS = {"SHA": "SHA", "SHA256": "SHA256", "SHA384": "SHA384", "MD5": "MD5"}
_SPECIAL = {"TLS_FALLBACK_SCSV": "TLS_FALLBACK_SCSV",
            # SSLv2 suites have their own naming
            "DES-CBC-MD5": "SSL_CK_DES_64_CBC_WITH_MD5", "DES-CBC3-MD5": "SSL_CK_DES_192_EDE3_CBC_WITH_MD5",
            "RC4-64-MD5": "SSL_CK_RC4_64_WITH_MD5",
            "IDEA-CBC-MD5": "SSL_CK_IDEA_128_CBC_WITH_MD5", "RC2-CBC-MD5": "SSL_CK_RC2_128_CBC_WITH_MD5",
            # GOST suites do not follow the <kx>_WITH_<cipher>_<mac> pattern
            "GOST2001-GOST89-GOST89": "TLS_GOSTR341001_WITH_28147_CNT_IMIT",
            "GOST94-GOST89-GOST89": "TLS_GOSTR341094_WITH_28147_CNT_IMIT",
            "GOST94-NULL-GOST94": "TLS_GOSTR341094_WITH_NULL_GOSTR3411"}


def _split_openssl(name: str) -> Optional[Tuple[str, str, Optional[str]]]:
    kx = "RSA"
    rest = name
    for prefix, rfc in _KX_PREFIXES:
        if name.startswith(prefix):
            kx, rest = rfc, name[len(prefix):]
            break
    for ossl, rfc in _CIPHERS:
        if rest == ossl or rest.startswith(ossl + "-"):
            mac = rest[len(ossl) + 1:] or None
            return kx, rfc, mac
    return None


def _export_rfc(openssl_name: str) -> Optional[str]:
    grade, _, rest = openssl_name.partition("-")
    kx = "RSA"
    for prefix, rfc in _KX_PREFIXES:
        if rest.startswith(prefix):
            kx, rest = rfc, rest[len(prefix):]
            break
    for ossl, cipher in _EXPORT_CIPHERS[grade]:
        if rest.startswith(ossl + "-") and rest[len(ossl) + 1:] in _MACS:
            if kx == "KRB5" and cipher == "DES40_CBC":
                cipher = "DES_CBC_40"                  # the Kerberos export suites spell it so
            return f"TLS_{kx}_{'EXPORT' if grade == 'EXP' else 'EXPORT1024'}_WITH_{cipher}_{rest[len(ossl) + 1:]}"
    return None


def rfc_name(openssl_name: str) -> Optional[str]:
    """The IANA name of an OpenSSL cipher-suite name, or None if its parts are not recognised."""
    if openssl_name in _SPECIAL:
        return _SPECIAL[openssl_name]
    if openssl_name.startswith(("EXP-", "EXP1024-")):
        return _export_rfc(openssl_name)
    if openssl_name.startswith("TLS_"):           # TLS 1.3: the same name
        return openssl_name
    parts = _split_openssl(openssl_name)
    if parts is None:
        return None
    kx, cipher, mac = parts
    if cipher.endswith(("_GCM", "_CCM", "_CCM_8")) or cipher == "CHACHA20_POLY1305":
        # AEAD: the RFC name carries the PRF hash (SHA256 unless OpenSSL names SHA384)
        suffix = "_" + (_MACS.get(mac or "", "SHA256") if mac else "SHA256")
        if cipher.endswith(("_CCM", "_CCM_8")):
            suffix = ""                                # AES-CCM suites name no hash
    elif mac in _MACS:
        suffix = "_" + _MACS[mac]
    else:
        return None
    return f"TLS_{kx}_WITH_{cipher}{suffix}"


_RFC = re.compile(r"^TLS_(?P<kx>.+?)_WITH_(?P<rest>.+)$")


def _export_openssl(kx_rfc: str, rest: str) -> Optional[str]:
    kx, _, grade = kx_rfc.rpartition("_")
    grade = "EXP" if grade == "EXPORT" else "EXP1024"
    rest = rest.replace("DES_CBC_40", "DES40_CBC")
    prefixes = [p for p, r in _KX_PREFIXES if r == kx]
    # OpenSSL calls the ephemeral-DH export suites EDH-, their 1024-bit variants DHE-
    prefix = "" if kx == "RSA" else next((p for p in prefixes if p.startswith("EDH") == (grade == "EXP")),
                                         prefixes[0] if prefixes else None)
    if prefix is None:
        return None
    for ossl, cipher in _EXPORT_CIPHERS[grade]:
        if rest.startswith(cipher + "_") and rest[len(cipher) + 1:] in _MACS:
            return f"{grade}-{prefix}{ossl}-{rest[len(cipher) + 1:]}"
    return None


def openssl_name(rfc: str) -> Optional[str]:
    """The OpenSSL name of an IANA cipher-suite name (the inverse of ``rfc_name``)."""
    if rfc in _SPECIAL.values():
        return next(k for k, v in _SPECIAL.items() if v == rfc)
    m = _RFC.match(rfc)
    if m is None:
        return rfc if rfc.startswith("TLS_") else None
    kx_rfc, rest = m.group("kx"), m.group("rest")
    if kx_rfc.endswith(("_EXPORT", "_EXPORT1024")):
        return _export_openssl(kx_rfc, rest)
    # OpenSSL names the ephemeral-DH DES suites EDH-..., the others DHE-...
    edh = kx_rfc in ("DHE_RSA", "DHE_DSS") and rest.split("_WITH_")[-1].startswith(("DES_CBC", "3DES_EDE_CBC"))
    prefix = next((p for p, r in _KX_PREFIXES if r == kx_rfc and p.startswith("EDH") == edh), None)
    if prefix is None and kx_rfc != "RSA":
        return None
    plain = [c for c in _CIPHERS if "-CBC" not in c[0] or c[0].startswith(("DES", "IDEA"))]
    plain = [c for c in plain if c[0] != "IDEA"]
    if kx_rfc.endswith("PSK") or kx_rfc.startswith("SRP"):
        plain = [c for c in _CIPHERS if c[0] not in ("AES128", "AES256", "DES-CBC3")]   # OpenSSL names these with "-CBC"
        if kx_rfc.startswith("SRP"):
            plain = [c for c in plain if c[0] not in ("AES128-CBC", "AES256-CBC")]
        else:
            plain = [c for c in plain if c[0] not in ("AES-128-CBC", "AES-256-CBC")]
    for ossl, cipher in sorted(plain, key=lambda c: -len(c[1])):
        if rest == cipher or rest.startswith(cipher + "_"):
            mac = rest[len(cipher) + 1:]
            aead = cipher.endswith(("_GCM", "_CCM", "_CCM_8")) or cipher == "CHACHA20_POLY1305"
            name = (prefix or "") + ossl
            if aead:
                if mac in ("", "SHA256") and (cipher.endswith(("_CCM", "_CCM_8")) or cipher == "CHACHA20_POLY1305"):
                    return name
                return f"{name}-{mac or 'SHA256'}"
            return f"{name}-{mac}" if mac in _MACS.values() else None
    return None


def missing_openssl_ciphers(openssl_ciphers: Set[str]) -> Set[str]:
    """The OpenSSL names this module cannot translate (reference API)."""
    return {c for c in openssl_ciphers if rfc_name(c) is None}


def local_openssl_ciphers() -> Dict[str, Optional[str]]:
    """OpenSSL name -> RFC name of every suite this Python's OpenSSL offers."""
    import ssl

    ctx = ssl.SSLContext(ssl.PROTOCOL_TLS_CLIENT)
    ctx.set_ciphers("ALL:@SECLEVEL=0")
    return {c["name"]: rfc_name(c["name"]) for c in ctx.get_ciphers()}
