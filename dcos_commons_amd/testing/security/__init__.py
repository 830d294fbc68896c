"""Security helpers of the integration tier (reference ``testing/security/``): TLS service accounts
and artifacts signed by the cluster CA (``transport_encryption``), Kerberos principal and krb5.conf
helpers (``kerberos``) and OpenSSL <-> RFC cipher-suite names (``cipher_suites``), all against the
local DC/OS stand-in (``testing.cluster``)."""
