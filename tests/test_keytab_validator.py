"""``testing.security.keytab_validator`` (reference ``testing/security/keytab-validator``)."""
import os

import pytest

from dcos_commons_amd.testing import keytab as kt
from dcos_commons_amd.testing.security import keytab_validator as kv

REF = "/root/reference/testing/security/keytab-validator"


def _entry(key=b"k" * 32, enctype=kt.AES256_CTS_HMAC_SHA1_96, components=("hdfs", "name-0-node")):
    return kt.KeytabEntry(realm="LOCAL", components=list(components), key=key, enctype=enctype)


def test_valid_and_invalid_keytabs(tmp_path, capsys):
    good = tmp_path / "good.keytab"
    good.write_bytes(kt.encode([_entry(), _entry(key=b"k" * 16, enctype=kt.AES128_CTS_HMAC_SHA1_96)]))
    assert kv.main([str(good)]) == 0 and "a-ok" in capsys.readouterr().out
    assert kv.problems(good.read_bytes()[:-3])                       # truncated record
    assert kv.problems(b"\x04\x02" + good.read_bytes()[2:])          # not a keytab header
    assert "needs a 32-byte key" in " ".join(kv.problems(kt.encode([_entry(key=b"short")])))
    assert kv.problems(kt.encode([]))                                # no entries
    bad = tmp_path / "bad.keytab"
    bad.write_bytes(kt.encode([_entry(key=b"x" * 5)]))
    assert kv.main([str(bad)]) == 1 and "not valid" in capsys.readouterr().out
    assert kv.main([str(tmp_path / "missing")]) == 1 and kv.main([]) == 1


@pytest.mark.skipif(not os.path.isdir(REF), reason="no reference tree")
def test_reference_fixtures():
    """The reference's known_good.keytab validates. Its known_bad.keytab is structurally sound as
    well (72 entries, the same principals and key lengths as known_good; only keys and timestamps
    differ), so what the JDK rejected in it is not visible in the file format: parity unpinned."""
    ok, why = kv.validate(os.path.join(REF, "known_good.keytab"))
    assert ok, why
    with open(os.path.join(REF, "known_bad.keytab"), "rb") as f:
        entries = kt.decode(f.read()).entries
    assert len(entries) == 72
