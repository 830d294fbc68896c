"""Keytab validation (reference ``testing/security/keytab-validator``: a Java tool that loads a
keytab with the JDK's ``KeyTab`` and reports whether it is valid).

Here the MIT keytab format is checked directly (``testing.keytab``): a 0x0501/0x0502 header, records
that decode to the end of the file, a realm and at least one component per principal, and a key
of the length its encryption type requires. Exit status and messages follow the Java tool.

    python -m dcos_commons_amd.testing.security.keytab_validator <keytab>
"""
from __future__ import annotations

import os
import sys
from typing import List, Optional, Sequence, Tuple

from dcos_commons_amd.testing import keytab as kt

# RFC 3961/3962/4757 key lengths per encryption type
KEY_LENGTHS = {1: 8, 3: 8, 16: 24, 17: 16, 18: 32, 19: 16, 20: 32, 23: 16, 24: 16, 25: 16, 26: 32}


def problems(data: bytes) -> List[str]:
    """Everything wrong with a keytab's bytes (empty: valid)."""
    if len(data) < 2 or data[:2] not in (b"\x05\x02", b"\x05\x01"):
        return ["not an MIT keytab (expected a 0x0501/0x0502 header)"]
    try:
        parsed = kt.decode(data)
    except Exception as e:  # noqa: BLE001 (any decoding failure makes the file invalid)
        return [f"unreadable record: {e}"]
    out = []
    if not parsed.entries:
        out.append("no entries")
    for i, e in enumerate(parsed.entries):
        if not e.realm or not e.components or not all(e.components):
            out.append(f"entry {i}: incomplete principal {e.components}@{e.realm}")
        want = KEY_LENGTHS.get(e.enctype)
        if want is not None and len(e.key) != want:
            out.append(f"entry {i}: enctype {e.enctype} needs a {want}-byte key, has {len(e.key)}")
    return out


def validate(path: str) -> Tuple[bool, Optional[str]]:
    with open(path, "rb") as f:
        found = problems(f.read())
    return (not found), ("; ".join(found) if found else None)


def main(argv: Optional[Sequence[str]] = None) -> int:
    args = list(sys.argv[1:] if argv is None else argv)
    if len(args) != 1 or args[0] in ("-h", "--help", "help"):
        print("Usage: keytab-validator <path to file>")
        return 1
    if not os.path.exists(args[0]):
        print("Supplied file does not exist!")
        return 1
    ok, why = validate(args[0])
    print("This keytab is a-ok" if ok else f"Keytab not valid :( ({why})")
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
