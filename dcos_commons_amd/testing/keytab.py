"""MIT keytab encoding for test fixtures and keytab secrets of Kerberized test services.

A minimal writer/reader of the file format ``keytab-fix`` (``native/keytab/keytab_fix.cpp``, the
counterpart of the reference's hdfs ``keytab-fix`` tool) rewrites: a big-endian ``u16`` version
(0x0502 or 0x0501) followed by size-prefixed records (``i32``; negative = a deleted hole) holding
the principal (component count, counted realm and components, ``u32`` name type for 0x0502),
``u32`` timestamp, ``u8`` kvno, ``u16`` enctype, counted key, and optionally a trailing ``u32``
kvno (what MIT kadmin/ktutil write and Hadoop 3.2.0 cannot read, HADOOP-16283).
"""
from __future__ import annotations

import struct
from dataclasses import dataclass, field
from typing import List, Optional, Tuple

KRB5_NT_PRINCIPAL = 1
AES256_CTS_HMAC_SHA1_96 = 18
AES128_CTS_HMAC_SHA1_96 = 17


@dataclass
class KeytabEntry:
    realm: str
    components: List[str]
    key: bytes
    kvno: int = 1
    enctype: int = AES256_CTS_HMAC_SHA1_96
    timestamp: int = 1_700_000_000
    name_type: int = KRB5_NT_PRINCIPAL
    kvno32: Optional[int] = None      # the optional trailing 32-bit kvno (None: not written)
    padding: bytes = b""              # bytes after the record body, counted in its size

    @property
    def principal(self) -> Tuple[str, Tuple[str, ...]]:
        return self.realm, tuple(self.components)


def _counted(b: bytes) -> bytes:
    return struct.pack(">H", len(b)) + b


def encode_entry(e: KeytabEntry, version: int = 0x0502) -> bytes:
    n = len(e.components) + (1 if version == 0x0501 else 0)
    body = struct.pack(">H", n) + _counted(e.realm.encode())
    for c in e.components:
        body += _counted(c.encode())
    if version == 0x0502:
        body += struct.pack(">I", e.name_type)
    body += struct.pack(">IBH", e.timestamp, e.kvno & 0xFF, e.enctype) + _counted(e.key)
    if e.kvno32 is not None:
        body += struct.pack(">I", e.kvno32)
    body += e.padding
    return struct.pack(">i", len(body)) + body


def encode(entries: List[KeytabEntry], version: int = 0x0502, holes: Tuple[Tuple[int, int], ...] = ()) -> bytes:
    """A keytab of ``entries``; ``holes`` = ((before entry index, hole size), ...) deleted records."""
    out = struct.pack(">H", version)
    hole_at = dict(holes)
    for i, e in enumerate(entries):
        if i in hole_at:
            out += struct.pack(">i", -hole_at[i]) + b"\0" * hole_at[i]
        out += encode_entry(e, version)
    return out


@dataclass
class Keytab:
    version: int
    entries: List[KeytabEntry] = field(default_factory=list)


def decode(data: bytes) -> Keytab:
    (version,) = struct.unpack_from(">H", data, 0)
    pos = 2
    kt = Keytab(version)
    while pos + 4 <= len(data):
        (size,) = struct.unpack_from(">i", data, pos)
        pos += 4
        if size == 0:
            break
        if size < 0:
            pos += -size
            continue
        end = pos + size
        (n,) = struct.unpack_from(">H", data, pos)
        pos += 2
        if version == 0x0501:
            n -= 1

        def counted():
            nonlocal pos
            (ln,) = struct.unpack_from(">H", data, pos)
            pos += 2
            s = data[pos:pos + ln]
            pos += ln
            return s
        realm = counted().decode()
        comps = [counted().decode() for _ in range(n)]
        name_type = KRB5_NT_PRINCIPAL
        if version == 0x0502:
            (name_type,) = struct.unpack_from(">I", data, pos)
            pos += 4
        ts, kvno, enctype = struct.unpack_from(">IBH", data, pos)
        pos += 7
        key = counted()
        kvno32 = None
        if end - pos >= 4:
            (kvno32,) = struct.unpack_from(">I", data, pos)
        kt.entries.append(KeytabEntry(realm, comps, key, kvno, enctype, ts, name_type, kvno32))
        pos = end
    return kt
