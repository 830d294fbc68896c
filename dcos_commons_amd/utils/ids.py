"""Random (version 4) UUID strings for resource, persistence, task and step IDs.

``uuid4_str()`` returns the same format as ``str(uuid.uuid4())`` (reference: ``UUID.randomUUID()``)
from a pooled ``os.urandom`` buffer, skipping the per-call syscall and ``uuid.UUID`` object. Offer
evaluation mints several IDs per pod per offer; this keeps them off the hot-path profile.
"""
from __future__ import annotations

import os
import threading

_POOL = 4096
_lock = threading.Lock()
_buf = b""
_pos = 0


def uuid4_str() -> str:
    global _buf, _pos
    with _lock:
        if _pos + 16 > len(_buf):
            _buf, _pos = os.urandom(_POOL), 0
        b = bytearray(_buf[_pos:_pos + 16])
        _pos += 16
    b[6] = (b[6] & 0x0F) | 0x40   # version 4
    b[8] = (b[8] & 0x3F) | 0x80   # RFC 4122 variant
    h = b.hex()
    return f"{h[:8]}-{h[8:12]}-{h[12:16]}-{h[16:20]}-{h[20:]}"
