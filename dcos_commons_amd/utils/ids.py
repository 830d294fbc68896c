"""Random (version 4) UUIDs for resource, persistence, task, offer and plan-element IDs.

``uuid4_str()`` returns the same format as ``str(uuid.uuid4())`` (reference: ``UUID.randomUUID()``)
and ``uuid4()`` a ``uuid.UUID``, both from a pooled ``os.urandom`` buffer. Besides the syscall
itself, ``uuid.uuid4()``'s ``os.urandom`` releases the GIL: in a process where the offer loop, the
master's dispatcher and the status path share the interpreter, every such call can park the
calling thread for a whole GIL switch interval (5 ms) behind a busy peer. Offer evaluation mints
several IDs per pod per offer and the recovery plan is rebuilt (new element IDs) on every cycle, so
these calls sat on the deploy critical path.
"""
from __future__ import annotations

import os
import threading
import uuid as _uuid

_POOL = 4096
_lock = threading.Lock()
_buf = b""
_pos = 0


def _reset_after_fork() -> None:
    """A forked child must not replay its parent's pooled random bytes (duplicate IDs)."""
    global _buf, _pos, _lock
    _lock = threading.Lock()
    _buf, _pos = b"", 0


if hasattr(os, "register_at_fork"):
    os.register_at_fork(after_in_child=_reset_after_fork)


def _random16() -> bytearray:
    global _buf, _pos
    with _lock:
        if _pos + 16 > len(_buf):
            _buf, _pos = os.urandom(_POOL), 0
        b = bytearray(_buf[_pos:_pos + 16])
        _pos += 16
    b[6] = (b[6] & 0x0F) | 0x40   # version 4
    b[8] = (b[8] & 0x3F) | 0x80   # RFC 4122 variant
    return b


def uuid4_str() -> str:
    h = _random16().hex()
    return f"{h[:8]}-{h[8:12]}-{h[12:16]}-{h[16:20]}-{h[20:]}"


def uuid4() -> _uuid.UUID:
    """Drop-in for ``uuid.uuid4()``."""
    return _uuid.UUID(bytes=bytes(_random16()))


def uuid4_bytes() -> bytes:
    return bytes(_random16())


def uuid4_hex() -> str:
    return _random16().hex()
