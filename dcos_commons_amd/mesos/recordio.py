"""RecordIO framing used by the Mesos v1 HTTP event stream: ``<decimal length>\\n<record bytes>``.

The reference gets this from the external ``mesos-http-adapter`` dependency
(sdk/scheduler/build.gradle:165-166); here it is a small incremental codec so the
scheduler can speak the v1 API directly.
"""
from __future__ import annotations

from typing import Callable, Iterator, List, Optional


class RecordIOError(ValueError):
    pass


MAX_RECORD_BYTES = 64 << 20
_MAX_HEADER_DIGITS = 20


def encode(record: bytes) -> bytes:
    return str(len(record)).encode("ascii") + b"\n" + record


class Decoder:
    """Incremental decoder: ``feed(chunk)`` returns every record completed by that chunk."""

    def __init__(self, max_record_bytes: int = MAX_RECORD_BYTES):
        self.max_record_bytes = max_record_bytes
        self._buf = bytearray()
        self._need: Optional[int] = None

    def feed(self, data: bytes) -> List[bytes]:
        self._buf += data
        out: List[bytes] = []
        while True:
            if self._need is None:
                nl = self._buf.find(b"\n")
                if nl < 0:
                    if len(self._buf) > _MAX_HEADER_DIGITS:
                        raise RecordIOError("record length header too long")
                    return out
                header = bytes(self._buf[:nl]).strip()
                if not header.isdigit():
                    raise RecordIOError(f"bad record length header {header[:32]!r}")
                self._need = int(header)
                if self._need > self.max_record_bytes:
                    raise RecordIOError(f"record of {self._need} bytes exceeds limit {self.max_record_bytes}")
                del self._buf[:nl + 1]
            if len(self._buf) < self._need:
                return out
            out.append(bytes(self._buf[:self._need]))
            del self._buf[:self._need]
            self._need = None

    @property
    def pending_bytes(self) -> int:
        return len(self._buf)


def iter_records(read: Callable[[int], bytes], chunk: int = 65536) -> Iterator[bytes]:
    """Yields records from a ``read(n)`` callable until it returns ``b""`` (end of stream)."""
    dec = Decoder()
    while True:
        data = read(chunk)
        if not data:
            if dec.pending_bytes:
                raise RecordIOError("stream ended inside a record")
            return
        yield from dec.feed(data)
