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


class ChunkedDecoder:
    """Incremental HTTP/1.1 ``Transfer-Encoding: chunked`` decoder (``<hex size>[;ext]\\r\\n<data>\\r\\n``
    ... ``0\\r\\n<trailers>\\r\\n``). ``http.client`` hands a chunked body over one chunk per
    ``read1``; reading the socket directly and de-chunking here returns everything that has
    arrived, so a reader that fell behind gets every queued event in one pass. ``done`` turns true
    after the last (zero-size) chunk; bytes after it are ignored."""

    _MAX_LINE = 4096

    def __init__(self):
        self._buf = bytearray()
        self._left = 0            # data bytes still to come in the current chunk
        self._crlf = False        # the CRLF that ends a chunk's data is still to come
        self.done = False

    def feed(self, data: bytes) -> bytes:
        self._buf += data
        out = bytearray()
        while not self.done:
            if self._left:
                take = min(self._left, len(self._buf))
                if not take:
                    break
                out += self._buf[:take]
                del self._buf[:take]
                self._left -= take
                if self._left:
                    break
                self._crlf = True
            if self._crlf:
                if len(self._buf) < 2:
                    break
                if self._buf[:2] != b"\r\n":
                    raise RecordIOError("chunk data not followed by CRLF")
                del self._buf[:2]
                self._crlf = False
            nl = self._buf.find(b"\r\n")
            if nl < 0:
                if len(self._buf) > self._MAX_LINE:
                    raise RecordIOError("chunk size line too long")
                break
            line = bytes(self._buf[:nl]).split(b";", 1)[0].strip()
            try:
                size = int(line, 16)
            except ValueError:
                raise RecordIOError(f"bad chunk size {line[:32]!r}") from None
            del self._buf[:nl + 2]
            if size == 0:
                self.done = True
                break
            self._left = size
        return bytes(out)
