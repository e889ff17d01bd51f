"""Byte buffer for the packet builder and the header parser.

The subset of aioquic's ``Buffer`` (src/aioquic/buffer.py, backed by
``_buffer.c``) that packet assembly and header parsing use: a fixed-capacity
cursor over a ``bytearray`` with big-endian integers and QUIC variable-length
integers (RFC 9000 sec. 16).  Host-side framing only; nothing here touches
packet protection.
"""

from __future__ import annotations

UINT_VAR_MAX = (1 << 62) - 1
UINT_VAR_MAX_SIZE = 8


class BufferReadError(ValueError):
    pass


class BufferWriteError(ValueError):
    pass


def size_uint_var(value: int) -> int:
    """Encoded size of a variable-length integer."""
    if value < 0x40:
        return 1
    if value < 0x4000:
        return 2
    if value < 0x40000000:
        return 4
    if value <= UINT_VAR_MAX:
        return 8
    raise ValueError("Integer is too big for a variable-length integer")


def encode_uint_var(value: int) -> bytes:
    b = Buffer(capacity=UINT_VAR_MAX_SIZE)
    b.push_uint_var(value)
    return b.data


class Buffer:
    def __init__(self, capacity: int = 0, data: bytes | None = None) -> None:
        if data is not None:
            self._b = bytearray(data)
        else:
            self._b = bytearray(capacity)
        self._cap = len(self._b)
        self._pos = 0

    # -- cursor
    @property
    def capacity(self) -> int:
        return self._cap

    @property
    def data(self) -> bytes:
        """Bytes written so far (up to the cursor)."""
        return bytes(self._b[: self._pos])

    def data_slice(self, start: int, end: int) -> bytes:
        if start < 0 or end > self._cap or start > end:
            raise BufferReadError("Read out of bounds")
        return bytes(self._b[start:end])

    def eof(self) -> bool:
        return self._pos == self._cap

    def seek(self, pos: int) -> None:
        if pos < 0 or pos > self._cap:
            raise BufferReadError("Seek out of bounds")
        self._pos = pos

    def tell(self) -> int:
        return self._pos

    # -- reads
    def _take(self, n: int) -> memoryview:
        if n < 0 or self._pos + n > self._cap:
            raise BufferReadError("Read out of bounds")
        v = memoryview(self._b)[self._pos : self._pos + n]
        self._pos += n
        return v

    def pull_bytes(self, length: int) -> bytes:
        return bytes(self._take(length))

    def pull_uint8(self) -> int:
        return self._take(1)[0]

    def pull_uint16(self) -> int:
        return int.from_bytes(self._take(2), "big")

    def pull_uint32(self) -> int:
        return int.from_bytes(self._take(4), "big")

    def pull_uint64(self) -> int:
        return int.from_bytes(self._take(8), "big")

    def pull_uint_var(self) -> int:
        if self._pos >= self._cap:
            raise BufferReadError("Read out of bounds")
        size = 1 << (self._b[self._pos] >> 6)
        raw = int.from_bytes(self._take(size), "big")
        return raw & ((1 << (8 * size - 2)) - 1)

    # -- writes
    def _put(self, raw: bytes) -> None:
        end = self._pos + len(raw)
        if end > self._cap:
            raise BufferWriteError("Write out of bounds")
        self._b[self._pos : end] = raw
        self._pos = end

    def push_bytes(self, value: bytes) -> None:
        self._put(value)

    def push_uint8(self, value: int) -> None:
        self._put(value.to_bytes(1, "big"))

    def push_uint16(self, value: int) -> None:
        self._put(value.to_bytes(2, "big"))

    def push_uint32(self, value: int) -> None:
        self._put(value.to_bytes(4, "big"))

    def push_uint64(self, value: int) -> None:
        self._put(value.to_bytes(8, "big"))

    def push_uint_var(self, value: int) -> None:
        size = size_uint_var(value)
        tag = {1: 0x00, 2: 0x40, 4: 0x80, 8: 0xC0}[size]
        raw = bytearray(value.to_bytes(size, "big"))
        raw[0] |= tag
        self._put(bytes(raw))
