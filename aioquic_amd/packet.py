"""Packet-number and header helpers used by the packet-protection path.

Mirrors aioquic src/aioquic/quic/packet.py: the first-byte bits :13-15,
QuicProtocolVersion, decode_packet_number :118-132, is_long_header :166-167,
the Retry integrity tag :135-159 (AES-128-GCM, computed on the GPU), and for
the batched callers the packet types and
long-header type codes :47-87, the header parser pull_quic_header :181-267
(which yields the encrypted offset the receive path needs), the long-header
first byte :270-285 and the frame-type table :532-577.
"""

from dataclasses import dataclass, field
from enum import Enum, IntEnum
from typing import Optional

from .buffer import Buffer

PACKET_LONG_HEADER = 0x80
PACKET_FIXED_BIT = 0x40
PACKET_SPIN_BIT = 0x20
PACKET_NUMBER_MAX_SIZE = 4
CONNECTION_ID_MAX_SIZE = 20

RETRY_AEAD_KEY_VERSION_1 = bytes.fromhex("be0c690b9f66575a1d766b54e368c84e")
RETRY_AEAD_KEY_VERSION_2 = bytes.fromhex("8fb4b01b56ac48e260fbcbcead7ccc92")
RETRY_AEAD_NONCE_VERSION_1 = bytes.fromhex("461599d35d632bf2239825bb")
RETRY_AEAD_NONCE_VERSION_2 = bytes.fromhex("d86969bc2d7c6d9990efb04a")
RETRY_INTEGRITY_TAG_SIZE = 16


class QuicProtocolVersion(IntEnum):
    NEGOTIATION = 0
    VERSION_1 = 0x00000001
    VERSION_2 = 0x6B3343CF


class QuicPacketType(Enum):
    INITIAL = 0
    ZERO_RTT = 1
    HANDSHAKE = 2
    RETRY = 3
    VERSION_NEGOTIATION = 4
    ONE_RTT = 5


# long-header type field (bits 4-5 of the first byte) per version:
# RFC 9000 sec. 17.2 and RFC 9369 sec. 3.2
_LONG_TYPES = {
    QuicProtocolVersion.VERSION_1: (QuicPacketType.INITIAL, QuicPacketType.ZERO_RTT,
                                    QuicPacketType.HANDSHAKE, QuicPacketType.RETRY),
    QuicProtocolVersion.VERSION_2: (QuicPacketType.RETRY, QuicPacketType.INITIAL,
                                    QuicPacketType.ZERO_RTT, QuicPacketType.HANDSHAKE),
}
PACKET_LONG_TYPE_DECODE_VERSION_1 = dict(enumerate(_LONG_TYPES[QuicProtocolVersion.VERSION_1]))
PACKET_LONG_TYPE_DECODE_VERSION_2 = dict(enumerate(_LONG_TYPES[QuicProtocolVersion.VERSION_2]))
PACKET_LONG_TYPE_ENCODE_VERSION_1 = {t: c for c, t in PACKET_LONG_TYPE_DECODE_VERSION_1.items()}
PACKET_LONG_TYPE_ENCODE_VERSION_2 = {t: c for c, t in PACKET_LONG_TYPE_DECODE_VERSION_2.items()}


class QuicFrameType(IntEnum):
    PADDING = 0x00
    PING = 0x01
    ACK = 0x02
    ACK_ECN = 0x03
    RESET_STREAM = 0x04
    STOP_SENDING = 0x05
    CRYPTO = 0x06
    NEW_TOKEN = 0x07
    STREAM_BASE = 0x08
    MAX_DATA = 0x10
    MAX_STREAM_DATA = 0x11
    MAX_STREAMS_BIDI = 0x12
    MAX_STREAMS_UNI = 0x13
    DATA_BLOCKED = 0x14
    STREAM_DATA_BLOCKED = 0x15
    STREAMS_BLOCKED_BIDI = 0x16
    STREAMS_BLOCKED_UNI = 0x17
    NEW_CONNECTION_ID = 0x18
    RETIRE_CONNECTION_ID = 0x19
    PATH_CHALLENGE = 0x1A
    PATH_RESPONSE = 0x1B
    TRANSPORT_CLOSE = 0x1C
    APPLICATION_CLOSE = 0x1D
    HANDSHAKE_DONE = 0x1E
    DATAGRAM = 0x30
    DATAGRAM_WITH_LENGTH = 0x31


# RFC 9002 sec. 2: frames that do not elicit an ACK / do not count in flight
_CLOSE_AND_ACK = (QuicFrameType.ACK, QuicFrameType.ACK_ECN, QuicFrameType.TRANSPORT_CLOSE,
                  QuicFrameType.APPLICATION_CLOSE)
NON_IN_FLIGHT_FRAME_TYPES = frozenset(_CLOSE_AND_ACK)
NON_ACK_ELICITING_FRAME_TYPES = frozenset(_CLOSE_AND_ACK + (QuicFrameType.PADDING,))


@dataclass
class QuicHeader:
    version: Optional[int]
    packet_type: QuicPacketType
    packet_length: int          # bytes from the first byte to the end of the packet
    destination_cid: bytes
    source_cid: bytes
    token: bytes = b""
    integrity_tag: bytes = b""
    supported_versions: list = field(default_factory=list)


def encode_long_header_first_byte(version: int, packet_type: QuicPacketType, bits: int) -> int:
    codes = (PACKET_LONG_TYPE_ENCODE_VERSION_2 if version == QuicProtocolVersion.VERSION_2
             else PACKET_LONG_TYPE_ENCODE_VERSION_1)
    return PACKET_LONG_HEADER | PACKET_FIXED_BIT | codes[packet_type] << 4 | bits


def _pull_cid(buf: Buffer, what: str) -> bytes:
    n = buf.pull_uint8()
    if n > CONNECTION_ID_MAX_SIZE:
        raise ValueError("%s CID is too long (%d bytes)" % (what, n))
    return buf.pull_bytes(n)


def pull_quic_header(buf: Buffer, host_cid_length: Optional[int] = None) -> QuicHeader:
    """Parse one packet header at the cursor; on return the cursor sits at
    the packet number (the encrypted offset), and packet_length covers the
    whole packet, so coalesced packets are walked by seeking past it
    (RFC 9000 sec. 12.2, 17)."""
    start = buf.tell()
    first = buf.pull_uint8()
    if not is_long_header(first):
        if not first & PACKET_FIXED_BIT:
            raise ValueError("Packet fixed bit is zero")
        dcid = buf.pull_bytes(host_cid_length)
        return QuicHeader(None, QuicPacketType.ONE_RTT, buf.capacity - start, dcid, b"")
    version = buf.pull_uint32()
    dcid = _pull_cid(buf, "Destination")
    scid = _pull_cid(buf, "Source")
    if version == QuicProtocolVersion.NEGOTIATION:
        versions = []
        while not buf.eof():
            versions.append(buf.pull_uint32())
        return QuicHeader(version, QuicPacketType.VERSION_NEGOTIATION, buf.tell() - start, dcid, scid,
                          supported_versions=versions)
    if not first & PACKET_FIXED_BIT:
        raise ValueError("Packet fixed bit is zero")
    table = (PACKET_LONG_TYPE_DECODE_VERSION_2 if version == QuicProtocolVersion.VERSION_2
             else PACKET_LONG_TYPE_DECODE_VERSION_1)
    ptype = table[(first >> 4) & 3]
    token, tag = b"", b""
    if ptype == QuicPacketType.RETRY:
        token = buf.pull_bytes(buf.capacity - buf.tell() - RETRY_INTEGRITY_TAG_SIZE)
        tag = buf.pull_bytes(RETRY_INTEGRITY_TAG_SIZE)
        rest = 0
    else:
        if ptype == QuicPacketType.INITIAL:
            token = buf.pull_bytes(buf.pull_uint_var())
        rest = buf.pull_uint_var()
    end = buf.tell() + rest
    if end > buf.capacity:
        raise ValueError("Packet payload is truncated")
    return QuicHeader(version, ptype, end - start, dcid, scid, token=token, integrity_tag=tag)


def decode_packet_number(truncated: int, num_bits: int, expected: int) -> int:
    """Recover a packet number from a truncated packet number (RFC 9000 App. A.3)."""
    window = 1 << num_bits
    half_window = window // 2
    candidate = (expected & ~(window - 1)) | truncated
    if candidate <= expected - half_window and candidate < (1 << 62) - window:
        return candidate + window
    elif candidate > expected + half_window and candidate >= window:
        return candidate - window
    else:
        return candidate


def is_long_header(first_byte: int) -> bool:
    return bool(first_byte & PACKET_LONG_HEADER)


def get_spin_bit(first_byte: int) -> bool:
    return bool(first_byte & PACKET_SPIN_BIT)


def get_retry_integrity_tag(
    packet_without_tag: bytes, original_destination_cid: bytes, version: int
) -> bytes:
    """Retry integrity tag (RFC 9001 sec. 5.8): AES-128-GCM over the Retry
    pseudo-packet with an empty plaintext, on the GPU."""
    from ._crypto import AEAD

    pseudo = bytes([len(original_destination_cid)]) + original_destination_cid + packet_without_tag
    if version == QuicProtocolVersion.VERSION_2:
        key, nonce = RETRY_AEAD_KEY_VERSION_2, RETRY_AEAD_NONCE_VERSION_2
    else:
        key, nonce = RETRY_AEAD_KEY_VERSION_1, RETRY_AEAD_NONCE_VERSION_1
    # packet number 0 leaves nonce = iv (_crypto.c:173-176)
    tag = AEAD(b"aes-128-gcm", key, nonce).encrypt(b"", pseudo, 0)
    assert len(tag) == RETRY_INTEGRITY_TAG_SIZE
    return tag
