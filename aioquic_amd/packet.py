"""Packet-number and header helpers used by the packet-protection path.

Mirrors aioquic src/aioquic/quic/packet.py: the first-byte bits :13-15,
QuicProtocolVersion, decode_packet_number :118-132, is_long_header :166-167,
and the Retry integrity tag :135-159 (AES-128-GCM, computed on the GPU).
"""

from enum import IntEnum

PACKET_LONG_HEADER = 0x80
PACKET_FIXED_BIT = 0x40
PACKET_SPIN_BIT = 0x20
PACKET_NUMBER_MAX_SIZE = 4

RETRY_AEAD_KEY_VERSION_1 = bytes.fromhex("be0c690b9f66575a1d766b54e368c84e")
RETRY_AEAD_KEY_VERSION_2 = bytes.fromhex("8fb4b01b56ac48e260fbcbcead7ccc92")
RETRY_AEAD_NONCE_VERSION_1 = bytes.fromhex("461599d35d632bf2239825bb")
RETRY_AEAD_NONCE_VERSION_2 = bytes.fromhex("d86969bc2d7c6d9990efb04a")
RETRY_INTEGRITY_TAG_SIZE = 16


class QuicProtocolVersion(IntEnum):
    NEGOTIATION = 0
    VERSION_1 = 0x00000001
    VERSION_2 = 0x6B3343CF


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
