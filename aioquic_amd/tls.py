"""Key-schedule helpers of the packet-protection path.

Restates the pieces of aioquic src/aioquic/tls.py that the path touches
(hkdf_label :164-171, hkdf_expand_label :174-185, hkdf_extract :188-193,
CipherSuite :294-298, CIPHER_SUITES hash map :1108-1112, cipher_suite_hash
:1135-1136) on the standard library, since these run once per key, on the host.
"""

import hashlib
import hmac
import struct
from enum import Enum, IntEnum


class Epoch(Enum):
    """Encryption levels (tls.py:129-133)."""

    INITIAL = 0
    ZERO_RTT = 1
    HANDSHAKE = 2
    ONE_RTT = 3


class CipherSuite(IntEnum):
    AES_128_GCM_SHA256 = 0x1301
    AES_256_GCM_SHA384 = 0x1302
    CHACHA20_POLY1305_SHA256 = 0x1303


class HashAlgorithm:
    """Minimal stand-in for a cryptography hash algorithm object."""

    def __init__(self, name: str):
        self.name = name
        self.digest_size = hashlib.new(name).digest_size

    def __eq__(self, other):
        return isinstance(other, HashAlgorithm) and other.name == self.name

    def __hash__(self):
        return hash(self.name)

    def __repr__(self):
        return f"HashAlgorithm({self.name!r})"


SHA256 = HashAlgorithm("sha256")
SHA384 = HashAlgorithm("sha384")

CIPHER_SUITES = {
    CipherSuite.AES_128_GCM_SHA256: SHA256,
    CipherSuite.AES_256_GCM_SHA384: SHA384,
    CipherSuite.CHACHA20_POLY1305_SHA256: SHA256,
}


def cipher_suite_hash(cipher_suite: CipherSuite) -> HashAlgorithm:
    return CIPHER_SUITES[cipher_suite]


def hkdf_label(label: bytes, hash_value: bytes, length: int) -> bytes:
    full_label = b"tls13 " + label
    return (
        struct.pack("!HB", length, len(full_label))
        + full_label
        + struct.pack("!B", len(hash_value))
        + hash_value
    )


def hkdf_expand(algorithm: HashAlgorithm, secret: bytes, info: bytes, length: int) -> bytes:
    """RFC 5869 HKDF-Expand."""
    if length > 255 * algorithm.digest_size:
        raise ValueError("HKDF-Expand length too large")
    out = b""
    block = b""
    counter = 1
    while len(out) < length:
        block = hmac.new(secret, block + info + bytes([counter]), algorithm.name).digest()
        out += block
        counter += 1
    return out[:length]


def hkdf_expand_label(
    algorithm: HashAlgorithm, secret: bytes, label: bytes, hash_value: bytes, length: int
) -> bytes:
    return hkdf_expand(algorithm, secret, hkdf_label(label, hash_value, length), length)


def hkdf_extract(algorithm: HashAlgorithm, salt: bytes, key_material: bytes) -> bytes:
    return hmac.new(salt, key_material, algorithm.name).digest()
