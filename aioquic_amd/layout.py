"""numpy views of the C ABI records in include/quic_pp.h."""

import numpy as np

AES_128_GCM, AES_256_GCM, CHACHA20_POLY1305 = 0, 1, 2

PACKET_MAX = 1500
TAG_LEN = 16
MAX_HDR = 1500

# the message of a packet the engine gave up on (S_INTERNAL: a kernel's
# bounded wait ran out; never expected)
INTERNAL_ERROR = "Internal error: the packet was not processed"

F_NO_HP = 1
F_RFC_PN = 2

S_OK, S_LENGTH, S_DECRYPT, S_KEY_PHASE, S_NO_KEY, S_INTERNAL = 0, 1, 2, 3, 4, 5

DESC = np.dtype(
    [
        ("in_off", "<u8"),
        ("out_off", "<u8"),
        ("len", "<u4"),
        ("hdr_len", "<u2"),
        ("flags", "<u2"),
        ("pn", "<u8"),
        ("slot", "<u4"),
        ("rsv", "<u4"),
    ]
)
RESULT = np.dtype([("pn", "<u8"), ("status", "<u2"), ("hdr_len", "<u2"), ("out_len", "<u4")])
KEY_MATERIAL = np.dtype(
    [
        ("slot", "<u4"),
        ("suite", "u1"),
        ("key_phase", "u1"),
        ("rsv", "u1", (2,)),
        ("iv", "u1", (12,)),
        ("key", "u1", (32,)),
        ("hp", "u1", (32,)),
    ]
)
SECRET = np.dtype(
    [
        ("slot", "<u4"),
        ("suite", "u1"),
        ("key_phase", "u1"),
        ("flags", "u1"),
        ("secret_len", "u1"),
        ("updates", "<u4"),
        ("rsv", "<u4"),
        ("secret", "u1", (64,)),
    ]
)
DERIVE_V2 = 1
assert DESC.itemsize == 40 and RESULT.itemsize == 16 and KEY_MATERIAL.itemsize == 84
assert SECRET.itemsize == 80


def key_material(slot: int, suite: int, key: bytes, iv: bytes, hp: bytes, key_phase: int = 0):
    rec = np.zeros(1, dtype=KEY_MATERIAL)
    rec["slot"] = slot
    rec["suite"] = suite
    rec["key_phase"] = key_phase
    rec["iv"][0, : len(iv)] = np.frombuffer(iv, dtype=np.uint8)
    rec["key"][0, : len(key)] = np.frombuffer(key, dtype=np.uint8)
    rec["hp"][0, : len(hp)] = np.frombuffer(hp, dtype=np.uint8)
    return rec


def secret_record(slot: int, suite: int, secret: bytes, *, key_phase: int = 0, v2: bool = False,
                  updates: int = 0):
    """One qpp_secret: a connection's traffic secret for KeyTable.derive."""
    if not 1 <= len(secret) <= 64:
        raise ValueError("secret must be 1..64 bytes")
    rec = np.zeros(1, dtype=SECRET)
    rec["slot"] = slot
    rec["suite"] = suite
    rec["key_phase"] = key_phase
    rec["flags"] = DERIVE_V2 if v2 else 0
    rec["secret_len"] = len(secret)
    rec["updates"] = updates
    rec["secret"][0, : len(secret)] = np.frombuffer(secret, dtype=np.uint8)
    return rec
