"""ctypes view of the CPU oracle (oracle/libqpp_oracle.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg, never by the product package ``aioquic_amd``.

Every function mirrors a reference call (see qpp_oracle.c for file:line).
Key derivation here is an independent stdlib restatement of
aioquic src/aioquic/quic/crypto.py:34-56 and src/aioquic/tls.py:164-193, so the
oracle checks the product's HKDF instead of sharing it.
"""

from __future__ import annotations

import ctypes
import hashlib
import hmac
import os
import struct

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = os.path.join(_HERE, "libqpp_oracle.so")

AES_128_GCM, AES_256_GCM, CHACHA20_POLY1305 = 0, 1, 2
VERSION_1, VERSION_2 = 0x00000001, 0x6B3343CF
SALT_V1 = bytes.fromhex("38762cf7f55934b34d179ae6a4c80cadccbb7f0a")
SALT_V2 = bytes.fromhex("0dede3def700a6db819381be6e269dcbf9bd2ed9")

# numpy mirrors of include/quic_pp.h structs
DESC_DTYPE = np.dtype(
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
RESULT_DTYPE = np.dtype(
    [("pn", "<u8"), ("status", "<u2"), ("hdr_len", "<u2"), ("out_len", "<u4")]
)
KEY_DTYPE = np.dtype(
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
assert DESC_DTYPE.itemsize == 40 and RESULT_DTYPE.itemsize == 16
assert KEY_DTYPE.itemsize == 84


def load() -> ctypes.CDLL:
    if not os.path.exists(_LIB):
        raise RuntimeError(f"oracle not built: run `make -C {_HERE}`")
    lib = ctypes.CDLL(_LIB)
    c = ctypes
    lib.qo_aead_encrypt.restype = c.c_long
    lib.qo_aead_decrypt.restype = c.c_long
    lib.qo_protect.restype = c.c_long
    lib.qo_unprotect.restype = c.c_long
    lib.qo_decode_pn.restype = c.c_uint64
    lib.qo_decode_pn.argtypes = [c.c_int64, c.c_int, c.c_uint64]
    for f in ("qo_aead_encrypt", "qo_aead_decrypt"):
        getattr(lib, f).argtypes = [
            c.c_int, c.c_char_p, c.c_char_p, c.c_char_p, c.c_size_t,
            c.c_char_p, c.c_size_t, c.c_uint64, c.c_void_p,
        ]
    lib.qo_protect.argtypes = [
        c.c_int, c.c_char_p, c.c_char_p, c.c_char_p, c.c_char_p, c.c_size_t,
        c.c_char_p, c.c_size_t, c.c_uint64, c.c_void_p,
    ]
    lib.qo_unprotect.argtypes = [
        c.c_int, c.c_char_p, c.c_char_p, c.c_char_p, c.c_char_p, c.c_size_t,
        c.c_size_t, c.c_uint64, c.c_void_p, c.POINTER(c.c_size_t), c.POINTER(c.c_uint64),
    ]
    lib.qo_hp_mask.argtypes = [c.c_int, c.c_char_p, c.c_char_p, c.c_void_p]
    for f in ("qo_protect_batch", "qo_unprotect_batch"):
        getattr(lib, f).argtypes = [c.c_void_p, c.c_uint32, c.c_void_p, c.c_uint32,
                                    c.c_void_p, c.c_void_p, c.c_void_p]
        getattr(lib, f).restype = None
    return lib


_lib = None


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        _lib = load()
    return _lib


# ---------------------------------------------------------------- keys ----


def _hash(suite: int):
    return hashlib.sha384 if suite == AES_256_GCM else hashlib.sha256


def hkdf_extract(hashfn, salt: bytes, ikm: bytes) -> bytes:
    return hmac.new(salt, ikm, hashfn).digest()


def hkdf_expand_label(hashfn, secret: bytes, label: bytes, context: bytes, length: int) -> bytes:
    full = b"tls13 " + label
    info = struct.pack("!HB", length, len(full)) + full + struct.pack("!B", len(context)) + context
    out, t, i = b"", b"", 1
    while len(out) < length:
        t = hmac.new(secret, t + info + bytes([i]), hashfn).digest()
        out += t
        i += 1
    return out[:length]


def derive_key_iv_hp(suite: int, secret: bytes, version: int = VERSION_1):
    h = _hash(suite)
    ks = 16 if suite == AES_128_GCM else 32
    p = b"quicv2 " if version == VERSION_2 else b"quic "
    return (
        hkdf_expand_label(h, secret, p + b"key", b"", ks),
        hkdf_expand_label(h, secret, p + b"iv", b"", 12),
        hkdf_expand_label(h, secret, p + b"hp", b"", ks),
    )


def initial_secrets(cid: bytes, version: int = VERSION_1):
    """(client_secret, server_secret) -- quic/crypto.py:201-227"""
    salt = SALT_V2 if version == VERSION_2 else SALT_V1
    init = hkdf_extract(hashlib.sha256, salt, cid)
    return (
        hkdf_expand_label(hashlib.sha256, init, b"client in", b"", 32),
        hkdf_expand_label(hashlib.sha256, init, b"server in", b"", 32),
    )


def next_secret(suite: int, secret: bytes) -> bytes:
    h = _hash(suite)
    return hkdf_expand_label(h, secret, b"quic ku", b"", h().digest_size)


# --------------------------------------------------------- per packet ----


def protect(suite, key, iv, hp, header: bytes, payload: bytes, pn: int) -> bytes:
    out = ctypes.create_string_buffer(len(header) + len(payload) + 16)
    n = lib().qo_protect(suite, key, iv, hp, header, len(header), payload, len(payload), pn, out)
    if n < 0:
        raise ValueError("oracle protect failed")
    return out.raw[:n]


def unprotect(suite, key, iv, hp, packet: bytes, pn_off: int, expected_pn: int):
    """-> (header, payload, pn) or raises ValueError('length'|'decrypt')"""
    out = ctypes.create_string_buffer(len(packet) + 16)
    hl, pn = ctypes.c_size_t(), ctypes.c_uint64()
    n = lib().qo_unprotect(suite, key, iv, hp, packet, len(packet), pn_off, expected_pn, out,
                           ctypes.byref(hl), ctypes.byref(pn))
    if n == -1:
        raise ValueError("length")
    if n == -2:
        raise ValueError("decrypt")
    return out.raw[: hl.value], out.raw[hl.value : hl.value + n], pn.value


def aead_encrypt(suite, key, iv, data: bytes, aad: bytes, pn: int) -> bytes:
    out = ctypes.create_string_buffer(len(data) + 16)
    n = lib().qo_aead_encrypt(suite, key, iv, data, len(data), aad, len(aad), pn, out)
    if n < 0:
        raise ValueError("length")
    return out.raw[:n]


def aead_decrypt(suite, key, iv, data: bytes, aad: bytes, pn: int) -> bytes:
    out = ctypes.create_string_buffer(max(len(data), 1))
    n = lib().qo_aead_decrypt(suite, key, iv, data, len(data), aad, len(aad), pn, out)
    if n == -1:
        raise ValueError("length")
    if n == -2:
        raise ValueError("decrypt")
    return out.raw[:n]


def hp_mask(suite, hp, sample: bytes) -> bytes:
    out = ctypes.create_string_buffer(16)
    lib().qo_hp_mask(suite, hp, sample, out)
    return out.raw


def decode_pn(truncated: int, num_bits: int, expected: int) -> int:
    return lib().qo_decode_pn(truncated, num_bits, expected)


# -------------------------------------------------------------- batch ----


def protect_batch(keys: np.ndarray, desc: np.ndarray, inbuf: np.ndarray, out_size: int):
    out = np.zeros(out_size, dtype=np.uint8)
    res = np.zeros(len(desc), dtype=RESULT_DTYPE)
    lib().qo_protect_batch(keys.ctypes.data, len(keys), desc.ctypes.data, len(desc),
                           inbuf.ctypes.data, out.ctypes.data, res.ctypes.data)
    return out, res


def unprotect_batch(keys: np.ndarray, desc: np.ndarray, inbuf: np.ndarray, out_size: int):
    out = np.zeros(out_size, dtype=np.uint8)
    res = np.zeros(len(desc), dtype=RESULT_DTYPE)
    lib().qo_unprotect_batch(keys.ctypes.data, len(keys), desc.ctypes.data, len(desc),
                             inbuf.ctypes.data, out.ctypes.data, res.ctypes.data)
    return out, res
