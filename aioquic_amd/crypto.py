"""QUIC packet protection contexts whose packet work runs on the GPU.

Public surface = aioquic's ``quic/crypto.py`` (suite table :12-16, initial
salts :18-19, ``KeyUnavailableError`` :30, ``derive_key_iv_hp`` :34-56,
``CryptoContext`` :59-145, ``apply_key_phase`` / ``next_key_phase``
:148-168, ``CryptoPair`` :171-246), so the connection code can import this
module in its place.  The design underneath differs:

* A context owns a two-slot device key table (``_PhaseSlots``).  Slot 0 is
  its current (AEAD key/IV, HP key, key phase); slot 1 is the next-phase
  candidate, installed when the device reports a flipped key-phase bit
  (``S_KEY_PHASE``; the reference tries ``next_key_phase`` at :91-96).
* ``encrypt_packet`` / ``decrypt_packet`` are one fused device call each:
  AEAD, header protection and packet-number recovery together, instead of
  the reference's ``aead`` call followed by an ``hp`` call.
* The ``aead`` / ``hp`` attributes stay the ``_crypto`` objects the
  reference exposes; the slots are filled from their key material.
"""

from __future__ import annotations

import struct
from dataclasses import dataclass
from typing import Callable, Dict, Optional, Tuple


from . import layout as L
from ._crypto import AEAD, CryptoError, HeaderProtection, KeyTable, protect_host, unprotect_host
from .packet import QuicProtocolVersion, decode_packet_number, is_long_header  # noqa: F401
from .tls import CipherSuite, cipher_suite_hash, hkdf_expand_label, hkdf_extract


@dataclass(frozen=True)
class _Suite:
    hp_name: bytes
    aead_name: bytes
    key_len: int


_SUITES: Dict[CipherSuite, _Suite] = {
    CipherSuite.AES_128_GCM_SHA256: _Suite(b"aes-128-ecb", b"aes-128-gcm", 16),
    CipherSuite.AES_256_GCM_SHA384: _Suite(b"aes-256-ecb", b"aes-256-gcm", 32),
    CipherSuite.CHACHA20_POLY1305_SHA256: _Suite(b"chacha20", b"chacha20-poly1305", 32),
}
# (hp cipher, aead cipher) per suite, as the reference publishes it
CIPHER_SUITES = {cs: (s.hp_name, s.aead_name) for cs, s in _SUITES.items()}

INITIAL_CIPHER_SUITE = CipherSuite.AES_128_GCM_SHA256
INITIAL_SALT_VERSION_1 = bytes.fromhex("38762cf7f55934b34d179ae6a4c80cadccbb7f0a")  # RFC 9001 5.2
INITIAL_SALT_VERSION_2 = bytes.fromhex("0dede3def700a6db819381be6e269dcbf9bd2ed9")  # RFC 9369 3.3.1
SAMPLE_SIZE = 16

Callback = Callable[[str], None]


def NoCallback(trigger: str) -> None:
    """Default setup / teardown hook: does nothing."""


# called with the AEAD / HP objects a context lets go of (teardown, or the
# AEAD replaced by a key update), so batch key tables drop them too
_KEY_RELEASE_HOOKS: list = []


def _release(*objs) -> None:
    for hook in _KEY_RELEASE_HOOKS:
        hook(*objs)


class KeyUnavailableError(CryptoError):
    """No key installed for the packet (decrypt before setup)."""


def _label_prefix(version: int) -> bytes:
    # RFC 9369 sec. 3.3.2: QUIC v2 renames the packet-protection labels
    return b"quicv2 " if version == QuicProtocolVersion.VERSION_2 else b"quic "


def derive_key_iv_hp(*, cipher_suite: CipherSuite, secret: bytes, version: int) -> Tuple[bytes, bytes, bytes]:
    """(AEAD key, IV, HP key) of a traffic secret (RFC 9001 sec. 5.1)."""
    hash_alg = cipher_suite_hash(cipher_suite)
    klen = _SUITES[cipher_suite].key_len
    pre = _label_prefix(version)
    sizes = ((b"key", klen), (b"iv", 12), (b"hp", klen))
    out = tuple(hkdf_expand_label(hash_alg, secret, pre + name, b"", size) for name, size in sizes)
    return out  # type: ignore[return-value]


def _status_error(status: int) -> Exception:
    if status == L.S_NO_KEY:
        return KeyUnavailableError("Decryption key is not available")
    if status == L.S_DECRYPT:
        return CryptoError("Payload decryption failed")
    if status == L.S_INTERNAL:
        return CryptoError(L.INTERNAL_ERROR)
    return CryptoError("Invalid payload length")


# one qpp_desc / qpp_result (layout.DESC / layout.RESULT) by struct: the
# per-packet calls build and read one record each, where numpy's structured
# arrays cost microseconds per call
_DESC = struct.Struct("<QQIHHQII")
_RESULT = struct.Struct("<QHHI")
assert _DESC.size == L.DESC.itemsize and _RESULT.size == L.RESULT.itemsize


def _one_desc(length: int, hdr_len: int, pn: int, slot: int) -> bytes:
    return _DESC.pack(0, 0, length, hdr_len, 0, pn & 0xFFFFFFFFFFFFFFFF, slot, 0)


class _Result:
    """One qpp_result, read from the library's bytes."""

    __slots__ = ("pn", "status", "hdr_len", "out_len")

    def __init__(self, raw: bytes) -> None:
        self.pn, self.status, self.hdr_len, self.out_len = _RESULT.unpack_from(raw)

    def __getitem__(self, field: str) -> int:
        return getattr(self, field)


class _PhaseSlots:
    """Device key table of one context: slot 0 = current keys, slot 1 = the
    next key phase's.  A slot is rewritten only when the objects bound to it
    change (identity of the AEAD / HP objects and the phase bit)."""

    __slots__ = ("table", "_bound")

    def __init__(self) -> None:
        self.table = KeyTable(2)
        self._bound: list = [None, None]

    def ensure(self, slot: int, aead: AEAD, hp: HeaderProtection, phase: int) -> None:
        held = self._bound[slot]
        if held is not None and held[0] is aead and held[1] is hp and held[2] == phase:
            return
        suite, key, iv = aead._material()
        hp_key = hp._material()[1]
        self.table.set(L.key_material(slot, suite, key, iv, hp_key, phase).tobytes())
        # holding the objects keeps the identity test sound
        self._bound[slot] = (aead, hp, phase)


def _unprotect_once(table: KeyTable, packet: bytes, offset: int, expected: int, slot: int):
    desc = _one_desc(len(packet), offset, expected, slot)
    out, res = unprotect_host(table, desc, packet, len(packet))
    return out, _Result(res)


class CryptoContext:
    """Keys of one direction at one encryption level."""

    def __init__(self, key_phase: int = 0, setup_cb: Callback = NoCallback,
                 teardown_cb: Callback = NoCallback) -> None:
        self._setup_cb, self._teardown_cb = setup_cb, teardown_cb
        self._slots: Optional[_PhaseSlots] = None
        self.version: Optional[int] = None
        self._forget()
        self.key_phase = key_phase

    def _forget(self) -> None:
        # what teardown clears (the version stays, as in the reference)
        self.aead: Optional[AEAD] = None
        self.hp: Optional[HeaderProtection] = None
        self.cipher_suite: Optional[CipherSuite] = None
        self.secret: Optional[bytes] = None

    def setup(self, *, cipher_suite: CipherSuite, secret: bytes, version: int) -> None:
        suite = _SUITES[cipher_suite]
        key, iv, hp_key = derive_key_iv_hp(cipher_suite=cipher_suite, secret=secret, version=version)
        self.cipher_suite, self.secret, self.version = cipher_suite, secret, version
        self.aead = AEAD(suite.aead_name, key, iv)
        self.hp = HeaderProtection(suite.hp_name, hp_key)
        self._setup_cb("tls")

    def teardown(self) -> None:
        held = (self.aead, self.hp)
        self._forget()
        self._slots = None
        _release(*held)
        self._teardown_cb("tls")

    def is_valid(self) -> bool:
        return self.aead is not None

    def _device(self) -> _PhaseSlots:
        if self._slots is None:
            self._slots = _PhaseSlots()
        self._slots.ensure(0, self.aead, self.hp, self.key_phase)
        return self._slots

    def encrypt_packet(self, plain_header: bytes, plain_payload: bytes, packet_number: int) -> bytes:
        """Header + protected payload + tag, header protection applied."""
        assert self.is_valid(), "Encryption key is not available"
        dev = self._device()
        total = len(plain_header) + len(plain_payload) + L.TAG_LEN
        desc = _one_desc(len(plain_payload), len(plain_header), packet_number, 0)
        out, res = protect_host(dev.table, desc, plain_header + plain_payload, total)
        status = _RESULT.unpack_from(res)[1]
        if status != L.S_OK:
            raise _status_error(status)
        return out

    def decrypt_packet(self, packet: bytes, encrypted_offset: int,
                       expected_packet_number: int) -> Tuple[bytes, bytes, int, bool]:
        """(plain header, payload, packet number, key phase changed)."""
        if not self.is_valid():
            raise KeyUnavailableError("Decryption key is not available")
        if encrypted_offset > L.MAX_HDR:
            raise CryptoError("Invalid payload length")
        dev = self._device()
        out, r = _unprotect_once(dev.table, packet, encrypted_offset, expected_packet_number, 0)
        rotated = False
        if r["status"] == L.S_KEY_PHASE:
            # the peer moved to the next phase: same HP key, next AEAD key
            candidate = next_key_phase(self)
            dev.ensure(1, candidate.aead, self.hp, candidate.key_phase)
            out, r = _unprotect_once(dev.table, packet, encrypted_offset, expected_packet_number, 1)
            rotated = True
        if r["status"] != L.S_OK:
            raise _status_error(int(r["status"]))
        cut, end = int(r["hdr_len"]), int(r["out_len"])
        return out[:cut], out[cut:end], int(r["pn"]), rotated


def apply_key_phase(self: CryptoContext, crypto: CryptoContext, trigger: str) -> None:
    """Adopt `crypto`'s AEAD key, phase and secret (the HP key is kept)."""
    old = self.aead
    self.aead, self.key_phase, self.secret = crypto.aead, crypto.key_phase, crypto.secret
    if old is not None and old is not self.aead:
        _release(old)
    hook = self._setup_cb
    hook(trigger)


def _updated_secret(ctx: CryptoContext) -> bytes:
    # RFC 9001 sec. 6.1: "quic ku" (kept for QUIC v2 too, RFC 9369 sec. 3.3.2)
    hash_alg = cipher_suite_hash(ctx.cipher_suite)
    return hkdf_expand_label(hash_alg, ctx.secret, b"quic ku", b"", hash_alg.digest_size)


def next_key_phase(self: CryptoContext) -> CryptoContext:
    """A fresh context on the next key phase of `self`."""
    nxt = CryptoContext(key_phase=1 - int(bool(self.key_phase)))
    nxt.setup(cipher_suite=self.cipher_suite, secret=_updated_secret(self), version=self.version)
    return nxt


# (receive label, send label) by role, RFC 9001 sec. 5.2
_INITIAL_LABELS: Dict[bool, Tuple[bytes, bytes]] = {
    True: (b"server in", b"client in"),
    False: (b"client in", b"server in"),
}


def _initial_salt(version: int) -> bytes:
    if version == QuicProtocolVersion.VERSION_2:
        return INITIAL_SALT_VERSION_2
    return INITIAL_SALT_VERSION_1


class CryptoPair:
    """Receive and send contexts of one encryption level, with key updates."""

    def __init__(self, recv_setup_cb: Callback = NoCallback, recv_teardown_cb: Callback = NoCallback,
                 send_setup_cb: Callback = NoCallback, send_teardown_cb: Callback = NoCallback) -> None:
        self.recv = CryptoContext(setup_cb=recv_setup_cb, teardown_cb=recv_teardown_cb)
        self.send = CryptoContext(setup_cb=send_setup_cb, teardown_cb=send_teardown_cb)
        self.aead_tag_size = L.TAG_LEN
        self._update_key_requested = False

    @property
    def key_phase(self) -> int:
        phase = self.recv.key_phase
        return int(not phase) if self._update_key_requested else phase

    def update_key(self) -> None:
        """Start a key update with the next packet sent."""
        self._update_key_requested = True

    def _update_key(self, trigger: str) -> None:
        for ctx in (self.recv, self.send):
            apply_key_phase(ctx, next_key_phase(ctx), trigger=trigger)
        self._update_key_requested = False

    def setup_initial(self, cid: bytes, is_client: bool, version: int) -> None:
        hash_alg = cipher_suite_hash(INITIAL_CIPHER_SUITE)
        root = hkdf_extract(hash_alg, _initial_salt(version), cid)
        for ctx, label in zip((self.recv, self.send), _INITIAL_LABELS[is_client]):
            ctx.setup(
                cipher_suite=INITIAL_CIPHER_SUITE,
                secret=hkdf_expand_label(hash_alg, root, label, b"", hash_alg.digest_size),
                version=version,
            )

    def teardown(self) -> None:
        for ctx in (self.recv, self.send):
            ctx.teardown()

    def encrypt_packet(self, plain_header: bytes, plain_payload: bytes, packet_number: int) -> bytes:
        if self._update_key_requested:
            self._update_key("local_update")
        return self.send.encrypt_packet(plain_header, plain_payload, packet_number)

    def decrypt_packet(self, packet: bytes, encrypted_offset: int,
                       expected_packet_number: int) -> Tuple[bytes, bytes, int]:
        header, payload, pn, rotated = self.recv.decrypt_packet(packet, encrypted_offset,
                                                                expected_packet_number)
        if rotated:
            self._update_key("remote_update")
        return header, payload, pn
