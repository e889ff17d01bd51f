"""Packet protection with aioquic's API, executed on the GPU.

Mirrors aioquic src/aioquic/quic/crypto.py (CIPHER_SUITES :12-16, salts :18-19,
KeyUnavailableError :30, derive_key_iv_hp :34-56, CryptoContext :59-154,
apply_key_phase / next_key_phase :148-168, CryptoPair :171-246) so it can
replace that module under the QUIC connection machinery.

CryptoContext keeps the reference's ``aead`` / ``hp`` attributes, but
encrypt_packet / decrypt_packet run the FUSED device path (one launch does
AEAD + header protection + packet-number decode), through a per-context
two-slot key table: slot 0 = (aead, hp, key_phase), slot 1 = the transient
next-phase key tried when a short header's key-phase bit flips
(crypto.py:91-96).
"""

import binascii
from typing import Callable, Optional

import numpy as np

from . import layout as L
from ._crypto import AEAD, CryptoError, HeaderProtection, KeyTable, protect_host, unprotect_host
from .packet import QuicProtocolVersion, decode_packet_number, is_long_header  # noqa: F401
from .tls import CipherSuite, cipher_suite_hash, hkdf_expand_label, hkdf_extract

CIPHER_SUITES = {
    CipherSuite.AES_128_GCM_SHA256: (b"aes-128-ecb", b"aes-128-gcm"),
    CipherSuite.AES_256_GCM_SHA384: (b"aes-256-ecb", b"aes-256-gcm"),
    CipherSuite.CHACHA20_POLY1305_SHA256: (b"chacha20", b"chacha20-poly1305"),
}
INITIAL_CIPHER_SUITE = CipherSuite.AES_128_GCM_SHA256
INITIAL_SALT_VERSION_1 = binascii.unhexlify("38762cf7f55934b34d179ae6a4c80cadccbb7f0a")
INITIAL_SALT_VERSION_2 = binascii.unhexlify("0dede3def700a6db819381be6e269dcbf9bd2ed9")
SAMPLE_SIZE = 16

Callback = Callable[[str], None]


def NoCallback(trigger: str) -> None:
    pass


class KeyUnavailableError(CryptoError):
    pass


def derive_key_iv_hp(
    *, cipher_suite: CipherSuite, secret: bytes, version: int
) -> tuple[bytes, bytes, bytes]:
    algorithm = cipher_suite_hash(cipher_suite)
    if cipher_suite in [
        CipherSuite.AES_256_GCM_SHA384,
        CipherSuite.CHACHA20_POLY1305_SHA256,
    ]:
        key_size = 32
    else:
        key_size = 16
    prefix = b"quicv2 " if version == QuicProtocolVersion.VERSION_2 else b"quic "
    return (
        hkdf_expand_label(algorithm, secret, prefix + b"key", b"", key_size),
        hkdf_expand_label(algorithm, secret, prefix + b"iv", b"", 12),
        hkdf_expand_label(algorithm, secret, prefix + b"hp", b"", key_size),
    )


def _raise_for(status: int) -> None:
    if status == L.S_DECRYPT:
        raise CryptoError("Payload decryption failed")
    if status == L.S_NO_KEY:
        raise KeyUnavailableError("Decryption key is not available")
    raise CryptoError("Invalid payload length")


class _FusedSlots:
    """Two device key slots holding (AEAD key/iv, HP key, key phase)."""

    def __init__(self) -> None:
        self.table = KeyTable(2)
        self.ident = [None, None]

    def bind(self, slot: int, aead: AEAD, hp: HeaderProtection, key_phase: int) -> None:
        ident = (id(aead), id(hp), key_phase)
        if self.ident[slot] == ident:
            return
        suite, key, iv = aead._material()
        _, hp_key = hp._material()
        self.table.set(L.key_material(slot, suite, key, iv, hp_key, key_phase).tobytes())
        # keep the objects alive so their ids stay unique while bound
        self.ident[slot] = ident
        setattr(self, f"_keep{slot}", (aead, hp))


def _desc(length: int, hdr_len: int, pn: int, slot: int, flags: int = 0) -> bytes:
    d = np.zeros(1, dtype=L.DESC)
    d["len"] = length
    d["hdr_len"] = hdr_len
    d["pn"] = pn & 0xFFFFFFFFFFFFFFFF
    d["slot"] = slot
    d["flags"] = flags
    return d.tobytes()


class CryptoContext:
    def __init__(
        self,
        key_phase: int = 0,
        setup_cb: Callback = NoCallback,
        teardown_cb: Callback = NoCallback,
    ) -> None:
        self.aead: Optional[AEAD] = None
        self.cipher_suite: Optional[CipherSuite] = None
        self.hp: Optional[HeaderProtection] = None
        self.key_phase = key_phase
        self.secret: Optional[bytes] = None
        self.version: Optional[int] = None
        self._setup_cb = setup_cb
        self._teardown_cb = teardown_cb
        self._slots: Optional[_FusedSlots] = None

    def _fused(self) -> _FusedSlots:
        if self._slots is None:
            self._slots = _FusedSlots()
        return self._slots

    def decrypt_packet(
        self, packet: bytes, encrypted_offset: int, expected_packet_number: int
    ) -> tuple[bytes, bytes, int, bool]:
        if self.aead is None:
            raise KeyUnavailableError("Decryption key is not available")
        if encrypted_offset > L.MAX_HDR:
            raise CryptoError("Invalid payload length")
        slots = self._fused()
        slots.bind(0, self.aead, self.hp, self.key_phase)
        desc = _desc(len(packet), encrypted_offset, expected_packet_number, 0)
        out, res = unprotect_host(slots.table, desc, packet, len(packet))
        r = np.frombuffer(res, dtype=L.RESULT)[0]
        crypto = self
        if r["status"] == L.S_KEY_PHASE:
            # detect key phase change (quic/crypto.py:91-96): the HP key stays
            crypto = next_key_phase(self)
            slots.bind(1, crypto.aead, self.hp, crypto.key_phase)
            desc = _desc(len(packet), encrypted_offset, expected_packet_number, 1)
            out, res = unprotect_host(slots.table, desc, packet, len(packet))
            r = np.frombuffer(res, dtype=L.RESULT)[0]
        if r["status"] != L.S_OK:
            _raise_for(int(r["status"]))
        hl, n = int(r["hdr_len"]), int(r["out_len"])
        return out[:hl], out[hl:n], int(r["pn"]), crypto is not self

    def encrypt_packet(
        self, plain_header: bytes, plain_payload: bytes, packet_number: int
    ) -> bytes:
        assert self.is_valid(), "Encryption key is not available"
        slots = self._fused()
        slots.bind(0, self.aead, self.hp, self.key_phase)
        desc = _desc(len(plain_payload), len(plain_header), packet_number, 0)
        n = len(plain_header) + len(plain_payload) + L.TAG_LEN
        out, res = protect_host(slots.table, desc, plain_header + plain_payload, n)
        r = np.frombuffer(res, dtype=L.RESULT)[0]
        if r["status"] != L.S_OK:
            _raise_for(int(r["status"]))
        return out

    def is_valid(self) -> bool:
        return self.aead is not None

    def setup(self, *, cipher_suite: CipherSuite, secret: bytes, version: int) -> None:
        hp_cipher_name, aead_cipher_name = CIPHER_SUITES[cipher_suite]

        key, iv, hp = derive_key_iv_hp(
            cipher_suite=cipher_suite,
            secret=secret,
            version=version,
        )
        self.aead = AEAD(aead_cipher_name, key, iv)
        self.cipher_suite = cipher_suite
        self.hp = HeaderProtection(hp_cipher_name, hp)
        self.secret = secret
        self.version = version

        # trigger callback
        self._setup_cb("tls")

    def teardown(self) -> None:
        self.aead = None
        self.cipher_suite = None
        self.hp = None
        self.secret = None
        self._slots = None

        # trigger callback
        self._teardown_cb("tls")


def apply_key_phase(self: CryptoContext, crypto: CryptoContext, trigger: str) -> None:
    self.aead = crypto.aead
    self.key_phase = crypto.key_phase
    self.secret = crypto.secret

    # trigger callback
    self._setup_cb(trigger)


def next_key_phase(self: CryptoContext) -> CryptoContext:
    algorithm = cipher_suite_hash(self.cipher_suite)

    crypto = CryptoContext(key_phase=int(not self.key_phase))
    crypto.setup(
        cipher_suite=self.cipher_suite,
        secret=hkdf_expand_label(
            algorithm, self.secret, b"quic ku", b"", algorithm.digest_size
        ),
        version=self.version,
    )
    return crypto


class CryptoPair:
    def __init__(
        self,
        recv_setup_cb: Callback = NoCallback,
        recv_teardown_cb: Callback = NoCallback,
        send_setup_cb: Callback = NoCallback,
        send_teardown_cb: Callback = NoCallback,
    ) -> None:
        self.aead_tag_size = 16
        self.recv = CryptoContext(setup_cb=recv_setup_cb, teardown_cb=recv_teardown_cb)
        self.send = CryptoContext(setup_cb=send_setup_cb, teardown_cb=send_teardown_cb)
        self._update_key_requested = False

    def decrypt_packet(
        self, packet: bytes, encrypted_offset: int, expected_packet_number: int
    ) -> tuple[bytes, bytes, int]:
        plain_header, payload, packet_number, update_key = self.recv.decrypt_packet(
            packet, encrypted_offset, expected_packet_number
        )
        if update_key:
            self._update_key("remote_update")
        return plain_header, payload, packet_number

    def encrypt_packet(
        self, plain_header: bytes, plain_payload: bytes, packet_number: int
    ) -> bytes:
        if self._update_key_requested:
            self._update_key("local_update")
        return self.send.encrypt_packet(plain_header, plain_payload, packet_number)

    def setup_initial(self, cid: bytes, is_client: bool, version: int) -> None:
        if is_client:
            recv_label, send_label = b"server in", b"client in"
        else:
            recv_label, send_label = b"client in", b"server in"

        if version == QuicProtocolVersion.VERSION_2:
            initial_salt = INITIAL_SALT_VERSION_2
        else:
            initial_salt = INITIAL_SALT_VERSION_1

        algorithm = cipher_suite_hash(INITIAL_CIPHER_SUITE)
        initial_secret = hkdf_extract(algorithm, initial_salt, cid)
        self.recv.setup(
            cipher_suite=INITIAL_CIPHER_SUITE,
            secret=hkdf_expand_label(
                algorithm, initial_secret, recv_label, b"", algorithm.digest_size
            ),
            version=version,
        )
        self.send.setup(
            cipher_suite=INITIAL_CIPHER_SUITE,
            secret=hkdf_expand_label(
                algorithm, initial_secret, send_label, b"", algorithm.digest_size
            ),
            version=version,
        )

    def teardown(self) -> None:
        self.recv.teardown()
        self.send.teardown()

    def update_key(self) -> None:
        self._update_key_requested = True

    @property
    def key_phase(self) -> int:
        if self._update_key_requested:
            return int(not self.recv.key_phase)
        else:
            return self.recv.key_phase

    def _update_key(self, trigger: str) -> None:
        apply_key_phase(self.recv, next_key_phase(self.recv), trigger=trigger)
        apply_key_phase(self.send, next_key_phase(self.send), trigger=trigger)
        self._update_key_requested = False
