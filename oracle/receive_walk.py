"""CPU restatement of aioquic's receive walk, for the batched-receive parity
tests.

TEST INFRASTRUCTURE ONLY: imported by tests/, never by the product package.

It restates, one packet at a time and independently of aioquic_amd:
  * pull_quic_header           src/aioquic/quic/packet.py:181-267
  * QuicConnection.receive_datagram's loop, up to the decrypt, the
    reserved-bits check and the expected-packet-number update
    src/aioquic/quic/connection.py:756-757,793-960,984-985
    (drop triggers: header_parse_error :800-810, initial_packet_datagram_too_small
    :814-828, unknown_connection_id :830-848, unsupported_version :856-869,
    key_unavailable :914-935, payload_decrypt_error :936-947; Version
    Negotiation :851-853 and Retry :872-880 are handed back unprotected;
    "reserved_bits" is the close of :949-960, which ends the datagram and
    leaves the expected packet number alone; "connection_closed" stands for a
    datagram that :756-757 ignores because the connection is closing)
  * CryptoPair / CryptoContext.decrypt_packet with the key-phase roll
    src/aioquic/quic/crypto.py:75-103,148-168,184-192,243-246
with the packet arithmetic from the C oracle (oracle.unprotect / hp_mask).
The connection-ID match (:830-848) runs when the connection lists its host
CIDs; without them the batched caller's datagrams are taken as already
demultiplexed per connection (asyncio/server.py:60-152).
"""

from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, List, Optional

from . import oracle as O

LONG, FIXED = 0x80, 0x40
VERSION_NEGOTIATION = 0
# long-header packet types by the two type bits (packet.py:41-56)
_TYPES_V1 = {0: "INITIAL", 1: "ZERO_RTT", 2: "HANDSHAKE", 3: "RETRY"}
_TYPES_V2 = {1: "INITIAL", 2: "ZERO_RTT", 3: "HANDSHAKE", 0: "RETRY"}
_EPOCH = {"INITIAL": "INITIAL", "ZERO_RTT": "ZERO_RTT", "HANDSHAKE": "HANDSHAKE", "ONE_RTT": "ONE_RTT"}


class ParseError(ValueError):
    pass


class _Cursor:
    def __init__(self, data: bytes, pos: int = 0):
        self.data, self.pos = data, pos

    def take(self, n: int) -> bytes:
        if n < 0 or self.pos + n > len(self.data):
            raise ParseError("read out of bounds")
        out = self.data[self.pos : self.pos + n]
        self.pos += n
        return out

    def u8(self) -> int:
        return self.take(1)[0]

    def u32(self) -> int:
        return int.from_bytes(self.take(4), "big")

    def varint(self) -> int:
        first = self.data[self.pos] if self.pos < len(self.data) else None
        if first is None:
            raise ParseError("read out of bounds")
        n = 1 << (first >> 6)
        v = int.from_bytes(self.take(n), "big")
        return v & ((1 << (8 * n - 2)) - 1)


@dataclass
class Header:
    version: Optional[int]
    packet_type: str
    packet_length: int
    encrypted_offset: int  # bytes from the packet start to the packet number
    destination_cid: bytes = b""


def parse_header(data: bytes, start: int, host_cid_length: int) -> Header:
    """pull_quic_header (packet.py:181-267) at `start`."""
    c = _Cursor(data, start)
    first = c.u8()
    if not first & LONG:
        if not first & FIXED:
            raise ParseError("Packet fixed bit is zero")
        dcid = c.take(host_cid_length)
        return Header(None, "ONE_RTT", len(data) - start, c.pos - start, dcid)
    version = c.u32()
    cids = []
    for what in ("Destination", "Source"):
        n = c.u8()
        if n > 20:
            raise ParseError(f"{what} CID is too long ({n} bytes)")
        cids.append(c.take(n))
    if version == VERSION_NEGOTIATION:
        return Header(version, "VERSION_NEGOTIATION", len(data) - start, c.pos - start, cids[0])
    if not first & FIXED:
        raise ParseError("Packet fixed bit is zero")
    ptype = (_TYPES_V2 if version == O.VERSION_2 else _TYPES_V1)[(first >> 4) & 3]
    if ptype == "RETRY":
        c.take(len(data) - c.pos - 16)
        c.take(16)
        rest = 0
    else:
        if ptype == "INITIAL":
            c.take(c.varint())
        rest = c.varint()
    end = c.pos + rest
    if end > len(data):
        raise ParseError("Packet payload is truncated")
    return Header(version, ptype, end - start, c.pos - start, cids[0])


class KeyUnavailable(Exception):
    pass


class DecryptError(Exception):
    pass


@dataclass
class Ctx:
    """One receive CryptoContext: suite, traffic secret, version, phase; the
    HP key stays the first one's across key updates (crypto.py:148-154)."""

    suite: int
    secret: bytes
    version: int
    key_phase: int = 0
    hp: Optional[bytes] = None

    def __post_init__(self):
        self.key, self.iv, hp = O.derive_key_iv_hp(self.suite, self.secret, self.version)
        if self.hp is None:
            self.hp = hp

    def next(self) -> "Ctx":
        """next_key_phase (crypto.py:157-168): "quic ku", same HP key."""
        return Ctx(self.suite, O.next_secret(self.suite, self.secret), self.version,
                   1 - self.key_phase, hp=self.hp)


@dataclass
class Pair:
    recv: Optional[Ctx] = None

    def decrypt_packet(self, packet: bytes, enc_off: int, expected: int):
        """CryptoPair.decrypt_packet (crypto.py:184-192 -> :75-103); the
        reference's undefined domain (a sample past the packet) is an error
        here, as in the product (Defined domain)."""
        ctx = self.recv
        if ctx is None:
            raise KeyUnavailable("Decryption key is not available")
        if enc_off + 20 > len(packet):
            raise DecryptError("Invalid payload length")
        mask = O.hp_mask(ctx.suite, ctx.hp, packet[enc_off + 4 : enc_off + 20])
        first = packet[0] ^ (mask[0] & (0x0F if packet[0] & LONG else 0x1F))
        use = ctx
        flipped = not first & LONG and ((first >> 2) & 1) != ctx.key_phase
        if flipped:
            use = ctx.next()
        try:
            hdr, payload, pn = O.unprotect(use.suite, use.key, use.iv, ctx.hp, packet, enc_off, expected)
        except ValueError as e:
            raise DecryptError(str(e)) from None
        if flipped:
            self.recv = use  # _update_key("remote_update")
        return hdr, payload, pn


@dataclass
class Conn:
    """What receive_datagram consults: pairs per epoch (Initial per version),
    expected packet numbers per space, CID length, role, versions; the host
    CIDs (None: not checked) and whether the connection is closing."""

    pairs: Dict[str, Pair]
    expected: Dict[str, int] = field(default_factory=lambda: {"INITIAL": 0, "HANDSHAKE": 0, "ONE_RTT": 0})
    initial_pairs: Optional[Dict[int, Pair]] = None
    host_cid_length: int = 8
    is_client: bool = False
    supported_versions: List[int] = field(default_factory=lambda: [O.VERSION_1, O.VERSION_2])
    host_cids: Optional[List[bytes]] = None
    closed: bool = False


@dataclass
class Outcome:
    datagram: int
    offset: int
    packet_type: str
    dropped: Optional[str] = None
    plain_header: bytes = b""
    plain_payload: bytes = b""
    packet_number: int = -1


def receive(items) -> List[Outcome]:
    """items: [(Conn, datagram bytes)] in arrival order -> one Outcome per
    packet (or per dropped remainder of a datagram)."""
    out: List[Outcome] = []
    for d, (conn, data) in enumerate(items):
        if conn.closed:
            # connection.py:756-757: a closing connection ignores the datagram
            out.append(Outcome(d, 0, "ONE_RTT", "connection_closed"))
            continue
        pos = 0
        while pos < len(data):
            try:
                h = parse_header(data, pos, conn.host_cid_length)
            except ParseError:
                out.append(Outcome(d, pos, "ONE_RTT", "header_parse_error"))
                break
            if not conn.is_client and h.packet_type == "INITIAL" and len(data) < 1200:
                out.append(Outcome(d, pos, h.packet_type, "initial_packet_datagram_too_small"))
                break
            # connection.py:830-848: clients check every packet's DCID,
            # servers their Handshake packets'
            if (conn.host_cids is not None and (conn.is_client or h.packet_type == "HANDSHAKE")
                    and h.destination_cid not in conn.host_cids):
                out.append(Outcome(d, pos, h.packet_type, "unknown_connection_id"))
                break
            if h.packet_type == "VERSION_NEGOTIATION":
                out.append(Outcome(d, pos, h.packet_type))
                break
            if h.version is not None and h.version not in conn.supported_versions:
                out.append(Outcome(d, pos, h.packet_type, "unsupported_version"))
                break
            if h.packet_type == "RETRY":
                out.append(Outcome(d, pos, h.packet_type))
                break
            epoch = _EPOCH[h.packet_type]
            if epoch == "INITIAL" and conn.initial_pairs is not None:
                pair = conn.initial_pairs.get(h.version, conn.pairs.get("INITIAL"))
            else:
                pair = conn.pairs[epoch]
            space = "ONE_RTT" if epoch == "ZERO_RTT" else epoch
            end = pos + h.packet_length
            o = Outcome(d, pos, h.packet_type)
            try:
                o.plain_header, o.plain_payload, o.packet_number = pair.decrypt_packet(
                    data[pos:end], h.encrypted_offset, conn.expected[space])
            except KeyUnavailable:
                o.dropped = "key_unavailable"
            except DecryptError:
                o.dropped = "payload_decrypt_error"
            if o.dropped is None:
                # connection.py:949-960: reserved bits set close the connection
                # (a key update inside decrypt_packet stands) and end the
                # datagram before :984-985 raises the expected number
                if o.plain_header[0] & (0x18 if h.packet_type == "ONE_RTT" else 0x0C):
                    out.append(Outcome(d, pos, h.packet_type, "reserved_bits"))
                    conn.closed = True
                    break
                if o.packet_number > conn.expected[space]:
                    conn.expected[space] = o.packet_number + 1
            out.append(o)
            pos = end
    return out
