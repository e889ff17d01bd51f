"""QUIC packet builder with deferred, batched encryption.

Same public surface as aioquic's ``quic/packet_builder.py``
(``QuicPacketBuilder`` :51-384, ``QuicSentPacket`` :30-44,
``QuicDeliveryState`` :25-27, ``QuicPacketBuilderStop`` :47-48,
``PACKET_LENGTH_SEND_SIZE`` / ``PACKET_NUMBER_SEND_SIZE`` :19-20), with one
difference in *when* packets are encrypted.

The reference encrypts each packet in place as soon as it is closed
(``_end_packet`` :341-350, one ``CryptoPair.encrypt_packet`` call per
packet).  Encryption never changes a packet's size (ciphertext = plaintext +
16-byte tag), so every datagram boundary, padding decision and
``sent_bytes`` figure is known before any byte is encrypted.  This builder
therefore writes the *plaintext* packet with a 16-byte hole for the tag,
records the key material the reference would have used at that moment
(including a pending local key update, crypto.py:194-199), and encrypts
everything at ``flush()`` in one device launch.  ``flush_builders`` does the
same across many connections' builders (a server's ``datagrams_to_send``
pass), still one launch.  The datagrams returned are byte-identical to the
reference's.
"""

from __future__ import annotations

from array import array
from dataclasses import dataclass, field
from enum import Enum
from typing import Any, Callable, Optional, Sequence

import numpy as np

from . import layout as L
from ._crypto import protect_datagrams
from .batch_io import KeySlots, _raise_status, default_slots
from .buffer import Buffer, size_uint_var
from .tls import Epoch
from .packet import (
    NON_ACK_ELICITING_FRAME_TYPES,
    NON_IN_FLIGHT_FRAME_TYPES,
    PACKET_FIXED_BIT,
    PACKET_NUMBER_MAX_SIZE,
    QuicFrameType,
    QuicPacketType,
    encode_long_header_first_byte,
)

PACKET_LENGTH_SEND_SIZE = 2
PACKET_NUMBER_SEND_SIZE = 2

QuicDeliveryHandler = Callable[..., None]


class QuicDeliveryState(Enum):
    ACKED = 0
    LOST = 1


@dataclass
class QuicSentPacket:
    epoch: Epoch
    in_flight: bool
    is_ack_eliciting: bool
    is_crypto_packet: bool
    packet_number: int
    packet_type: QuicPacketType
    sent_time: Optional[float] = None
    sent_bytes: int = 0
    delivery_handlers: list = field(default_factory=list)
    quic_logger_frames: list = field(default_factory=list)


class QuicPacketBuilderStop(Exception):
    pass


_EPOCH_OF = {QuicPacketType.INITIAL: Epoch.INITIAL, QuicPacketType.HANDSHAKE: Epoch.HANDSHAKE}
_EPOCH_ONE_RTT = Epoch.ONE_RTT
# a packet closer than this to the end of the datagram starts a new one
# (the reference's arbitrary limit, packet_builder.py:197-199)
_MIN_PACKET_ROOM = 128


class _Pending:
    """The closed packets of a builder awaiting encryption, one entry per
    packet in flat lists: its datagram (index among the builder's closed
    datagrams), offset in it, header size, plaintext header + payload size,
    packet number, and the key material the reference would have encrypted
    it with -- an index into `keys`, the builder's distinct (aead, hp,
    key_phase) triples, so that slots are resolved per key, not per packet."""

    __slots__ = ("dg", "off", "hsize", "size", "pn", "ref", "keys", "_key_ix")

    def __init__(self) -> None:
        # typed arrays: appended per packet, handed to numpy without a copy
        self.dg = array("I")
        self.off = array("I")
        self.hsize = array("I")
        self.size = array("I")
        self.pn = array("Q")
        self.ref = array("I")
        self.keys: list = []
        self._key_ix: dict = {}

    def __len__(self) -> int:
        return len(self.dg)

    def add(self, dg: int, off: int, hsize: int, size: int, pn: int, keys: tuple) -> None:
        k = (id(keys[0]), id(keys[1]), keys[2])
        r = self._key_ix.get(k)
        if r is None:
            r = self._key_ix[k] = len(self.keys)
            self.keys.append(keys)
        self.dg.append(dg)
        self.off.append(off)
        self.hsize.append(hsize)
        self.size.append(size)
        self.pn.append(pn & 0xFFFFFFFFFFFFFFFF)
        self.ref.append(r)

    def packets(self):
        """(datagram, offset, header size, size, packet number, keys) per packet."""
        return zip(self.dg, self.off, self.hsize, self.size, self.pn, (self.keys[r] for r in self.ref))


def _default_slots() -> KeySlots:
    return default_slots()


class QuicPacketBuilder:
    """Builds QUIC packets into datagrams; encryption is deferred to flush()."""

    def __init__(self, *, host_cid: bytes, peer_cid: bytes, version: int, is_client: bool,
                 max_datagram_size: int, packet_number: int = 0, peer_token: bytes = b"",
                 quic_logger=None, spin_bit: bool = False, slots: Optional[KeySlots] = None):
        self.max_flight_bytes: Optional[int] = None
        self.max_total_bytes: Optional[int] = None
        self.quic_logger_frames: Optional[list] = None

        self._host_cid, self._peer_cid, self._peer_token = host_cid, peer_cid, peer_token
        self._is_client, self._version, self._spin_bit = is_client, version, spin_bit
        self._quic_logger = quic_logger
        self._slots = slots

        # finished datagrams (plaintext, tag holes) and their pending packets
        self._datagrams: list = []
        self._pending = _Pending()
        self._packets: list = []
        self._flight_bytes = 0
        self._total_bytes = 0

        # the datagram being filled
        self._buffer = Buffer(max_datagram_size)
        self._buffer_capacity = max_datagram_size
        self._flight_capacity = max_datagram_size
        self._datagram_fresh = True
        self._datagram_flight_bytes = 0
        self._datagram_needs_padding = False

        # the packet being filled
        self._packet: Optional[QuicSentPacket] = None
        self._packet_crypto = None
        self._packet_type: Optional[QuicPacketType] = None
        self._packet_start = 0
        self._header_size = 0
        self._packet_number = packet_number

    # ---------------------------------------------------------- properties
    @property
    def packet_is_empty(self) -> bool:
        assert self._packet is not None
        return self._buffer.tell() - self._packet_start <= self._header_size

    @property
    def packet_number(self) -> int:
        return self._packet_number

    @property
    def remaining_buffer_space(self) -> int:
        return self._buffer_capacity - self._buffer.tell() - self._packet_crypto.aead_tag_size

    @property
    def remaining_flight_space(self) -> int:
        return self._flight_capacity - self._buffer.tell() - self._packet_crypto.aead_tag_size

    # ------------------------------------------------------------ packets
    def _header_size_for(self, packet_type: QuicPacketType) -> int:
        if packet_type == QuicPacketType.ONE_RTT:
            return 1 + len(self._peer_cid) + PACKET_NUMBER_SEND_SIZE
        # first byte, version, two CID lengths, length field, packet number
        size = 1 + 4 + 1 + len(self._peer_cid) + 1 + len(self._host_cid)
        size += PACKET_LENGTH_SEND_SIZE + PACKET_NUMBER_SEND_SIZE
        if packet_type == QuicPacketType.INITIAL:
            size += size_uint_var(len(self._peer_token)) + len(self._peer_token)
        return size

    def _open_datagram(self) -> None:
        cap = self._buffer_capacity
        if self.max_total_bytes is not None:
            cap = min(cap, self.max_total_bytes - self._total_bytes)
        self._buffer_capacity = cap
        flight = cap
        if self.max_flight_bytes is not None:
            flight = min(flight, self.max_flight_bytes - self._flight_bytes)
        self._flight_capacity = flight
        self._datagram_flight_bytes = 0
        self._datagram_needs_padding = False
        self._datagram_fresh = False

    def start_packet(self, packet_type: QuicPacketType, crypto) -> None:
        assert packet_type in (QuicPacketType.INITIAL, QuicPacketType.HANDSHAKE,
                               QuicPacketType.ZERO_RTT, QuicPacketType.ONE_RTT), "Invalid packet type"
        if self._packet is not None:
            self._end_packet()
        start = self._buffer.tell()
        if self._buffer_capacity - start < _MIN_PACKET_ROOM:
            self._flush_current_datagram()
            start = 0
        if self._datagram_fresh:
            self._open_datagram()
        hsize = self._header_size_for(packet_type)
        if start + hsize >= self._buffer_capacity:
            raise QuicPacketBuilderStop
        self._packet = QuicSentPacket(
            epoch=_EPOCH_OF.get(packet_type, _EPOCH_ONE_RTT), in_flight=False, is_ack_eliciting=False,
            is_crypto_packet=False, packet_number=self._packet_number, packet_type=packet_type)
        self._packet_crypto, self._packet_type = crypto, packet_type
        self._packet_start, self._header_size = start, hsize
        self.quic_logger_frames = self._packet.quic_logger_frames
        self._buffer.seek(start + hsize)

    def start_frame(self, frame_type: int, capacity: int = 1, handler: Optional[QuicDeliveryHandler] = None,
                    handler_args: Sequence[Any] = []) -> Buffer:
        counts_in_flight = frame_type not in NON_IN_FLIGHT_FRAME_TYPES
        if self.remaining_buffer_space < capacity or (counts_in_flight and self.remaining_flight_space < capacity):
            raise QuicPacketBuilderStop
        self._buffer.push_uint_var(frame_type)
        pkt = self._packet
        pkt.is_ack_eliciting |= frame_type not in NON_ACK_ELICITING_FRAME_TYPES
        pkt.in_flight |= counts_in_flight
        pkt.is_crypto_packet |= frame_type == QuicFrameType.CRYPTO
        if handler is not None:
            pkt.delivery_handlers.append((handler, handler_args))
        return self._buffer

    def _padding_for(self, packet_size: int) -> int:
        # enough bytes after the packet number for a 16-byte HP sample
        # (RFC 9001 sec. 5.4.2)
        pad = PACKET_NUMBER_MAX_SIZE - PACKET_NUMBER_SEND_SIZE + self._header_size - packet_size
        if self._packet_type == QuicPacketType.INITIAL and (self._is_client or self._packet.is_ack_eliciting):
            self._datagram_needs_padding = True  # RFC 9000 sec. 14.1
        if self._datagram_needs_padding and self._packet_type == QuicPacketType.ONE_RTT:
            # a 1-RTT packet cannot be followed by datagram padding: pad inside it
            pad = max(pad, self.remaining_flight_space)
            self._datagram_needs_padding = False
        return pad

    def _write_header(self, packet_size: int) -> None:
        buf, crypto = self._buffer, self._packet_crypto
        buf.seek(self._packet_start)
        pn16 = self._packet_number & 0xFFFF
        if self._packet_type == QuicPacketType.ONE_RTT:
            buf.push_uint8(PACKET_FIXED_BIT | (self._spin_bit << 5) | (crypto.key_phase << 2)
                           | (PACKET_NUMBER_SEND_SIZE - 1))
            buf.push_bytes(self._peer_cid)
        else:
            rest = packet_size - self._header_size + PACKET_NUMBER_SEND_SIZE + crypto.aead_tag_size
            buf.push_uint8(encode_long_header_first_byte(self._version, self._packet_type,
                                                         PACKET_NUMBER_SEND_SIZE - 1))
            buf.push_uint32(self._version)
            for cid in (self._peer_cid, self._host_cid):
                buf.push_uint8(len(cid))
                buf.push_bytes(cid)
            if self._packet_type == QuicPacketType.INITIAL:
                buf.push_uint_var(len(self._peer_token))
                buf.push_bytes(self._peer_token)
            buf.push_uint16(rest | 0x4000)
        buf.push_uint16(pn16)

    def _end_packet(self) -> None:
        buf, pkt = self._buffer, self._packet
        size = buf.tell() - self._packet_start
        if size <= self._header_size:
            buf.seek(self._packet_start)  # nothing written: cancel the packet
        else:
            pad = self._padding_for(size)
            if pad > 0:
                buf.push_bytes(bytes(pad))
                size += pad
                pkt.in_flight = True
                if self._quic_logger is not None:
                    pkt.quic_logger_frames.append(self._quic_logger.encode_padding_frame())
            self._write_header(size)
            # the key material encrypt_packet would use now, with a pending
            # local key update applied first (crypto.py:194-199)
            pair = self._packet_crypto
            if getattr(pair, "_update_key_requested", False):
                pair._update_key("local_update")
            ctx = getattr(pair, "send", pair)
            assert ctx.is_valid(), "Encryption key is not available"
            # (the current datagram becomes datagram len(self._datagrams))
            self._pending.add(len(self._datagrams), self._packet_start, self._header_size, size,
                              self._packet_number, (ctx.aead, ctx.hp, ctx.key_phase))
            # leave the tag's room: the cursor ends where the reference's would
            buf.seek(self._packet_start + size)
            buf.push_bytes(bytes(pair.aead_tag_size))
            pkt.sent_bytes = size + pair.aead_tag_size
            self._packets.append(pkt)
            if pkt.in_flight:
                self._datagram_flight_bytes += pkt.sent_bytes
            if self._packet_type == QuicPacketType.ONE_RTT:
                self._flush_current_datagram()  # short headers end the datagram
            self._packet_number += 1
        self._packet = None
        self.quic_logger_frames = None

    def _flush_current_datagram(self) -> None:
        buf = self._buffer
        used = buf.tell()
        if not used:
            return
        if self._datagram_needs_padding:
            extra = self._flight_capacity - used
            if extra > 0:
                buf.push_bytes(bytes(extra))
                self._datagram_flight_bytes += extra
                used += extra
        self._datagrams.append(buf.data)
        self._flight_bytes += self._datagram_flight_bytes
        self._total_bytes += used
        self._datagram_fresh = True
        buf.seek(0)

    def _close(self):
        """End the packet and datagram in progress; hand over (plaintext
        datagrams, pending packets per datagram, sent packets)."""
        if self._packet is not None:
            self._end_packet()
        self._flush_current_datagram()
        out = (self._datagrams, self._pending, self._packets)
        self._datagrams, self._pending, self._packets = [], _Pending(), []
        return out

    def flush(self) -> tuple:
        """(datagrams, sent packets), every packet encrypted in one launch."""
        return flush_builders([self], slots=self._slots)[0]


def flush_builders(builders: Sequence[QuicPacketBuilder], slots: Optional[KeySlots] = None) -> list:
    """flush() of many builders (e.g. every connection of a server) with ONE
    device launch for all their packets; returns [(datagrams, packets)] in
    builder order."""
    closed = [b._close() for b in builders]
    plains = [d for c in closed for d in c[0]]
    wire = _protect_datagrams(plains, [(len(c[0]), c[1]) for c in closed], slots) if plains else []
    out, k = [], 0
    for dgrams, _, packets in closed:
        out.append((wire[k : k + len(dgrams)], packets))
        k += len(dgrams)
    return out


def _protect_datagrams(plains: list, pending: list, slots: Optional[KeySlots]) -> list:
    """Encrypt every pending packet of the given plaintext datagrams in one
    launch (_crypto.protect_datagrams: descriptors and pinned staging built in
    C, one bytes object per wire datagram).  `pending` holds, per builder in
    datagram order, (its datagram count, its _Pending).  The slots are
    resolved once per distinct key of a builder."""
    slots = slots or _default_slots()
    # every builder's distinct keys, assigned slots in one call
    triples, firsts = [], []
    for _, pend in pending:
        firsts.append(len(triples))
        triples += pend.keys
    per_key = np.asarray(slots.assign(triples), dtype=np.uint32) if triples else np.zeros(0, np.uint32)
    cols = {k: [] for k in ("dg", "off", "hsize", "size", "pn", "slot")}
    base = 0
    for (count, pend), first in zip(pending, firsts):
        if len(pend):
            cols["dg"].append(np.frombuffer(pend.dg, np.uint32) + np.uint32(base))
            cols["off"].append(np.frombuffer(pend.off, np.uint32))
            cols["hsize"].append(np.frombuffer(pend.hsize, np.uint32))
            cols["size"].append(np.frombuffer(pend.size, np.uint32))
            cols["pn"].append(np.frombuffer(pend.pn, np.uint64))
            cols["slot"].append(per_key[first + np.frombuffer(pend.ref, np.uint32)])
        base += count
    arr = {k: (np.concatenate(v) if v else np.zeros(0, np.uint64 if k == "pn" else np.uint32)).tobytes()
           for k, v in cols.items()}
    wire, res = protect_datagrams(slots.table, plains, arr["dg"], arr["off"], arr["hsize"], arr["size"],
                                  arr["pn"], arr["slot"])
    status = np.frombuffer(res, dtype=L.RESULT)["status"]
    bad = np.flatnonzero(status != L.S_OK)
    if len(bad):
        raise _raise_status(int(status[bad[0]]))
    return wire
