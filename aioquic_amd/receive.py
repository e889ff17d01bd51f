"""Batched receive of many datagrams.

QuicConnection.receive_datagram (quic/connection.py:793-947) walks the
coalesced packets of ONE datagram: pull_quic_header (packet.py:181-267)
gives each packet's header and the offset of its packet number (the
"encrypted offset"), the packet's epoch picks the crypto pair and packet
number space (:889-899), and CryptoPair.decrypt_packet runs per packet
(:905-947).  receive_datagrams does the same walk for a whole batch of
datagrams, possibly of many connections, then decrypts every packet in one
ReceiveBatch (one device launch, a second only for key-phase flips), with
the sequential semantics of the per-packet loop: a packet's expected packet
number reflects the packets before it, and a peer key update rolls the
pair's keys before later packets (batch_io.ReceiveBatch).

Datagrams whose first byte is a short header (the 1-RTT bulk) take a
vectorised path: encrypted offset = 1 + host CID length, one packet per
datagram (a short-header packet always runs to the end of its datagram,
RFC 9000 sec. 12.2), no per-packet header parse.

The connection-level checks around the decrypt follow the reference too:
a connection that lists its host CIDs drops packets for other CIDs (clients:
every packet, servers: Handshake packets, "unknown_connection_id",
connection.py:830-848); a packet that authenticates with a reserved header bit
set closes its connection ("reserved_bits", :949-960: the rest of the datagram
is not read and the expected packet number is not raised), and a closed
connection's datagrams are ignored ("connection_closed", :756-757; one record
per datagram, where the reference logs nothing).
"""

from __future__ import annotations

from dataclasses import dataclass, field
from typing import Any, Dict, List, NamedTuple, Optional, Sequence, Tuple

import numpy as np

from . import _crypto
from ._crypto import CryptoError
from .batch_io import ConnectionClosedError, ReceiveBatch, ReservedBitsError, default_slots
from .buffer import Buffer
from .crypto import KeyUnavailableError
from .packet import (
    PACKET_FIXED_BIT,
    PACKET_LONG_HEADER,
    QuicHeader,
    QuicPacketType,
    QuicProtocolVersion,
    pull_quic_header,
)
from .tls import Epoch

SMALLEST_MAX_DATAGRAM_SIZE = 1200  # quic/configuration.py; RFC 9000 sec. 14.1

_EPOCH_OF_TYPE = {
    QuicPacketType.INITIAL: Epoch.INITIAL,
    QuicPacketType.ZERO_RTT: Epoch.ZERO_RTT,
    QuicPacketType.HANDSHAKE: Epoch.HANDSHAKE,
    QuicPacketType.ONE_RTT: Epoch.ONE_RTT,
}


@dataclass
class ConnectionKeys:
    """What receive_datagram consults per packet: the crypto pairs per epoch
    (Initial ones per version), the packet number spaces, the CID length,
    the role and the versions the configuration accepts
    (QuicConfiguration.supported_versions, configuration.py:115-120); the
    host CIDs a packet's destination CID must match (connection.py:830-848;
    None: not checked, the batch is already demultiplexed per connection) and
    whether the connection is closing (set by a reserved-bit violation)."""

    cryptos: Dict[Epoch, Any]
    spaces: Dict[Epoch, Any]
    cryptos_initial: Optional[Dict[int, Any]] = None
    host_cid_length: int = 8
    is_client: bool = False
    supported_versions: List[int] = field(
        default_factory=lambda: [QuicProtocolVersion.VERSION_1, QuicProtocolVersion.VERSION_2])
    host_cids: Optional[Sequence[bytes]] = None
    closed: bool = False

    def cid_unknown(self, packet_type: QuicPacketType, dcid: bytes) -> bool:
        """connection.py:830-848: clients check every packet, servers their
        Handshake packets."""
        return (self.host_cids is not None and (self.is_client or packet_type == QuicPacketType.HANDSHAKE)
                and dcid not in self.host_cids)

    def pair_and_space(self, epoch: Epoch, version: Optional[int]):
        if epoch == Epoch.INITIAL:
            pair = (self.cryptos_initial or {}).get(version, self.cryptos.get(Epoch.INITIAL))
        else:
            pair = self.cryptos[epoch]
        space = self.spaces[Epoch.ONE_RTT if epoch == Epoch.ZERO_RTT else epoch]
        return pair, space


class ReceivedPacket(NamedTuple):
    """One packet's outcome, in datagram order (an immutable record; tuple
    construction keeps the batched walk cheap per packet)."""

    datagram: int                 # index of the datagram in the batch
    offset: int                   # packet start within the datagram
    header: Optional[QuicHeader]  # None on the short-header fast path
    packet_type: QuicPacketType
    epoch: Optional[Epoch]
    plain_header: bytes = b""
    plain_payload: bytes = b""
    packet_number: int = -1
    dropped: Optional[str] = None  # the reference's packet_dropped trigger, if any

    @property
    def ok(self) -> bool:
        return self.dropped is None


_new = tuple.__new__
# reserved header bits (connection.py:949-953)
_RSV_SHORT, _RSV_LONG = 0x18, 0x0C
_DROP_OF = {ReservedBitsError: "reserved_bits", ConnectionClosedError: "connection_closed",
            KeyUnavailableError: "key_unavailable"}


def _record(f: tuple, res) -> ReceivedPacket:
    """The record of a queued packet from its ReceiveBatch outcome."""
    if isinstance(res, tuple):
        return _new(ReceivedPacket, f + res + (None,))
    drop = _DROP_OF.get(type(res), "payload_decrypt_error")
    if drop == "connection_closed":
        f = (f[0], 0, None, QuicPacketType.ONE_RTT, None)
    return _new(ReceivedPacket, f + (b"", b"", -1, drop))


def _closed_record(d: int) -> ReceivedPacket:
    return ReceivedPacket(d, 0, None, QuicPacketType.ONE_RTT, None, dropped="connection_closed")


def _walk_long(conn: ConnectionKeys, d: int, data: bytes, out: list, queued: list, add) -> None:
    """One datagram through the header parser, packet by packet.  Packets to
    decrypt go to `add(pair, packet, encrypted_offset, space)` and their
    record fields (datagram, offset, header, type, epoch) to `queued` with a
    placeholder in `out`."""
    buf = Buffer(data=data)
    while not buf.eof():
        start = buf.tell()
        try:
            header = pull_quic_header(buf, host_cid_length=conn.host_cid_length)
        except ValueError:
            out.append(ReceivedPacket(d, start, None, QuicPacketType.ONE_RTT, None, dropped="header_parse_error"))
            return
        ptype = header.packet_type
        if not conn.is_client and ptype == QuicPacketType.INITIAL and len(data) < SMALLEST_MAX_DATAGRAM_SIZE:
            out.append(ReceivedPacket(d, start, header, ptype, Epoch.INITIAL,
                                      dropped="initial_packet_datagram_too_small"))
            return
        if conn.cid_unknown(ptype, header.destination_cid):
            out.append(ReceivedPacket(d, start, header, ptype, None, dropped="unknown_connection_id"))
            return
        if ptype == QuicPacketType.VERSION_NEGOTIATION:
            # not packet-protected: handed back for the connection's own handler
            out.append(ReceivedPacket(d, start, header, ptype, None))
            return
        # a long header of a version the configuration does not accept ends
        # the datagram (connection.py:855-869)
        if header.version is not None and header.version not in conn.supported_versions:
            out.append(ReceivedPacket(d, start, header, ptype, None, dropped="unsupported_version"))
            return
        if ptype == QuicPacketType.RETRY:
            out.append(ReceivedPacket(d, start, header, ptype, None))
            return
        epoch = _EPOCH_OF_TYPE[ptype]
        pair, space = conn.pair_and_space(epoch, header.version)
        enc_off = buf.tell() - start
        end = start + header.packet_length
        buf.seek(end)
        queued.append((len(out), (d, start, header, ptype, epoch)))
        out.append(None)
        add(pair, data[start:end], enc_off, space, conn, _RSV_SHORT if ptype == QuicPacketType.ONE_RTT else _RSV_LONG)


def _receive_short(items: list) -> Optional[List[ReceivedPacket]]:
    """The steady state in C (_crypto.receive_short): every datagram one
    short-header packet.  None (nothing launched) when any is not; the
    caller then walks the batch in Python."""
    conns = _crypto.first_of_each(items)
    if any(c.is_client and c.host_cids is not None for c in conns):
        return None  # DCID checks: the general walk
    pix: dict = {}
    six: dict = {}
    upairs, uspaces, c_pair, c_space, c_cid = [], [], [], [], []
    for conn in conns:
        pair, space = conn.pair_and_space(Epoch.ONE_RTT, None)
        if id(pair) not in pix:
            pix[id(pair)] = len(upairs)
            upairs.append(pair)
        if id(space) not in six:
            six[id(space)] = len(uspaces)
            uspaces.append(space)
        c_pair.append(pix[id(pair)])
        c_space.append(six[id(space)])
        c_cid.append(conn.host_cid_length)
    slots = default_slots()
    keyed = [k for k, p in enumerate(upairs) if p.recv.aead is not None]
    pslot = np.full(len(upairs), 0xFFFFFFFF, np.uint32)
    if keyed:
        rc = [upairs[k].recv for k in keyed]
        pslot[keyed] = slots.assign([(c.aead, c.hp, c.key_phase) for c in rc])
    sexp = np.asarray([sp.expected_packet_number & 0xFFFFFFFFFFFFFFFF for sp in uspaces], np.uint64)
    got = _crypto.receive_short(slots.table, items, conns, np.asarray(c_cid, np.uint32).tobytes(),
                                np.asarray(c_pair, np.uint32).tobytes(), np.asarray(c_space, np.uint32).tobytes(),
                                pslot.tobytes(), sexp.tobytes(), ReceivedPacket, QuicPacketType.ONE_RTT,
                                Epoch.ONE_RTT, bytes(bool(c.closed) for c in conns))
    if got is None:
        return None
    recs, deferred, sexp2, closed = got
    new = np.frombuffer(sexp2, dtype=np.uint64)
    for k in np.flatnonzero(new != sexp).tolist():
        uspaces[k].expected_packet_number = int(new[k])
    for k, f in enumerate(closed):
        if f:
            conns[k].closed = True
    if deferred:
        # key-phase flips and numbers decoded under a stale expected number:
        # the general walk takes them in order from the state left above
        rb = ReceiveBatch(slots=slots)
        for d in deferred:
            conn, data = items[d]
            pair, space = conn.pair_and_space(Epoch.ONE_RTT, None)
            rb.add(pair, data, 1 + conn.host_cid_length, space=space, conn=conn, reserved_mask=_RSV_SHORT)
        for d, res in zip(deferred, rb.run()):
            recs[d] = _record((d, 0, None, QuicPacketType.ONE_RTT, Epoch.ONE_RTT), res)
            if isinstance(res, ReservedBitsError):
                items[d][0].closed = True
    return recs


def receive_datagrams(items: Sequence[Tuple[ConnectionKeys, bytes]],
                      batch: Optional[ReceiveBatch] = None) -> List[ReceivedPacket]:
    """Parse and unprotect every packet of every (connection, datagram) in
    order; returns one ReceivedPacket per packet (or per dropped remainder of
    a datagram, like the reference's early returns).

    Short-header datagrams (the 1-RTT bulk) skip the header parser: their
    encrypted offset is 1 + the host CID length and the packet runs to the
    end of the datagram.  Every packet goes into one ReceiveBatch, whose first
    round (one launch and the in-order walk) runs in C."""
    own = batch is None
    if not items:
        return []
    if own:
        fast = _receive_short(items if isinstance(items, list) else list(items))
        if fast is not None:
            return fast
    batch = batch or ReceiveBatch(slots=default_slots())
    first = np.fromiter((dg[0] if dg else 0 for _, dg in items), np.uint8, len(items))
    short = ((first & (PACKET_LONG_HEADER | PACKET_FIXED_BIT)) == PACKET_FIXED_BIT).tolist()
    out: list = []
    queued: list = []  # (position in out, record fields) of every packet to decrypt
    # runs of short-header datagrams go to the batch in bulk
    r_pairs: list = []
    r_packets: list = []
    r_offs: list = []
    r_spaces: list = []
    r_conns: list = []
    by_conn: dict = {}
    bulk = own or hasattr(batch, "_extend")

    def flush_run():
        if r_pairs:
            if bulk:
                batch._extend(r_pairs, r_packets, r_offs, r_spaces, r_conns, _RSV_SHORT)
            else:
                for a, b, c, e, g in zip(r_pairs, r_packets, r_offs, r_spaces, r_conns):
                    batch.add(a, b, c, space=e, conn=g, reserved_mask=_RSV_SHORT)
            r_pairs.clear(), r_packets.clear(), r_offs.clear(), r_spaces.clear(), r_conns.clear()

    def add(pair, packet, enc_off, space, conn, rsv):
        flush_run()
        batch.add(pair, packet, enc_off, space=space, conn=conn, reserved_mask=rsv)

    one_rtt, ep1 = QuicPacketType.ONE_RTT, Epoch.ONE_RTT
    for d, ((conn, data), is_short) in enumerate(zip(items, short)):
        if conn.closed:
            out.append(_closed_record(d))  # connection.py:756-757
            continue
        if is_short:
            c = by_conn.get(id(conn))
            if c is None:
                pair, space = conn.pair_and_space(ep1, None)
                c = by_conn[id(conn)] = (pair, space, 1 + conn.host_cid_length, conn,
                                         conn.is_client and conn.host_cids is not None)
            if len(data) >= c[2]:
                if c[4] and data[1:c[2]] not in conn.host_cids:
                    out.append(ReceivedPacket(d, 0, None, one_rtt, None, dropped="unknown_connection_id"))
                    continue
                queued.append((len(out), (d, 0, None, one_rtt, ep1)))
                out.append(None)
                r_pairs.append(c[0])
                r_packets.append(data)
                r_offs.append(c[2])
                r_spaces.append(c[1])
                r_conns.append(conn)
                continue
        _walk_long(conn, d, data, out, queued, add)
    flush_run()
    results = batch.run()
    cut = False
    for (pos, f), res in zip(queued, results):
        out[pos] = _record(f, res)
        cut = cut or not isinstance(res, tuple) and isinstance(res, (ReservedBitsError, ConnectionClosedError))
    return _apply_closes(items, out) if cut else out


def _apply_closes(items, out: list) -> list:
    """A reserved-bit violation closes its connection (connection.py:949-960):
    the rest of its datagram is not read, and every later datagram of the
    connection is ignored (:756-757), one "connection_closed" record each."""
    new: list = []
    closed: set = set()
    k = 0
    while k < len(out):
        d = out[k].datagram
        conn = items[d][0]
        e = k
        while e < len(out) and out[e].datagram == d:
            e += 1
        if id(conn) in closed:
            new.append(_closed_record(d))
        else:
            for r in out[k:e]:
                new.append(r)
                if r.dropped == "reserved_bits":
                    closed.add(id(conn))
                    conn.closed = True
                    break
        k = e
    return new
