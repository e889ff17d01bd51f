"""Batched receive (aioquic_amd.receive.receive_datagrams): header walk of
coalesced datagrams, epoch -> (pair, space) dispatch, drops with the
reference's triggers (connection.py:797-947), and one ReceiveBatch for all.

The CPU test swaps the device batch for the oracle (tests only); the GPU
test runs datagrams built by the deferred-encryption builder through the
real device path and checks every plaintext."""

from __future__ import annotations

import numpy as np
import pytest

from aioquic_amd import layout as L
from aioquic_amd import packet_builder as PB
from aioquic_amd import receive as R
from aioquic_amd.packet import QuicFrameType, QuicPacketType, QuicProtocolVersion
from aioquic_amd.tls import Epoch

from tests.test_packet_builder_batched import _oracle_protect, _Pair


class _Space:
    def __init__(self):
        self.expected_packet_number = 0


class _OracleBatch:
    """ReceiveBatch stand-in: decrypts each added packet with the oracle."""

    def __init__(self, oracle, keys):
        self.o, self.keys, self.items = oracle, keys, []

    def add(self, pair, packet, enc_off, space=None, conn=None, reserved_mask=0):
        self.items.append((pair, packet, enc_off, space))

    def run(self):
        out = []
        for pair, packet, enc_off, space in self.items:
            if pair is None:
                out.append(R.KeyUnavailableError("Decryption key is not available"))
                continue
            suite, key, iv, hp = self.keys
            try:
                h, p, pn = self.o.unprotect(suite, key, iv, hp, packet, enc_off, space.expected_packet_number)
            except ValueError:
                out.append(R.CryptoError("Payload decryption failed"))
                continue
            space.expected_packet_number = max(space.expected_packet_number, pn + 1)
            out.append((h, p, pn))
        return out


def _build(monkeypatch, oracle, pair):
    monkeypatch.setattr(PB, "_protect_datagrams", _oracle_protect(oracle))
    b = PB.QuicPacketBuilder(host_cid=bytes(8), peer_cid=bytes(8), version=QuicProtocolVersion.VERSION_1,
                             is_client=True, max_datagram_size=1200)
    b.start_packet(QuicPacketType.INITIAL, pair)
    b.start_frame(QuicFrameType.CRYPTO).push_bytes(b"\x11" * 100)
    b.start_packet(QuicPacketType.HANDSHAKE, pair)
    b.start_frame(QuicFrameType.CRYPTO).push_bytes(b"\x22" * 200)
    for k in range(3):
        b.start_packet(QuicPacketType.ONE_RTT, pair)
        b.start_frame(QuicFrameType.STREAM_BASE).push_bytes(bytes([k]) * (300 + k))
    return b.flush()


def test_receive_walk_and_drops_cpu(monkeypatch, oracle):
    pair = _Pair(oracle)
    datagrams, packets = _build(monkeypatch, oracle, pair)
    # Initial + Handshake + the first 1-RTT packet (padded inside itself to
    # fill the client's Initial datagram, RFC 9000 sec. 14.1), then two 1-RTT
    assert [len(d) for d in datagrams][0] == 1200 and len(datagrams) == 3
    suite, key, iv = pair.send.aead._material()
    keys = (suite, key, iv, pair.send.hp._material()[1])
    spaces = {e: _Space() for e in (Epoch.INITIAL, Epoch.HANDSHAKE, Epoch.ONE_RTT)}
    conn = R.ConnectionKeys(cryptos={e: pair for e in Epoch}, spaces=spaces)
    tampered = bytearray(datagrams[2])
    tampered[-1] ^= 1
    items = [(conn, d) for d in datagrams] + [(conn, bytes(tampered)), (conn, bytes([0x40]))]
    got = R.receive_datagrams(items, batch=_OracleBatch(oracle, keys))
    kinds = [(p.datagram, p.packet_type, p.dropped) for p in got]
    assert kinds[:5] == [(0, QuicPacketType.INITIAL, None), (0, QuicPacketType.HANDSHAKE, None),
                         (0, QuicPacketType.ONE_RTT, None), (1, QuicPacketType.ONE_RTT, None),
                         (2, QuicPacketType.ONE_RTT, None)]
    assert got[5].dropped == "payload_decrypt_error"
    assert got[6].dropped == "header_parse_error"
    assert [p.packet_number for p in got[:5]] == [p.packet_number for p in packets]
    assert got[0].plain_payload.startswith(b"\x06")  # CRYPTO frame type, then the bytes
    assert b"\x22" * 200 in got[1].plain_payload
    # the coalesced short-header packet runs to the end of the datagram
    assert got[2].offset + got[2].header.packet_length == 1200


def test_server_drops_small_initial_datagram(monkeypatch, oracle):
    pair = _Pair(oracle)
    datagrams, _ = _build(monkeypatch, oracle, pair)
    conn = R.ConnectionKeys(cryptos={e: pair for e in Epoch}, spaces={e: _Space() for e in Epoch})
    short_dg = datagrams[0][:1100]
    got = R.receive_datagrams([(conn, short_dg)], batch=_OracleBatch(oracle, None))
    assert [p.dropped for p in got] == ["initial_packet_datagram_too_small"]


@pytest.mark.gpu
def test_receive_datagrams_gpu_round_trip():
    """Client builders -> datagrams (one launch) -> server receive (one
    batch): every packet decrypts to what was written, packet numbers
    advance per space, and a connection with no 1-RTT keys drops its 1-RTT
    packets as key_unavailable."""
    from aioquic_amd.crypto import CryptoPair

    rng = np.random.default_rng(0x5EC)
    builders, conns, payloads = [], [], []
    for c in range(5):
        cid = bytes([c + 1]) * 8
        client, server = CryptoPair(), CryptoPair()
        client.setup_initial(cid, is_client=True, version=QuicProtocolVersion.VERSION_1)
        server.setup_initial(cid, is_client=False, version=QuicProtocolVersion.VERSION_1)
        b = PB.QuicPacketBuilder(host_cid=bytes(8), peer_cid=bytes(8), version=QuicProtocolVersion.VERSION_1,
                                 is_client=True, max_datagram_size=1200)
        sent = []
        for k in range(30):
            ptype = QuicPacketType.INITIAL if k == 0 else QuicPacketType.ONE_RTT
            b.start_packet(ptype, client)
            frame = b.start_frame(QuicFrameType.STREAM_BASE)
            body = rng.bytes(min(int(rng.integers(20, 900)), b.remaining_flight_space))
            frame.push_bytes(body)
            sent.append(body)
        builders.append(b)
        payloads.append(sent)
        one_rtt = server if c != 3 else CryptoPair()  # connection 3: no 1-RTT keys yet
        conns.append(R.ConnectionKeys(
            cryptos={Epoch.INITIAL: server, Epoch.HANDSHAKE: server, Epoch.ZERO_RTT: one_rtt,
                     Epoch.ONE_RTT: one_rtt},
            spaces={e: _Space() for e in (Epoch.INITIAL, Epoch.HANDSHAKE, Epoch.ONE_RTT)},
            is_client=False))
    flushed = PB.flush_builders(builders)
    items = []
    for c, (dgrams, _) in enumerate(flushed):
        items += [(conns[c], d) for d in dgrams]
    # interleave connections as a server socket would see them
    order = rng.permutation(len(items))
    got = R.receive_datagrams([items[i] for i in order])
    by_conn = {}
    for p in got:
        conn = items[order[p.datagram]][0]
        by_conn.setdefault(conns.index(conn), []).append(p)
    for c, pkts in by_conn.items():
        if c == 3:
            assert all(p.dropped == "key_unavailable" for p in pkts if p.epoch == Epoch.ONE_RTT)
            assert all(p.ok for p in pkts if p.epoch == Epoch.INITIAL)
            continue
        assert all(p.ok for p in pkts), [p.dropped for p in pkts]
        for p in pkts:
            assert payloads[c][p.packet_number][:50] in p.plain_payload
