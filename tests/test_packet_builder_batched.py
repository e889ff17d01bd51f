"""Deferred-encryption packet builder (aioquic_amd.packet_builder) and the
header parser (aioquic_amd.packet.pull_quic_header).

CPU tests drive the builder with stand-in key objects and protect the
datagrams with the oracle (tests only), and check the datagram / packet
accounting against the figures the reference's own builder tests hold
(tests/test_packet_builder.py: remaining space 1156 / 1173 / 995 / 1157 /
973 / 773, datagram sizes, sent_bytes).  GPU tests run the real device path
and compare every datagram with the oracle, byte for byte, across several
connections flushed in one launch.
"""

from __future__ import annotations

import numpy as np
import pytest

from aioquic_amd import layout as L
from aioquic_amd import packet_builder as PB
from aioquic_amd.buffer import Buffer
from aioquic_amd.packet import QuicFrameType, QuicPacketType, QuicProtocolVersion, pull_quic_header
from aioquic_amd.tls import Epoch


class _Mat:
    def __init__(self, *m):
        self._m = m

    def _material(self):
        return self._m


class _Ctx:
    def __init__(self, suite, key, iv, hp, phase=0):
        self.aead = _Mat(suite, key, iv)
        self.hp = _Mat(suite, hp)
        self.key_phase = phase

    def is_valid(self):
        return True


class _Pair:
    """Stand-in CryptoPair: client Initial keys of DCID 00..00 (RFC 9001 A.1
    derivation, via the oracle)."""

    aead_tag_size = 16
    _update_key_requested = False

    def __init__(self, oracle, cid=bytes(8)):
        client, _ = oracle.initial_secrets(cid)
        key, iv, hp = oracle.derive_key_iv_hp(0, client)
        self.send = _Ctx(L.AES_128_GCM, key, iv, hp)

    @property
    def key_phase(self):
        return self.send.key_phase


def _oracle_protect(oracle):
    """Stand-in for packet_builder._protect_datagrams: each pending packet
    protected by the oracle.  pending = [(datagram count, _Pending)] per
    builder, as flush_builders passes it."""
    def protect(plains, pending, slots):
        out = [bytearray(d) for d in plains]
        base = 0
        for count, pend in pending:
            for dg, off, hsize, size, pn, keys in pend.packets():
                d = out[base + dg]
                suite, key, iv = keys[0]._material()
                _, hp = keys[1]._material()
                hdr = bytes(d[off : off + hsize])
                pay = bytes(d[off + hsize : off + size])
                wire = oracle.protect(suite, key, iv, hp, hdr, pay, pn)
                d[off : off + len(wire)] = wire
            base += count
        return [bytes(d) for d in out]

    return protect


@pytest.fixture
def cpu_builder(oracle, monkeypatch):
    monkeypatch.setattr(PB, "_protect_datagrams", _oracle_protect(oracle))

    def make(is_client=False):
        return PB.QuicPacketBuilder(host_cid=bytes(8), peer_cid=bytes(8), version=QuicProtocolVersion.VERSION_1,
                                    is_client=is_client, max_datagram_size=1200, packet_number=0)

    return make


def _sent(epoch, pn, ptype, nbytes, crypto=True, in_flight=True, ack=True):
    return PB.QuicSentPacket(epoch=epoch, in_flight=in_flight, is_ack_eliciting=ack,
                             is_crypto_packet=crypto, packet_number=pn, packet_type=ptype, sent_bytes=nbytes)


def _walk(datagram, cid_len=8):
    """Headers of the coalesced packets of a datagram (encrypted offsets)."""
    buf = Buffer(data=datagram)
    out = []
    while not buf.eof():
        start = buf.tell()
        if not any(datagram[start:]):
            break  # datagram padding (RFC 9000 sec. 14.1)
        h = pull_quic_header(buf, host_cid_length=cid_len)
        out.append((h, start, buf.tell() - start))
        buf.seek(start + h.packet_length)
    return out


def _check_decrypts(oracle, pair, datagrams, packets):
    """Every packet of every datagram unprotects under the pair's keys to
    the plaintext the builder wrote, with the packet numbers of `packets`."""
    suite, key, iv = pair.send.aead._material()
    _, hp = pair.send.hp._material()
    pns = iter(p.packet_number for p in packets)
    for dg in datagrams:
        for h, start, enc_off in _walk(dg):
            pkt = dg[start : start + h.packet_length]
            got = oracle.unprotect(suite, key, iv, hp, pkt, enc_off, 0)
            assert got is not None
            plain_header, payload, pn = got[0], got[1], got[2]
            assert pn == next(pns)
            assert len(plain_header) + len(payload) + 16 == len(pkt)


def test_initial_client_padded(cpu_builder, oracle):
    b, pair = cpu_builder(is_client=True), _Pair(oracle)
    b.start_packet(QuicPacketType.INITIAL, pair)
    assert b.remaining_flight_space == 1156
    b.start_frame(QuicFrameType.CRYPTO).push_bytes(bytes(100))
    assert not b.packet_is_empty
    b.start_packet(QuicPacketType.INITIAL, pair)
    assert b.packet_is_empty
    datagrams, packets = b.flush()
    assert [len(d) for d in datagrams] == [1200]
    assert packets == [_sent(Epoch.INITIAL, 0, QuicPacketType.INITIAL, 145)]
    assert b.packet_number == 1
    _check_decrypts(oracle, pair, datagrams, packets)


def test_initial_server_coalesced(cpu_builder, oracle):
    b, pair = cpu_builder(), _Pair(oracle)
    b.start_packet(QuicPacketType.INITIAL, pair)
    assert b.remaining_flight_space == 1156
    b.start_frame(QuicFrameType.ACK).push_bytes(bytes(16))
    b.start_frame(QuicFrameType.CRYPTO).push_bytes(bytes(100))
    b.start_packet(QuicPacketType.INITIAL, pair)
    assert b.packet_is_empty
    b.start_packet(QuicPacketType.HANDSHAKE, pair)
    assert b.remaining_flight_space == 995
    b.start_frame(QuicFrameType.CRYPTO).push_bytes(bytes(994))
    b.start_packet(QuicPacketType.HANDSHAKE, pair)
    assert b.remaining_flight_space == 1157
    b.start_frame(QuicFrameType.CRYPTO).push_bytes(bytes(800))
    b.start_packet(QuicPacketType.HANDSHAKE, pair)
    assert b.packet_is_empty
    datagrams, packets = b.flush()
    assert [len(d) for d in datagrams] == [1200, 844]
    assert packets == [
        _sent(Epoch.INITIAL, 0, QuicPacketType.INITIAL, 162),
        _sent(Epoch.HANDSHAKE, 1, QuicPacketType.HANDSHAKE, 1038),
        _sent(Epoch.HANDSHAKE, 2, QuicPacketType.HANDSHAKE, 844),
    ]
    # coalesced: Initial + Handshake in datagram 0, the parser walks both
    hs = _walk(datagrams[0])
    assert [h.packet_type for h, _, _ in hs] == [QuicPacketType.INITIAL, QuicPacketType.HANDSHAKE]
    assert [h.packet_length for h, _, _ in hs] == [162, 1038]
    _check_decrypts(oracle, pair, datagrams, packets)


def test_long_then_short(cpu_builder, oracle):
    b, pair = cpu_builder(), _Pair(oracle)
    b.start_packet(QuicPacketType.INITIAL, pair)
    assert b.remaining_flight_space == 1156
    b.start_frame(QuicFrameType.CRYPTO).push_bytes(bytes(b.remaining_flight_space))
    b.start_packet(QuicPacketType.INITIAL, pair)
    b.start_packet(QuicPacketType.ONE_RTT, pair)
    assert b.remaining_flight_space == 1173
    b.start_frame(QuicFrameType.STREAM_BASE).push_bytes(bytes(b.remaining_flight_space))
    b.start_packet(QuicPacketType.ONE_RTT, pair)
    assert b.packet_is_empty
    datagrams, packets = b.flush()
    assert [len(d) for d in datagrams] == [1200, 1200]
    assert packets == [
        _sent(Epoch.INITIAL, 0, QuicPacketType.INITIAL, 1200),
        _sent(Epoch.ONE_RTT, 1, QuicPacketType.ONE_RTT, 1200, crypto=False),
    ]
    assert b.packet_number == 2
    _check_decrypts(oracle, pair, datagrams, packets)


@pytest.mark.parametrize("limit,field,space,sizes", [
    (1000, "max_flight_bytes", 973, [1000]),
    (800, "max_total_bytes", 773, [800]),
])
def test_short_header_limits(cpu_builder, oracle, limit, field, space, sizes):
    b, pair = cpu_builder(), _Pair(oracle)
    setattr(b, field, limit)
    b.start_packet(QuicPacketType.ONE_RTT, pair)
    assert b.remaining_flight_space == space
    b.start_frame(QuicFrameType.CRYPTO).push_bytes(bytes(b.remaining_flight_space))
    with pytest.raises(PB.QuicPacketBuilderStop):
        b.start_packet(QuicPacketType.ONE_RTT, pair)
        b.start_frame(QuicFrameType.CRYPTO)
    datagrams, packets = b.flush()
    assert [len(d) for d in datagrams] == sizes
    assert packets == [_sent(Epoch.ONE_RTT, 0, QuicPacketType.ONE_RTT, sizes[0])]
    _check_decrypts(oracle, pair, datagrams, packets)


def test_short_header_total_bytes_two_datagrams(cpu_builder, oracle):
    b, pair = cpu_builder(), _Pair(oracle)
    b.max_total_bytes = 2000
    for want in (1173, 773):
        b.start_packet(QuicPacketType.ONE_RTT, pair)
        assert b.remaining_flight_space == want
        b.start_frame(QuicFrameType.CRYPTO).push_bytes(bytes(b.remaining_flight_space))
    with pytest.raises(PB.QuicPacketBuilderStop):
        b.start_packet(QuicPacketType.ONE_RTT, pair)
    datagrams, packets = b.flush()
    assert [len(d) for d in datagrams] == [1200, 800]
    assert [p.sent_bytes for p in packets] == [1200, 800]
    _check_decrypts(oracle, pair, datagrams, packets)


def test_sample_padding_on_tiny_packet(cpu_builder, oracle):
    """A 1-byte PING payload gets padded so that the HP sample exists
    (PACKET_NUMBER_MAX_SIZE - PACKET_NUMBER_SEND_SIZE bytes)."""
    b, pair = cpu_builder(), _Pair(oracle)
    b.start_packet(QuicPacketType.ONE_RTT, pair)
    b.start_frame(QuicFrameType.PING)
    datagrams, packets = b.flush()
    # header 11 + PING 1 + padding 1 (2 bytes after the PN) + tag 16
    assert [len(d) for d in datagrams] == [29]
    assert packets[0].sent_bytes == 29 and packets[0].in_flight
    _check_decrypts(oracle, pair, datagrams, packets)


def test_pull_quic_header_errors():
    with pytest.raises(ValueError, match="fixed bit"):
        pull_quic_header(Buffer(data=bytes([0x00]) + bytes(8)), host_cid_length=8)
    with pytest.raises(ValueError, match="too long"):
        pull_quic_header(Buffer(data=bytes([0xC0, 0, 0, 0, 1, 21]) + bytes(30)), host_cid_length=8)
    # long header whose length field runs past the datagram
    bad = bytes([0xC0]) + (1).to_bytes(4, "big") + bytes([0, 0, 0]) + bytes([0x44, 0x00])
    with pytest.raises(ValueError, match="truncated"):
        pull_quic_header(Buffer(data=bad), host_cid_length=8)


# ------------------------------------------------------------------ GPU --


def _gpu_case(oracle, n_conn=6, per_conn=40):
    from aioquic_amd.crypto import CryptoPair

    rng = np.random.default_rng(0xB11D)
    builders, pairs = [], []
    for c in range(n_conn):
        pair = CryptoPair()
        pair.setup_initial(bytes([c]) * 8, is_client=bool(c & 1), version=QuicProtocolVersion.VERSION_1)
        b = PB.QuicPacketBuilder(host_cid=bytes([c]) * 8, peer_cid=bytes([c + 1]) * 8,
                                 version=QuicProtocolVersion.VERSION_1, is_client=bool(c & 1),
                                 max_datagram_size=1200, packet_number=int(rng.integers(0, 1 << 20)))
        for k in range(per_conn):
            if c == 2 and k == per_conn // 2:
                pair.update_key()  # a local key update half way through
            ptype = QuicPacketType.INITIAL if (k == 0 and c < 3) else QuicPacketType.ONE_RTT
            b.start_packet(ptype, pair)
            room = b.remaining_flight_space
            b.start_frame(QuicFrameType.STREAM_BASE).push_bytes(
                rng.bytes(int(rng.integers(1, max(2, room)))))
        builders.append(b)
        pairs.append(pair)
    return builders, pairs


@pytest.mark.gpu
def test_flush_builders_matches_oracle(oracle):
    """Several connections flushed in ONE launch: each datagram equals the
    oracle's encryption of the same plaintext packets."""
    builders, pairs = _gpu_case(oracle)
    twins, _ = _gpu_case(oracle)  # same packets, kept in plaintext
    got = PB.flush_builders(builders)
    for (dgrams, packets), twin in zip(got, twins):
        plains, pending, tpackets = twin._close()
        want = _oracle_protect(oracle)(plains, [(len(plains), pending)], None)
        assert [len(d) for d in dgrams] == [len(d) for d in want]
        assert dgrams == want
        assert [p.sent_bytes for p in packets] == [p.sent_bytes for p in tpackets]


@pytest.mark.gpu
def test_flush_builders_two_threads(oracle):
    """Two threads flushing builders at once on the default key tables (one
    per thread): every datagram still equals the oracle's."""
    import threading

    results, errors = {}, []

    def work(tag):
        try:
            for rep in range(3):
                builders, _ = _gpu_case(oracle, n_conn=4, per_conn=30)
                twins, _ = _gpu_case(oracle, n_conn=4, per_conn=30)
                got = PB.flush_builders(builders)
                for (dgrams, _), twin in zip(got, twins):
                    plains, pending, _ = twin._close()
                    if dgrams != _oracle_protect(oracle)(plains, [(len(plains), pending)], None):
                        errors.append((tag, rep))
            results[tag] = True
        except Exception as e:  # noqa: BLE001 - reported below
            errors.append((tag, repr(e)))

    ts = [threading.Thread(target=work, args=(t,)) for t in range(2)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=300)
    assert not errors, errors
    assert results == {0: True, 1: True}


@pytest.mark.gpu
def test_key_slots_release_on_teardown_and_update():
    """CryptoContext.teardown and a key update release the keys a batch table
    holds: the slots are freed, reused, and the table's device
    entries of released slots are cleared (a packet aimed at one reports
    KeyUnavailable), while live keys keep working."""
    from aioquic_amd._crypto import unprotect_host
    from aioquic_amd.batch_io import KeySlots, SendBatch
    from aioquic_amd.crypto import CryptoPair

    def pair(cid):
        p = CryptoPair()
        p.setup_initial(cid, is_client=True, version=QuicProtocolVersion.VERSION_1)
        return p

    slots = KeySlots(8)
    a, b = pair(bytes(8)), pair(bytes([1]) * 8)
    sb = SendBatch(slots)
    hdr = bytes([0x41]) + bytes(8) + bytes(2)
    sb.add(a, hdr, bytes(40), 0)
    sb.add(b, hdr, bytes(40), 0)
    sb.flush()
    assert len(slots._keep) == 2
    a_slot = slots._slot[(id(a.send.aead), id(a.send.hp), 0)]
    a.teardown()
    assert len(slots._keep) == 1 and slots._free == [a_slot]
    # the cleared device entry: unprotect aimed at it finds no key
    desc = np.zeros(1, dtype=L.DESC)
    desc["len"], desc["hdr_len"], desc["slot"] = 40, 9, a_slot
    _, res = unprotect_host(slots.table, desc.tobytes(), bytes(40), 40)
    assert np.frombuffer(res, dtype=L.RESULT)[0]["status"] == L.S_NO_KEY
    # a key update releases the old AEAD; the new one reuses the freed slot
    old = b.send.aead
    b.update_key()
    sb.add(b, bytes([0x45]) + bytes(8) + bytes(2), bytes(40), 1)
    w = sb.flush()
    assert len(w) == 1 and not any(k[0] == id(old) for k in slots._slot)
    assert len(slots._keep) == 1


@pytest.mark.gpu
def test_key_release_from_another_thread_is_queued():
    """A context torn down on another thread does not touch this thread's
    table there and then: the release is queued and applied at the
    table's next assign(), by its own thread."""
    import threading

    from aioquic_amd.batch_io import KeySlots, SendBatch
    from aioquic_amd.crypto import CryptoPair

    p = CryptoPair()
    p.setup_initial(bytes(8), is_client=True, version=QuicProtocolVersion.VERSION_1)
    slots = KeySlots(8)
    sb = SendBatch(slots)
    sb.add(p, bytes([0x41]) + bytes(8) + bytes(2), bytes(40), 0)
    sb.flush()
    assert len(slots._keep) == 1
    t = threading.Thread(target=p.teardown)
    t.start()
    t.join()
    assert len(slots._keep) == 1 and slots._inbox  # queued (recv and send), not applied
    slots.assign([])
    assert len(slots._keep) == 0 and not slots._inbox and not slots._by_obj
    # an owner that stops assigning: close() applies the queue and frees the rest
    p2, q = CryptoPair(), CryptoPair()
    p2.setup_initial(bytes(8), is_client=True, version=QuicProtocolVersion.VERSION_1)
    q.setup_initial(bytes(8), is_client=False, version=QuicProtocolVersion.VERSION_1)
    sb.add(p2, bytes([0x41]) + bytes(8) + bytes(2), bytes(40), 1)
    sb.add(q, bytes([0x41]) + bytes(8) + bytes(2), bytes(40), 0)
    sb.flush()
    assert len(slots._keep) == 2
    t = threading.Thread(target=q.teardown)
    t.start()
    t.join()
    assert slots._inbox
    slots.close()
    assert len(slots._keep) == 0 and not slots._inbox and not slots._by_obj and not slots._slot
