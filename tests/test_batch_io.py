"""GPU parity of the batched callers.

SendBatch.flush() must return exactly what per-packet CryptoPair.encrypt_packet
returns (and what the CPU oracle computes).  ReceiveBatch.run() must reproduce,
packet for packet and in order, the outcomes and the pair/space state changes
of calling CryptoPair.decrypt_packet one packet at a time (quic/crypto.py:184-192,
quic/connection.py:905-985): key-phase rolls, drops, packet-number decoding.
"""

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SUITES = ("AES_128_GCM_SHA256", "AES_256_GCM_SHA384", "CHACHA20_POLY1305_SHA256")


def _pairs(rng, suite_name, version=1):
    """(client, server) pairs sharing 1-RTT secrets, plus twins for the
    sequential per-packet replay."""
    from aioquic_amd.crypto import CryptoPair
    from aioquic_amd.tls import CipherSuite

    cs = CipherSuite[suite_name]
    n = 48 if cs == CipherSuite.AES_256_GCM_SHA384 else 32
    c2s, s2c = rng.bytes(n), rng.bytes(n)
    made = []
    for _ in range(2):
        client, server = CryptoPair(), CryptoPair()
        client.send.setup(cipher_suite=cs, secret=c2s, version=version)
        client.recv.setup(cipher_suite=cs, secret=s2c, version=version)
        server.recv.setup(cipher_suite=cs, secret=c2s, version=version)
        server.send.setup(cipher_suite=cs, secret=s2c, version=version)
        made.append((client, server))
    return made


def _short_header(key_phase, pn, pn_len=2, dcid=b"\x11" * 8):
    first = 0x40 | (key_phase << 2) | (pn_len - 1)
    return bytes([first]) + dcid + (pn & ((1 << (8 * pn_len)) - 1)).to_bytes(pn_len, "big")


def _outcome(fn):
    try:
        return ("ok",) + tuple(fn())
    except Exception as e:  # noqa: BLE001 - compared by type and message
        return (type(e).__name__, str(e))


def test_send_batch_matches_per_packet_and_oracle(oracle):
    from aioquic_amd.batch_io import SendBatch

    rng = np.random.default_rng(21)
    batch = SendBatch(capacity=64)
    expect, plan = [], []
    twins = []
    for suite in SUITES:
        for ver in (1, 0x6B3343CF):
            (cl, _), (cl2, _) = _pairs(rng, suite, ver)
            twins.append((cl, cl2))
    pn = [0] * len(twins)
    for k in range(300):
        j = int(rng.integers(0, len(twins)))
        cl, cl2 = twins[j]
        if rng.random() < 0.02:  # a local key update between packets (crypto.py:194-199)
            cl.update_key()
            cl2.update_key()
        pl = int(rng.choice([4, 5, 20, 300, 1173, 1400]))  # >= 4: the HP sample must exist
        hdr = _short_header(cl.key_phase, pn[j], pn_len=int(rng.integers(1, 5)))
        payload = rng.bytes(pl)
        batch.add(cl, hdr, payload, pn[j])
        expect.append(cl2.encrypt_packet(hdr, payload, pn[j]))
        ctx = cl2.send
        suite, key, iv = ctx.aead._material()
        _, hpk = ctx.hp._material()
        plan.append(oracle.protect(suite, key, iv, hpk, hdr, payload, pn[j]))
        pn[j] += 1
    got = batch.flush()
    assert len(batch) == 0
    assert got == expect
    assert got == plan


def test_send_batch_rejects_like_reference():
    from aioquic_amd._crypto import CryptoError
    from aioquic_amd.batch_io import SendBatch

    rng = np.random.default_rng(2)
    (cl, _), _ = _pairs(rng, "AES_128_GCM_SHA256")
    b = SendBatch(capacity=4)
    b.add(cl, _short_header(0, 1), b"x" * 100, 1)
    b.add(cl, _short_header(0, 2), b"x" * 1474, 2)  # 11 + 1474 + 16 > 1500: overruns the reference
    with pytest.raises(CryptoError, match="Invalid payload length"):
        b.flush()


def _traffic(rng, sender, n, update_at=(), tamper=(), old_phase_at=()):
    """Wire packets from `sender`, with local key updates before the indices in
    update_at; returns [(packet, pn_off)]."""
    out = []
    held = None
    for i in range(n):
        if i in update_at:
            held = sender.send.aead, sender.send.key_phase
            sender.update_key()
        hdr = _short_header(sender.key_phase, i)
        pkt = sender.encrypt_packet(hdr, rng.bytes(int(rng.integers(8, 1200))), i)
        if i in tamper:
            b = bytearray(pkt)
            b[-1] ^= 1
            pkt = bytes(b)
        out.append((pkt, 9))
    return out, held


@pytest.mark.parametrize("suite", SUITES)
def test_receive_batch_matches_sequential(suite):
    from aioquic_amd.batch_io import ReceiveBatch

    rng = np.random.default_rng(31)
    (cl, sv), (cl2, sv2) = _pairs(rng, suite)
    pkts, _ = _traffic(rng, cl, 120, update_at={40, 90}, tamper={5, 41, 77})
    # same traffic for the twin sender is not needed: the receiver twin replays
    # the same wire bytes one packet at a time
    batch = ReceiveBatch(capacity=16)

    class Space:
        expected_packet_number = 0

    sp, sp2 = Space(), Space()
    for pkt, off in pkts:
        batch.add(sv, pkt, off, space=sp)
    got = [(("ok",) + tuple(o)) if isinstance(o, tuple) else (type(o).__name__, str(o))
           for o in batch.run()]
    want = []
    for pkt, off in pkts:
        o = _outcome(lambda: sv2.decrypt_packet(pkt, off, sp2.expected_packet_number))
        if o[0] == "ok" and o[3] > sp2.expected_packet_number:
            sp2.expected_packet_number = o[3] + 1
        want.append(o)
    assert got == want
    assert sp.expected_packet_number == sp2.expected_packet_number
    assert sv.key_phase == sv2.key_phase == 0  # two updates: back to phase 0
    assert sv.recv.secret == sv2.recv.secret and sv.send.secret == sv2.send.secret
    assert sum(o[0] == "ok" for o in got) == 117
    assert batch.launches >= 3  # one per key roll at least


def test_receive_batch_old_phase_after_roll_and_no_key():
    """A reordered old-phase packet after a roll fails exactly as in the
    sequential path; a pair without receive keys yields KeyUnavailableError."""
    from aioquic_amd.batch_io import ReceiveBatch
    from aioquic_amd.crypto import CryptoPair

    rng = np.random.default_rng(41)
    (cl, sv), (_, sv2) = _pairs(rng, "AES_128_GCM_SHA256")
    pkts, _ = _traffic(rng, cl, 12, update_at={6})
    order = list(range(12))
    order[6], order[8] = order[8], order[6]
    order.insert(9, 3)  # a duplicate of an old-phase packet after the roll
    nokey = CryptoPair()
    batch = ReceiveBatch(capacity=8)
    for i in order:
        batch.add(sv, pkts[i][0], 9, expected_packet_number=i)
    batch.add(nokey, pkts[0][0], 9, expected_packet_number=0)
    got = [(("ok",) + tuple(o)) if isinstance(o, tuple) else (type(o).__name__, str(o))
           for o in batch.run()]
    want = [_outcome(lambda i=i: sv2.decrypt_packet(pkts[i][0], 9, i)) for i in order]
    want.append(_outcome(lambda: CryptoPair().decrypt_packet(pkts[0][0], 9, 0)))
    assert got == want
    assert got[-1] == ("KeyUnavailableError", "Decryption key is not available")


def test_receive_batch_many_connections():
    """Hundreds of connections in one batch: one launch when no key rolls."""
    from aioquic_amd.batch_io import ReceiveBatch, SendBatch

    rng = np.random.default_rng(51)
    conns = [_pairs(rng, SUITES[i % 3])[0] for i in range(200)]
    sb = SendBatch(capacity=512)
    meta = []
    for k, (cl, sv) in enumerate(conns):
        for pn in range(3):
            hdr = _short_header(0, pn, pn_len=1 + (k % 4))
            payload = rng.bytes(int(rng.integers(4, 1173)))
            sb.add(cl, hdr, payload, pn)
            meta.append((sv, 9, pn, hdr, payload))
    wires = sb.flush()
    rb = ReceiveBatch(capacity=512)
    for (sv, off, pn, _, _), w in zip(meta, wires):
        rb.add(sv, w, off, expected_packet_number=pn)
    got = rb.run()
    assert rb.launches == 1
    for (sv, off, pn, hdr, payload), o in zip(meta, got):
        assert o == (hdr, payload, pn)


@pytest.mark.parametrize("suite", SUITES)
def test_receive_batch_one_byte_pns_past_the_window(suite):
    """More than 256 packets of one connection with 1-byte packet numbers: a
    packet decoded under the batch's starting expected number would get the
    wrong packet number (pn 256 decodes as 0), fail authentication and be
    dropped, though the sequential decrypt_packet accepts it once earlier
    packets have advanced expected_packet_number (batch_io.py)."""
    from aioquic_amd.batch_io import ReceiveBatch

    rng = np.random.default_rng(61)
    (cl, sv), (_, sv2) = _pairs(rng, suite)
    pkts = []
    for pn in range(300):
        hdr = _short_header(0, pn, pn_len=1)
        pkts.append(cl.encrypt_packet(hdr, rng.bytes(int(rng.integers(8, 200))), pn))
    b = bytearray(pkts[200])
    b[-1] ^= 1
    pkts[200] = bytes(b)

    class Space:
        expected_packet_number = 0

    sp, sp2 = Space(), Space()
    batch = ReceiveBatch(capacity=8)
    for pkt in pkts:
        batch.add(sv, pkt, 9, space=sp)
    got = [(("ok",) + tuple(o)) if isinstance(o, tuple) else (type(o).__name__, str(o))
           for o in batch.run()]
    want = []
    for pkt in pkts:
        o = _outcome(lambda: sv2.decrypt_packet(pkt, 9, sp2.expected_packet_number))
        if o[0] == "ok" and o[3] > sp2.expected_packet_number:
            sp2.expected_packet_number = o[3] + 1
        want.append(o)
    assert got == want
    assert sum(o[0] == "ok" for o in got) == 299
    assert sp.expected_packet_number == sp2.expected_packet_number == 300
