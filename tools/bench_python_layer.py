#!/usr/bin/env python3
"""Packet protection through the Python layer:
per-call latency of the reference-shaped objects and batch throughput of the
callers, on a GPU box.  Prints one JSON object.

  latency_us   AEAD.encrypt / decrypt (1173 B payload, 11 B header),
               HeaderProtection.apply / remove, CryptoContext.encrypt_packet /
               decrypt_packet -- each a device round trip per call (the
               reference's CPU figures: 1.64 us encrypt_packet, 2.23 us
               decrypt_packet)
  send / recv  SendBatch / ReceiveBatch of N packets over C connections:
               add() loop and flush()/run() timed apart, packets/s overall
  builder      N packets through QuicPacketBuilder (frames written by the
               caller) + flush_builders (one launch), then receive_datagrams
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np


sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _lat(fn, reps):
    for _ in range(20):
        fn()
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    return (time.perf_counter() - t) / reps * 1e6


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--packets", type=int, default=65536)
    ap.add_argument("--conns", type=int, default=64)
    ap.add_argument("--reps", type=int, default=2000)
    ap.add_argument("--profile", action="store_true", help="cProfile of one receive + flush to stderr")
    a = ap.parse_args()

    from aioquic_amd._crypto import AEAD, HeaderProtection
    from aioquic_amd.batch_io import ReceiveBatch, SendBatch
    from aioquic_amd.crypto import CryptoPair
    from aioquic_amd import packet_builder as PB
    from aioquic_amd import receive as R
    from aioquic_amd.packet import QuicFrameType, QuicPacketType, QuicProtocolVersion
    from aioquic_amd.tls import Epoch

    rng = np.random.default_rng(7)
    out = {"packets": a.packets, "connections": a.conns}
    hdr = bytes([0x41]) + bytes(8) + b"\x00\x01"
    payload = rng.bytes(1173)

    # ------------------------------------------------ per-call latency
    lat = {}
    for name, klen in ((b"aes-128-gcm", 16), (b"chacha20-poly1305", 32)):
        aead = AEAD(name, rng.bytes(klen), rng.bytes(12))
        ct = aead.encrypt(payload, hdr, 1)
        lat[f"{name.decode()}.encrypt"] = _lat(lambda: aead.encrypt(payload, hdr, 1), a.reps)
        lat[f"{name.decode()}.decrypt"] = _lat(lambda: aead.decrypt(ct, hdr, 1), a.reps)
    hp = HeaderProtection(b"aes-128-ecb", rng.bytes(16))
    prot = hp.apply(hdr, payload + bytes(16))
    lat["hp.apply"] = _lat(lambda: hp.apply(hdr, payload + bytes(16)), a.reps)
    lat["hp.remove"] = _lat(lambda: hp.remove(prot, 9), a.reps)
    client, server = CryptoPair(), CryptoPair()
    client.setup_initial(bytes(8), is_client=True, version=QuicProtocolVersion.VERSION_1)
    server.setup_initial(bytes(8), is_client=False, version=QuicProtocolVersion.VERSION_1)
    wire = client.send.encrypt_packet(hdr, payload, 1)
    lat["CryptoContext.encrypt_packet"] = _lat(lambda: client.send.encrypt_packet(hdr, payload, 1), a.reps)
    lat["CryptoContext.decrypt_packet"] = _lat(lambda: server.recv.decrypt_packet(wire, 9, 1), a.reps)
    out["latency_us"] = {k: round(v, 2) for k, v in lat.items()}
    out["reference_cpu_us"] = {"CryptoContext.encrypt_packet": 1.64, "CryptoContext.decrypt_packet": 2.23}

    # ------------------------------------------------ batch throughput
    pairs = []
    for c in range(a.conns):
        cl, sv = CryptoPair(), CryptoPair()
        cid = int(c).to_bytes(8, "big")
        cl.setup_initial(cid, is_client=True, version=QuicProtocolVersion.VERSION_1)
        sv.setup_initial(cid, is_client=False, version=QuicProtocolVersion.VERSION_1)
        pairs.append((cl, sv))
    n = a.packets
    conn_of = np.arange(n) % a.conns
    pns = np.arange(n) // a.conns
    payloads = [payload] * n
    sb = SendBatch(capacity=2 * a.conns + 8)
    sb.flush() if len(sb) else None
    for rnd in range(2):  # first round warms up
        t0 = time.perf_counter()
        for i in range(n):
            sb.add(pairs[conn_of[i]][0], hdr[:9] + int(pns[i] & 0xFFFF).to_bytes(2, "big"), payloads[i], int(pns[i]))
        t1 = time.perf_counter()
        wires = sb.flush()
        t2 = time.perf_counter()
    out["send"] = {"add_s": round(t1 - t0, 4), "flush_s": round(t2 - t1, 4),
                   "packets_per_s": round(n / (t2 - t0)), "flush_packets_per_s": round(n / (t2 - t1))}
    rb = ReceiveBatch(capacity=2 * a.conns + 8)
    for rnd in range(2):
        t0 = time.perf_counter()
        for i in range(n):
            rb.add(pairs[conn_of[i]][1], wires[i], 9, expected_packet_number=int(pns[i]))
        t1 = time.perf_counter()
        res = rb.run()
        t2 = time.perf_counter()
    assert all(isinstance(r, tuple) for r in res)
    out["recv"] = {"add_s": round(t1 - t0, 4), "run_s": round(t2 - t1, 4),
                   "packets_per_s": round(n / (t2 - t0)), "run_packets_per_s": round(n / (t2 - t1))}

    # ------------------------------------------------ builder + receive
    per = n // a.conns
    body = rng.bytes(1200)
    for rnd in range(2):
        t0 = time.perf_counter()
        builders = []
        for c in range(a.conns):
            b = PB.QuicPacketBuilder(host_cid=bytes(8), peer_cid=bytes(8), version=QuicProtocolVersion.VERSION_1,
                                     is_client=True, max_datagram_size=1200)
            for _ in range(per):
                b.start_packet(QuicPacketType.ONE_RTT, pairs[c][0])
                b.start_frame(QuicFrameType.STREAM_BASE).push_bytes(body[: b.remaining_flight_space])
            builders.append(b)
        t1 = time.perf_counter()
        flushed = PB.flush_builders(builders)
        t2 = time.perf_counter()
    n_dg = sum(len(d) for d, _ in flushed)
    out["builder"] = {"datagrams": n_dg, "build_s": round(t1 - t0, 4), "flush_s": round(t2 - t1, 4),
                      "packets_per_s": round(n_dg / (t2 - t0)), "flush_packets_per_s": round(n_dg / (t2 - t1))}

    class _S:
        expected_packet_number = 0

    conns = [R.ConnectionKeys(cryptos={e: sv for e in Epoch}, spaces={e: _S() for e in Epoch})
             for _, sv in pairs]
    items = [(conns[c], d) for c, (dg, _) in enumerate(flushed) for d in dg]
    # arrival order of a server socket: the connections interleaved
    mixed = [items[i] for i in np.random.default_rng(11).permutation(len(items))]
    times = {}
    for name, its in (("in_order", items), ("interleaved", mixed)):
        ts = []
        for rnd in range(3):
            for sp in conns:  # a fresh batch of the same traffic each round
                for e in Epoch:
                    sp.spaces[e] = _S()
            t0 = time.perf_counter()
            got = R.receive_datagrams(its)
            ts.append(time.perf_counter() - t0)
            assert all(p.ok for p in got), {p.dropped for p in got}
        times[name] = float(np.median(ts))
    out["receive_datagrams"] = {"s": round(times["in_order"], 4),
                                "packets_per_s": round(len(items) / times["in_order"]),
                                "interleaved_packets_per_s": round(len(items) / times["interleaved"]),
                                "note": "median of 3 rounds, fresh packet-number spaces each round"}
    if a.profile:
        import cProfile
        import pstats

        pr = cProfile.Profile()
        pr.enable()
        R.receive_datagrams(mixed)
        PB.flush_builders(builders)
        pr.disable()
        pstats.Stats(pr, stream=sys.stderr).sort_stats("cumulative").print_stats(18)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
