"""Synthetic workloads of BASELINE.json / SURVEY.md sec. 8(d).

Packet = 1-RTT short header 0x41 | DCID(8, fixed) | PN16(pn) (11 B, the shape
QuicPacketBuilder emits: packet_builder.py:19-20,230), plaintext 1173 B from a
seeded PRNG, 16 B tag -> 1200 B on the wire (test_packet_builder.py:490-522).
Secrets are seeded random 32 B (48 B for AES-256) expanded with
derive_key_iv_hp semantics.  Packets are laid out one per 1200-byte slot in
arrival order.  Arrival order is one of
  "grouped"      packets of one key contiguous (a single connection's burst),
  "round_robin"  packet i on key i mod n_keys,
  "random"       every packet on a seeded random key -- what a server socket
                 sees when many connections send at once
                 (src/aioquic/asyncio/server.py:60-152); the engine buckets it
                 by (suite, key) on the device (qpp_plan) before launch.
Packet numbers count up per key in arrival order.
"""

from __future__ import annotations

from dataclasses import dataclass

import os

import numpy as np

from . import layout as L
from .crypto import derive_key_iv_hp
from .packet import QuicProtocolVersion
from .tls import CipherSuite

SLOT_BYTES = 1200
HDR_LEN = 11
PAYLOAD_LEN = 1173
PN_OFF = 9
DCID = bytes.fromhex("8394c8f03e515708")

_SUITE_TO_CS = {
    L.AES_128_GCM: CipherSuite.AES_128_GCM_SHA256,
    L.AES_256_GCM: CipherSuite.AES_256_GCM_SHA384,
    L.CHACHA20_POLY1305: CipherSuite.CHACHA20_POLY1305_SHA256,
}


@dataclass
class Workload:
    n: int
    n_keys: int
    keys: np.ndarray      # KEY_MATERIAL records
    desc: np.ndarray      # protect descriptors
    udesc: np.ndarray     # unprotect descriptors (expected pn = pn)
    plain: np.ndarray     # uint8 [n * 1200]: header | payload | 16 spare per slot
    plain_size: int
    wire_size: int
    suites: np.ndarray    # suite per packet


def make_keys(n_keys: int, suites, seed: int, version: int, random_suites: bool = False) -> np.ndarray:
    """Key slots 0..n_keys-1; suite of slot s = suites[s % len] or, with
    random_suites, a seeded uniform pick among `suites`."""
    rng = np.random.default_rng(seed)
    pick = np.random.default_rng(seed ^ 0x5EED).integers(0, len(suites), n_keys)
    recs = np.zeros(n_keys, dtype=L.KEY_MATERIAL)
    for s in range(n_keys):
        suite = int(suites[pick[s]] if random_suites else suites[s % len(suites)])
        secret = rng.bytes(48 if suite == L.AES_256_GCM else 32)
        key, iv, hp = derive_key_iv_hp(cipher_suite=_SUITE_TO_CS[suite], secret=secret,
                                       version=version)
        recs[s]["slot"] = s
        recs[s]["suite"] = suite
        recs[s]["iv"] = np.frombuffer(iv, np.uint8)
        recs[s]["key"][: len(key)] = np.frombuffer(key, np.uint8)
        recs[s]["hp"][: len(hp)] = np.frombuffer(hp, np.uint8)
    return recs


def _per_key_counter(key_of: np.ndarray, n_keys: int) -> np.ndarray:
    """pn[i] = number of earlier packets on the same key (arrival order)."""
    order = np.argsort(key_of, kind="stable")
    counts = np.bincount(key_of, minlength=n_keys)
    starts = np.concatenate([[0], np.cumsum(counts)[:-1]])
    rank = np.empty(len(key_of), np.int64)
    rank[order] = np.arange(len(key_of)) - np.repeat(starts, counts)
    return rank.astype(np.uint64)


def make_workload(n: int, suite=L.AES_128_GCM, n_keys: int = 1, seed: int = 0x9001,
                  version: int = QuicProtocolVersion.VERSION_1, mixed=None,
                  first_packet: int = 0, order: str = "grouped",
                  layout: str = "arrival") -> Workload:
    """n packets; `mixed` = list of suites (config 5): keys get a seeded
    random suite from it with order="random", else round-robin; without
    `mixed` every key uses `suite`.  `first_packet` offsets a rank's shard
    in the global stream.  layout="by_key" stores the packets of one key
    contiguously in memory whatever the arrival order (a study knob: it
    separates the cost of scattered memory from the cost of bucketing)."""
    suites = list(mixed) if mixed else [suite]
    keys = make_keys(n_keys, suites, seed, int(version), random_suites=order == "random")
    rng = np.random.default_rng(seed + 1)
    idx = np.arange(first_packet, first_packet + n, dtype=np.int64)
    if order == "random":
        # the global stream's key sequence, sliced for this shard
        krng = np.random.default_rng(seed + 2)
        key_of = krng.integers(0, n_keys, first_packet + n).astype(np.uint32)
        pn = _per_key_counter(key_of, n_keys)[first_packet:]
        key_of = key_of[first_packet:]
    else:
        key_of = (idx % n_keys).astype(np.uint32)
        pn = (idx // n_keys).astype(np.uint64)
        if order == "grouped":
            o = np.argsort(key_of, kind="stable")
            key_of, pn = key_of[o], pn[o]
        elif order != "round_robin":
            raise ValueError(f"unknown order {order!r}")

    # layout study only (QPP_BENCH_SHIFT=k): the whole batch starts k bytes
    # into its buffers, e.g. 5 puts every payload on a 16-byte boundary
    shift = int(os.environ.get("QPP_BENCH_SHIFT", "0"))
    plain = np.zeros(n * SLOT_BYTES + shift, dtype=np.uint8)
    view = plain[shift:].reshape(n, SLOT_BYTES)
    view[:, 0] = 0x41
    view[:, 1:9] = np.frombuffer(DCID, np.uint8)
    view[:, 9] = ((pn >> 8) & 0xFF).astype(np.uint8)
    view[:, 10] = (pn & 0xFF).astype(np.uint8)
    view[:, HDR_LEN : HDR_LEN + PAYLOAD_LEN] = rng.integers(0, 256, size=(n, PAYLOAD_LEN),
                                                            dtype=np.uint8)

    if layout == "by_key":
        pos = np.empty(n, np.int64)
        pos[np.argsort(key_of, kind="stable")] = np.arange(n)
        offs = pos.astype(np.uint64) * SLOT_BYTES
        view[pos] = view.copy()
    elif layout == "arrival":
        offs = np.arange(n, dtype=np.uint64) * SLOT_BYTES
    else:
        raise ValueError(f"unknown layout {layout!r}")
    offs = offs + np.uint64(shift)
    desc = np.zeros(n, dtype=L.DESC)
    desc["in_off"] = offs
    desc["out_off"] = offs
    desc["len"] = PAYLOAD_LEN
    desc["hdr_len"] = HDR_LEN
    desc["pn"] = pn
    desc["slot"] = key_of
    udesc = desc.copy()
    udesc["len"] = SLOT_BYTES
    udesc["hdr_len"] = PN_OFF
    return Workload(n=n, n_keys=n_keys, keys=keys, desc=desc, udesc=udesc, plain=plain,
                    plain_size=n * SLOT_BYTES + shift, wire_size=n * SLOT_BYTES + shift,
                    suites=keys["suite"][key_of])
