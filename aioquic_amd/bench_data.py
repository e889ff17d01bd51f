"""Synthetic workloads of BASELINE.json / SURVEY.md sec. 8(d).

Packet = 1-RTT short header 0x41 | DCID(8, fixed) | PN16(pn) (11 B, the shape
QuicPacketBuilder emits: packet_builder.py:19-20,230), plaintext 1173 B from a
seeded PRNG, 16 B tag -> 1200 B on the wire (test_packet_builder.py:490-522).
Secrets are seeded random 32 B (48 B for AES-256) expanded with
derive_key_iv_hp semantics.  Packets are laid out one per 1200-byte slot;
descriptors are grouped by key slot, which is how the engine's host side
buckets a multi-connection batch before launch.
"""

from __future__ import annotations

from dataclasses import dataclass

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


def make_keys(n_keys: int, suites, seed: int, version: int) -> np.ndarray:
    rng = np.random.default_rng(seed)
    recs = np.zeros(n_keys, dtype=L.KEY_MATERIAL)
    for s in range(n_keys):
        suite = int(suites[s % len(suites)])
        secret = rng.bytes(48 if suite == L.AES_256_GCM else 32)
        key, iv, hp = derive_key_iv_hp(cipher_suite=_SUITE_TO_CS[suite], secret=secret,
                                       version=version)
        recs[s]["slot"] = s
        recs[s]["suite"] = suite
        recs[s]["iv"] = np.frombuffer(iv, np.uint8)
        recs[s]["key"][: len(key)] = np.frombuffer(key, np.uint8)
        recs[s]["hp"][: len(hp)] = np.frombuffer(hp, np.uint8)
    return recs


def make_workload(n: int, suite=L.AES_128_GCM, n_keys: int = 1, seed: int = 0x9001,
                  version: int = QuicProtocolVersion.VERSION_1, mixed=None,
                  first_packet: int = 0) -> Workload:
    """n packets; `mixed` = list of suites assigned to keys round-robin
    (config 5), else every key uses `suite`."""
    suites = list(mixed) if mixed else [suite]
    keys = make_keys(n_keys, suites, seed, int(version))
    rng = np.random.default_rng(seed + 1)
    idx = np.arange(first_packet, first_packet + n, dtype=np.int64)
    key_of = (idx % n_keys).astype(np.uint32)
    pn = (idx // n_keys).astype(np.uint64)
    # group by key slot (stable), as the host side of the engine does
    order = np.argsort(key_of, kind="stable")
    key_of, pn = key_of[order], pn[order]

    plain = np.zeros(n * SLOT_BYTES, dtype=np.uint8)
    view = plain.reshape(n, SLOT_BYTES)
    view[:, 0] = 0x41
    view[:, 1:9] = np.frombuffer(DCID, np.uint8)
    view[:, 9] = ((pn >> 8) & 0xFF).astype(np.uint8)
    view[:, 10] = (pn & 0xFF).astype(np.uint8)
    view[:, HDR_LEN : HDR_LEN + PAYLOAD_LEN] = rng.integers(0, 256, size=(n, PAYLOAD_LEN),
                                                            dtype=np.uint8)

    offs = np.arange(n, dtype=np.uint64) * SLOT_BYTES
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
                    plain_size=n * SLOT_BYTES, wire_size=n * SLOT_BYTES,
                    suites=keys["suite"][key_of])
