"""Whole-batch checker built on the reference's own per-packet path.

oracle/_ref/aioquic_ref/_crypto*.so is /root/reference/src/aioquic/_crypto.c
compiled by `make -C oracle ref` against the system libcrypto (never part of
the package; it travels to the GPU box as a built file, the reference source
does not).  Test infrastructure only: the packets of a bench_data workload go
through AEAD.encrypt + HeaderProtection.apply and HeaderProtection.remove +
decode_packet_number + AEAD.decrypt one by one, exactly as
quic/crypto.py:75-116 drives them, at ~1-3 us per packet, so a 1 Mi batch is
checked whole in seconds where the plain-C restatement (oracle/qpp_oracle.c,
bitwise GHASH) would take minutes.
"""

import glob
import importlib.util
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
_NAMES = {0: (b"aes-128-gcm", b"aes-128-ecb", 16), 1: (b"aes-256-gcm", b"aes-256-ecb", 32),
          2: (b"chacha20-poly1305", b"chacha20", 32)}


# Written by `make -C oracle ref` (build(), in the build container where
# /root/reference exists) beside oracle/_ref/: it travels with the tree, so a
# GPU box that got the marker but not the library fails the whole-batch tests
# instead of silently checking them against the C oracle's small sample.
EXPECTED = os.path.join(ROOT, "oracle", "_ref_expected")

# (test id, checker) of every whole-batch check this session; conftest.py
# prints them in the terminal summary, so a -q log states which checker ran
USED = []


def load():
    """The reference's _crypto module, or None when oracle/_ref is not built."""
    so = glob.glob(os.path.join(ROOT, "oracle", "_ref", "aioquic_ref", "_crypto*.so"))
    if not so:
        return None
    spec = importlib.util.spec_from_file_location("_crypto", so[0])
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def checker(test_id: str):
    """The whole-batch checker for one test: the reference's _crypto when it
    is built, else None (the caller's C-oracle sample).  Fails when the build
    container built oracle/_ref (the marker is here) but the library is not,
    and records which checker ran."""
    ref = load()
    if ref is None and os.path.exists(EXPECTED):
        raise AssertionError(
            "oracle/_ref was built from /root/reference (oracle/_ref_expected) but is missing here: "
            "the whole-batch parity check would downgrade to the C oracle's sample")
    USED.append((test_id, "reference _crypto (oracle/_ref), every packet both directions" if ref is not None
                 else "C oracle (oracle/qpp_oracle.c), sample only: oracle/_ref not built"))
    return ref


def _objects(ref, keys):
    objs = []
    for k in keys:
        an, hn, kl = _NAMES[int(k["suite"])]
        objs.append((ref.AEAD(an, bytes(k["key"][:kl]), bytes(k["iv"])),
                     ref.HeaderProtection(hn, bytes(k["hp"][:kl]))))
    return objs


def protect_all(ref, w) -> np.ndarray:
    """The wire image of every packet of workload w (bench_data layout:
    dense 1200-byte slots, header at in_off, payload after it)."""
    objs = _objects(ref, w.keys)
    out = bytearray(w.wire_size)
    buf = w.plain.tobytes()
    d = w.desc
    for i, o, h, n, slot, pn in zip(d["in_off"].tolist(), d["out_off"].tolist(), d["hdr_len"].tolist(),
                                    d["len"].tolist(), d["slot"].tolist(), d["pn"].tolist()):
        aead, hp = objs[slot]
        hdr = buf[i : i + h]
        pkt = hp.apply(hdr, aead.encrypt(buf[i + h : i + h + n], hdr, pn))
        out[o : o + len(pkt)] = pkt
    return np.frombuffer(out, np.uint8)


def unprotect_all(ref, w, wire: np.ndarray):
    """(plaintext image, decoded packet numbers) of every packet of w's wire
    image; a failed packet raises (the batch is expected to authenticate)."""
    from aioquic_amd.packet import decode_packet_number

    objs = _objects(ref, w.keys)
    out = bytearray(w.plain_size)
    pns = []
    buf = wire.tobytes()
    d = w.udesc
    for i, o, n, pn_off, slot, exp in zip(d["in_off"].tolist(), d["out_off"].tolist(), d["len"].tolist(),
                                          d["hdr_len"].tolist(), d["slot"].tolist(), d["pn"].tolist()):
        aead, hp = objs[slot]
        hdr, trunc = hp.remove(buf[i : i + n], pn_off)
        pn = decode_packet_number(trunc, ((hdr[0] & 3) + 1) * 8, exp)
        pt = aead.decrypt(buf[i + len(hdr) : i + n], hdr, pn)
        h = len(hdr)
        out[o : o + h] = hdr
        out[o + h : o + h + len(pt)] = pt
        pns.append(pn)
    return np.frombuffer(out, np.uint8), np.array(pns, np.uint64)
