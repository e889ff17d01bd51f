"""Generate tests/golden/golden_vectors.json from the REFERENCE itself.

The reference's per-packet path (aioquic src/aioquic/_crypto.c) is compiled
from /root/reference by ``make -C oracle ref`` into oracle/_ref/ and loaded here
as a module.  The packet-level glue mirrors aioquic src/aioquic/quic/crypto.py
(CryptoContext.encrypt_packet :105-116, decrypt_packet :75-103,
derive_key_iv_hp :34-56, next_key_phase :157-168) and quic/packet.py
decode_packet_number :118-132, restated with stdlib hmac/hashlib because the
reference's tls.py needs the absent `cryptography` package.

Inputs are derived deterministically from a per-case seed with ``gen_bytes``
(SHA-256 in counter mode, reproduced by tests/golden_cases.py), so the fixture
only stores seeds, sizes and the reference's outputs (full hex when short,
SHA-256 otherwise).  Run in the build container:
    make -C oracle ref && python tests/golden/make_golden.py
"""

import glob
import hashlib
import hmac
import importlib.util
import json
import os
import struct
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "tests"))

from golden_cases import (  # noqa: E402
    AEAD_NAMES,
    HP_NAMES,
    build_cases,
    gen_bytes,
)


def load_ref():
    so = glob.glob(os.path.join(ROOT, "oracle", "_ref", "aioquic_ref", "_crypto*.so"))
    if not so:
        raise SystemExit("build the reference first: make -C oracle ref")
    spec = importlib.util.spec_from_file_location("_crypto", so[0])
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


REF = load_ref()


def _hash(suite):
    return hashlib.sha384 if suite == 1 else hashlib.sha256


def hkdf_expand_label(h, secret, label, ctx, length):
    full = b"tls13 " + label
    info = struct.pack("!HB", length, len(full)) + full + struct.pack("!B", len(ctx)) + ctx
    out, t, i = b"", b"", 1
    while len(out) < length:
        t = hmac.new(secret, t + info + bytes([i]), h).digest()
        out += t
        i += 1
    return out[:length]


def derive(suite, secret, version):
    h = _hash(suite)
    ks = 16 if suite == 0 else 32
    p = b"quicv2 " if version == 0x6B3343CF else b"quic "
    return (hkdf_expand_label(h, secret, p + b"key", b"", ks),
            hkdf_expand_label(h, secret, p + b"iv", b"", 12),
            hkdf_expand_label(h, secret, p + b"hp", b"", ks))


def next_secret(suite, secret):
    h = _hash(suite)
    return hkdf_expand_label(h, secret, b"quic ku", b"", h().digest_size)


def decode_packet_number(truncated, num_bits, expected):
    window = 1 << num_bits
    half_window = window // 2
    candidate = (expected & ~(window - 1)) | truncated
    if candidate <= expected - half_window and candidate < (1 << 62) - window:
        return candidate + window
    elif candidate > expected + half_window and candidate >= window:
        return candidate - window
    return candidate


def out_field(b: bytes):
    return {"hex": b.hex()} if len(b) <= 96 else {"sha256": hashlib.sha256(b).hexdigest(),
                                                 "len": len(b)}


def run_case(c):
    suite, version = c["suite"], c["version"]
    secret = gen_bytes(c["seed"] + ":secret", 48 if suite == 1 else 32)
    key, iv, hp = derive(suite, secret, version)
    aead = REF.AEAD(AEAD_NAMES[suite], key, iv)
    hpo = REF.HeaderProtection(HP_NAMES[suite], hp)
    hdr = bytes.fromhex(c["header"])
    payload = gen_bytes(c["seed"] + ":payload", c["payload_len"])
    res = {}
    # protect == CryptoContext.encrypt_packet; a sender in the next key phase
    # uses next_key_phase's AEAD but keeps the HP key (crypto.py:148-154)
    send = aead
    if c.get("send_phase"):
        k2, iv2, _ = derive(suite, next_secret(suite, secret), version)
        send = REF.AEAD(AEAD_NAMES[suite], k2, iv2)
    pkt = hpo.apply(hdr, send.encrypt(payload, hdr, c["pn"]))
    res["protected"] = out_field(pkt)
    # unprotect of the (possibly tampered) packet == CryptoContext.decrypt_packet
    wire = bytearray(pkt)
    for pos, bit in c.get("tamper", []):
        wire[pos] ^= 1 << bit
    wire = bytes(wire)
    pn_off = c["pn_off"]
    try:
        plain_header, trunc = hpo.remove(wire, pn_off)
        first = plain_header[0]
        pn_len = (first & 3) + 1
        pn = decode_packet_number(trunc, pn_len * 8, c["expected_pn"])
        use = aead
        phase_flip = False
        if not (first & 0x80) and ((first & 4) >> 2) != c["key_phase"]:
            k2, iv2, _ = derive(suite, next_secret(suite, secret), version)
            use = REF.AEAD(AEAD_NAMES[suite], k2, iv2)
            phase_flip = True
        body = use.decrypt(wire[len(plain_header):], plain_header, pn)
        res["unprotect"] = {"ok": True, "header": plain_header.hex(), "pn": pn,
                            "phase_flip": phase_flip, "pn_trunc": trunc,
                            "payload": out_field(body)}
    except REF.CryptoError as e:
        res["unprotect"] = {"ok": False, "error": str(e)}
    return res


def main():
    cases = build_cases()
    out = []
    for c in cases:
        r = dict(c)
        r.update(run_case(c))
        out.append(r)
    path = os.path.join(HERE, "golden_vectors.json")
    with open(path, "w") as f:
        json.dump({"generator": "tests/golden/make_golden.py", "reference": "aioquic _crypto.c compiled from /root/reference, "
                   + os.popen("openssl version").read().strip(),
                   "cases": out}, f, separators=(",", ":"))
    print("wrote", path, len(out), "cases", os.path.getsize(path), "bytes")


if __name__ == "__main__":
    main()
