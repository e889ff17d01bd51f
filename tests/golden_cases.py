"""Deterministic case list shared by tests/golden/make_golden.py (which runs the
reference on it) and the parity tests (which rebuild the same inputs).

Inputs come from ``gen_bytes`` (SHA-256 counter mode), so the fixture stores
seeds, not payloads.
"""

import hashlib
import random

AEAD_NAMES = {0: b"aes-128-gcm", 1: b"aes-256-gcm", 2: b"chacha20-poly1305"}
HP_NAMES = {0: b"aes-128-ecb", 1: b"aes-256-ecb", 2: b"chacha20"}
VERSION_1, VERSION_2 = 0x00000001, 0x6B3343CF


def gen_bytes(seed: str, n: int) -> bytes:
    out = bytearray()
    i = 0
    while len(out) < n:
        out += hashlib.sha256(f"{seed}/{i}".encode()).digest()
        i += 1
    return bytes(out[:n])


def _varint(v: int) -> bytes:
    if v < 0x40:
        return bytes([v])
    if v < 0x4000:
        return (v | 0x4000).to_bytes(2, "big")
    return (v | 0x80000000).to_bytes(4, "big")


def short_header(dcid: bytes, pn: int, pn_len: int, key_phase: int, spin: int = 0) -> bytes:
    first = 0x40 | (spin << 5) | (key_phase << 2) | (pn_len - 1)
    return bytes([first]) + dcid + (pn & ((1 << (8 * pn_len)) - 1)).to_bytes(pn_len, "big")


def long_header(version: int, dcid: bytes, scid: bytes, token: bytes, pn: int, pn_len: int,
                rest_len: int) -> bytes:
    """Initial packet header; rest_len = payload + tag length (for the Length field)."""
    first = 0xC0 | (pn_len - 1)
    return (bytes([first]) + version.to_bytes(4, "big") + bytes([len(dcid)]) + dcid +
            bytes([len(scid)]) + scid + _varint(len(token)) + token +
            (rest_len + pn_len | 0x4000).to_bytes(2, "big") +
            (pn & ((1 << (8 * pn_len)) - 1)).to_bytes(pn_len, "big"))


PAYLOAD_LENS = [1, 3, 4, 15, 16, 17, 31, 32, 33, 47, 63, 64, 65, 100, 255, 256, 1000, 1173,
                1184, 1232, 1440]


def build_cases():
    rnd = random.Random(0x9001)
    cases = []
    for suite in (0, 1, 2):
        for version in (VERSION_1, VERSION_2):
            for j, plen in enumerate(PAYLOAD_LENS):
                pn_len = 1 + (j % 4)
                long = j % 3 == 2
                pn = rnd.choice([0, 1, 2, 255, 256, 65535, 1 << 20, rnd.randrange(1 << 30),
                                 rnd.randrange(1 << 62)])
                seed = f"s{suite}-v{version:x}-{j}"
                if long:
                    dcid = gen_bytes(seed + ":dcid", rnd.choice([0, 8, 20]))
                    scid = gen_bytes(seed + ":scid", rnd.choice([0, 8]))
                    token = gen_bytes(seed + ":tok", rnd.choice([0, 5, 40]))
                    hdr = long_header(version, dcid, scid, token, pn, pn_len, plen + 16)
                else:
                    dcid = gen_bytes(seed + ":dcid", rnd.choice([0, 4, 8, 20]))
                    hdr = short_header(dcid, pn, pn_len, 0, spin=j & 1)
                if len(hdr) + plen + 16 > 1500 or plen + 16 < 20 - pn_len:
                    plen = min(plen, 1484 - len(hdr))
                    plen = max(plen, 4 - pn_len)
                # expected pn within the decodable window of pn
                win = 1 << (8 * pn_len)
                exp = max(0, pn + rnd.randrange(-(win // 2) + 1, win // 2))
                cases.append(dict(seed=seed, suite=suite, version=version, header=hdr.hex(),
                                  payload_len=plen, pn=pn, pn_off=len(hdr) - pn_len,
                                  expected_pn=exp, key_phase=0, send_phase=0))
            # tampered packets: ciphertext, tag, first byte, packet number
            for t, where in enumerate(("ct", "tag", "first", "pn")):
                seed = f"s{suite}-v{version:x}-tamper{t}"
                hdr = short_header(gen_bytes(seed + ":dcid", 8), 77, 2, 0)
                plen = 200
                pos = {"ct": len(hdr) + 50, "tag": len(hdr) + plen + 3, "first": 0,
                       "pn": len(hdr) - 1}[where]
                bit = {"first": 0}.get(where, 5)
                cases.append(dict(seed=seed, suite=suite, version=version, header=hdr.hex(),
                                  payload_len=plen, pn=77, pn_off=len(hdr) - 2, expected_pn=77,
                                  key_phase=0, send_phase=0, tamper=[[pos, bit]]))
            # sender moved to the next key phase: receiver must switch (crypto.py:91-96)
            for t in range(2):
                seed = f"s{suite}-v{version:x}-phase{t}"
                hdr = short_header(gen_bytes(seed + ":dcid", 8), 1000 + t, 2, 1)
                cases.append(dict(seed=seed, suite=suite, version=version, header=hdr.hex(),
                                  payload_len=300 + t, pn=1000 + t, pn_off=9,
                                  expected_pn=1000, key_phase=0, send_phase=1))
            # truncated pn 0xfffffffe: HeaderProtection.remove returns it as signed -2
            seed = f"s{suite}-v{version:x}-pnsign"
            pn = 0x1FFFFFFFE
            hdr = short_header(gen_bytes(seed + ":dcid", 8), pn, 4, 0)
            cases.append(dict(seed=seed, suite=suite, version=version, header=hdr.hex(),
                              payload_len=64, pn=pn, pn_off=9, expected_pn=pn, key_phase=0,
                              send_phase=0))
    return cases
