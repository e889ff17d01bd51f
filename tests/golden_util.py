"""Load tests/golden/golden_vectors.json and rebuild each case's inputs."""

import hashlib
import json
import os

from tests.golden_cases import gen_bytes

_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "golden_vectors.json")


def load_cases():
    with open(_PATH) as f:
        return json.load(f)["cases"]


def case_inputs(c, oracle):
    """-> dict(suite, key, iv, hp, next_key, next_iv, header, payload)"""
    suite = c["suite"]
    secret = gen_bytes(c["seed"] + ":secret", 48 if suite == 1 else 32)
    key, iv, hp = oracle.derive_key_iv_hp(suite, secret, c["version"])
    k2, iv2, _ = oracle.derive_key_iv_hp(suite, oracle.next_secret(suite, secret), c["version"])
    return dict(suite=suite, secret=secret, key=key, iv=iv, hp=hp, next_key=k2, next_iv=iv2,
                header=bytes.fromhex(c["header"]),
                payload=gen_bytes(c["seed"] + ":payload", c["payload_len"]))


def matches(field, data: bytes) -> bool:
    if "hex" in field:
        return data.hex() == field["hex"]
    return len(data) == field["len"] and hashlib.sha256(data).hexdigest() == field["sha256"]


def tamper(c, pkt: bytes) -> bytes:
    w = bytearray(pkt)
    for pos, bit in c.get("tamper", []):
        w[pos] ^= 1 << bit
    return bytes(w)
