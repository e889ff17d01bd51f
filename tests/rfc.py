"""RFC 9001 / RFC 9369 Appendix-A vectors, loaded from tests/golden/rfc_vectors.json
(extracted from the reference's tests/test_crypto_v{1,2}.py by
tests/golden/make_rfc_vectors.py)."""

import json
import os

_D = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "rfc_vectors.json")))

VERSIONS = {"v1": 0x00000001, "v2": 0x6B3343CF}


class V:
    def __init__(self, tag):
        d = _D[tag]
        self.tag = tag
        self.version = VERSIONS[tag]
        for k, v in d.items():
            if k.startswith("_"):
                continue
            setattr(k.lower(), v) if False else None
            setattr(self, k.lower(), bytes.fromhex(v) if isinstance(v, str) else v)
        lit = d["_literals"]
        self.cid = bytes.fromhex(lit["create_crypto"][0])
        self.chacha_secret = bytes.fromhex(lit["test_decrypt_chacha20"][0])
        self.short_secret = bytes.fromhex(lit["test_decrypt_short_server"][0])
        dk = [bytes.fromhex(x) for x in lit["test_derive_key_iv_hp"]]
        self.derive_client = dk[0:4]  # secret, key, iv, hp
        self.derive_server = dk[4:8]
        self.derive_chacha = [bytes.fromhex(x) for x in lit["test_derive_key_iv_hp_chacha20"]]


V1 = V("v1")
V2 = V("v2")
ALL = [V1, V2]
