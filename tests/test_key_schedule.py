"""GPU parity of the batched key schedule (qpp_keytab_derive, SURVEY.md sec. 8(f)
row 4): device HKDF-Expand-Label + slot expansion against the oracle's
independent stdlib restatement of derive_key_iv_hp / next_key_phase
(quic/crypto.py:34-56,157-168) and against the RFC 9001 / 9369 vectors."""

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

KEY_LEN = {0: 16, 1: 32, 2: 32}


def test_derive_matches_oracle_and_protects(oracle):
    import torch

    from aioquic_amd import layout as L
    from aioquic_amd.batch import PacketEngine, layout_packets
    from tests.golden_cases import short_header

    rng = np.random.default_rng(77)
    n = 300
    recs = np.concatenate([
        L.secret_record(i, i % 3, rng.bytes(48 if i % 3 == 1 else 32), key_phase=(i // 3) & 1,
                        v2=bool(i & 4), updates=int(rng.integers(0, 4)))
        for i in range(n)])
    eng = PacketEngine(n)
    km = eng.derive_keys(recs)
    for i, r in enumerate(recs):
        suite, secret = int(r["suite"]), bytes(r["secret"][: r["secret_len"]])
        for _ in range(int(r["updates"])):
            secret = oracle.next_secret(suite, secret)
        key, iv, hp = oracle.derive_key_iv_hp(suite, secret,
                                              oracle.VERSION_2 if r["flags"] & 1 else oracle.VERSION_1)
        kl = KEY_LEN[suite]
        assert km[i]["slot"] == i and km[i]["suite"] == suite and km[i]["key_phase"] == r["key_phase"]
        assert bytes(km[i]["key"][:kl]) == key and bytes(km[i]["iv"]) == iv
        assert bytes(km[i]["hp"][:kl]) == hp
    # the derived slots protect exactly like slots installed from the same material
    headers = [short_header(rng.bytes(8), j, 2, int(km[j % n]["key_phase"])) for j in range(600)]
    payloads = [rng.bytes(int(rng.integers(20, 1200))) for _ in range(600)]
    slots = [j % n for j in range(600)]
    inbuf, desc, size = layout_packets(headers, payloads, list(range(600)), slots)
    exp, eres = oracle.protect_batch(km, desc, inbuf, size)
    assert (eres["status"] == 0).all()
    d_out = torch.zeros(size, dtype=torch.uint8, device="cuda")
    res = torch.empty(600 * 16, dtype=torch.uint8, device="cuda")
    eng.protect(torch.from_numpy(desc.view(np.uint8).copy()).cuda(), 600,
                torch.from_numpy(inbuf).cuda(), d_out, res)
    torch.cuda.synchronize()
    assert (res.cpu().numpy().view(L.RESULT)["status"] == 0).all()
    assert np.array_equal(d_out.cpu().numpy(), exp)


def test_derive_rfc_initial_vectors():
    """RFC 9001 App. A.1 / RFC 9369 App. A.1: client / server initial secrets."""
    from aioquic_amd import layout as L
    from aioquic_amd.batch import PacketEngine
    from tests.rfc import V1, V2

    eng = PacketEngine(4)
    recs, want = [], []
    for v in (V1, V2):
        for secret, key, iv, hp in (v.derive_client, v.derive_server):
            recs.append(L.secret_record(len(recs), 0, secret, v2=v.version == 0x6B3343CF))
            want.append((key, iv, hp))
    km = eng.derive_keys(np.concatenate(recs))
    for r, (key, iv, hp) in zip(km, want):
        assert (bytes(r["key"][:16]), bytes(r["iv"]), bytes(r["hp"][:16])) == (key, iv, hp)


def test_derive_rejects_bad_records():
    from aioquic_amd import layout as L
    from aioquic_amd.batch import PacketEngine

    eng = PacketEngine(2)
    with pytest.raises(ValueError):
        eng.derive_keys(L.secret_record(2, 0, bytes(32)))  # slot out of range
    bad = L.secret_record(0, 0, bytes(32))
    bad["suite"] = 7
    with pytest.raises(ValueError):
        eng.derive_keys(bad)
