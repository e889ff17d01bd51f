"""GPU parity of the round-2 boundary work, through the C ABI:

* bucketing by (suite, key slot) on the device (qpp_plan_*): planned launches
  equal unplanned ones and the oracle, results land in the caller's order,
  unknown slots report NO_KEY; BASELINE config 4 (AES-256-GCM, 4096 keys,
  1 Mi packets) and config 5 (AES-128-GCM / ChaCha20-Poly1305, 1024 keys,
  2 Mi packets) in random arrival order at full size;
* standalone HeaderProtection.apply byte parity (_crypto.c:289-319);
* two threads in the library at once (one session per thread);
* the session's descriptor bounds checks (QPP_S_LENGTH, nothing touched);
* no unauthenticated plaintext left behind by a failed unprotect.
"""

import os
import threading

import numpy as np
import pytest

from tests.golden_cases import short_header

pytestmark = pytest.mark.gpu

KEY_LEN = {0: 16, 1: 32, 2: 32}
NAMES = {0: (b"aes-128-gcm", b"aes-128-ecb"), 1: (b"aes-256-gcm", b"aes-256-ecb"),
         2: (b"chacha20-poly1305", b"chacha20")}


def _keys(rng, n_slots, suites=(0, 1, 2)):
    from aioquic_amd import layout as L

    recs = np.zeros(n_slots, dtype=L.KEY_MATERIAL)
    for s in range(n_slots):
        suite = suites[s % len(suites)]
        kl = KEY_LEN[suite]
        recs[s]["slot"] = s
        recs[s]["suite"] = suite
        recs[s]["iv"] = np.frombuffer(rng.bytes(12), np.uint8)
        recs[s]["key"][:kl] = np.frombuffer(rng.bytes(kl), np.uint8)
        recs[s]["hp"][:kl] = np.frombuffer(rng.bytes(kl), np.uint8)
    return recs


def _dev(a):
    import torch

    return torch.from_numpy(np.ascontiguousarray(a).view(np.uint8).ravel().copy()).cuda()


def _run(eng, fn_name, desc, n, inbuf, out_size, plan):
    """One device launch; returns (out bytes, results)."""
    import torch

    from aioquic_amd import layout as L

    d_desc = _dev(desc)
    d_in = _dev(inbuf)
    d_out = torch.zeros(out_size, dtype=torch.uint8, device="cuda")
    d_res = torch.full((n * 16,), 0xEE, dtype=torch.uint8, device="cuda")
    p = eng.bucket(d_desc, n) if plan else None
    getattr(eng, fn_name)(d_desc, n, d_in, d_out, d_res, plan=p)
    torch.cuda.synchronize()
    return d_out.cpu().numpy(), d_res.cpu().numpy().view(L.RESULT)


@pytest.fixture(params=["counting", "radix"])
def plan_path(request, monkeypatch):
    """Both bucketing paths: the counting sort (tables of <= 4096 slots) and
    the rocPRIM radix sort (larger tables; forced by QPP_PLAN_RADIX)."""
    if request.param == "radix":
        monkeypatch.setenv("QPP_PLAN_RADIX", "1")
    else:
        monkeypatch.delenv("QPP_PLAN_RADIX", raising=False)
    return request.param


def test_planned_equals_unplanned_and_oracle(oracle, plan_path):
    """A random ragged batch over all suites, interleaved slots, some of them
    empty or out of range: the planned path gives the same bytes and results
    as the unplanned one and the oracle, in the caller's order."""
    from aioquic_amd import layout as L
    from aioquic_amd.batch import PacketEngine, layout_packets

    rng = np.random.default_rng(0xB0C)
    n_slots = 40
    recs = _keys(rng, n_slots)
    eng = PacketEngine(n_slots + 4)  # slots 40..43 never installed
    eng.set_key_records(recs)
    n = 4000
    headers, payloads, pns, slots = [], [], [], []
    for i in range(n):
        pn_len = 1 + i % 4
        pn = int(rng.integers(0, 1 << 30))
        headers.append(short_header(rng.bytes(int(rng.integers(0, 21))), pn, pn_len, 0))
        payloads.append(rng.bytes(int(rng.integers(4, 1400))))
        pns.append(pn)
        slots.append(int(rng.integers(0, n_slots + 6)))  # 44, 45: beyond capacity
    inbuf, desc, size = layout_packets(headers, payloads, pns, slots)
    out_u, res_u = _run(eng, "protect", desc, n, inbuf, size, False)
    out_p, res_p = _run(eng, "protect", desc, n, inbuf, size, True)
    assert res_p.tobytes() == res_u.tobytes()
    assert np.array_equal(out_p, out_u)
    nokey = np.array(slots) >= n_slots
    assert (res_p["status"][nokey] == L.S_NO_KEY).all()
    assert (res_p["status"][~nokey] == L.S_OK).all()
    keys_full = np.zeros(n_slots + 6, dtype=L.KEY_MATERIAL)
    keys_full[:n_slots] = recs
    ok = np.nonzero(~nokey)[0]
    o_out, o_res = oracle.protect_batch(recs, desc[ok], inbuf, size)
    for i in ok[::7]:
        o, m = int(desc[i]["out_off"]), int(res_p[i]["out_len"])
        assert np.array_equal(out_p[o : o + m], o_out[o : o + m]), i
    # unprotect of the planned output, planned and unplanned
    ud = desc.copy()
    ud["len"] = np.where(nokey, 1200, res_p["out_len"])
    ud["hdr_len"] = [len(h) - ((h[0] & 3) + 1) for h in headers]
    ud["pn"] = np.asarray(pns, np.uint64)
    back_u, r_u = _run(eng, "unprotect", ud, n, out_p, size, False)
    back_p, r_p = _run(eng, "unprotect", ud, n, out_p, size, True)
    assert r_p.tobytes() == r_u.tobytes()
    assert np.array_equal(back_p, back_u)
    assert (r_p["status"][~nokey] == L.S_OK).all() and (r_p["status"][nokey] == L.S_NO_KEY).all()
    for i in ok[::5]:
        o = int(desc[i]["in_off"])
        assert back_p[o : o + len(headers[i]) + len(payloads[i])].tobytes() == headers[i] + payloads[i]


def test_wave_items_ragged_runs(oracle, plan_path):
    """Key runs of 1, 15, 16, 17, 31, 33, 64, 255 and 257 packets (the plan's
    wave items split them at 16), all suites, shuffled arrival: planned ==
    unplanned == oracle for every packet."""
    from aioquic_amd import layout as L
    from aioquic_amd.batch import PacketEngine, layout_packets

    rng = np.random.default_rng(0x17E5)
    runs = [1, 15, 16, 17, 31, 33, 64, 255, 257]
    n_slots = 3 * len(runs)
    recs = _keys(rng, n_slots)
    eng = PacketEngine(n_slots)
    eng.set_key_records(recs)
    slots = np.concatenate([np.full(runs[s % len(runs)], s) for s in range(n_slots)])
    rng.shuffle(slots)
    n = len(slots)
    headers, payloads, pns = [], [], []
    for i in range(n):
        pn = int(rng.integers(0, 1 << 20))
        headers.append(short_header(rng.bytes(8), pn, 2, 0))
        payloads.append(rng.bytes(int(rng.integers(20, 300))))
        pns.append(pn)
    inbuf, desc, size = layout_packets(headers, payloads, pns, [int(x) for x in slots])
    out_u, res_u = _run(eng, "protect", desc, n, inbuf, size, False)
    out_p, res_p = _run(eng, "protect", desc, n, inbuf, size, True)
    assert (res_p["status"] == L.S_OK).all()
    assert res_p.tobytes() == res_u.tobytes()
    assert np.array_equal(out_p, out_u)
    o_out, o_res = oracle.protect_batch(recs, desc, inbuf, size)
    assert np.array_equal(o_res["out_len"], res_p["out_len"])
    for i in range(n):
        o, m = int(desc[i]["out_off"]), int(res_p[i]["out_len"])
        assert np.array_equal(out_p[o : o + m], o_out[o : o + m]), i


def _full_size(cfg, n, n_keys, seed, oracle):
    """Full-size random-arrival batch on device tensors, bucketed in the
    product: every tag verifies, the round trip is exact, decoded packet
    numbers are the sent ones, and every packet in both directions equals the
    reference's own _crypto byte for byte (the C oracle on the first packet of
    every key when oracle/_ref is not built)."""
    import torch

    from aioquic_amd import bench_data
    from aioquic_amd import layout as L
    from aioquic_amd.batch import PacketEngine

    w = bench_data.make_workload(n, n_keys=n_keys, seed=seed, order="random", **cfg)
    assert len(np.unique(w.desc["slot"][:4096])) > min(n_keys, 4096) // 2  # interleaved
    eng = PacketEngine(n_keys)
    eng.set_key_records(w.keys)
    d_in = torch.from_numpy(w.plain).cuda()
    d_desc = _dev(w.desc)
    d_udesc = _dev(w.udesc)
    d_wire = torch.zeros(w.wire_size, dtype=torch.uint8, device="cuda")
    d_back = torch.zeros(w.plain_size, dtype=torch.uint8, device="cuda")
    d_r1 = torch.zeros(n * 16, dtype=torch.uint8, device="cuda")
    d_r2 = torch.zeros(n * 16, dtype=torch.uint8, device="cuda")
    eng.protect(d_desc, n, d_in, d_wire, d_r1, plan=eng.bucket(d_desc, n))
    eng.unprotect(d_udesc, n, d_wire, d_back, d_r2, plan=eng.bucket(d_udesc, n))
    torch.cuda.synchronize()
    r1 = d_r1.cpu().numpy().view(L.RESULT)
    r2 = d_r2.cpu().numpy().view(L.RESULT)
    assert (r1["status"] == 0).all() and (r1["out_len"] == 1200).all()
    assert (r2["status"] == 0).all()
    assert (r2["pn"] == w.desc["pn"]).all()
    assert torch.equal(d_back, d_in)
    wire = d_wire.cpu().numpy()
    back = d_back.cpu().numpy()
    # whole-batch parity: every packet in both directions
    # against the reference's own _crypto (oracle/_ref: _crypto.c:115-194
    # driven as quic/crypto.py:75-116 drives it) when it is built; otherwise
    # the first packet of every key against the C oracle
    from tests import ref_crypto

    ref = ref_crypto.checker(os.environ.get("PYTEST_CURRENT_TEST", "?").split(" ")[0])
    if ref is not None:
        assert np.array_equal(ref_crypto.protect_all(ref, w), wire)
        r_back, r_pn = ref_crypto.unprotect_all(ref, w, wire)
        assert np.array_equal(r_back, back)
        assert np.array_equal(r_pn, r2["pn"])
        return w
    _, first = np.unique(w.desc["slot"], return_index=True)
    assert len(first) == n_keys
    sub = w.desc[first].copy()
    o_out, o_res = oracle.protect_batch(w.keys, sub, w.plain, w.wire_size)
    assert (o_res["status"] == 0).all()
    wire_rows = wire.reshape(n, 1200)[first]
    want_rows = o_out.reshape(n, 1200)[first]
    assert np.array_equal(wire_rows, want_rows)
    return w


def test_config4_aes256_4096_keys_random_order(oracle):
    w = _full_size(dict(suite=1), 1 << 20, 4096, 0x9005, oracle)
    assert (w.suites == 1).all()


def test_config5_mixed_1024_keys_random_order(oracle):
    w = _full_size(dict(suite=0, mixed=(0, 2)), 1 << 21, 1024, 0x9006, oracle)
    frac = float((w.suites == 2).mean())
    assert 0.35 < frac < 0.65  # both suites, interleaved packet by packet


def test_hp_apply_vs_oracle(oracle):
    """Standalone HeaderProtection.apply (_crypto.c:289-319): every suite,
    packet-number lengths 1-4, short and long headers, against the oracle's
    mask applied as the reference applies it."""
    from aioquic_amd._crypto import HeaderProtection

    rng = np.random.default_rng(0xA991)
    for suite in (0, 1, 2):
        hpk = rng.bytes(KEY_LEN[suite])
        hp = HeaderProtection(NAMES[suite][1], hpk)
        for pn_len in (1, 2, 3, 4):
            for long_hdr in (False, True):
                for _ in range(4):
                    if long_hdr:
                        hdr = (bytes([0xC0 | (pn_len - 1)]) + rng.bytes(4) + b"\x08" + rng.bytes(8) +
                               b"\x00" + bytes([5]) + rng.bytes(5) + b"\x44\x00" + rng.bytes(pn_len))
                    else:
                        hdr = bytes([0x40 | (pn_len - 1) | (int(rng.integers(0, 2)) << 2)]) + \
                            rng.bytes(8) + rng.bytes(pn_len)
                    payload = rng.bytes(int(rng.integers(20 - pn_len, 1300)))
                    got = hp.apply(hdr, payload)
                    m = oracle.hp_mask(suite, hpk, payload[4 - pn_len : 20 - pn_len])
                    want = bytearray(hdr + payload)
                    want[0] ^= m[0] & (0x0F if want[0] & 0x80 else 0x1F)
                    for i in range(pn_len):
                        want[len(hdr) - pn_len + i] ^= m[1 + i]
                    assert got == bytes(want), (suite, pn_len, long_hdr)
                    # and remove() undoes it
                    h2, _ = hp.remove(got, len(hdr) - pn_len)
                    assert h2 == hdr


def test_two_threads_in_the_library(oracle):
    """protect_host batches in one thread while another runs the object API
    (AEAD.encrypt) and per-packet CryptoContext.encrypt_packet: each thread
    has its own session, every result equals the oracle."""
    from aioquic_amd import layout as L
    from aioquic_amd._crypto import AEAD
    from aioquic_amd.batch import PacketEngine, layout_packets
    from aioquic_amd.crypto import CryptoContext
    from aioquic_amd.tls import CipherSuite

    rng = np.random.default_rng(0x7777)
    recs = _keys(rng, 6)
    eng = PacketEngine(6)
    eng.set_key_records(recs)
    headers = [short_header(rng.bytes(8), i, 2, 0) for i in range(700)]
    payloads = [rng.bytes(int(rng.integers(4, 1300))) for _ in range(700)]
    inbuf, desc, size = layout_packets(headers, payloads, list(range(700)), [i % 6 for i in range(700)])
    want_batch, _ = oracle.protect_batch(recs, desc, inbuf, size)
    key, iv = rng.bytes(16), rng.bytes(12)
    aead = AEAD(b"aes-128-gcm", key, iv)
    secret = rng.bytes(32)
    ctx = CryptoContext()
    ctx.setup(cipher_suite=CipherSuite.AES_128_GCM_SHA256, secret=secret, version=1)
    k2, iv2, hp2 = oracle.derive_key_iv_hp(0, secret)
    errors = []

    def batches():
        try:
            for _ in range(12):
                out, res = eng.protect_host(desc, inbuf.tobytes(), size)
                assert (res["status"] == L.S_OK).all()
                assert np.array_equal(out, want_batch)
        except Exception as e:  # noqa: BLE001
            errors.append(e)

    def singles():
        try:
            for i in range(150):
                data, aad = rng.bytes(200 + i), rng.bytes(11)
                assert aead.encrypt(data, aad, i) == oracle.aead_encrypt(0, key, iv, data, aad, i)
                hdr = short_header(b"\x22" * 8, i, 2, 0)
                assert ctx.encrypt_packet(hdr, data, i) == oracle.protect(0, k2, iv2, hp2, hdr, data, i)
        except Exception as e:  # noqa: BLE001
            errors.append(e)

    ts = [threading.Thread(target=batches), threading.Thread(target=singles)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=100)
    assert not any(t.is_alive() for t in ts)
    assert not errors, errors[0]


def test_session_rejects_descriptors_outside_the_buffers():
    """Host-buffer calls check every descriptor against in_len / out_len: a
    packet that does not fit reports QPP_S_LENGTH and nothing is written for
    it; the others are unaffected."""
    from aioquic_amd import layout as L
    from aioquic_amd.batch import PacketEngine, layout_packets

    rng = np.random.default_rng(3)
    recs = _keys(rng, 2)
    eng = PacketEngine(2)
    eng.set_key_records(recs)
    headers = [short_header(rng.bytes(8), i, 2, 0) for i in range(8)]
    payloads = [rng.bytes(300) for _ in range(8)]
    inbuf, desc, size = layout_packets(headers, payloads, list(range(8)), [i % 2 for i in range(8)])
    ref_out, ref_res = eng.protect_host(desc, inbuf.tobytes(), size)
    bad = desc.copy()
    bad[2]["in_off"] = 1 << 40                # input beyond the buffer
    bad[5]["out_off"] = size - 100            # output runs past out_len
    bad[6]["len"] = 1 << 20                   # payload longer than the buffer
    out, res = eng.protect_host(bad, inbuf.tobytes(), size)
    for i in range(8):
        o, m = int(desc[i]["out_off"]), int(ref_res[i]["out_len"])
        if i in (2, 5, 6):
            assert res[i]["status"] == L.S_LENGTH and res[i]["out_len"] == 0
            if i != 5:  # nothing written at the rejected packet's own (valid) output
                assert not out[o : o + m].any()
        else:
            assert res[i]["status"] == L.S_OK
            assert np.array_equal(out[o : o + m], ref_out[o : o + m])


@pytest.mark.parametrize("suite", [0, 1, 2])
def test_failed_unprotect_leaves_no_plaintext(suite):
    """Tampered packets: status DECRYPT and their payload regions zero in the
    output; untampered neighbours decrypt normally."""
    import torch

    from aioquic_amd import layout as L
    from aioquic_amd.batch import PacketEngine, layout_packets

    rng = np.random.default_rng(40 + suite)
    recs = _keys(rng, 1, suites=(suite,))
    eng = PacketEngine(1)
    eng.set_key_records(recs)
    n = 512
    headers = [short_header(rng.bytes(8), i, 2, 0) for i in range(n)]
    payloads = [rng.bytes(int(rng.integers(20, 1400))) for _ in range(n)]
    inbuf, desc, size = layout_packets(headers, payloads, list(range(n)), [0] * n)
    wire, res = _run(eng, "protect", desc, n, inbuf, size, False)
    assert (res["status"] == 0).all()
    bad = set(range(3, n, 17))
    wire = wire.copy()
    for i in bad:  # flip a ciphertext bit past the HP sample
        wire[int(desc[i]["out_off"]) + 11 + 30 + int(rng.integers(0, len(payloads[i]) - 16 + 1))] ^= 4
    ud = desc.copy()
    ud["len"] = res["out_len"]
    ud["hdr_len"] = 9
    fill = np.full(size, 0x5A, np.uint8)
    d_out = torch.from_numpy(fill).cuda()
    d_res = torch.zeros(n * 16, dtype=torch.uint8, device="cuda")
    eng.unprotect(_dev(ud), n, _dev(wire), d_out, d_res)
    torch.cuda.synchronize()
    out = d_out.cpu().numpy()
    r = d_res.cpu().numpy().view(L.RESULT)
    for i in range(n):
        o, hl, pl = int(desc[i]["out_off"]), 11, len(payloads[i])
        if i in bad:
            assert r[i]["status"] == L.S_DECRYPT and r[i]["out_len"] == 0
            assert not out[o + hl : o + hl + pl].any(), i
        else:
            assert r[i]["status"] == L.S_OK
            assert out[o + hl : o + hl + pl].tobytes() == payloads[i]
