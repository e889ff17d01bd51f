"""GPU parity: the HIP path against the reference's golden vectors and the CPU
oracle, through the C ABI (libquicpp via aioquic_amd._crypto).  Bit-exact."""

import hashlib
import os

import numpy as np
import pytest

from tests.golden_cases import gen_bytes, short_header

pytestmark = pytest.mark.gpu

SUITES = (0, 1, 2)
KEY_LEN = {0: 16, 1: 32, 2: 32}


@pytest.fixture(scope="module")
def L():
    from aioquic_amd import layout

    return layout


@pytest.fixture(scope="module")
def engine_cls():
    from aioquic_amd.batch import PacketEngine

    return PacketEngine


def _keys(rng, n_slots, suites=SUITES):
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


def test_golden_vectors_batch(oracle, L, engine_cls):
    """All reference golden cases in one protect batch and one unprotect batch."""
    from tests.golden_util import case_inputs, load_cases, matches, tamper

    cases = load_cases()
    n = len(cases)
    eng = engine_cls(2 * n)
    recs = np.zeros(2 * n, dtype=L.KEY_MATERIAL)
    xs = []
    for i, c in enumerate(cases):
        x = case_inputs(c, oracle)
        xs.append(x)
        kl = len(x["key"])
        for slot, (k, iv, ph) in ((2 * i, (x["key"], x["iv"], 0)),
                                  (2 * i + 1, (x["next_key"], x["next_iv"], 1))):
            recs[slot]["slot"] = slot
            recs[slot]["suite"] = c["suite"]
            recs[slot]["key_phase"] = ph
            recs[slot]["iv"] = np.frombuffer(iv, np.uint8)
            recs[slot]["key"][:kl] = np.frombuffer(k, np.uint8)
            recs[slot]["hp"][:kl] = np.frombuffer(x["hp"], np.uint8)
    eng.set_key_records(recs)

    from aioquic_amd.batch import layout_packets

    inbuf, desc, size = layout_packets(
        [x["header"] for x in xs], [x["payload"] for x in xs], [c["pn"] for c in cases],
        [2 * i + c["send_phase"] for i, c in enumerate(cases)], align=1)
    out, res = eng.protect_host(desc, inbuf.tobytes(), size)
    assert (res["status"] == L.S_OK).all()
    wires = []
    for i, c in enumerate(cases):
        o, ln = int(desc[i]["out_off"]), int(res[i]["out_len"])
        pkt = out[o : o + ln].tobytes()
        assert matches(c["protected"], pkt), c["seed"]
        wires.append(tamper(c, pkt))

    # unprotect: slot = receiver's current key (phase 0); KEY_PHASE -> retry with next
    ud = np.zeros(n, dtype=L.DESC)
    blob, pos = bytearray(), 0
    for i, (c, w) in enumerate(zip(cases, wires)):
        ud[i]["in_off"] = pos
        ud[i]["out_off"] = pos
        ud[i]["len"] = len(w)
        ud[i]["hdr_len"] = c["pn_off"]
        ud[i]["pn"] = c["expected_pn"]
        ud[i]["slot"] = 2 * i
        blob += w
        pos += len(w)
    out, res = eng.unprotect_host(ud, bytes(blob), pos)
    retry = np.nonzero(res["status"] == L.S_KEY_PHASE)[0]
    res = res.copy()
    out = out.copy()
    if len(retry):
        ud2 = ud[retry].copy()
        ud2["slot"] += 1
        out2, res2 = eng.unprotect_host(ud2, bytes(blob), pos)
        for j, i in enumerate(retry):
            res[i] = res2[j]
            o = int(ud[i]["out_off"])
            out[o : o + int(res2[j]["out_len"])] = out2[o : o + int(res2[j]["out_len"])]
    for i, c in enumerate(cases):
        exp = c["unprotect"]
        st = int(res[i]["status"])
        if not exp["ok"]:
            assert st == L.S_DECRYPT, (c["seed"], st)
            continue
        assert st == L.S_OK, (c["seed"], st)
        assert (i in retry) == exp["phase_flip"]
        o, hl, ln = int(ud[i]["out_off"]), int(res[i]["hdr_len"]), int(res[i]["out_len"])
        assert out[o : o + hl].tobytes().hex() == exp["header"], c["seed"]
        assert matches(exp["payload"], out[o + hl : o + ln].tobytes()), c["seed"]
        assert int(res[i]["pn"]) == exp["pn"], c["seed"]


def _random_batch(rng, n, n_slots, recs, *, max_payload=1400, pn_lens=(1, 2, 3, 4)):
    headers, payloads, pns, slots = [], [], [], []
    for i in range(n):
        pn_len = pn_lens[i % len(pn_lens)]
        pn = int(rng.integers(0, 1 << 40))
        if i % 5 == 4:
            dcid = rng.bytes(int(rng.integers(0, 21)))
            token = rng.bytes(int(rng.integers(0, 60)))
            hdr = (bytes([0xC0 | (pn_len - 1)]) + (1).to_bytes(4, "big") + bytes([len(dcid)]) +
                   dcid + b"\x00" + bytes([len(token)]) + token + b"\x44\x00" +
                   (pn & ((1 << (8 * pn_len)) - 1)).to_bytes(pn_len, "big"))
        else:
            hdr = short_header(rng.bytes(int(rng.integers(0, 21))), pn, pn_len, 0, spin=i & 1)
        plen = int(rng.integers(max(0, 4 - pn_len), max_payload))
        plen = min(plen, 1500 - 16 - len(hdr))
        headers.append(hdr)
        payloads.append(rng.bytes(plen))
        pns.append(pn)
        slots.append(int(rng.integers(0, n_slots)))
    return headers, payloads, pns, slots


@pytest.mark.parametrize("bpl", ["1", "2"], ids=["gcm-bpl1", "gcm-bpl2"])
@pytest.mark.parametrize("align", [1, 16, -16], ids=["align1", "align16", "payload16"])
def test_random_batch_vs_oracle(oracle, L, engine_cls, align, bpl):
    """Ragged, misaligned packets of all suites and mixed key slots vs the oracle,
    under both GCM step forms (QPP_GCM_BPL: one or two blocks per lane a step);
    align < 0: payloads on multiples of -align (layout_packets(payload_align=...)).
    The library reads QPP_GCM_BPL once per process, so the one-block form runs
    in a child process started with QPP_GCM_BPL=1."""
    if bpl == "1":
        import subprocess
        import sys

        root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
        code = ("import sys; sys.path.insert(0, %r); from tests.test_gpu_parity import random_batch_check; "
                "random_batch_check(%d, 'QPP_GCM_BPL=1')" % (root, align))
        r = subprocess.run([sys.executable, "-c", code], env=dict(os.environ, QPP_GCM_BPL="1"),
                           capture_output=True, text=True, timeout=180)
        assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
        assert "random_batch_check ok QPP_GCM_BPL=1" in r.stdout
        return
    random_batch_check(align, "", oracle, L, engine_cls)


def random_batch_check(align, tag, oracle=None, L=None, engine_cls=None):
    """Body of test_random_batch_vs_oracle (also run in a child process)."""
    from aioquic_amd.batch import PacketEngine, layout_packets

    if oracle is None:
        from oracle import oracle as orc

        orc.lib()
        oracle = orc
    if L is None:
        from aioquic_amd import layout as L
    engine_cls = engine_cls or PacketEngine
    rng = np.random.default_rng(0x9001 + abs(align))
    n_slots = 24
    recs = _keys(rng, n_slots)
    eng = engine_cls(n_slots)
    eng.set_key_records(recs)
    headers, payloads, pns, slots = _random_batch(rng, 3000, n_slots, recs)
    inbuf, desc, size = layout_packets(headers, payloads, pns, slots, align=max(align, 1),
                                       payload_align=max(-align, 1))
    out_g, res_g = eng.protect_host(desc, inbuf.tobytes(), size)
    out_o, res_o = oracle.protect_batch(recs, desc, inbuf, size)
    assert (res_g["status"] == res_o["status"]).all()
    assert (res_g["out_len"] == res_o["out_len"]).all()
    assert np.array_equal(out_g, out_o)

    # unprotect what the GPU produced, with expected pn = pn (+ jitter)
    ud = desc.copy()
    ud["len"] = res_g["out_len"]
    ud["hdr_len"] = [len(h) - ((h[0] & 3) + 1) for h in headers]
    ud["pn"] = np.asarray(pns, np.uint64) + rng.integers(0, 50, size=len(pns)).astype(np.uint64)
    u_g, r_g = eng.unprotect_host(ud, out_g.tobytes(), size)
    u_o, r_o = oracle.unprotect_batch(recs, ud, out_g, size)
    bad = np.nonzero(r_g != r_o)[0]
    assert len(bad) == 0, (bad[:10], r_g[bad[:3]], r_o[bad[:3]])
    # the only failures allowed are the reference's signed-pn quirk: 4-byte
    # packet number >= 2^32 whose truncated value has its top bit set
    quirk = np.array([((h[0] & 3) == 3) and pn >= (1 << 32) and (pn & 0x80000000) != 0
                      for h, pn in zip(headers, pns)])
    assert ((r_g["status"] == L.S_OK) | quirk).all()
    assert ((r_g["status"] == L.S_DECRYPT) == quirk).all()
    # round trip restores the input (header + payload); outputs equal the oracle's
    for i in range(len(headers)):
        o = int(desc[i]["in_off"])
        n_ = len(headers[i]) + len(payloads[i])
        if not quirk[i]:
            assert u_g[o : o + n_].tobytes() == headers[i] + payloads[i]
            assert np.array_equal(u_g[o : o + n_], u_o[o : o + n_])
    if tag:
        print("random_batch_check ok", tag)


def test_tamper_and_edge_status(oracle, L, engine_cls):
    """Corrupted tags/ciphertext -> DECRYPT for exactly those packets; bad
    lengths -> LENGTH; empty slot -> NO_KEY; key phase flip -> KEY_PHASE."""
    from aioquic_amd.batch import layout_packets

    rng = np.random.default_rng(7)
    recs = _keys(rng, 6)
    eng = engine_cls(8)
    eng.set_key_records(recs)
    n = 600
    headers = [short_header(rng.bytes(8), i, 2, 0) for i in range(n)]
    payloads = [rng.bytes(int(rng.integers(4, 1200))) for _ in range(n)]
    slots = [i % 6 for i in range(n)]
    inbuf, desc, size = layout_packets(headers, payloads, list(range(n)), slots)
    out, res = eng.protect_host(desc, inbuf.tobytes(), size)
    assert (res["status"] == L.S_OK).all()
    wire = out.copy()
    bad = set(int(i) for i in rng.choice(n, 60, replace=False))
    for i in bad:
        o = int(desc[i]["out_off"]) + 11 + int(rng.integers(0, len(payloads[i]) + 16))
        wire[o] ^= 1 << int(rng.integers(0, 8))
    ud = desc.copy()
    ud["len"] = res["out_len"]
    ud["hdr_len"] = 9
    ud[3]["len"] = 25          # too short for header + tag
    ud[5]["slot"] = 7          # never installed
    ud[7]["hdr_len"] = 0       # pn offset 0
    u, r = eng.unprotect_host(ud, wire.tobytes(), size)
    uo, ro = oracle.unprotect_batch(recs, ud, wire, size)
    for i in range(n):
        st = int(r[i]["status"])
        if i == 5:
            assert st == L.S_NO_KEY
        elif i in (3, 7):
            assert st == L.S_LENGTH
        elif i in bad:
            # a flipped sample bit changes the unmasked first byte, which can
            # flip the key-phase bit or the pn length; the oracle agrees
            assert st != L.S_OK, i
        else:
            assert st == L.S_OK, i
        assert st == int(ro[i]["status"]), i
        if st == L.S_OK:
            assert r[i] == ro[i]
    # key-phase: flip the receiver's phase for slot 0
    recs2 = recs.copy()
    recs2[0]["key_phase"] = 1
    eng.set_key_records(recs2[:1])
    u, r = eng.unprotect_host(ud, wire.tobytes(), size)
    for i in range(0, n, 6):
        if i not in bad and i not in (3, 5, 7):
            assert int(r[i]["status"]) == L.S_KEY_PHASE


def test_aead_only_batch(oracle, L, engine_cls):
    """QPP_F_NO_HP: AEAD.encrypt / AEAD.decrypt semantics, arbitrary AAD incl. empty."""
    from aioquic_amd.batch import layout_packets

    rng = np.random.default_rng(11)
    recs = _keys(rng, 3)
    eng = engine_cls(3)
    eng.set_key_records(recs)
    aads = [rng.bytes(int(rng.integers(0, 70))) for _ in range(400)]
    datas = [rng.bytes(int(rng.integers(0, 1500))) for _ in range(400)]
    pns = [int(rng.integers(0, 1 << 63)) for _ in range(400)]
    inbuf, desc, size = layout_packets(aads, datas, pns, [i % 3 for i in range(400)],
                                       flags=L.F_NO_HP)
    out, res = eng.protect_host(desc, inbuf.tobytes(), size)
    out_o, res_o = oracle.protect_batch(recs, desc, inbuf, size)
    assert (res["status"] == 0).all() and (res == res_o).all()
    diff = np.nonzero(out != out_o)[0]
    if len(diff):
        starts = desc["out_off"].astype(np.int64)
        k = int(np.searchsorted(starts, diff[0], side="right") - 1)
        raise AssertionError(f"first diff at byte {diff[0]} ({len(diff)} total) in packet {k}: "
                             f"aad {len(aads[k])} data {len(datas[k])} slot {k % 3} "
                             f"suite {recs[k % 3]['suite']} off {diff[0] - starts[k]}")
    ud = desc.copy()
    ud["len"] = res["out_len"]
    u, r = eng.unprotect_host(ud, out.tobytes(), size)
    uo, ro = oracle.unprotect_batch(recs, ud, out, size)
    # data (ct||tag) longer than 1500 B is "Invalid payload length" (_crypto.c:126-129)
    too_long = np.array([len(x) + 16 > 1500 for x in datas])
    assert (r == ro).all()
    assert ((r["status"] == L.S_LENGTH) == too_long).all()
    assert ((r["status"] == L.S_OK) == ~too_long).all()
    # output bytes are defined for authenticated packets only
    for i in np.nonzero(~too_long)[0]:
        o, ln = int(ud[i]["out_off"]), int(r[i]["out_len"])
        assert np.array_equal(u[o : o + ln], uo[o : o + ln]), i


@pytest.mark.parametrize("suite,version,n", [(0, 1, 1 << 16), (2, 0x6B3343CF, 1 << 16), (0, 1, 1 << 20)],
                         ids=["config2-aes128", "config3-chacha-v2", "north-star-aes128-1Mi"])
def test_full_size_round_trip(L, engine_cls, suite, version, n):
    """BASELINE configs 2 and 3 on device tensors: 64Ki x 1200 B, one key,
    AES-128-GCM (QUIC v1) or ChaCha20-Poly1305 (QUIC v2 labels); and the
    north-star shape itself, AES-128-GCM 1Mi x 1200 B with one key (the
    1200-byte datagram of tests/test_packet_builder.py:490-522).
    Size-independent properties: round trip identity, all tags verify, every
    ciphertext differs from its plaintext; then the whole batch against the C
    oracle in both directions (not a sample): every protected byte
    and result record, and the oracle's unprotect of the device's wire against
    the device's unprotect (plaintext and result records)."""
    import torch

    from aioquic_amd import bench_data

    w = bench_data.make_workload(n, suite=suite, n_keys=1, seed=0x9002, version=version)
    eng = engine_cls(w.n_keys)
    eng.set_key_records(w.keys)
    dev = torch.device("cuda")
    d_in = torch.from_numpy(w.plain).to(dev)
    d_desc = torch.from_numpy(w.desc.view(np.uint8)).to(dev)
    d_wire = torch.empty(w.wire_size, dtype=torch.uint8, device=dev)
    d_res = torch.empty(n * 16, dtype=torch.uint8, device=dev)
    eng.protect(d_desc, n, d_in, d_wire, d_res)
    d_udesc = torch.from_numpy(w.udesc.view(np.uint8)).to(dev)
    d_back = torch.zeros(w.plain_size, dtype=torch.uint8, device=dev)
    d_res2 = torch.empty(n * 16, dtype=torch.uint8, device=dev)
    eng.unprotect(d_udesc, n, d_wire, d_back, d_res2)
    torch.cuda.synchronize()
    r1 = d_res.cpu().numpy().view(L.RESULT)
    r2 = d_res2.cpu().numpy().view(L.RESULT)
    assert (r1["status"] == 0).all() and (r1["out_len"] == 1200).all()
    assert (r2["status"] == 0).all() and (r2["pn"] == w.desc["pn"]).all()
    back = d_back.cpu().numpy()
    assert np.array_equal(back, w.plain)
    wire = d_wire.cpu().numpy()
    assert hashlib.sha256(wire.tobytes()).hexdigest() != hashlib.sha256(back.tobytes()).hexdigest()
    # whole-batch parity: the reference's own _crypto (oracle/_ref) over every
    # packet in both directions when it is built; otherwise the C oracle on a
    # 4096-packet prefix (its bitwise GHASH runs ~3.5 MB/s)
    from tests import ref_crypto

    ref = ref_crypto.checker(os.environ.get("PYTEST_CURRENT_TEST", "?").split(" ")[0])
    if ref is not None:
        assert np.array_equal(ref_crypto.protect_all(ref, w), wire)
        r_back, r_pn = ref_crypto.unprotect_all(ref, w, wire)
        assert np.array_equal(r_back, back)
        assert np.array_equal(r_pn, r2["pn"])
    else:
        from oracle import oracle as orc

        m = 4096
        o_wire, o_res = orc.protect_batch(w.keys, w.desc[:m], w.plain, w.wire_size)
        assert np.array_equal(o_res, r1[:m])
        assert np.array_equal(o_wire[: m * 1200], wire[: m * 1200])
        o_back, o_res2 = orc.unprotect_batch(w.keys, w.udesc[:m], wire, w.plain_size)
        assert np.array_equal(o_res2, r2[:m])
        assert np.array_equal(o_back[: m * 1200], back[: m * 1200])


def test_object_api():
    """aioquic._crypto object semantics (errors, signed pn from remove)."""
    from aioquic_amd._crypto import AEAD, CryptoError, HeaderProtection

    with pytest.raises(CryptoError, match="Invalid cipher name: foo"):
        AEAD(b"foo", bytes(16), bytes(12))
    with pytest.raises(CryptoError, match="Invalid key length"):
        AEAD(b"aes-128-gcm", bytes(33), bytes(12))
    with pytest.raises(CryptoError, match="Invalid iv length"):
        AEAD(b"aes-128-gcm", bytes(16), bytes(13))
    with pytest.raises(CryptoError, match="OpenSSL call failed"):
        AEAD(b"aes-128-gcm", bytes(32), bytes(12))
    a = AEAD(b"aes-128-gcm", bytes(16), bytes(12))
    with pytest.raises(CryptoError, match="Invalid payload length"):
        a.decrypt(b"x" * 15, b"", 0)
    with pytest.raises(CryptoError, match="Invalid payload length"):
        a.encrypt(b"x" * 1501, b"", 0)
    with pytest.raises(CryptoError, match="Payload decryption failed"):
        a.decrypt(b"x" * 16, b"", 0)
    ct = a.encrypt(b"hello", b"hdr", 5)
    assert a.decrypt(ct, b"hdr", 5) == b"hello"
    # short iv is zero padded (reference: memcpy into a zeroed object)
    assert AEAD(b"aes-128-gcm", bytes(16), bytes(8)).encrypt(b"abc", b"", 0) == \
        a.encrypt(b"abc", b"", 0)
    with pytest.raises(CryptoError, match="OpenSSL call failed"):
        HeaderProtection(b"aes-128-ecb", bytes(32))
    hp = HeaderProtection(b"aes-128-ecb", bytes(16))
    # known value from the reference build (aes-128-ecb of zeros under key 0)
    hdr, pn = hp.remove(bytes(30), 5)
    assert hdr.hex() == "0600000000e94bd4" and pn == 15289300


def test_object_api_vs_oracle(oracle):
    from aioquic_amd._crypto import AEAD, CryptoError, HeaderProtection

    rng = np.random.default_rng(5)
    names = {0: (b"aes-128-gcm", b"aes-128-ecb"), 1: (b"aes-256-gcm", b"aes-256-ecb"),
             2: (b"chacha20-poly1305", b"chacha20")}
    for suite in SUITES:
        kl = KEY_LEN[suite]
        key, iv, hpk = rng.bytes(kl), rng.bytes(12), rng.bytes(kl)
        a = AEAD(names[suite][0], key, iv)
        h = HeaderProtection(names[suite][1], hpk)
        for ln in (0, 1, 15, 16, 17, 100, 1484, 1500):
            data, aad, pn = rng.bytes(ln), rng.bytes(int(rng.integers(0, 40))), int(rng.integers(0, 1 << 62))
            ct = a.encrypt(data, aad, pn)
            assert ct == oracle.aead_encrypt(suite, key, iv, data, aad, pn)
            if len(ct) <= 1500:
                assert a.decrypt(ct, aad, pn) == data
            else:  # the reference rejects data (ct||tag) longer than 1500 bytes
                with pytest.raises(CryptoError, match="Invalid payload length"):
                    a.decrypt(ct, aad, pn)
        for _ in range(10):
            sample = rng.bytes(16)
            pkt = rng.bytes(5) + sample + rng.bytes(3)
            hdr, pn = h.remove(pkt, 1)
            m = oracle.hp_mask(suite, hpk, sample)
            b0 = pkt[0] ^ (m[0] & (0x0F if pkt[0] & 0x80 else 0x1F))
            pl = (b0 & 3) + 1
            assert hdr[0] == b0 and len(hdr) == 1 + pl
            t = int.from_bytes(bytes(x ^ y for x, y in zip(pkt[1 : 1 + pl], m[1 : 1 + pl])), "big")
            assert pn == (t - (1 << 32) if t >= 1 << 31 else t)


def test_retry_integrity_tag():
    """Retry tags of RFC 9001 / RFC 9369 App. A.4 (reference tests/test_packet.py:111-189)."""
    from aioquic_amd.packet import QuicProtocolVersion, get_retry_integrity_tag

    odcid = bytes.fromhex("8394c8f03e515708")
    v1 = bytes.fromhex("ff000000010008f067a5502a4262b5746f6b656e04a265ba2eff4d829058fb3f0f2496ba")
    v2 = bytes.fromhex("cf6b3343cf0008f067a5502a4262b5746f6b656ec8646ce8bfe33952d955543665dcc7b6")
    assert get_retry_integrity_tag(v1[:20], odcid, QuicProtocolVersion.VERSION_1) == v1[20:]
    assert get_retry_integrity_tag(v2[:20], odcid, QuicProtocolVersion.VERSION_2) == v2[20:]


def test_in_place(oracle, L, engine_cls):
    """out buffer == in buffer (the builder encrypts in place, packet_builder.py:341-350)."""
    import torch

    from aioquic_amd.batch import layout_packets

    rng = np.random.default_rng(9)
    recs = _keys(rng, 3)
    eng = engine_cls(3)
    eng.set_key_records(recs)
    headers = [short_header(rng.bytes(8), i, 2, 0) for i in range(256)]
    payloads = [rng.bytes(int(rng.integers(4, 1300))) for _ in range(256)]
    inbuf, desc, size = layout_packets(headers, payloads, list(range(256)), [i % 3 for i in range(256)])
    exp, _ = oracle.protect_batch(recs, desc, inbuf, size)
    buf = torch.from_numpy(inbuf.copy()).cuda()
    d = torch.from_numpy(desc.view(np.uint8).copy()).cuda()
    res = torch.empty(256 * 16, dtype=torch.uint8, device="cuda")
    eng.protect(d, 256, buf, buf, res)
    torch.cuda.synchronize()
    got = buf.cpu().numpy()
    for i in range(256):
        o, n = int(desc[i]["out_off"]), len(headers[i]) + len(payloads[i]) + 16
        assert np.array_equal(got[o : o + n], exp[o : o + n])


def test_fused_protect_length_boundary(oracle, L, engine_cls):
    """hdr + payload + tag = 1500 is the last defined size of the reference's
    encrypt_packet (buffer[1500], _crypto.c:168-171,305-306); one byte more is
    "Invalid payload length" in the kernel, the oracle and the object API."""
    import torch

    from aioquic_amd._crypto import CryptoError, HeaderProtection
    from aioquic_amd.batch import layout_packets

    rng = np.random.default_rng(13)
    recs = _keys(rng, 3)
    eng = engine_cls(3)
    eng.set_key_records(recs)
    headers, payloads, slots = [], [], []
    for s in range(3):
        for hl, extra in ((11, 0), (11, 1), (40, 0), (40, 1), (5, 0)):
            headers.append(short_header(rng.bytes(hl - 3), s, 2, 0))
            payloads.append(rng.bytes(1500 - 16 - hl + extra))
            slots.append(s)
    n = len(headers)
    inbuf, desc, size = layout_packets(headers, payloads, list(range(n)), slots)
    exp, eres = oracle.protect_batch(recs, desc, inbuf, size)
    d_in = torch.from_numpy(inbuf).cuda()
    d_out = torch.zeros(size, dtype=torch.uint8, device="cuda")
    d = torch.from_numpy(desc.view(np.uint8).copy()).cuda()
    res = torch.empty(n * 16, dtype=torch.uint8, device="cuda")
    eng.protect(d, n, d_in, d_out, res)
    torch.cuda.synchronize()
    r = res.cpu().numpy().view(L.RESULT)
    assert list(r["status"]) == list(eres["status"])
    want = [0 if len(h) + len(p) + 16 <= 1500 else L.S_LENGTH for h, p in zip(headers, payloads)]
    assert list(r["status"]) == want
    got = d_out.cpu().numpy()
    for i in range(n):
        if want[i] == 0:
            o, m = int(desc[i]["out_off"]), int(r[i]["out_len"])
            assert np.array_equal(got[o : o + m], exp[o : o + m])
    hp = HeaderProtection(b"aes-128-ecb", bytes(16))
    assert len(hp.apply(b"\x40" + bytes(10), bytes(1489))) == 1500
    with pytest.raises(CryptoError, match="Invalid payload length"):
        hp.apply(b"\x40" + bytes(10), bytes(1490))


def test_session_pipelined_unaligned_ragged(oracle, L, engine_cls):
    """The pipelined host path (>= 64 MiB of output) over ragged packets at
    odd offsets: chunk tiles start and end mid-word, so the library's D2H copy
    kernel (k_xfer) copies unaligned heads and tails of every tile.  Protect
    and unprotect through the host path must equal the device-resident launch
    on the same descriptors byte for byte, and the round trip must be exact."""
    import torch

    from aioquic_amd.batch import MultiDeviceEngine, layout_packets

    rng = np.random.default_rng(0x6A1)
    recs = _keys(rng, 5)
    n = 100000
    headers, payloads, pns, slots = _random_batch(rng, n, 5, recs, max_payload=1450)
    inbuf, desc, size = layout_packets(headers, payloads, pns, slots)
    assert size >= 64 << 20 and (desc["out_off"] % 16 != 0).sum() > n // 2
    host = MultiDeviceEngine(5, devices=[0])
    host.set_key_records(recs)
    host.trace(True)
    out_h, res_h = host.protect_host(desc, inbuf.tobytes(), size)
    assert host.trace()[0]["pipelined"] == 1
    dev = torch.device("cuda")
    eng = engine_cls(5)
    eng.set_key_records(recs)
    d_out = torch.zeros(size, dtype=torch.uint8, device=dev)
    d_res = torch.zeros(n * 16, dtype=torch.uint8, device=dev)
    eng.protect(torch.from_numpy(desc.view(np.uint8)).to(dev), n, torch.from_numpy(inbuf).to(dev), d_out, d_res)
    torch.cuda.synchronize()
    assert np.array_equal(out_h, d_out.cpu().numpy())
    assert res_h.tobytes() == d_res.cpu().numpy().tobytes()
    assert (res_h["status"] == L.S_OK).all()
    ud = desc.copy()
    ud["len"] = res_h["out_len"]
    ud["hdr_len"] = [len(h) - ((h[0] & 3) + 1) for h in headers]
    # 4-byte packet numbers up to 2^40: decode them unsigned (RFC 9000 A.3)
    # rather than with the reference's signed-int32 quirk (_crypto.c:349),
    # under which such packets fail to authenticate
    ud["flags"] |= L.F_RFC_PN
    back_h, r2_h = host.unprotect_host(ud, out_h.tobytes(), size)
    assert host.trace()[0]["pipelined"] == 1
    host.trace(False)
    d_back = torch.zeros(size, dtype=torch.uint8, device=dev)
    d_res2 = torch.zeros(n * 16, dtype=torch.uint8, device=dev)
    eng.unprotect(torch.from_numpy(ud.view(np.uint8)).to(dev), n, d_out, d_back, d_res2)
    torch.cuda.synchronize()
    assert np.array_equal(back_h, d_back.cpu().numpy())
    assert r2_h.tobytes() == d_res2.cpu().numpy().tobytes()
    assert (r2_h["status"] == L.S_OK).all()
    for i in range(0, n, 997):
        o, h, p = int(desc[i]["in_off"]), len(headers[i]), len(payloads[i])
        assert back_h[o : o + h + p].tobytes() == headers[i] + payloads[i], i
    # QPP_F_RFC_PN against the oracle's unsigned decode on a prefix (the
    # oracle's bitwise GHASH is slow), and the protect side too
    m = 2000
    o_wire, o_res = oracle.protect_batch(recs, desc[:m], inbuf, size)
    assert np.array_equal(o_res, res_h[:m])
    end = int(desc[m]["out_off"])
    assert np.array_equal(o_wire[:end], out_h[:end])
    o_back, o_res2 = oracle.unprotect_batch(recs, ud[:m], out_h, size)
    assert np.array_equal(o_res2, r2_h[:m])
    assert (o_res2["pn"] == np.array(pns[:m], np.uint64)).all()
    assert np.array_equal(o_back[:end], back_h[:end])


@pytest.mark.parametrize("mixed,n", [(False, 98304), (True, 98304), (False, 262144)],
                         ids=["3-chunks", "3-chunks-mixed", "tapered-13-chunks"])
def test_session_pipelined_host_batch(L, engine_cls, mixed, n):
    """Host-buffer batches of >= 64 MiB go through the session's three-stage
    pipeline (chunked H2D / kernels / D2H, qpp_engine.hip session_run_pipelined;
    from 8 regular chunks on, the first and last are cut into quarter /
    quarter / half pieces: 262144 packets, 315 MB, run as 13 chunks).
    Its output and results must equal the serial session path
    (QPP_SESSION_SERIAL=1) and the device-resident path byte for byte; a
    tampered packet in a late chunk reports its status in place; a
    non-monotone descriptor order (serial fallback) gives the same bytes."""
    import torch

    from aioquic_amd import bench_data

    kw = dict(mixed=[0, 2]) if mixed else {}
    w = bench_data.make_workload(n, suite=0, n_keys=7, seed=0x51 + int(mixed), **kw)
    eng = engine_cls(w.n_keys)
    eng.set_key_records(w.keys)
    plain = w.plain.tobytes()
    out_p, res_p = eng.protect_host(w.desc, plain, w.wire_size)
    os.environ["QPP_SESSION_SERIAL"] = "1"
    try:
        out_s, res_s = eng.protect_host(w.desc, plain, w.wire_size)
    finally:
        del os.environ["QPP_SESSION_SERIAL"]
    assert np.array_equal(out_p, out_s)
    assert res_p.tobytes() == res_s.tobytes()
    # caller-owned, reused buffers (protect_into), stale contents overwritten
    out_i = np.full(w.wire_size, 0xA5, np.uint8)
    res_i = np.zeros(n, dtype=L.RESULT)
    eng.protect_into(w.desc, w.plain, out_i, res_i)
    assert np.array_equal(out_i, out_p)
    assert res_i.tobytes() == res_p.tobytes()
    assert (res_p["status"] == L.S_OK).all()
    dev = torch.device("cuda")
    d_wire = torch.zeros(w.wire_size, dtype=torch.uint8, device=dev)
    d_res = torch.empty(n * 16, dtype=torch.uint8, device=dev)
    eng.protect(torch.from_numpy(w.desc.view(np.uint8)).to(dev), n,
                torch.from_numpy(w.plain).to(dev), d_wire, d_res)
    torch.cuda.synchronize()
    assert np.array_equal(d_wire.cpu().numpy(), out_p)
    # unprotect through the pipeline, one packet of the last chunk tampered
    wire = out_p.copy()
    bad = n - 5
    wire[int(w.udesc[bad]["in_off"]) + 600] ^= 1
    back, r = eng.unprotect_host(w.udesc, wire.tobytes(), w.plain_size)
    assert r["status"][bad] == L.S_DECRYPT
    ok = np.ones(n, bool)
    ok[bad] = False
    assert (r["status"][ok] == L.S_OK).all()
    assert (r["pn"][ok] == w.udesc["pn"][ok]).all()
    for i in (0, 1, n // 3, n // 2, n - 6, n - 1):
        o = int(w.udesc[i]["out_off"])
        ln = int(r["hdr_len"][i]) + int(r["out_len"][i])
        assert np.array_equal(back[o : o + ln], w.plain[o : o + ln])
    plain_ok = back.copy()
    po = int(w.udesc[bad]["out_off"])
    plain_ok[po : po + 1200] = 0
    ref = w.plain.copy()
    ref[po : po + 1200] = 0
    assert np.array_equal(plain_ok, ref)
    # reversed descriptor order: not monotone, served by the serial path
    rev = w.desc[::-1].copy()
    out_r, res_r = eng.protect_host(rev, plain, w.wire_size)
    assert np.array_equal(out_r, out_p)
    assert res_r.tobytes() == res_p[::-1].tobytes()
