"""Lone-packet kernels (k_lone_gcm / k_lone_chacha: one wave per packet, for
unplanned launches of up to a few thousand packets -- the object API's one
packet per call, small flushes) against the C oracle, chunk by chunk: every suite, short and long
headers, AEAD-only with associated data up to 1500 bytes, payloads from 0 to
the 1500-byte limit, tiny inputs, in-place operation, tampered tags and the
status paths (LENGTH, NO_KEY, KEY_PHASE).  Reference: _crypto.c:115-204 and
quic/crypto.py:75-116 through the same C ABI as the quad kernels."""

import os

import numpy as np
import pytest

from tests.golden_cases import short_header
from tests.test_gpu_parity import _keys, _random_batch

pytestmark = pytest.mark.gpu

CHUNK = 16


@pytest.fixture(scope="module")
def L():
    from aioquic_amd import layout

    return layout


def _chunks(n, rng, chunk=CHUNK):
    """Chunk sizes 1..chunk covering n packets (the lone kernels' launch sizes)."""
    out, i = [], 0
    while i < n:
        k = int(rng.integers(1, chunk + 1))
        out.append(slice(i, min(n, i + k)))
        i += k
    return out


def _check_round_trip(oracle, L, eng, recs, headers, payloads, pns, slots, rng, flags=0, chunk=CHUNK):
    from aioquic_amd.batch import layout_packets

    n_ok = 0
    for sl in _chunks(len(headers), rng, chunk):
        h, p, pn, s = headers[sl], payloads[sl], pns[sl], slots[sl]
        inbuf, desc, size = layout_packets(h, p, pn, s, flags=flags)
        out_g, res_g = eng.protect_host(desc, inbuf.tobytes(), size)
        out_o, res_o = oracle.protect_batch(recs, desc, inbuf, size)
        assert (res_g == res_o).all(), (res_g, res_o)
        assert np.array_equal(out_g, out_o), sl
        ud = desc.copy()
        ud["len"] = res_g["out_len"]
        if not flags:
            ud["hdr_len"] = [len(x) - ((x[0] & 3) + 1) for x in h]
            ud["pn"] = np.asarray(pn, np.uint64) + rng.integers(0, 50, size=len(pn)).astype(np.uint64)
        wire = out_g.copy()
        # a tampered packet in about every other chunk
        t = int(rng.integers(0, 2 * len(h)))
        if t < len(h) and res_g[t]["status"] == L.S_OK:
            o = int(desc[t]["out_off"]) + int(rng.integers(len(h[t]), int(res_g[t]["out_len"])))
            wire[o] ^= 1 << int(rng.integers(0, 8))
        u_g, r_g = eng.unprotect_host(ud, wire.tobytes(), size)
        u_o, r_o = oracle.unprotect_batch(recs, ud, wire, size)
        assert (r_g == r_o).all(), (sl, r_g, r_o)
        for j in range(len(h)):
            if r_g[j]["status"] == L.S_OK:
                o, ln = int(ud[j]["out_off"]), int(r_g[j]["out_len"])
                assert np.array_equal(u_g[o : o + ln], u_o[o : o + ln]), (sl, j)
                n_ok += 1
            elif r_g[j]["status"] == L.S_DECRYPT:
                # no plaintext after a failed tag (launches of <= 8 packets
                # split a packet over two waves, each zeroing its own blocks):
                # past the longest header (pn offset + 4) up to the tag, zeros
                o = int(ud[j]["out_off"])
                lo, hi = o + int(ud[j]["hdr_len"]) + 4, o + int(ud[j]["len"]) - 16
                assert not u_g[lo:hi].any(), (sl, j)
    return n_ok


@pytest.mark.parametrize("suites", [(0,), (1,), (2,), (0, 1, 2)], ids=["aes128", "aes256", "chacha", "mixed"])
def test_lone_random_packets_vs_oracle(oracle, L, suites):
    """Short and long headers, pn lengths 1-4, payloads 0..1400 B, several
    keys: protect and unprotect in launches of 1-16 packets."""
    from aioquic_amd.batch import PacketEngine

    rng = np.random.default_rng(0x10E + len(suites) + 7 * suites[0])
    recs = _keys(rng, 6, suites)
    eng = PacketEngine(6)
    eng.set_key_records(recs)
    headers, payloads, pns, slots = _random_batch(rng, 300, 6, recs)
    # the reference's 4-byte signed-pn quirk packets fail on both sides alike
    n_ok = _check_round_trip(oracle, L, eng, recs, headers, payloads, pns, slots, rng)
    assert n_ok > 200  # ~1 in 8 quirk packets, ~1 tampered per 2 chunks


@pytest.mark.parametrize("suite", [0, 1, 2])
def test_lone_aead_only_long_aad(oracle, L, suite):
    """AEAD.encrypt / decrypt (QPP_F_NO_HP) with associated data up to 1500
    bytes and data up to the 1500-byte limit: up to 188 GHASH / Poly1305
    blocks, three per lane, 24 associated-data groups."""
    from aioquic_amd.batch import PacketEngine

    rng = np.random.default_rng(0xAAD + suite)
    recs = _keys(rng, 2, (suite,))
    eng = PacketEngine(2)
    eng.set_key_records(recs)
    sizes = [(0, 0), (0, 1), (1, 0), (15, 1), (16, 16), (17, 47), (0, 1484), (1500, 0), (1500, 1484),
             (1000, 400), (63, 64), (64, 63), (300, 1200), (13, 3)]
    sizes += [(int(rng.integers(0, 1500)), int(rng.integers(0, 1485))) for _ in range(50)]
    aads = [rng.bytes(a) for a, _ in sizes]
    datas = [rng.bytes(b) for _, b in sizes]
    pns = [int(rng.integers(0, 1 << 62)) for _ in sizes]
    slots = [i % 2 for i in range(len(sizes))]
    _check_round_trip(oracle, L, eng, recs, aads, datas, pns, slots, rng, flags=L.F_NO_HP)


@pytest.mark.parametrize("suite", [0, 1, 2])
def test_lone_long_header_hp(oracle, L, suite):
    """Header protection with long headers (1000-1480 B, up to QPP_MAX_HDR
    with the packet's 1500-byte limit) and short payloads (clen < 20 and
    < 32: the sample then overlaps the tag), in launches of 1-8 packets (pair
    launches: for AES-GCM the header is past the first wave's 64 positions,
    so CT blocks 0-1 come from the second wave through LDS), both
    directions, against the oracle."""
    from aioquic_amd.batch import PacketEngine

    rng = np.random.default_rng(0x10A6 + suite)
    recs = _keys(rng, 3, (suite,))
    eng = PacketEngine(3)
    eng.set_key_records(recs)
    headers, payloads, pns, slots = [], [], [], []
    for i in range(96):
        pn_len = 1 + i % 4
        pn = int(rng.integers(0, 1 << 30))
        hlen = int(rng.choice([1000, 1008, 1023, 1024, 1200, 1399, 1400, 1450, 1479]))
        clen = int(rng.choice([4 - pn_len, 3, 7, 15, 16, 17, 19, 20, 24, 31, 32, 33, 40]))
        clen = max(4 - pn_len, min(clen, 1500 - 16 - hlen))
        # an Initial whose token pads the header to hlen
        fixed = 1 + 4 + 1 + 8 + 1 + 2 + 2 + pn_len
        tok = hlen - fixed
        hdr = (bytes([0xC0 | (pn_len - 1)]) + (1).to_bytes(4, "big") + b"\x08" + rng.bytes(8) + b"\x00" +
               bytes([0x40 | (tok >> 8), tok & 0xFF]) + rng.bytes(tok) + bytes([0x40 | ((clen + pn_len + 16) >> 8),
                                                                                    (clen + pn_len + 16) & 0xFF]) +
               (pn & ((1 << (8 * pn_len)) - 1)).to_bytes(pn_len, "big"))
        assert len(hdr) == hlen
        headers.append(hdr)
        payloads.append(rng.bytes(clen))
        pns.append(pn)
        slots.append(i % 3)
    n_ok = _check_round_trip(oracle, L, eng, recs, headers, payloads, pns, slots, rng, chunk=8)
    assert n_ok > 60


def test_lone_status_paths(oracle, L):
    """LENGTH (short data, pn offset 0), NO_KEY (empty and out-of-table
    slots), KEY_PHASE, DECRYPT, in one launch of 16 packets per suite."""
    from aioquic_amd.batch import PacketEngine, layout_packets

    rng = np.random.default_rng(0x5747)
    recs = _keys(rng, 3)
    eng = PacketEngine(4)
    eng.set_key_records(recs)
    n = 16
    headers = [short_header(rng.bytes(8), i, 2, 0) for i in range(n)]
    payloads = [rng.bytes(int(rng.integers(4, 1200))) for _ in range(n)]
    slots = [i % 3 for i in range(n)]
    inbuf, desc, size = layout_packets(headers, payloads, list(range(n)), slots)
    out, res = eng.protect_host(desc, inbuf.tobytes(), size)
    assert (res["status"] == L.S_OK).all()
    wire = out.copy()
    o = int(desc[2]["out_off"]) + int(res[2]["out_len"]) - 1
    wire[o] ^= 4  # the tag's last byte (beyond the HP sample): DECRYPT
    ud = desc.copy()
    ud["len"] = res["out_len"]
    ud["hdr_len"] = 9
    ud[3]["len"] = 25    # too short for header + tag
    ud[5]["slot"] = 3    # never installed
    ud[6]["slot"] = 9    # beyond the table
    ud[7]["hdr_len"] = 0
    u, r = eng.unprotect_host(ud, wire.tobytes(), size)
    uo, ro = oracle.unprotect_batch(recs, ud, wire, size)
    assert (r == ro).all()
    assert r[2]["status"] == L.S_DECRYPT and r[3]["status"] == L.S_LENGTH
    assert r[5]["status"] == L.S_NO_KEY and r[6]["status"] == L.S_NO_KEY
    assert r[7]["status"] == L.S_LENGTH
    recs2 = recs.copy()
    recs2[0]["key_phase"] = 1
    eng.set_key_records(recs2[:1])
    u, r = eng.unprotect_host(ud, wire.tobytes(), size)
    for i in range(0, n, 3):
        if i not in (3, 6):
            assert int(r[i]["status"]) == L.S_KEY_PHASE, i


def test_lone_matches_quad_kernels_on_device(L):
    """The same 16-packet device batch through the lone kernels and, in a child
    process with QPP_LONE=0, through the quad kernels: identical bytes."""
    import os
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = ("import sys; sys.path.insert(0, %r); from tests.test_gpu_lone import _device_digest; "
            "print('digest', _device_digest())" % root)
    outs = []
    for lone in ("1", "0"):
        r = subprocess.run([sys.executable, "-c", code], env=dict(os.environ, QPP_LONE=lone),
                           capture_output=True, text=True, timeout=180)
        assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
        outs.append([x for x in r.stdout.splitlines() if x.startswith("digest")][-1])
    assert outs[0] == outs[1]


def _device_digest():
    import hashlib

    import torch

    from aioquic_amd import bench_data
    from aioquic_amd.batch import PacketEngine

    h = hashlib.sha256()
    for suite in (0, 1, 2):
        w = bench_data.make_workload(16, suite=suite, n_keys=2, seed=0x1E + suite)
        eng = PacketEngine(w.n_keys)
        eng.set_key_records(w.keys)
        dev = torch.device("cuda")
        d_in = torch.from_numpy(w.plain).to(dev)
        d_desc = torch.from_numpy(w.desc.view(np.uint8)).to(dev)
        d_wire = torch.zeros(w.wire_size, dtype=torch.uint8, device=dev)
        d_res = torch.zeros(16 * 16, dtype=torch.uint8, device=dev)
        eng.protect(d_desc, 16, d_in, d_wire, d_res)
        d_udesc = torch.from_numpy(w.udesc.view(np.uint8)).to(dev)
        d_back = torch.zeros(w.plain_size, dtype=torch.uint8, device=dev)
        d_res2 = torch.zeros(16 * 16, dtype=torch.uint8, device=dev)
        eng.unprotect(d_udesc, 16, d_wire, d_back, d_res2)
        torch.cuda.synchronize()
        for t in (d_wire, d_res, d_back, d_res2):
            h.update(t.cpu().numpy().tobytes())
        assert np.array_equal(d_back.cpu().numpy(), w.plain)
    return h.hexdigest()


def test_lone_in_place(oracle, L):
    """out buffer == in buffer for a 16-packet device launch (the builder
    encrypts in place, packet_builder.py:341-350), then decrypt in place."""
    import torch

    from aioquic_amd.batch import PacketEngine, layout_packets

    rng = np.random.default_rng(0x19)
    recs = _keys(rng, 3)
    eng = PacketEngine(3)
    eng.set_key_records(recs)
    n = 16
    headers = [short_header(rng.bytes(8), i, 1 + i % 4, 0) for i in range(n)]
    payloads = [rng.bytes(int(rng.integers(4, 1400))) for _ in range(n)]
    inbuf, desc, size = layout_packets(headers, payloads, list(range(n)), [i % 3 for i in range(n)])
    exp, _ = oracle.protect_batch(recs, desc, inbuf, size)
    buf = torch.from_numpy(inbuf.copy()).cuda()
    d = torch.from_numpy(desc.view(np.uint8).copy()).cuda()
    res = torch.zeros(n * 16, dtype=torch.uint8, device="cuda")
    eng.protect(d, n, buf, buf, res)
    torch.cuda.synchronize()
    got = buf.cpu().numpy()
    for i in range(n):
        o, ln = int(desc[i]["out_off"]), len(headers[i]) + len(payloads[i]) + 16
        assert np.array_equal(got[o : o + ln], exp[o : o + ln]), i
    ud = desc.copy()
    ud["len"] = [len(h) + len(p) + 16 for h, p in zip(headers, payloads)]
    ud["hdr_len"] = [len(h) - ((h[0] & 3) + 1) for h in headers]
    eng.unprotect(torch.from_numpy(ud.view(np.uint8).copy()).cuda(), n, buf, buf, res)
    torch.cuda.synchronize()
    back = buf.cpu().numpy()
    r = res.cpu().numpy().view(L.RESULT)
    assert (r["status"] == L.S_OK).all()
    for i in range(n):
        o = int(desc[i]["out_off"])
        assert back[o : o + len(headers[i]) + len(payloads[i])].tobytes() == headers[i] + payloads[i], i


@pytest.mark.parametrize("switch", ["QPP_ZERO_COPY", "QPP_LONE_STAGE"])
def test_lone_through_staging_copies(switch):
    """The same small host calls with QPP_ZERO_COPY=0 (both copies of the
    session's staging, no writes into pinned memory from the kernel) or
    QPP_LONE_STAGE=0 (the input by a copy instead of the kernel's own staging
    read), in a child process, against the oracle."""
    import os
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = ("import sys; sys.path.insert(0, %r); from tests.test_gpu_lone import _child_check; _child_check()" % root)
    r = subprocess.run([sys.executable, "-c", code], env=dict(os.environ, **{switch: "0"}),
                       capture_output=True, text=True, timeout=180)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "lone child ok" in r.stdout


def _child_check():
    from aioquic_amd import layout as L
    from aioquic_amd.batch import PacketEngine
    from oracle import oracle as orc

    orc.lib()
    rng = np.random.default_rng(0xC0B1)
    recs = _keys(rng, 6)
    eng = PacketEngine(6)
    eng.set_key_records(recs)
    headers, payloads, pns, slots = _random_batch(rng, 120, 6, recs)
    _check_round_trip(orc, L, eng, recs, headers, payloads, pns, slots, rng)
    print("lone child ok")


def test_quad_kernels_at_small_sizes():
    """With the lone kernels taking unplanned launches of up to a few thousand
    packets, the quad kernels' small-launch paths (golden vectors, in place,
    tampering) run in a child process with QPP_LONE=0, against the oracle."""
    import os
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = ("import sys; sys.path.insert(0, %r); from tests.test_gpu_lone import _quad_child; _quad_child()" % root)
    r = subprocess.run([sys.executable, "-c", code], env=dict(os.environ, QPP_LONE="0"),
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "quad child ok" in r.stdout


def _quad_child():
    from aioquic_amd import layout as L
    from aioquic_amd.batch import PacketEngine
    from oracle import oracle as orc
    from tests import test_gpu_parity as T

    orc.lib()
    T.test_golden_vectors_batch(orc, L, PacketEngine)
    T.test_in_place(orc, L, PacketEngine)
    T.test_tamper_and_edge_status(orc, L, PacketEngine)
    rng = np.random.default_rng(0x0AD)
    recs = _keys(rng, 6)
    eng = PacketEngine(6)
    eng.set_key_records(recs)
    headers, payloads, pns, slots = _random_batch(rng, 120, 6, recs)
    _check_round_trip(orc, L, eng, recs, headers, payloads, pns, slots, rng)
    print("quad child ok")


@pytest.mark.parametrize("suite,n", [(0, 8192), (0, 8193), (1, 4096), (2, 64), (2, 65)],
                         ids=["aes128-8192-lone", "aes128-8193-quad", "aes256-4096-lone", "chacha-64-lone",
                              "chacha-65-quad"])
def test_lone_threshold_sizes_whole_batch(L, suite, n):
    """Device launches on either side of the lone / quad thresholds
    (launch_packets: 8192 AES-GCM, 64 ChaCha20-Poly1305 packets), every
    packet in both directions against the reference's own _crypto
    (tests/ref_crypto.py; the C oracle on a prefix without oracle/_ref)."""
    import torch

    from aioquic_amd import bench_data
    from aioquic_amd.batch import PacketEngine
    from tests import ref_crypto

    w = bench_data.make_workload(n, suite=suite, n_keys=3, seed=0x7E + n, order="random")
    eng = PacketEngine(w.n_keys)
    eng.set_key_records(w.keys)
    dev = torch.device("cuda")
    d_in = torch.from_numpy(w.plain).to(dev)
    d_wire = torch.zeros(w.wire_size, dtype=torch.uint8, device=dev)
    d_back = torch.zeros(w.plain_size, dtype=torch.uint8, device=dev)
    d_res = torch.zeros(n * 16, dtype=torch.uint8, device=dev)
    d_res2 = torch.zeros(n * 16, dtype=torch.uint8, device=dev)
    eng.protect(torch.from_numpy(w.desc.view(np.uint8)).to(dev), n, d_in, d_wire, d_res)
    eng.unprotect(torch.from_numpy(w.udesc.view(np.uint8)).to(dev), n, d_wire, d_back, d_res2)
    torch.cuda.synchronize()
    wire, back = d_wire.cpu().numpy(), d_back.cpu().numpy()
    r1, r2 = d_res.cpu().numpy().view(L.RESULT), d_res2.cpu().numpy().view(L.RESULT)
    assert (r1["status"] == 0).all() and (r2["status"] == 0).all()
    assert np.array_equal(back, w.plain)
    ref = ref_crypto.checker(os.environ.get("PYTEST_CURRENT_TEST", "?").split(" ")[0])
    if ref is not None:
        assert np.array_equal(ref_crypto.protect_all(ref, w), wire)
        r_back, r_pn = ref_crypto.unprotect_all(ref, w, wire)
        assert np.array_equal(r_back, back) and np.array_equal(r_pn, r2["pn"])
    else:
        from oracle import oracle as orc

        m = min(n, 512)
        o_wire, _ = orc.protect_batch(w.keys, w.desc[:m], w.plain, w.wire_size)
        assert np.array_equal(o_wire[: m * 1200], wire[: m * 1200])
