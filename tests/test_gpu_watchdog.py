"""The kernels' bounded waits never leave a stale result.

Two waits inside the kernels are bounded as a watchdog: a wave waiting for a
GHASH table entry (k_gcm's tab_acquire) and the two waves of a packet in a
pair launch handing the tag over (k_lone_gcm, launches of <= 8 packets).  A
correct run never reaches either bound.  When one is reached, every packet
concerned reports QPP_S_INTERNAL (no plaintext left at out_off), never a
leftover QPP_S_OK from an earlier launch, and the object API raises
CryptoError -- the reference's convention that a failed call raises and
returns no bytes (_crypto.c:17-29, :148-152).

QPP_SPIN_LIMIT=0 (read once per process, so in a child process) makes every
bounded wait give up at once:
- k_gcm: no wave ever gets a table entry, so every packet of every launch,
  planned or not, must come back QPP_S_INTERNAL, into result buffers that
  were filled with QPP_S_OK records beforehand;
- pair launches: a wave gives up only if its partner has not yet reached the
  hand-over, so each packet is either QPP_S_INTERNAL (unprotect: zeroed
  plaintext) or QPP_S_OK and byte-equal to the oracle.
"""

import os
import subprocess
import sys

import numpy as np
import pytest

from tests.test_gpu_parity import _keys, _random_batch

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run_child(fn: str, **env):
    code = "import sys; sys.path.insert(0, %r); from tests.test_gpu_watchdog import %s; %s()" % (ROOT, fn, fn)
    r = subprocess.run([sys.executable, "-c", code], env=dict(os.environ, **env), capture_output=True, text=True,
                       timeout=240)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "child ok" in r.stdout
    return r.stdout


def test_table_watchdog_reports_internal():
    out = _run_child("_table_child", QPP_SPIN_LIMIT="0", QPP_LONE="0")
    assert "watchdog events" in out


def test_pair_watchdog_never_stale():
    _run_child("_pair_child", QPP_SPIN_LIMIT="0")


def test_pair_watchdog_fires():
    """The pair hand-over's give-up path, taken deterministically: the second
    wave of every pair launch sleeps before handing its share over
    (QPP_PAIR_DELAY, a test switch) while the first wave's wait is 0, so the
    first wave always gives up (flag 0 -> 4) and the second wave finds the
    flag taken: every packet QPP_S_INTERNAL, no plaintext on either wave, and
    the watchdog counts the events."""
    out = _run_child("_pair_forced_child", QPP_SPIN_LIMIT="0", QPP_PAIR_DELAY="64")
    assert "pair forced" in out


def _table_child():
    import torch

    from aioquic_amd import _crypto
    from aioquic_amd import layout as L
    from aioquic_amd.batch import PacketEngine, layout_packets
    from oracle import oracle as orc

    rng = np.random.default_rng(0xD06)
    recs = _keys(rng, 4, (0, 1))  # AES-GCM suites only: k_gcm holds the tables
    eng = PacketEngine(4)
    eng.set_key_records(recs)
    headers, payloads, pns, slots = _random_batch(rng, 300, 4, recs)
    inbuf, desc, size = layout_packets(headers, payloads, pns, slots)
    n = len(desc)
    dev = torch.device("cuda")
    ok = np.zeros(n, L.RESULT)  # a stale record would read as S_OK
    ok["out_len"] = 1
    for planned in (False, True):
        d_desc = torch.from_numpy(desc.view(np.uint8).copy()).to(dev)
        d_in = torch.from_numpy(inbuf.copy()).to(dev)
        d_out = torch.zeros(size, dtype=torch.uint8, device=dev)
        d_res = torch.from_numpy(ok.view(np.uint8).copy()).to(dev)
        plan = eng.bucket(d_desc, n) if planned else None
        eng.protect(d_desc, n, d_in, d_out, d_res, plan=plan)
        torch.cuda.synchronize()
        r = d_res.cpu().numpy().view(L.RESULT)
        assert (r["status"] == L.S_INTERNAL).all(), (planned, np.unique(r["status"]))
        assert (r["out_len"] == 0).all()
        # unprotect of a correct wire image: no plaintext anywhere
        wire, res_o = orc.protect_batch(recs, desc, inbuf, size)
        ud = desc.copy()
        ud["len"] = res_o["out_len"]
        ud["hdr_len"] = [len(x) - ((x[0] & 3) + 1) for x in headers]
        d_udesc = torch.from_numpy(ud.view(np.uint8).copy()).to(dev)
        d_wire = torch.from_numpy(wire.copy()).to(dev)
        d_back = torch.zeros(size, dtype=torch.uint8, device=dev)
        d_res2 = torch.from_numpy(ok.view(np.uint8).copy()).to(dev)
        plan = eng.bucket(d_udesc, n) if planned else None
        eng.unprotect(d_udesc, n, d_wire, d_back, d_res2, plan=plan)
        torch.cuda.synchronize()
        r2 = d_res2.cpu().numpy().view(L.RESULT)
        assert (r2["status"] == L.S_INTERNAL).all(), (planned, np.unique(r2["status"]))
        assert not d_back.cpu().numpy().any()
    # the host-buffer form maps it the same way
    _, r3 = eng.protect_host(desc, inbuf.tobytes(), size)
    assert (r3["status"] == L.S_INTERNAL).all()
    print("watchdog events", _crypto.watchdog_count())
    assert _crypto.watchdog_count() > 0
    print("table child ok")


def _pair_child():
    from aioquic_amd import layout as L
    from aioquic_amd._crypto import AEAD, CryptoError
    from aioquic_amd.batch import PacketEngine, layout_packets
    from oracle import oracle as orc

    orc.lib()
    rng = np.random.default_rng(0x9A1)
    recs = _keys(rng, 4, (0, 1))
    eng = PacketEngine(4)
    eng.set_key_records(recs)
    counts = {"ok": 0, "internal": 0}
    for rep in range(60):
        k = int(rng.integers(1, 9))  # pair launches: at most 8 packets
        headers, payloads, pns, slots = _random_batch(rng, k, 4, recs)
        inbuf, desc, size = layout_packets(headers, payloads, pns, slots)
        out_g, res_g = eng.protect_host(desc, inbuf.tobytes(), size)
        out_o, res_o = orc.protect_batch(recs, desc, inbuf, size)
        for j in range(k):
            st = int(res_g[j]["status"])
            assert st in (L.S_OK, L.S_INTERNAL, int(res_o[j]["status"])), st
            if st == L.S_OK:
                assert res_o[j]["status"] == L.S_OK
                o, ln = int(desc[j]["out_off"]), int(res_g[j]["out_len"])
                assert np.array_equal(out_g[o : o + ln], out_o[o : o + ln])
                counts["ok"] += 1
            elif st == L.S_INTERNAL:
                assert res_g[j]["out_len"] == 0
                counts["internal"] += 1
        ud = desc.copy()
        ud["len"] = res_o["out_len"]
        ud["hdr_len"] = [len(x) - ((x[0] & 3) + 1) for x in headers]
        u_g, r_g = eng.unprotect_host(ud, out_o.tobytes(), size)
        u_o, r_o = orc.unprotect_batch(recs, ud, out_o, size)
        for j in range(k):
            st = int(r_g[j]["status"])
            o = int(ud[j]["out_off"])
            if st == L.S_OK:
                assert r_o[j]["status"] == L.S_OK
                ln = int(r_g[j]["out_len"])
                assert np.array_equal(u_g[o : o + ln], u_o[o : o + ln])
                counts["ok"] += 1
            elif st == L.S_INTERNAL:
                # no plaintext: past the longest header (pn offset + 4) up to the tag
                lo, hi = o + int(ud[j]["hdr_len"]) + 4, o + int(ud[j]["len"]) - 16
                assert not u_g[lo:hi].any(), (rep, j)
                counts["internal"] += 1
            else:
                assert st == int(r_o[j]["status"])
    # the object API: correct bytes or CryptoError, never wrong bytes
    key, iv = rng.bytes(16), rng.bytes(12)
    aead = AEAD(b"aes-128-gcm", key, iv)
    for i in range(40):
        data, aad = rng.bytes(300 + i), rng.bytes(13)
        try:
            ct = aead.encrypt(data, aad, i)
        except CryptoError as e:
            assert "Internal error" in str(e)
            counts["internal"] += 1
            continue
        assert ct == orc.aead_encrypt(0, key, iv, data, aad, i)
        counts["ok"] += 1
    print("pair outcomes", counts)
    print("pair child ok")


def _pair_forced_child():
    from aioquic_amd import _crypto
    from aioquic_amd import layout as L
    from aioquic_amd._crypto import AEAD, CryptoError
    from aioquic_amd.batch import PacketEngine, layout_packets
    from oracle import oracle as orc

    orc.lib()
    rng = np.random.default_rng(0x9A2)
    recs = _keys(rng, 4, (0, 1))
    eng = PacketEngine(4)
    eng.set_key_records(recs)
    w0 = _crypto.watchdog_count()
    packets = 0
    for rep in range(12):
        k = int(rng.integers(1, 9))  # pair launches: at most 8 packets
        headers, payloads, pns, slots = _random_batch(rng, k, 4, recs)
        inbuf, desc, size = layout_packets(headers, payloads, pns, slots)
        _, res_g = eng.protect_host(desc, inbuf.tobytes(), size)
        out_o, res_o = orc.protect_batch(recs, desc, inbuf, size)
        ok = res_o["status"] == L.S_OK
        assert (res_g["status"][ok] == L.S_INTERNAL).all(), (rep, res_g["status"])
        assert (res_g["out_len"][ok] == 0).all()
        ud = desc.copy()
        ud["len"] = res_o["out_len"]
        ud["hdr_len"] = [len(x) - ((x[0] & 3) + 1) for x in headers]
        u_g, r_g = eng.unprotect_host(ud, out_o.tobytes(), size)
        for j in range(k):
            if not ok[j]:
                continue
            assert int(r_g[j]["status"]) == L.S_INTERNAL, (rep, j, int(r_g[j]["status"]))
            # no plaintext from either wave: past the longest header up to the tag
            o = int(ud[j]["out_off"])
            lo, hi = o + int(ud[j]["hdr_len"]) + 4, o + int(ud[j]["len"]) - 16
            assert not u_g[lo:hi].any(), (rep, j)
            packets += 2
    key, iv = rng.bytes(16), rng.bytes(12)
    aead = AEAD(b"aes-128-gcm", key, iv)
    for i in range(4):
        try:
            aead.encrypt(rng.bytes(300 + i), rng.bytes(13), i)
        except CryptoError as e:
            assert "Internal error" in str(e)
        else:
            raise AssertionError("a forced give-up returned bytes")
    fired = _crypto.watchdog_count() - w0
    assert fired >= packets, (fired, packets)
    print("pair forced", packets, "packets, watchdog events", fired)
    print("pair child ok")
