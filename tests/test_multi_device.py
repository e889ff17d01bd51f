"""Library-level multi-device host path (qpp_multi, aioquic_amd.batch.MultiDeviceEngine).

One host batch split into contiguous ranges, one session and key-table
replica per device; on the one-GPU box the "devices" are sessions on the same
GPU.  The bytes and results must equal one session's (PacketEngine) and the
oracle's, for protect and unprotect, mixed suites, rejected descriptors, and
a layout whose ranges would overlap (run on one device)."""

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _workload(n, seed):
    from aioquic_amd import bench_data

    return bench_data.make_workload(n, suite=0, n_keys=6, seed=seed, mixed=(0, 1, 2))


@pytest.mark.parametrize("devices", [[0, 0], [0, 0, 0]], ids=["2-sessions", "3-sessions"])
def test_multi_equals_single_session(oracle, devices):
    from aioquic_amd import layout as L
    from aioquic_amd.batch import MultiDeviceEngine, PacketEngine

    w = _workload(3001, 0x51)
    one = PacketEngine(w.n_keys)
    one.set_key_records(w.keys)
    multi = MultiDeviceEngine(w.n_keys, devices=devices)
    assert multi.multi.devices == len(devices)
    multi.set_key_records(w.keys)
    wire1, r1 = one.protect_host(w.desc, w.plain, w.wire_size)
    wire2, r2 = multi.protect_host(w.desc, w.plain, w.wire_size)
    assert (r1["status"] == L.S_OK).all()
    assert np.array_equal(wire1, wire2) and np.array_equal(r1, r2)
    exp, _ = oracle.protect_batch(w.keys, w.desc, w.plain, w.wire_size)
    assert np.array_equal(wire2, exp)
    back1, u1 = one.unprotect_host(w.udesc, wire1, w.plain_size)
    back2, u2 = multi.unprotect_host(w.udesc, wire2, w.plain_size)
    assert np.array_equal(back1, back2) and np.array_equal(u1, u2)
    assert np.array_equal(back2, w.plain)


def test_multi_rejects_and_overlap_like_one_session():
    from aioquic_amd import layout as L
    from aioquic_amd.batch import MultiDeviceEngine, PacketEngine

    w = _workload(800, 0x52)
    one = PacketEngine(w.n_keys)
    one.set_key_records(w.keys)
    multi = MultiDeviceEngine(w.n_keys, devices=[0, 0])
    multi.set_key_records(w.keys)
    d = w.desc.copy()
    d[5]["in_off"] = w.plain_size + 10  # outside the input: QPP_S_LENGTH, nothing touched
    d[600]["out_off"] = w.wire_size - 3  # output past the end
    a = one.protect_host(d, w.plain, w.wire_size)
    b = multi.protect_host(d, w.plain, w.wire_size)
    assert a[1][5]["status"] == L.S_LENGTH and a[1][600]["status"] == L.S_LENGTH
    assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])
    # descriptors out of output order: the ranges' extents overlap -> one device
    rev = w.desc[::-1].copy()
    a = one.protect_host(rev, w.plain, w.wire_size)
    b = multi.protect_host(rev, w.plain, w.wire_size)
    assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])


def test_multi_into_caller_buffers():
    """The caller-owned-buffer form (the bench's host path) writes the same
    bytes and results as the bytes-returning form."""
    from aioquic_amd import layout as L
    from aioquic_amd.batch import MultiDeviceEngine

    w = _workload(2048, 0x53)
    multi = MultiDeviceEngine(w.n_keys, devices=[0, 0])
    multi.set_key_records(w.keys)
    wire, r1 = multi.protect_host(w.desc, w.plain, w.wire_size)
    out = np.full(w.wire_size, 0xAA, np.uint8)
    res = np.zeros(len(w.desc), L.RESULT)
    multi.protect_into(w.desc, w.plain, out, res)
    assert np.array_equal(out, wire) and np.array_equal(res, r1)
    back = np.empty(w.plain_size, np.uint8)
    res2 = np.zeros(len(w.desc), L.RESULT)
    multi.unprotect_into(w.udesc, out, back, res2)
    assert (res2["status"] == 0).all() and np.array_equal(back, w.plain)


def test_multi_empty_middle_range_out_of_order():
    """A middle range whose packets are all rejected has no extent: the
    ranges around it must still be checked against each other.
    Descriptors by thirds in reverse output order, the middle third rejected:
    the outer ranges' extents are out of order, so the batch runs on one
    device, byte for byte as one session."""
    from aioquic_amd import layout as L
    from aioquic_amd.batch import MultiDeviceEngine, PacketEngine

    w = _workload(900, 0x54)
    one = PacketEngine(w.n_keys)
    one.set_key_records(w.keys)
    multi = MultiDeviceEngine(w.n_keys, devices=[0, 0, 0])
    multi.set_key_records(w.keys)
    d = np.concatenate([w.desc[600:], w.desc[300:600], w.desc[:300]]).copy()
    d["in_off"][300:600] = w.plain_size + 1  # every packet of range 1 rejected
    a = one.protect_host(d, w.plain, w.wire_size)
    b = multi.protect_host(d, w.plain, w.wire_size)
    assert (a[1]["status"][300:600] == L.S_LENGTH).all() and (a[1]["status"][:300] == L.S_OK).all()
    assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])


def test_trace_reports_pipeline_phases():
    """qpp_multi_trace / MultiDeviceEngine.trace: a host batch large enough
    for the chunked pipeline (>= 64 MiB of output) reports its phases, and
    tracing changes no byte.  Untraced and small calls report pipelined = 0."""
    from aioquic_amd import bench_data
    from aioquic_amd import layout as L
    from aioquic_amd.batch import MultiDeviceEngine

    n = 65536  # 75 MiB of wire
    w = bench_data.make_workload(n, suite=0, n_keys=1, seed=0x54)
    eng = MultiDeviceEngine(w.n_keys, devices=[0])
    eng.set_key_records(w.keys)
    wire0 = np.empty(w.wire_size, np.uint8)
    r0 = np.empty(n, L.RESULT)
    eng.protect_into(w.desc, w.plain, wire0, r0)
    assert eng.trace()[0]["pipelined"] == 0  # tracing was off
    eng.trace(True)
    wire = np.empty(w.wire_size, np.uint8)
    r1 = np.empty(n, L.RESULT)
    eng.protect_into(w.desc, w.plain, wire, r1)
    (t,) = eng.trace()
    assert np.array_equal(wire, wire0) and np.array_equal(r1, r0)
    assert t["pipelined"] == 1 and t["chunks"] >= 2
    assert t["in_bytes"] >= w.plain_size and t["out_bytes"] >= w.wire_size
    for k in ("total_ms", "submit_ms", "copy_in_ms", "copy_out_ms", "h2d_ms", "kernel_ms", "d2h_ms", "gpu_span_ms"):
        assert t[k] > 0, (k, t)
    assert t["total_ms"] >= t["submit_ms"] and t["gpu_span_ms"] >= max(t["h2d_ms"], t["kernel_ms"], t["d2h_ms"]) * 0.99
    back = np.empty(w.plain_size, np.uint8)
    r2 = np.empty(n, L.RESULT)
    eng.unprotect_into(w.udesc, wire, back, r2)
    assert eng.trace()[0]["pipelined"] == 1
    assert (r2["status"] == 0).all() and np.array_equal(back, w.plain)
    eng.trace(False)


def test_multi_pipelined_ranges_equal_one_session():
    """Large host batches split over two sessions (the one-GPU stand-in for two
    devices): each range is big enough for its session's chunked pipeline
    (D2H legs by k_xfer), the two run at once on their own threads, and the
    bytes and results equal one session's, both directions."""
    from aioquic_amd import bench_data
    from aioquic_amd import layout as L
    from aioquic_amd.batch import MultiDeviceEngine

    n = 160000  # 2 x ~96 MB of wire: both ranges pipelined
    w = bench_data.make_workload(n, suite=0, n_keys=3, seed=0x55, mixed=(0, 2))
    one = MultiDeviceEngine(w.n_keys, devices=[0])
    two = MultiDeviceEngine(w.n_keys, devices=[0, 0])
    for e in (one, two):
        e.set_key_records(w.keys)
    two.trace(True)
    outs = []
    for e in (one, two):
        wire = np.empty(w.wire_size, np.uint8)
        r1 = np.empty(n, L.RESULT)
        e.protect_into(w.desc, w.plain, wire, r1)
        back = np.empty(w.plain_size, np.uint8)
        r2 = np.empty(n, L.RESULT)
        e.unprotect_into(w.udesc, wire, back, r2)
        outs.append((wire, r1, back, r2))
    assert [t["pipelined"] for t in two.trace()] == [1, 1]
    two.trace(False)
    (w1, a1, b1, c1), (w2, a2, b2, c2) = outs
    assert np.array_equal(w1, w2) and a1.tobytes() == a2.tobytes()
    assert np.array_equal(b1, b2) and c1.tobytes() == c2.tobytes()
    assert (a2["status"] == L.S_OK).all() and (c2["status"] == L.S_OK).all()
    assert np.array_equal(b2, w.plain)
