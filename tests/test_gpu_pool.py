"""The launch-wide item pool of the persistent GCM kernel (qpp_engine.hip,
PoolRing / k_gcm's pool argument).

A single-key AES-GCM launch of more than 4096 wave items (> 64 Ki packets)
runs 1024-thread workgroups whose contiguous shares leave the last 1/12 of the
items to a counter in one of the key table's 32 pool slots.  A slot is taken
only when the launch that held it before has completed, and that launch's
last workgroup zeroed it.  So launches on two streams, interleaved, more of
them than there are slots, must each process every packet exactly once:
every status OK and every output byte-equal to a launch run alone (which the
oracle's whole-batch parity tests pin), and the round trip exact.
"""

import ctypes
import glob
import os

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

pytestmark = pytest.mark.gpu


def test_pool_slots_many_launches_two_streams():
    import torch

    from aioquic_amd import bench_data
    from aioquic_amd import layout as L
    from aioquic_amd.batch import PacketEngine

    n = 65536 + 8192  # 4608 wave items: the 1024-thread shape
    w = bench_data.make_workload(n, suite=0, n_keys=1, seed=0x9007, version=1)
    eng = PacketEngine(w.n_keys)
    eng.set_key_records(w.keys)
    dev = torch.device("cuda")
    d_in = torch.from_numpy(w.plain).to(dev)
    d_desc = torch.from_numpy(w.desc.view(np.uint8)).to(dev)
    d_udesc = torch.from_numpy(w.udesc.view(np.uint8)).to(dev)
    ref = torch.zeros(w.wire_size, dtype=torch.uint8, device=dev)
    ref_res = torch.zeros(n * 16, dtype=torch.uint8, device=dev)
    eng.protect(d_desc, n, d_in, ref, ref_res)
    torch.cuda.synchronize()
    assert (ref_res.cpu().numpy().view(L.RESULT)["status"] == L.S_OK).all()

    lib = ctypes.CDLL(glob.glob(os.path.join(ROOT, "aioquic_amd", "libquicpp.so"))[0])
    lib.qpp_pool_fallbacks.restype = ctypes.c_uint64
    fb0 = lib.qpp_pool_fallbacks()
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    # 24 buffers per stream, every launch of a round enqueued before the round
    # synchronizes: 96 pooled launches in flight at once, three times the
    # ring's 32 slots, so launches find slots whose event has not fired
    # (skipped) and rounds where every slot is held (pool = null, static
    # shares only) -- each must still process every packet exactly once
    k = 24
    wires = [[torch.empty_like(ref) for _ in range(k)] for _ in streams]
    backs = [[torch.empty(w.plain_size, dtype=torch.uint8, device=dev) for _ in range(k)] for _ in streams]
    res = [[torch.empty(n * 32, dtype=torch.uint8, device=dev) for _ in range(k)] for _ in streams]
    launches = 0
    for rnd in range(3):  # 3 x 2 streams x 24 x (protect + unprotect) = 288 launches
        for si, st in enumerate(streams):
            with torch.cuda.stream(st):
                for b in range(k):
                    wires[si][b].fill_(0xA5)
                    backs[si][b].fill_(0x5A)
                    res[si][b].fill_(0xFF)
        for b in range(k):  # the two streams' launches interleaved
            for si, st in enumerate(streams):
                with torch.cuda.stream(st):
                    eng.protect(d_desc, n, d_in, wires[si][b], res[si][b][: n * 16], stream=st)
                    eng.unprotect(d_udesc, n, wires[si][b], backs[si][b], res[si][b][n * 16:], stream=st)
                    launches += 2
        torch.cuda.synchronize()
        for si in range(len(streams)):
            for b in range(k):
                assert torch.equal(wires[si][b], ref), (rnd, si, b)
                st = res[si][b].cpu().numpy().view(L.RESULT)
                assert (st["status"] == L.S_OK).all(), (rnd, si, b)
                back = backs[si][b].view(n, 1200)[:, :1184]
                assert torch.equal(back, d_in.view(n, 1200)[:, :1184]), (rnd, si, b)
    assert launches > 3 * 32
    # with 96 launches queued per round, some ran without a slot
    assert lib.qpp_pool_fallbacks() > fb0


def test_pool_planned_single_key():
    """A bucketed (planned) single-key launch takes the pool too: its pooled
    items index the plan's item list.  Against an unplanned launch of the
    same batch, whose outputs the oracle-pinned parity tests cover."""
    import torch

    from aioquic_amd import bench_data
    from aioquic_amd import layout as L
    from aioquic_amd.batch import PacketEngine

    n = 65536 + 12288 + 77  # > 4096 wave items, a ragged last item
    w = bench_data.make_workload(n, suite=1, n_keys=1, seed=0x9008, version=1)
    eng = PacketEngine(w.n_keys)
    eng.set_key_records(w.keys)
    dev = torch.device("cuda")
    d_in = torch.from_numpy(w.plain).to(dev)
    d_desc = torch.from_numpy(w.desc.view(np.uint8)).to(dev)
    d_udesc = torch.from_numpy(w.udesc.view(np.uint8)).to(dev)
    outs, backs, ress = [], [], []
    for planned in (False, True, True):
        wire = torch.full((w.wire_size,), 0xA5, dtype=torch.uint8, device=dev)
        back = torch.full((w.plain_size,), 0x5A, dtype=torch.uint8, device=dev)
        r1 = torch.zeros(n * 16, dtype=torch.uint8, device=dev)
        r2 = torch.zeros(n * 16, dtype=torch.uint8, device=dev)
        eng.protect(d_desc, n, d_in, wire, r1, plan=eng.bucket(d_desc, n) if planned else None)
        eng.unprotect(d_udesc, n, wire, back, r2, plan=eng.bucket(d_udesc, n) if planned else None)
        outs.append(wire)
        backs.append(back)
        ress.append((r1, r2))
    torch.cuda.synchronize()
    for i in (1, 2):
        assert torch.equal(outs[i], outs[0])
        assert torch.equal(backs[i], backs[0])
    for r1, r2 in ress:
        assert (r1.cpu().numpy().view(L.RESULT)["status"] == L.S_OK).all()
        assert (r2.cpu().numpy().view(L.RESULT)["status"] == L.S_OK).all()
    assert torch.equal(backs[0].view(n, 1200)[:, :1184], d_in.view(n, 1200)[:, :1184])
