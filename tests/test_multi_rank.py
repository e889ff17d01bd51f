"""world_size-2 gloo checks of the multi-GPU path (CPU, no GPU needed).

The bench shards packets across ranks with no data-path collective
(SURVEY.md sec. 8(e)); only the barrier and the max-over-ranks time use gloo.
Here every rank builds its shard exactly as bench.py does, the ranks gather
their (slot, pn) sets, and rank 0 checks they are disjoint and together equal
the single-GPU workload of 2n packets.  Each shard is also a self-contained
batch (its own keys and descriptors round-trip through the oracle).
"""

import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

N_PER_RANK = 96


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, cfg, q):
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from aioquic_amd.bench_data import make_workload
        from aioquic_amd.shard import shard_range
        from oracle import oracle as orc

        first, n = shard_range(rank, world, N_PER_RANK)
        w = make_workload(n, suite=cfg["suite"], n_keys=cfg["n_keys"], seed=7,
                          mixed=cfg.get("mixed"), first_packet=first,
                          order=cfg.get("order", "grouped"))
        pairs = sorted(zip(w.desc["slot"].tolist(), w.desc["pn"].tolist()))
        gathered = [None] * world
        dist.all_gather_object(gathered, pairs)
        # each rank's shard is a whole batch of its own: protect and unprotect
        # it (the oracle stands in for the GPU launch here), then gather the
        # per-rank statuses and a checksum of the wire bytes
        wire, r1 = orc.protect_batch(w.keys, w.desc, w.plain, w.wire_size)
        back, r2 = orc.unprotect_batch(w.keys, w.udesc, wire, w.plain_size)
        v = back.reshape(n, 1200)[:, :1184]
        rt = bool(np.array_equal(v, w.plain.reshape(n, 1200)[:, :1184]))
        import hashlib

        mine = (int((r1["status"] != 0).sum()), int((r2["status"] != 0).sum()), rt,
                hashlib.sha256(wire.tobytes()).hexdigest())
        stats = [None] * world
        dist.all_gather_object(stats, mine)
        # the timing reduction bench.py performs (max over ranks)
        import torch

        t = torch.tensor([float(rank + 1)], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        if rank == 0:
            q.put((gathered, float(t.item()), stats))
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("cfg", [dict(suite=0, n_keys=1), dict(suite=1, n_keys=5),
                                 dict(suite=0, n_keys=4, mixed=(0, 2)),
                                 dict(suite=1, n_keys=9, order="random"),
                                 dict(suite=0, n_keys=6, mixed=(0, 2), order="random")],
                         ids=["aes128-1key", "aes256-5keys", "mixed-4keys", "aes256-random",
                              "mixed-random"])
def test_two_rank_shards_cover_the_stream(cfg):
    from aioquic_amd.bench_data import make_workload

    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, cfg, q)) for r in range(world)]
    for p in procs:
        p.start()
    gathered, tmax, stats = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert tmax == float(world)
    sets = [set(map(tuple, g)) for g in gathered]
    assert sets[0].isdisjoint(sets[1])
    whole = make_workload(world * N_PER_RANK, suite=cfg["suite"], n_keys=cfg["n_keys"], seed=7,
                          mixed=cfg.get("mixed"), order=cfg.get("order", "grouped"))
    assert sets[0] | sets[1] == set(zip(whole.desc["slot"].tolist(), whole.desc["pn"].tolist()))
    # per rank: every packet authenticated, round trip exact, distinct wire bytes
    for bad_p, bad_u, rt, _ in stats:
        assert (bad_p, bad_u, rt) == (0, 0, True)
    assert stats[0][3] != stats[1][3]


def test_shard_range_rejects_bad_rank():
    from aioquic_amd.shard import shard_range

    assert shard_range(3, 4, 10) == (30, 10)
    with pytest.raises(ValueError):
        shard_range(4, 4, 10)


def test_shard_protect_matches_oracle_per_rank(oracle):
    """Each shard is a self-contained batch: its keys and descriptors protect
    and unprotect on their own (oracle as the checker)."""
    from aioquic_amd.bench_data import make_workload
    from aioquic_amd.shard import shard_range

    for rank in range(2):
        first, n = shard_range(rank, 2, 32)
        w = make_workload(n, suite=2, n_keys=3, seed=11, first_packet=first)
        wire, res = oracle.protect_batch(w.keys, w.desc, w.plain, w.wire_size)
        assert (res["status"] == 0).all()
        back, res2 = oracle.unprotect_batch(w.keys, w.udesc, wire, w.plain_size)
        assert (res2["status"] == 0).all()
        v = back.reshape(n, 1200)[:, :1184]
        assert np.array_equal(v, w.plain.reshape(n, 1200)[:, :1184])


def test_bench_workload_label_follows_packet_override():
    """bench.py names the packet count it ran, not only the config's default."""
    import bench

    c2 = bench.CONFIGS["2"]
    assert bench._workload_name(c2, c2["n"]) == c2["name"]
    assert bench._workload_name(c2, 1 << 20) == "aes-128-gcm 1Mi x 1200B, 1 key"
    assert bench._workload_name(c2, 1 << 17) == "aes-128-gcm 128Ki x 1200B, 1 key"
