"""Packet sharding across GPUs.

Packets are independent, so a batch splits into contiguous ranges of the
global packet stream, one per rank, with no collective on the data path.
Rank r of `world` owns global packets [r * n_per_rank, (r + 1) * n_per_rank);
packet i uses key slot i mod n_keys and packet number i // n_keys, so the union
over ranks is exactly the single-GPU workload of world * n_per_rank packets.
"""


def shard_range(rank: int, world: int, n_per_rank: int) -> tuple[int, int]:
    if not (0 <= rank < world) or n_per_rank < 0:
        raise ValueError("bad shard arguments")
    return rank * n_per_rank, n_per_rank
