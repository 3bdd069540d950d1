"""Multi-GPU partitioning of the hot path.

Windows are independent, so N GPUs split the clip index space with no
collective on the data path: rank r of R owns a contiguous range of global
clip indices.  The synthetic generator is keyed on the GLOBAL clip index, so a
sharded run reproduces the unsharded run clip for clip.  torch.distributed is
used only for the start/stop barriers and the max-over-ranks timing.
"""
from typing import Tuple


def shard_range(n_total: int, rank: int, world: int) -> Tuple[int, int]:
    """(first, count) of rank's clips when n_total clips are split over world
    ranks as evenly as possible (the first n_total % world ranks get one more)."""
    if world <= 0 or not 0 <= rank < world or n_total < 0:
        raise ValueError(f"bad shard request: n_total={n_total} rank={rank} world={world}")
    base, extra = divmod(n_total, world)
    first = rank * base + min(rank, extra)
    return first, base + (1 if rank < extra else 0)


def weak_shard(batch_per_rank: int, rank: int) -> Tuple[int, int]:
    """Weak scaling (bench.py): every rank processes batch_per_rank clips,
    rank r the global indices [r*batch_per_rank, (r+1)*batch_per_rank)."""
    return rank * batch_per_rank, batch_per_rank
