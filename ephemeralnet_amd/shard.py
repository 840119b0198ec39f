"""Record sharding across GPUs: records are independent, so a batch is split into
one contiguous record range per rank, balanced by bytes (not record count) so mixed-size batches
(C5: 512 B - 64 KiB) give every GPU the same work.  No collective touches the data path; ranks
only agree on timing (barrier / max) and optionally sum failure counts."""
from __future__ import annotations

from bisect import bisect_left
from typing import Sequence


def shard_ranges(lengths: Sequence[int], world: int) -> list[tuple[int, int]]:
    """Split records 0..n-1 into `world` contiguous [lo, hi) ranges with ~equal byte totals.
    Every record lands in exactly one range; ranges are ordered by rank."""
    n = len(lengths)
    if world <= 0:
        raise ValueError("world must be positive")
    prefix = [0]
    for L in lengths:
        prefix.append(prefix[-1] + int(L))
    total = prefix[-1]
    cuts = [0]
    for r in range(1, world):
        target = total * r // world
        # first record boundary at or after the byte target, never moving backwards
        k = bisect_left(prefix, target)
        k = min(max(k, cuts[-1]), n)
        cuts.append(k)
    cuts.append(n)
    return [(cuts[r], cuts[r + 1]) for r in range(world)]


def shard_of(lengths: Sequence[int], world: int, rank: int) -> tuple[int, int]:
    return shard_ranges(lengths, world)[rank]
