"""Multi-GPU block replay (configs[4]): squares are independent units, so a
replay of N consecutive blocks is sharded across ranks with NO data-path
collective; only the 32-B DAHs are gathered at the end (for the caller to
compare with the stored DataHash, as app/test/integration_test.go:355-379
does per block).  One process per GPU (torch.distributed.run).
"""
from __future__ import annotations

from typing import Callable, List, Sequence


def shard_range(n: int, rank: int, world: int) -> range:
    """Contiguous, balanced shard of [0, n) for `rank` (sizes differ by <= 1)."""
    base, extra = divmod(n, world)
    start = rank * base + min(rank, extra)
    return range(start, start + base + (1 if rank < extra else 0))


def replay(n_blocks: int, dah_of: Callable[[int], bytes], rank: int, world: int,
           dist=None) -> List[bytes]:
    """Compute dah_of(i) for this rank's shard; gather every DAH on every rank
    (all_gather_object), in block order.  `dist` = torch.distributed or None."""
    mine = [(i, dah_of(i)) for i in shard_range(n_blocks, rank, world)]
    if dist is None or world == 1:
        return [d for _, d in mine]
    parts: List[Sequence] = [None] * world
    dist.all_gather_object(parts, mine)
    out = [None] * n_blocks
    for part in parts:
        for i, d in part:
            out[i] = d
    return out
