"""Multi-GPU plumbing: one process per GPU, the state batch sharded by rows.

The reference is a single process (``trpo_inksci.py:23``).  Here each rank owns a
contiguous, path-aligned block of the concatenated batch (so the discounted
scan needs no carry across ranks), every rank holds the full parameter vector,
and the engine all-reduces the per-rank FVP / gradient / loss partial sums with
RCCL (the engine's own communicator; ``torch.distributed`` is used only to
hand rank 0's RCCL id to the others and for barriers/timing).
"""
from __future__ import annotations

from typing import List, Optional, Sequence, Tuple

import numpy as np


def shard_bounds(n_total: int, world: int, starts: Optional[Sequence[int]] = None) -> List[Tuple[int, int]]:
    """Contiguous row ranges, one per rank.  With ``starts`` (1 = first step of a path),
    every cut is moved forward to the next path start so no path spans two ranks."""
    cuts = [0]
    st = None if starts is None else np.flatnonzero(np.asarray(starts))
    for r in range(1, world):
        target = (n_total * r) // world
        if st is not None and st.size:
            i = np.searchsorted(st, target)
            target = int(st[i]) if i < st.size else n_total
        cuts.append(max(cuts[-1], min(target, n_total)))
    cuts.append(n_total)
    return [(cuts[r], cuts[r + 1]) for r in range(world)]


def init_engine_comm(engine, rank: int, world: int, group=None):
    """Create the engine's RCCL communicator: rank 0 draws the id, torch.distributed
    broadcasts it (any backend, e.g. gloo), every rank joins."""
    if world <= 1:
        return
    import torch.distributed as dist
    obj = [engine.comm_unique_id() if rank == 0 else None]
    dist.broadcast_object_list(obj, src=0, group=group)
    engine.comm_init(obj[0], rank, world)


def broadcast_unique_id(uid_factory, rank: int, group=None) -> bytes:
    import torch.distributed as dist
    obj = [uid_factory() if rank == 0 else None]
    dist.broadcast_object_list(obj, src=0, group=group)
    return obj[0]
