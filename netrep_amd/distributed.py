"""Multi-GPU sharding of the permutation procedure (one process per GPU).

Permutations are independent: the reference splits nPerm into contiguous
per-thread chunks, remainder to the first threads (src/permutations.cpp:
338-354), and merges runs by concatenating nulls along the permutation axis
(combineAnalyses, R/multi-machine.R:114). Here a rank plays a thread: it gets
the same contiguous chunk of global permutation indices, and because each
permutation's shuffle is keyed by (seed, global index) the merged cube is
bitwise identical for any number of ranks.

The only collectives are setup-time broadcasts of the test matrices (RCCL over
xGMI with backend "nccl"; gloo on CPU in tests) and the final gather of the
null slices to rank 0. There is no collective on the data path.
"""
from __future__ import annotations

import numpy as np


def perm_range(rank: int, world: int, n_perm: int):
    """[begin, end) of rank's contiguous chunk (src/permutations.cpp:338-354)."""
    base, rem = divmod(int(n_perm), int(world))
    begin = rank * base + min(rank, rem)
    return begin, begin + base + (1 if rank < rem else 0)


def broadcast_tensors(tensors, src: int = 0):
    """Broadcast a list of same-device tensors from `src` (in place)."""
    import torch.distributed as dist
    for t in tensors:
        dist.broadcast(t, src=src)


def gather_nulls(local_nulls: np.ndarray, rank: int, world: int, n_perm: int, dst: int = 0):
    """Concatenate each rank's (rows, stats, chunk) null slice along the
    permutation axis on `dst` (combineAnalyses' abind(..., along=3)).
    Returns the full cube on dst, None elsewhere."""
    import torch
    import torch.distributed as dist
    rows, stats = local_nulls.shape[:2]
    width = max(perm_range(r, world, n_perm)[1] - perm_range(r, world, n_perm)[0] for r in range(world))
    buf = np.full((width, rows, stats), np.nan)
    buf[: local_nulls.shape[2]] = np.moveaxis(local_nulls, 2, 0)
    t = torch.from_numpy(buf)
    if dist.get_backend() == "nccl":
        t = t.cuda()
    out = [torch.empty_like(t) for _ in range(world)] if rank == dst else None
    dist.gather(t, out, dst=dst)
    if rank != dst:
        return None
    parts = []
    for r in range(world):
        b, e = perm_range(r, world, n_perm)
        parts.append(out[r].cpu().numpy()[: e - b])
    return np.asfortranarray(np.moveaxis(np.concatenate(parts, axis=0), 0, 2))
