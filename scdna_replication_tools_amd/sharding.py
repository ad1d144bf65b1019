"""Cell sharding across ranks (one process per GPU, torch.distributed over RCCL).

The PERT log joint factorises over cells given the shared sites (per-bin rho, global
a / lambda / beta_means / beta_stds, pert_model.py:553-574), so cells are split into
contiguous, balanced ranges with every bin on every rank.  Per SVI step the only
exchange is one sum all-reduce of the shared-gradient block (engine.PertShard
``grad_shared``: d loss / d shared params, then the loss); global priors are added by
the root rank only (``is_root``).
"""
from __future__ import annotations

from typing import Callable, List, Optional, Tuple

import numpy as np


def cell_bounds(n_cells: int, world: int) -> List[Tuple[int, int]]:
    """Contiguous [start, end) ranges, sizes differing by at most one cell."""
    if world < 1 or n_cells < world:
        raise ValueError("need at least one cell per rank ({} cells, {} ranks)".format(n_cells, world))
    b = np.linspace(0, n_cells, world + 1).round().astype(int)
    return [(int(b[i]), int(b[i + 1])) for i in range(world)]


def shard_slice(n_cells: int, world: int, rank: int) -> slice:
    s, e = cell_bounds(n_cells, world)[rank]
    return slice(s, e)


def make_allreduce(group=None) -> Optional[Callable]:
    """Sum all-reduce over ``group`` (None when not distributed or world size 1)."""
    import torch.distributed as dist
    if not dist.is_available() or not dist.is_initialized() or dist.get_world_size(group) == 1:
        return None

    def allreduce(t):
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
    return allreduce
