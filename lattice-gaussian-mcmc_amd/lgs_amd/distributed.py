"""Multi-GPU IMHK: chains sharded over ranks, one collective for the statistics.

The reference parallelises only with ``multiprocessing.Pool`` over independent
chains, each reseeded with ``seed + 1000 * chain_id``
(``experiments/dimension_scaling.py:841-845, 879``) and stacked with
``np.vstack`` afterwards (``experiments/cryptographic_experiments.py:268``).
Here one process drives one GPU; global chain ids are split contiguously, and
because every draw is addressed by (seed, global chain, step, slot) the union of
the ranks' chains is bit-identical for any world size.  The only exchange is one
all-reduce (RCCL over xGMI with the "nccl" backend, gloo on CPU) of the integer
accumulators: accepted proposals and sum z / sum z^2 over kept states.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Callable

import numpy as np


def shard_range(n_total: int, rank: int, world: int):
    """Contiguous split of [0, n_total): (first, count) for `rank`."""
    base, rem = divmod(int(n_total), int(world))
    first = rank * base + min(rank, rem)
    return first, base + (1 if rank < rem else 0)


@dataclass
class ShardResult:
    accepts: int
    moments: np.ndarray  # 2*d int64: sum z_i, sum z_i^2 over kept states
    kept: int            # number of kept states


def gpu_compute(ctx, seed: int, d: int, *, thin: int = 1, flags: int = 0, device=None):
    """Per-rank compute on the HIP C-ABI: returns a callable for `imhk_sharded`.

    Chain state lives on the device (coordinate-major), every call continues
    the same chains."""
    import torch
    from . import _capi

    state = {}

    def compute(first_chain, n_chains, first_step, n_steps):
        dev = device if device is not None else torch.device("cuda", ctx.device)
        if not state:
            state["z"] = torch.zeros((d, n_chains), dtype=torch.int32, device=dev)
            state["lw"] = torch.zeros(n_chains, dtype=torch.float64, device=dev)
            state["init"] = torch.zeros(n_chains, dtype=torch.int32, device=dev)
        acc = torch.zeros(n_chains, dtype=torch.int64, device=dev)
        mom = torch.zeros(2 * d, dtype=torch.int64, device=dev)
        torch.cuda.synchronize(dev)
        ctx.imhk(seed, first_chain, n_chains, first_step, n_steps, thin, state["z"], state["lw"],
                 state["init"], acc, moments=mom,
                 flags=flags | _capi.LGS_DEVICE_PTRS | _capi.LGS_COORD_MAJOR)
        return ShardResult(int(acc.sum().item()), mom.cpu().numpy(), n_chains * (n_steps // thin))

    return compute


def imhk_sharded(compute: Callable, n_chains: int, n_steps: int, *, rank: int, world: int,
                 first_step: int = 1, group=None, device=None):
    """Run this rank's shard of an IMHK job and all-reduce the statistics.

    Returns (global accepts, global moments (2d int64), global kept states)."""
    import torch
    import torch.distributed as dist

    first, count = shard_range(n_chains, rank, world)
    r = compute(first_chain=first, n_chains=count, first_step=first_step, n_steps=n_steps)
    stats = torch.from_numpy(np.concatenate([[r.accepts, r.kept], r.moments]).astype(np.int64))
    if device is not None:
        stats = stats.to(device)
    if world > 1:
        dist.all_reduce(stats, group=group)  # the single collective
    s = stats.cpu().numpy()
    return int(s[0]), s[2:], int(s[1])
