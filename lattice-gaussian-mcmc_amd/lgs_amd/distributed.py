"""Multi-GPU IMHK: chains sharded over ranks, one collective for the statistics.

The reference parallelises only with ``multiprocessing.Pool`` over independent
chains, each reseeded with ``seed + 1000 * chain_id``
(``experiments/dimension_scaling.py:841-845, 879``) and stacked with
``np.vstack`` afterwards (``experiments/cryptographic_experiments.py:268``).
Here one process drives one GPU; global chain ids are split contiguously, and
because every draw is addressed by (seed, global chain, step, slot) the union of
the ranks' chains is bit-identical for any world size.  The only exchange is one
all-reduce (RCCL over xGMI with the "nccl" backend, gloo on CPU) of the integer
accumulators: accepted proposals and sum z / sum z^2 over kept states (plus,
on request, the exact d x d second-moment matrix sum z z^T -- SURVEY §2.2 K4, about
8 MB at d = 1024), and one all-gather of per-chain scalar statistics (mean and
sum of squared deviations of a chosen coordinate over each chain's kept states)
for the Gelman-Rubin statistic across every chain of the job.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Callable, Optional

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
    gram: Optional[np.ndarray] = None         # d x d int64: sum z z^T over kept states
    chain_stats: Optional[np.ndarray] = None  # n_chains x 2 float64: mean, sum (x - mean)^2


@dataclass
class JobStats:
    accepts: int
    moments: np.ndarray
    kept: int
    gram: Optional[np.ndarray] = None
    chain_stats: Optional[np.ndarray] = None  # all chains of the job, global order

    def covariance(self) -> np.ndarray:
        """Unbiased covariance of the kept coefficient vectors (np.cov convention)."""
        d = self.moments.size // 2
        s = self.moments[:d].astype(np.float64)
        return (self.gram.astype(np.float64) - np.outer(s, s) / self.kept) / (self.kept - 1)

    def gelman_rubin(self, n_per_chain: int) -> float:
        """R-hat of convergence_diag.py:176-213 from the gathered per-chain statistics."""
        m = self.chain_stats.shape[0]
        n = n_per_chain
        means = list(self.chain_stats[:, 0])
        overall = np.mean(means)
        B = n / (m - 1) * sum((mu - overall) ** 2 for mu in means)
        W = np.mean([c0 / (n - 1) for c0 in self.chain_stats[:, 1]])
        return float(np.sqrt((((n - 1) / n) * W + (1 / n) * B) / W))


def gpu_compute(ctx, seed: int, d: int, *, thin: int = 1, flags: int = 0, device=None,
                want_gram: bool = False, gr_coord: Optional[int] = None):
    """Per-rank compute on the HIP C-ABI: returns a callable for `imhk_sharded`.

    Chain state lives on the device (coordinate-major), every call continues
    the same chains.  want_gram: exact sum z z^T of the kept states (lgs_gram);
    gr_coord: per-chain mean / squared deviations of that coordinate over the kept
    states (lgs_series_stats) for Gelman-Rubin."""
    import torch
    from . import _capi

    state = {}

    def compute(first_chain, n_chains, first_step, n_steps):
        dev = device if device is not None else torch.device("cuda", ctx.device)
        if not state:
            state["z"] = torch.zeros((n_chains, d), dtype=torch.int32, device=dev)
            state["lw"] = torch.zeros(n_chains, dtype=torch.float64, device=dev)
            state["init"] = torch.zeros(n_chains, dtype=torch.int32, device=dev)
        acc = torch.zeros(n_chains, dtype=torch.int64, device=dev)
        mom = torch.zeros(2 * d, dtype=torch.int64, device=dev)
        keep = n_steps // thin
        need_trace = want_gram or gr_coord is not None
        zs = torch.zeros((n_chains, keep, d), dtype=torch.int32, device=dev) if need_trace else None
        torch.cuda.synchronize(dev)
        ctx.imhk(seed, first_chain, n_chains, first_step, n_steps, thin, state["z"], state["lw"],
                 state["init"], acc, z_samples=zs, moments=mom, flags=flags | _capi.LGS_DEVICE_PTRS)
        gram = cs = None
        if want_gram:
            g = torch.zeros((d, d), dtype=torch.int64, device=dev)
            ctx.gram(zs.reshape(-1, d), gram_out=g, flags=_capi.LGS_DEVICE_PTRS)
            gram = g.cpu().numpy()
        if gr_coord is not None:
            mean = torch.empty(n_chains, dtype=torch.float64, device=dev)
            c0 = torch.empty(n_chains, dtype=torch.float64, device=dev)
            view = zs.reshape(-1)[gr_coord:]
            ctx.series_stats(view, n_chains, keep, 1, keep * d, 0, d, max_lag=0, mean=mean, c0=c0,
                             flags=_capi.LGS_DEVICE_PTRS)
            cs = torch.stack([mean, c0], 1).cpu().numpy()
        return ShardResult(int(acc.sum().item()), mom.cpu().numpy(), n_chains * keep, gram, cs)

    return compute


def imhk_sharded(compute: Callable, n_chains: int, n_steps: int, *, rank: int, world: int,
                 first_step: int = 1, group=None, device=None):
    """Run this rank's shard of an IMHK job and combine the statistics.

    One all-reduce of the integer accumulators (accepts, kept, moments and, when
    the shards computed it, the d x d second-moment matrix) and, when the shards
    computed per-chain statistics, one all-gather of them (padded to the largest
    shard), returned in global chain order.  Returns JobStats."""
    import torch
    import torch.distributed as dist

    first, count = shard_range(n_chains, rank, world)
    r = compute(first_chain=first, n_chains=count, first_step=first_step, n_steps=n_steps)
    parts = [[r.accepts, r.kept], r.moments.ravel()]
    if r.gram is not None:
        parts.append(r.gram.ravel())
    stats = torch.from_numpy(np.concatenate(parts).astype(np.int64))
    if device is not None:
        stats = stats.to(device)
    if world > 1:
        dist.all_reduce(stats, group=group)  # the single reduction
    s = stats.cpu().numpy()
    d2 = r.moments.size
    gram = None
    if r.gram is not None:
        d = d2 // 2
        gram = s[2 + d2:].reshape(d, d)
    chain_stats = None
    if r.chain_stats is not None:
        width = max(shard_range(n_chains, k, world)[1] for k in range(world))
        buf = np.zeros((width, 2))
        buf[:count] = r.chain_stats
        t = torch.from_numpy(buf)
        if device is not None:
            t = t.to(device)
        if world > 1:
            out = [torch.zeros_like(t) for _ in range(world)]
            dist.all_gather(out, t, group=group)  # the single gather
        else:
            out = [t]
        chain_stats = np.concatenate([o.cpu().numpy()[:shard_range(n_chains, k, world)[1]]
                                      for k, o in enumerate(out)])
    return JobStats(int(s[0]), s[2:2 + d2], int(s[1]), gram, chain_stats)
