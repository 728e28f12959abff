"""Multi-GPU IMHK: chains sharded over ranks, one collective for the statistics.

The reference parallelises only with ``multiprocessing.Pool`` over independent
chains, each reseeded with ``seed + 1000 * chain_id``
(``experiments/dimension_scaling.py:841-845, 879``) and stacked with
``np.vstack`` afterwards (``experiments/cryptographic_experiments.py:268``).
Here one process drives one GPU; global chain ids are split contiguously, and
because every draw is addressed by (seed, global chain, step, slot) the union of
the ranks' chains is bit-identical for any world size.  The only exchange is one
all-reduce (RCCL over xGMI with the "nccl" backend, gloo on CPU) of the
accumulators, packed into one fp64 tensor (``allreduce_parts``; int64 sums split
into exact 32-bit halves): accepted proposals and sum z / sum z^2 over kept
states, plus on request the exact d x d second-moment matrix sum z z^T (SURVEY
§2.2 K4, about 8 MB at d = 1024) or the lag-L autocovariance sums of scalar
functionals of the kept states (``LagSums``); and one all-gather of
per-chain scalar statistics (mean and sum of squared deviations of a chosen
coordinate over each chain's kept states) for the Gelman-Rubin statistic.

Two drivers share that reduction: ``imhk_sharded`` (one job, statistics back on
the host) and ``StreamingShard`` (the benchmark's timed path: chains advanced
block by block on the device, lag sums carried across blocks, one all-reduce at
the end).  Both take the per-rank compute as a callable, so the CPU tests drive
them with the oracle over gloo and the GPU path with the HIP C-ABI over RCCL.

The collective is deliberately host-side ``torch.distributed`` rather than a
C-ABI entry: the process group owns the RCCL communicator (one
process per GPU), and the reduced data is a few KB once per job.
"""
from __future__ import annotations

import os
import socket
from dataclasses import dataclass
from typing import Callable, Optional

import numpy as np


def shard_range(n_total: int, rank: int, world: int):
    """Contiguous split of [0, n_total): (first, count) for `rank`."""
    base, rem = divmod(int(n_total), int(world))
    first = rank * base + min(rank, rem)
    return first, base + (1 if rank < rem else 0)


def collective_active() -> bool:
    """A torch.distributed process group is initialised (any world size, 1 included:
    the all-reduce then runs through the backend too)."""
    import torch.distributed as dist
    return dist.is_available() and dist.is_initialized()


def init_process_group(backend: str, local_rank: int, world: int, rank: int = 0):
    """Initialise torch.distributed for this rank: "nccl" (= RCCL on ROCm) binds the
    communicator to cuda:local_rank; gloo on CPU.  Without a launcher's environment
    a one-rank group gets a private TCP store on 127.0.0.1; several ranks need the
    launcher's MASTER_ADDR / MASTER_PORT (a per-process random port would leave
    every rank waiting at its own rendezvous)."""
    import torch
    import torch.distributed as dist
    kw = {}
    if "RANK" not in os.environ or "WORLD_SIZE" not in os.environ:
        kw = dict(rank=rank, world_size=world)
    if "MASTER_ADDR" not in os.environ or "MASTER_PORT" not in os.environ:
        if world > 1:
            raise RuntimeError(f"world size {world} needs MASTER_ADDR and MASTER_PORT in the environment "
                               "(e.g. python -m torch.distributed.run --master-addr 127.0.0.1 ...)")
        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
        s.close()
        kw["init_method"] = f"tcp://127.0.0.1:{port}"
    if backend == "nccl":
        torch.cuda.set_device(local_rank)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank), **kw)
    else:
        dist.init_process_group(backend, **kw)


def pack_f64(torch, parts):
    """One fp64 tensor for the single all-reduce: int64 parts split into exact
    32-bit halves (each sum of halves over <= 2^20 ranks stays below 2^53)."""
    out, layout = [], []
    for p in parts:
        if p.dtype == torch.int64:
            out += [(p >> 32).double(), (p & 0xFFFFFFFF).double()]
            layout.append(("i", p.numel(), tuple(p.shape)))
        else:
            out.append(p.double().reshape(-1))
            layout.append(("f", p.numel(), tuple(p.shape)))
    return torch.cat([o.reshape(-1) for o in out]), layout


def unpack_f64(torch, flat, layout):
    res, o = [], 0
    for kind, n, shape in layout:
        if kind == "i":
            hi, lo = flat[o:o + n], flat[o + n:o + 2 * n]
            res.append(((hi.round().long() << 32) + lo.round().long()).reshape(shape))
            o += 2 * n
        else:
            res.append(flat[o:o + n].reshape(shape))
            o += n
    return res


def allreduce_parts(parts, group=None):
    """Sum a list of int64 / fp64 tensors (one device) over all ranks with ONE
    all-reduce; int64 parts stay exact.  Without a process group: the local values."""
    import torch
    import torch.distributed as dist
    flat, layout = pack_f64(torch, parts)
    if collective_active():
        dist.all_reduce(flat, group=group)  # the single collective (RCCL over xGMI / gloo)
    return unpack_f64(torch, flat, layout)


class LagSums:
    """Lag-L autocovariance sums of per-chain scalar series, continued across
    blocks through a ring of each chain's last L values.  int64 sums
    (exact, order-independent) for integer series, fp64 otherwise.  One update is a
    handful of device kernels: the ring starts as zeros, so pairs reaching before
    the first step contribute nothing and only the pair counts (host integers)
    need the history length."""

    def __init__(self, torch, n_chains, L, dtype, device):
        self.t, self.L = torch, L
        self.ring = torch.zeros((n_chains, L), dtype=dtype, device=device)
        self.have = 0
        # one buffer [S | S1] (the library's fused update adds to it in place)
        self.sums = torch.zeros(L + 2, dtype=dtype, device=device)
        self.S = self.sums[:L + 1]                                 # sum_t x_t x_{t-k}
        self.N = np.zeros(L + 1, dtype=np.int64)                  # pairs per lag
        self.S1 = self.sums[L + 1:]
        self.n = 0

    def update(self, x):
        self.update_device(x)
        self.update_host(*x.shape)

    def update_device(self, x):
        """The device part: sums and ring updated in place (graph-capturable)."""
        torch, L = self.t, self.L
        T = x.shape[1]
        xs = torch.cat([self.ring, x], 1)                      # (nc, L + T)
        win = xs.unfold(1, T, 1).flip(1)                       # win[:, k] = xs[:, L - k : L - k + T]
        # (the time axis first -- the contiguous one -- then the chains: one reduction
        # over both axes runs as a strided reduction with a few dozen workgroups)
        self.S += (win * x[:, None, :]).sum(2).sum(0)
        self.S1 += x.sum()
        self.ring.copy_(xs[:, T:] if T < L else x[:, T - L:])

    def update_host(self, nc, T):
        """The host part: pair counts (the ring starts as zeros, so pairs reaching
        before the first step add nothing to S but must not be counted)."""
        k = np.arange(self.L + 1)
        self.N += nc * np.maximum(T - np.maximum(k - self.have, 0), 0)
        self.n += nc * T
        self.have = min(self.L, self.have + T)

    def parts(self):
        t = self.t
        dev = self.S.device
        return [self.S, t.from_numpy(self.N).to(dev), self.S1, t.tensor([self.n], dtype=t.int64, device=dev)]

    @staticmethod
    def acf(S, N, S1, n):
        """ACF_k = (mean of lag-k products - mean^2) / (mean of squares - mean^2)."""
        m = S1 / n
        c = S / np.maximum(N, 1) - m * m
        return (c / c[0]).tolist() if c[0] > 0 else None


class StreamingShard:
    """One rank's shard of a streaming IMHK job -- the benchmark's timed path.

    ``advance(first_step, n_steps, acc, mom)`` advances this rank's chains by
    n_steps (adding accepted proposals per chain to ``acc`` and sum z / sum z^2 of
    the kept states to ``mom``) and returns their kept lattice points v
    (n_chains x n_steps x d, fp64 tensor), or a dict with the two functionals
    computed by the library ("zk": n_chains x n_steps int64, "vn2": ||v||^2 fp64 --
    gpu_advance, lgs_imhk_ex), or None.  The shard carries the lag-L
    autocovariance sums of two scalar functionals of the first ``lag_chains``
    chains' kept states -- the coefficient z_k = round(<binv_row, v>) and
    1e-6 ||v||^2 -- across blocks, and ``reduce`` combines everything over the
    ranks with one all-reduce.

    ``gram_every`` = k > 0 (needs ``advance.gram(G, S)``, which ADDS sum z z^T and
    sum z over the chains' current states to int64 G (d x d) / S (d)): after every
    k-th block the states the chains hold at that block's end -- kept states,
    thinned to one per chain per k blocks -- enter an exact second-moment sum, so
    the job's empirical covariance (base.py:154-160) comes back from the same
    single all-reduce (``covariance``)."""

    def __init__(self, advance: Callable, n_chains: int, d: int, *, binv_row, device, lag_chains: int = 1024,
                 lags: int = 16, first_step: int = 1, gram_every: int = 0, fused_lag: bool = True):
        import torch
        self.t = torch
        self.advance = advance
        self.nc, self.d, self.dev = n_chains, d, device
        self.lag_chains = min(n_chains, lag_chains)
        self.lags = lags
        if gram_every and not hasattr(advance, "gram"):
            raise ValueError("gram_every needs an advance callable with a gram(G, S) method")
        self.gram_every = int(gram_every)
        self.fused_lag = fused_lag
        self.binv = torch.as_tensor(np.asarray(binv_row, dtype=np.float64)).to(device)
        self.next_step = first_step
        # the per-block lag-sum update is ~20 small kernels; on a GPU it is replayed
        # as one captured graph from the second block on (the host would otherwise
        # launch them one by one after lgs_imhk's final synchronisation, with the
        # GPU idle in between).  LGS_NO_GRAPH=1: eager.
        self._graph = None
        self._graph_key = None
        self._graph_ok = str(device).startswith("cuda") and os.environ.get("LGS_NO_GRAPH", "0") != "1"
        self.reset_stats()

    def reset_stats(self):
        t = self.t
        self.acc = t.zeros(self.nc, dtype=t.int64, device=self.dev)
        self.mom = t.zeros(2 * self.d, dtype=t.int64, device=self.dev)
        self.lag_z = LagSums(t, self.lag_chains, self.lags, t.int64, self.dev)
        self.lag_v = LagSums(t, self.lag_chains, self.lags, t.float64, self.dev)
        # an advance that continues the lag sums itself (gpu_advance: inside lgs_imhk_ex,
        # before its final synchronisation) gets the sums' device buffers
        self._fused_lag = False
        if hasattr(self.advance, "bind_lag"):
            self._fused_lag = self.advance.bind_lag(self.lag_z if self.fused_lag else None, self.lag_v,
                                                    self.lag_chains, self.lags, 1e-6)
        self.steps_done = 0
        self.blocks = 0
        if self.gram_every:
            self.G = t.zeros((self.d, self.d), dtype=t.int64, device=self.dev)
            self.S = t.zeros(self.d, dtype=t.int64, device=self.dev)
            self.n_gram = 0
        self._graph = None  # captured against the previous sums' buffers

    def step(self, n_steps: int):
        v = self.advance(self.next_step, n_steps, self.acc, self.mom)
        self.next_step += n_steps
        self.steps_done += n_steps
        self.blocks += 1
        if v is not None:
            if not (isinstance(v, dict) and v.get("lag_done")):
                self._lag_update(v)
            self.lag_z.update_host(self.lag_chains, n_steps)
            self.lag_v.update_host(self.lag_chains, n_steps)
        if self.gram_every and self.blocks % self.gram_every == 0:
            self.advance.gram(self.G, self.S)
            self.n_gram += self.nc

    def _lag_device(self, v):
        if isinstance(v, dict):  # the library's functionals of the kept states (no re-read of v)
            self.lag_z.update_device(v["zk"][:self.lag_chains])
            self.lag_v.update_device(v["vn2"][:self.lag_chains] * 1e-6)
            return
        vs = v[:self.lag_chains]
        self.lag_z.update_device(self.t.round(vs @ self.binv).long())
        # ||v||^2 in one fused multiply-reduce pass over v (no v*v temporary); v is
        # integer, so every partial sum is an exact integer below 2^53 and the result
        # equals (v * v).sum(-1) in any summation order
        self.lag_v.update_device(self.t.linalg.vecdot(vs, vs) * 1e-6)

    def _lag_update(self, v):
        t = self.t
        k0 = v["zk"] if isinstance(v, dict) else v
        key = (k0.data_ptr(), tuple(k0.shape))
        if not self._graph_ok:
            self._lag_device(v)
        elif self._graph is not None and self._graph_key == key:
            self._graph.replay()
        elif self._graph_key == key:  # second block on the same buffer: capture, then replay
            g = t.cuda.CUDAGraph()
            with t.cuda.graph(g):
                self._lag_device(v)
            self._graph = g
            g.replay()
        else:  # first block (or a new buffer): eager, which also warms the kernels up
            self._graph = None
            self._graph_key = key
            self._lag_device(v)

    def reduce(self, group=None) -> dict:
        """One all-reduce of [accepts, moments, lag sums of both functionals, and
        (gram_every) the thinned states' sum z z^T, sum z and count]."""
        t = self.t
        parts = [self.acc.sum().reshape(1), self.mom] + self.lag_z.parts() + self.lag_v.parts()
        if self.gram_every:
            parts += [self.G, self.S, t.tensor([self.n_gram], dtype=t.int64, device=self.S.device)]
        r = allreduce_parts(parts, group=group)
        out = {"accepts": r[0], "moments": r[1], "lag_z": r[2:6], "lag_v": r[6:10]}
        if self.gram_every:
            out["gram"] = r[10:13]
        return out

    @staticmethod
    def acf(parts):
        S, N, S1, n = [x.cpu().numpy() for x in parts]
        return LagSums.acf(S.astype(np.float64), N, float(S1[0]), float(n[0]))

    @staticmethod
    def covariance(parts) -> np.ndarray:
        """Unbiased covariance (np.cov convention) of the thinned states from the
        exact reduced sums (G, S, n) of ``reduce()["gram"]``."""
        G, S, n = [x.cpu().numpy() for x in parts]
        n = int(n[0])
        s = S.astype(np.float64)
        return (G.astype(np.float64) - np.outer(s, s) / n) / (n - 1)


def gpu_advance(ctx, seed: int, first_chain: int, n_chains: int, d: int, device, *, flags: int = 0,
                block_steps: int = 0, want_v: bool = True, fn_chains: int = 0):
    """StreamingShard's advance over the HIP C-ABI: chain state resident on the
    device (coordinate-major z), one lgs_imhk call per block; v of every kept state
    into a preallocated (n_chains, block_steps, d) buffer.  The state tensors are
    exposed as ``advance.state``; ``advance.gram(G, S)`` adds sum z z^T / sum z of
    the chains' current states (lgs_gram, exact int8-digit MFMA).  The lag
    functionals ("zk", "vn2") cover the leading ``fn_chains`` chains (0: all; a
    StreamingShard reads its first ``lag_chains``).

    Streams: the library runs on the caller's current stream when that is not the
    null stream at creation (bench.py: one work stream, no cross-stream waits);
    otherwise on a dedicated torch stream.  A call made from any other current
    stream makes the library's stream wait (on the GPU, no host synchronisation) for
    everything enqueued there -- the lag-sum update still reading the reused v
    buffer, the zeroed accumulators -- and that stream wait for the library's work
    after it.  On a stream set this way lgs_imhk waits only for each
    block's Klein launch (its flags decide a redo), not for the accept / moments /
    B z launches behind it: the host enqueues the next step while they run."""
    import torch
    from . import _capi
    st = {"z": torch.zeros((d, n_chains), dtype=torch.int32, device=device),
          "lw": torch.zeros(n_chains, dtype=torch.float64, device=device),
          "init": torch.zeros(n_chains, dtype=torch.int32, device=device),
          "v": torch.empty((n_chains, block_steps, d), dtype=torch.float64, device=device)
          if want_v and block_steps else None,
          "zk": None, "vn2": None}
    fl = flags | _capi.LGS_DEVICE_PTRS | _capi.LGS_COORD_MAJOR
    nfn = n_chains if fn_chains <= 0 else min(int(fn_chains), n_chains)
    cur = torch.cuda.current_stream(device)
    lib_stream = cur if cur.cuda_stream else torch.cuda.Stream(device=device)
    ctx.set_stream(lib_stream.cuda_stream)

    def _enter():
        cur = torch.cuda.current_stream(device)
        if cur != lib_stream:
            lib_stream.wait_stream(cur)

    def _leave():
        cur = torch.cuda.current_stream(device)
        if cur != lib_stream:
            cur.wait_stream(lib_stream)

    lag = {}

    def bind_lag(lag_z, lag_v, lag_chains, L, v_scale):
        """StreamingShard hands over its LagSums: lgs_imhk_ex continues them (fused);
        lag_z None: unbind (the shard updates its sums from the returned series)."""
        lag.clear()
        if lag_z is None or not want_v or lag_chains != nfn:  # (the library's series: exactly nfn chains)
            return False
        lag.update(z=lag_z, v=lag_v, L=int(L), scale=float(v_scale))
        return True

    def advance(first_step, n_steps, acc, mom):
        v = st["v"]
        if want_v and (v is None or v.shape[1] != n_steps):
            v = st["v"] = torch.empty((n_chains, n_steps, d), dtype=torch.float64, device=device)
        if want_v and (st["zk"] is None or st["zk"].shape[1] != n_steps):
            st["zk"] = torch.empty((nfn, n_steps), dtype=torch.int64, device=device)
            st["vn2"] = torch.empty((nfn, n_steps), dtype=torch.float64, device=device)
        _enter()
        # the lag functionals z_{d-1} and ||v||^2 of every kept state come from the
        # library (coefficient store / B z epilogue), not from re-reading v
        ctx.imhk(seed, first_chain, n_chains, first_step, n_steps, 1, st["z"], st["lw"], st["init"], acc,
                 v_samples=v if want_v else None, moments=mom, flags=fl,
                 vnorm2_samples=st["vn2"] if want_v else None, zk_samples=st["zk"] if want_v else None,
                 zk_index=d - 1, fn_chains=nfn,
                 lag=(lag["L"], lag["z"].ring, lag["z"].sums, lag["v"].ring, lag["v"].sums, lag["scale"])
                 if lag else None)
        _leave()
        return {"v": v, "zk": st["zk"], "vn2": st["vn2"], "lag_done": bool(lag)} if want_v else None

    def gram(G, S):
        _enter()
        ctx.gram(st["z"], sum_out=S, gram_out=G, coord_major=True, flags=_capi.LGS_DEVICE_PTRS)
        _leave()

    advance.state = st
    advance.gram = gram
    advance.bind_lag = bind_lag
    advance.stream = lib_stream
    return advance


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

    if collective_active() and dist.get_world_size(group) != world:
        raise ValueError(f"imhk_sharded: world={world} but the active process group has "
                         f"{dist.get_world_size(group)} ranks")
    first, count = shard_range(n_chains, rank, world)
    r = compute(first_chain=first, n_chains=count, first_step=first_step, n_steps=n_steps)
    parts = [torch.tensor([r.accepts, r.kept], dtype=torch.int64),
             torch.from_numpy(np.ascontiguousarray(r.moments, dtype=np.int64))]
    if r.gram is not None:
        parts.append(torch.from_numpy(np.ascontiguousarray(r.gram, dtype=np.int64)))
    if device is not None:
        parts = [p.to(device) for p in parts]
    red = [p.cpu().numpy() for p in allreduce_parts(parts, group=group)]  # the single reduction
    s = red[0]
    gram = red[2] if r.gram is not None else None
    chain_stats = None
    if r.chain_stats is not None:
        width = max(shard_range(n_chains, k, world)[1] for k in range(world))
        buf = np.zeros((width, 2))
        buf[:count] = r.chain_stats
        t = torch.from_numpy(buf)
        if device is not None:
            t = t.to(device)
        if collective_active():
            out = [torch.zeros_like(t) for _ in range(world)]
            dist.all_gather(out, t, group=group)  # the single gather
        else:
            out = [t]
        chain_stats = np.concatenate([o.cpu().numpy()[:shard_range(n_chains, k, world)[1]]
                                      for k, o in enumerate(out)])
    return JobStats(int(s[0]), red[1], int(s[1]), gram, chain_stats)
