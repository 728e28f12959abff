"""Test helper: an oracle-backed per-rank compute for lgs_amd.distributed (CPU, gloo)."""
from typing import Optional

import numpy as np

from lgs_amd.distributed import ShardResult


def oracle_compute_factory(oracle, R, cp, B, sigma, seed, *, thin: int = 1, mode: int = 0,
                           center: Optional[np.ndarray] = None, want_gram: bool = False,
                           gr_coord: Optional[int] = None):
    """CPU stand-in for `gpu_compute` (the oracle module is passed in by the test)."""
    d = R.shape[0]

    def compute(first_chain, n_chains, first_step, n_steps):
        st = oracle.imhk(R, cp, B, sigma, n_chains, n_steps, center=center, seed=seed,
                         first_chain=first_chain, first_step=first_step, mode=mode, trace=True)
        tr = st["trace"][:, thin - 1::thin]
        kept = tr.reshape(-1, d)
        mom = np.concatenate([kept.sum(0), (kept * kept).sum(0)]).astype(np.int64)
        gram = kept.T.astype(np.int64) @ kept.astype(np.int64) if want_gram else None
        cs = None
        if gr_coord is not None:
            x = tr[:, :, gr_coord].astype(np.float64)
            m = x.mean(1)
            cs = np.stack([m, ((x - m[:, None]) ** 2).sum(1)], 1)
        return ShardResult(int(st["accepts"].sum()), mom, kept.shape[0], gram, cs)

    return compute


def oracle_advance_factory(oracle, R, cp, B, sigma, seed, first_chain, n_chains, *, mode: int = 0):
    """CPU stand-in for `gpu_advance` (StreamingShard's per-rank compute): the
    oracle's resumable IMHK chains, kept lattice points v = B z as a CPU tensor."""
    import torch
    d = R.shape[0]
    st = {"state": None}

    def advance(first_step, n_steps, acc, mom):
        prev = st["state"]["accepts"].copy() if st["state"] is not None else np.zeros(n_chains, dtype=np.int64)
        r = oracle.imhk(R, cp, B, sigma, n_chains, n_steps, seed=seed, first_chain=first_chain,
                        first_step=first_step, state=st["state"], mode=mode, trace=True)  # resumes in place
        tr = r.pop("trace")
        st["state"] = r
        acc += torch.from_numpy((r["accepts"] - prev).astype(np.int64))
        kept = tr.reshape(-1, d).astype(np.int64)
        mom += torch.from_numpy(np.concatenate([kept.sum(0), (kept * kept).sum(0)]))
        return torch.from_numpy(tr.astype(np.float64) @ B.T)

    def gram(G, S):  # the chains' current states (gpu_advance: lgs_gram of z_state)
        z = torch.from_numpy(st["state"]["z"].astype(np.int64))
        G += z.T @ z
        S += z.sum(0)

    advance.state = st
    advance.gram = gram
    return advance
