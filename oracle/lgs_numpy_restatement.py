"""ORACLE / TEST INFRASTRUCTURE ONLY -- the reference's NumPy Klein loop, restated.

The CPU baseline of BASELINE.md: the reference Python cannot travel
to the GPU box, so ``bench.py``'s ``cpu_baseline`` leg times this restatement,
which keeps the reference's algorithm AND loop structure, one process per host
core as ``experiments/dimension_scaling.py:841-845`` runs chains:

* ``sample_single`` (``src/samplers/klein.py:181-220``): coordinates i = d-1..0,
  the conditional sum as a Python loop over j > i, the 1e-10 / 1e10 sigma rules;
* ``_compute_1d_probabilities`` (``klein.py:101-139``): the support window with
  its 1000-point cap, log-space weights normalised by ``scipy.special.logsumexp``;
* ``_sample_1d_discrete_gaussian`` (``klein.py:141-179``): the table cache keyed
  on ``round(mean, 6)``, renormalisation, and ``np.random.choice`` -- replaced
  by the inverse-CDF rule ``searchsorted(cumsum(p) / cumsum[-1], u, 'right')``
  fed with the Philox uniform of the build's counter layout;
* ``basis @ x`` (``klein.py:218``).

It exists for timing; decisions match the oracle except where the reference's
approximate ``_sample_cache`` serves a table built for another mean.
"""
from __future__ import annotations

import os
import time

import numpy as np


def _philox_uniform(oracle, seed, slot, step, chain):
    return oracle.philox_u(seed, slot, step, chain, 0)


class NumpyKlein:
    def __init__(self, R, cprime, B, sigma, precision=10):
        from scipy.special import logsumexp
        self._lse = logsumexp
        self.R = np.asarray(R, dtype=np.float64)
        self.cp = np.asarray(cprime, dtype=np.float64)
        self.B = np.asarray(B, dtype=np.float64)
        self.R_diag = np.diag(self.R).copy()
        self.sigma = float(sigma)
        self.precision = int(precision)
        self.d = self.R.shape[0]
        self.P = np.arange(self.d)
        self._cache = {}

    def _probabilities(self, mean, sigma):  # klein.py:101-139 (log space)
        rf = max(3, self.precision) if sigma < 0.1 else self.precision
        lower = int(np.floor(mean - rf * sigma))
        upper = int(np.ceil(mean + rf * sigma))
        if upper - lower > 1000:
            c = int(np.round(mean))
            lower, upper = c - 500, c + 500
        support = np.arange(lower, upper + 1)
        lp = -0.5 * ((support - mean) / sigma) ** 2
        return support, lp - self._lse(lp)

    def _sample_1d(self, mean, sigma, u):  # klein.py:141-179
        key = (round(mean, 6), round(sigma, 6), self.precision)
        hit = self._cache.get(key)
        if hit is None:
            hit = self._probabilities(mean, sigma)
            if len(self._cache) >= 10000:
                self._cache.clear()
            self._cache[key] = hit
        support, lp = hit
        p = np.exp(lp)
        p = p / np.sum(p)
        cdf = np.cumsum(p)
        cdf /= cdf[-1]
        return int(support[np.searchsorted(cdf, u, side="right")])

    def sample_single(self, uniform):  # klein.py:181-220, same statements and indexing
        x = np.zeros(self.d, dtype=int)
        for i in range(self.d - 1, -1, -1):
            conditional_sum = 0.0
            for j in range(i + 1, self.d):
                conditional_sum += self.R[i, j] * x[j]
            mean = (self.cp[i] - conditional_sum) / self.R_diag[i]
            s = self.sigma / abs(self.R_diag[i])
            if s < 1e-10:
                x[i] = int(np.round(mean))
            else:
                x[i] = self._sample_1d(mean, min(s, 1e6) if s > 1e10 else s, uniform(self.d - 1 - i))
        x_permuted = np.zeros_like(x)  # klein.py:214-218 (P = identity)
        x_permuted[self.P] = x
        return self.B @ x_permuted


def _worker(args):
    R, cp, B, sigma, seed, chain, n = args
    import sys
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import lgs_oracle
    k = NumpyKlein(R, cp, B, sigma)
    t0 = time.perf_counter()
    for s in range(n):
        k.sample_single(lambda slot, s=s: _philox_uniform(lgs_oracle, seed, slot, s, chain))
    return n, time.perf_counter() - t0


def timed_run(R, cp, B, sigma, *, processes, samples_per_process, seed=1):
    """Klein samples/s of the restatement over `processes` worker processes (one per
    core, each drawing its own chain's samples); the sample loop is timed inside the
    workers, so interpreter start-up is excluded.  Returns (rate, total_samples,
    mean_wall_s)."""
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    jobs = [(R, cp, B, sigma, seed, c, samples_per_process) for c in range(processes)]
    # one core per worker: the spawned interpreters must not fan B @ x out over
    # BLAS threads (OMP_NUM_THREADS = 16 on the GPU box would oversubscribe the cores)
    keys = ("OPENBLAS_NUM_THREADS", "OMP_NUM_THREADS", "MKL_NUM_THREADS")
    saved = {k: os.environ.get(k) for k in keys}
    os.environ.update({k: "1" for k in keys})
    try:
        with ctx.Pool(processes) as pool:
            out = pool.map(_worker, jobs)
    finally:
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    total = sum(n for n, _ in out)
    wall = max(t for _, t in out)
    return total / wall, total, float(np.mean([t for _, t in out]))
