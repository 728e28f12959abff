"""IMHK sampler drop-in -- the reference's ``IMHKSampler``
(``src/samplers/imhk.py:19-317``): independent Metropolis-Hastings with Klein
proposals (Wang & Ling 2019).

Every step runs on the device (``lgs_imhk``): the Klein proposal, its
importance weight, the Metropolis test and the state bookkeeping.  Because the
proposals are independent of the chain state, a call of ``sample(N, thin)``
draws all ``N*thin`` proposals in one parallel launch and then runs the
sequential accept/reject scan; the result is identical to stepping one at a
time (every draw has a fixed Philox counter).

Weights: by default the reference's ``_compute_importance_weight``
(imhk.py:102-124), which is a constant up to rounding, so the acceptance rate
is 1.0 exactly as in the reference.  ``wang_ling=True`` selects the exact
Wang-Ling weight (product of the 1-D normalisers), an opt-in mode that the
reference does not have.
"""
from __future__ import annotations

import logging
import time
from typing import List, Optional, Tuple

import numpy as np

from .. import _capi
from ..diagnostics import moments as _moments
from .base import DiscreteGaussianSampler
from .klein import RefinedKleinSampler, _default_seed

logger = logging.getLogger(__name__)


class IMHKSampler(DiscreteGaussianSampler):
    """Independent Metropolis-Hastings-Klein chain on MI355X (imhk.py:19-66)."""

    def __init__(self, lattice, sigma: float, center: Optional[np.ndarray] = None,
                 precision: int = 10, burn_in: Optional[int] = None, *,
                 seed: Optional[int] = None, device: int = 0, wang_ling: bool = False,
                 exact_order: bool = False, chain_id: int = 0):
        super().__init__(lattice, sigma, center)
        self.seed = _default_seed() if seed is None else int(seed)
        self.proposal_sampler = RefinedKleinSampler(lattice, sigma, center, precision,
                                                    seed=self.seed, device=device,
                                                    exact_order=exact_order)
        self.wang_ling = wang_ling
        self.chain_id = int(chain_id)
        self.burn_in = burn_in if burn_in is not None else self._estimate_burn_in()
        self.total_proposals = 0
        self.accepted_proposals = 0
        self.current_state = None
        self.current_coeffs = None
        self.current_log_weight = None
        self._precompute_partition_bounds()
        d = self.dimension
        self._z = np.zeros((1, d), dtype=np.int64)
        self._lw = np.zeros(1)
        self._init = np.zeros(1, dtype=np.int32)
        self._next_step = 1
        self._sbuf = None  # look-ahead block served by step() (see _fill_steps)
        self._step_block = 16
        logger.info(f"Initialized IMHK with burn-in={self.burn_in}")

    # ------------------------------------------------------------ set-up (imhk.py:68-100)
    def _estimate_burn_in(self) -> int:
        """Same formula as the reference, including its OverflowError at large d."""
        epsilon = 0.01
        dimension_factor = self.dimension
        sigma_factor = (float(self.sigma) / float(self.lattice.min_gram_schmidt_norm)) ** self.dimension
        inv_delta_estimate = dimension_factor * sigma_factor
        mixing_time = int(np.ceil(-np.log(epsilon) * inv_delta_estimate))
        return min(mixing_time * 2, 10000)

    def _precompute_partition_bounds(self):
        R = self.proposal_sampler.R
        sig = self.sigma / np.abs(np.diag(R))
        self.klein_log_partition = float(np.sum(0.5 * np.log(2 * np.pi) + np.log(sig)))

    @property
    def context(self) -> _capi.Context:
        return self.proposal_sampler.context

    def _flags(self):
        f = _capi.LGS_WANG_LING if self.wang_ling else 0
        if self.proposal_sampler.exact_order:
            f |= _capi.LGS_EXACT_ORDER
        return f

    # ------------------------------------------------------------ device steps
    def _run(self, n_steps: int, thin: int = 1, keep: bool = True):
        """Advance the chain n_steps; returns kept coefficient vectors (n_steps//thin, d)."""
        ctx = self.context
        n_keep = n_steps // thin
        self._sbuf = None  # the chain moves past any look-ahead block
        for z64 in (False, True):
            zt = np.int64 if z64 else np.int32
            z_state = self._z.astype(zt)
            lw = self._lw.copy()
            init = self._init.copy()
            acc = np.zeros(1, dtype=np.int64)
            zs = np.zeros((1, max(n_keep, 1), self.dimension), dtype=zt) if keep and n_keep else None
            try:
                ctx.imhk(self.seed, self.chain_id, 1, self._next_step, n_steps, thin, z_state, lw,
                         init, acc, z_samples=zs, flags=self._flags() | (_capi.LGS_Z64 if z64 else 0))
            except _capi.LgsError as e:
                if e.code == _capi.LGS_ERR_OVERFLOW and not z64:
                    continue
                raise
            break
        first_init = not bool(self._init[0])
        self._z = z_state.astype(np.int64)
        self._lw = lw
        self._init = init
        self._next_step += n_steps
        self.total_proposals += n_steps
        self.accepted_proposals += int(acc[0])
        self.current_coeffs = self._z[0].astype(int)
        self.current_state = ctx.lattice_points(self._z)[0]
        self.current_log_weight = float(self._lw[0])
        if first_init:
            logger.debug(f"Initialized chain at state with log weight {self.current_log_weight:.4f}")
        out = None if zs is None else zs[0, :n_keep].astype(np.int64)
        return out, int(acc[0])

    def _fill_steps(self, k: int):
        """Draw the next k steps of the chain in one lgs_imhk_trace call: kept states,
        their log weights, the per-step accept decisions and the lattice points.  The
        chain's own state is not advanced here: step() moves it through the block one
        step at a time, so the other methods continue from wherever step() left it
        (every draw has a fixed Philox counter, so the block equals k single steps)."""
        ctx = self.context
        d = self.dimension
        flags = self._flags()
        for z64 in (False, True):
            zt = np.int64 if z64 else np.int32
            z_state = self._z.astype(zt)
            lw = self._lw.copy()
            init = self._init.copy()
            acc = np.zeros(1, dtype=np.int64)
            zs = np.zeros((1, k, d), dtype=zt)
            lws = np.zeros((1, k))
            accd = np.zeros((1, k), dtype=np.uint8)
            try:
                ctx.imhk(self.seed, self.chain_id, 1, self._next_step, k, 1, z_state, lw, init, acc,
                         z_samples=zs, flags=flags | (_capi.LGS_Z64 if z64 else 0),
                         logw_samples=lws, accepted=accd)
            except _capi.LgsError as e:
                if e.code == _capi.LGS_ERR_OVERFLOW and not z64:
                    continue
                raise
            break
        z = zs[0].astype(np.int64)
        self._sbuf = {"z": z, "lw": lws[0].copy(), "acc": accd[0].astype(bool),
                      "v": ctx.lattice_points(z), "first": self._next_step, "pos": 0, "key": self._block_key()}

    def _block_key(self):
        """What a look-ahead block was drawn with: the counters (seed, chain id), the
        call flags and the context (basis) -- a block is served only while all match."""
        return (self.seed, self.chain_id, self._flags(), id(self.context))

    def step(self) -> Tuple[np.ndarray, bool]:
        """One MCMC step (imhk.py:141-177): (new_state, accepted).  Served from a
        look-ahead block drawn in one launch (16 steps, doubling up to 1024 while the
        caller keeps stepping), identical to launching every step on its own."""
        b = self._sbuf
        if (b is None or b["pos"] >= len(b["lw"]) or b["first"] + b["pos"] != self._next_step
                or b["key"] != self._block_key()):
            if b is not None and b["pos"] >= len(b["lw"]):
                self._step_block = min(2 * self._step_block, 1024)
            self._fill_steps(self._step_block)
            b = self._sbuf
        j = b["pos"]
        b["pos"] = j + 1
        first_init = not bool(self._init[0])
        self._z = b["z"][j:j + 1].copy()
        self._lw = b["lw"][j:j + 1].copy()
        self._init = np.ones(1, dtype=np.int32)
        self._next_step += 1
        accepted = bool(b["acc"][j])
        self.total_proposals += 1
        self.accepted_proposals += int(accepted)
        self.current_coeffs = self._z[0].astype(int)
        self.current_state = b["v"][j].copy()
        self.current_log_weight = float(self._lw[0])
        if first_init:
            logger.debug(f"Initialized chain at state with log weight {self.current_log_weight:.4f}")
        return self.current_state.copy(), accepted

    def sample_single(self) -> np.ndarray:
        """imhk.py:179-194: burn-in on first use, then one step."""
        if self.current_state is None and self.burn_in > 0:
            self._run(self.burn_in, 1, keep=False)
        state, _ = self.step()
        return state

    def sample(self, num_samples: int = 1, thin: int = 1) -> np.ndarray:
        """imhk.py:196-229: num_samples states, thin steps apart (no burn-in)."""
        start = time.time()
        zs, _ = self._run(num_samples * thin, thin, keep=True)
        samples = self.context.lattice_points(zs) if num_samples else np.zeros((0, self.dimension))
        self.stats.samples_generated += num_samples
        self.stats.time_elapsed += time.time() - start
        self.stats.acceptance_rate = (self.accepted_proposals / self.total_proposals
                                      if self.total_proposals > 0 else 0.0)
        return samples

    def run_chain(self, num_steps: int, save_every: int = 1) -> List[np.ndarray]:
        """imhk.py:231-250: states of steps i with i % save_every == 0."""
        zs, _ = self._run(num_steps, 1, keep=True)
        if num_steps == 0:
            return []
        idx = np.arange(0, num_steps, save_every)
        pts = self.context.lattice_points(zs[idx])
        return [p.copy() for p in pts]

    def estimate_spectral_gap(self, num_samples: int = 1000) -> float:
        """imhk.py:252-284: 1 / max importance weight over Klein proposals."""
        r = self.proposal_sampler._draw(num_samples, want_v=False, want_logw=True,
                                        flags=_capi.LGS_WANG_LING if self.wang_ling else 0)
        lw = r["logw"]
        w = np.where(lw > 700, np.inf, np.where(lw < -700, 0.0, np.exp(np.clip(lw, -700, 700))))
        w = w[np.isfinite(w)]
        if w.size == 0:
            logger.warning("All importance weights were infinite")
            return 0.0
        mx = float(np.max(w))
        return 1.0 / mx if mx > 0 else 0.0

    # ------------------------------------------------------------ Wang-Ling delta
    def _log_normaliser_max(self) -> float:
        """log prod_i rho_{sigma_i}(Z) over the drawn coordinates (sigma_i >= 1e-10):
        each 1-D normaliser is largest at an integer mean (Poisson summation), so this
        is the maximum of the Wang-Ling weight.  Evaluated by the device SampleZ
        normaliser (lgs_sample_z) at mu = 0 with the sampler's window rules."""
        if getattr(self, "_lnmax", None) is None:
            R = self.proposal_sampler.R
            sig = self.sigma / np.abs(np.diag(R))
            sig = sig[sig >= 1e-10]
            sig = np.where(sig > 1e10, 1e6, sig)
            _, ln = self.context.sample_z(np.zeros(sig.size), sig, np.full(sig.size, 0.5),
                                          precision=self.proposal_sampler.precision)
            self._lnmax = float(np.sum(ln))
        return self._lnmax

    def compute_delta(self, num_samples: int = 1 << 16) -> float:
        """Monte Carlo estimate of Wang & Ling's delta = rho_{sigma,c}(L) / prod_i rho_{sigma_i}(Z)
        (the quantity of imhk.py:256-258 and the aspirational IndependentMHK.compute_delta of
        experiments/cryptographic_experiments.py:288): rho(L) = E_Klein[w(x)] with the exact
        weight w(x) = prod_i rho_{sigma_i}(Z - mu_i(x)), drawn on the GPU
        (lgs_klein with LGS_WANG_LING log-weights)."""
        r = self.proposal_sampler._draw(int(num_samples), want_v=False, want_logw=True,
                                        flags=_capi.LGS_WANG_LING)
        lw = r["logw"]
        m = float(np.max(lw))
        log_mean = m + float(np.log(np.mean(np.exp(lw - m))))
        return float(np.exp(log_mean - self._log_normaliser_max()))

    def spectral_gap(self, num_samples: int = 1 << 16) -> float:
        """Spectral gap of the IMHK kernel: delta (uniform ergodicity, ||P^t - pi|| <= (1-delta)^t)."""
        return self.compute_delta(num_samples)

    def mixing_time(self, epsilon: float = 0.25, num_samples: int = 1 << 16) -> int:
        """t_mix(epsilon) <= ceil(ln(epsilon) / ln(1 - delta))."""
        delta = self.compute_delta(num_samples)
        if delta >= 1.0:
            return 1
        if delta <= 0.0:
            return int(np.iinfo(np.int64).max)
        return int(np.ceil(np.log(epsilon) / np.log1p(-delta)))

    def diagnose_convergence(self, num_samples: int = 1000) -> dict:
        """imhk.py:286-313."""
        old_stats = self.stats
        self.reset_stats()
        samples = self.sample(num_samples)
        diagnostics = {
            "acceptance_rate": self.stats.acceptance_rate,
            "spectral_gap_estimate": self.estimate_spectral_gap(100),
            "empirical_mean": self.empirical_mean(samples),
            "empirical_std": _moments.empirical_std(samples),
            "theoretical_std": self.sigma * np.ones(self.dimension),
            "samples_per_second": num_samples / max(self.stats.time_elapsed, 1e-12),
        }
        self.stats = old_stats
        return diagnostics

    def __repr__(self) -> str:
        rate = self.stats.acceptance_rate or 0.0
        name = getattr(self.lattice, "name", type(self.lattice).__name__)
        return f"IMHKSampler(lattice={name}, σ={self.sigma:.4f}, burn_in={self.burn_in}, acceptance_rate={rate:.2%})"
