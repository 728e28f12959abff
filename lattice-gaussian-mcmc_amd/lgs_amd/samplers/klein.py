"""Klein sampler drop-in -- the reference's ``RefinedKleinSampler``
(``src/samplers/klein.py:21-354``), exported as ``KleinSampler``.

Host side (this file): the QR set-up of ``_precompute_qr_stable``
(klein.py:56-79, NumPy LAPACK, identical to the reference), parameter
validation and bookkeeping.  Device side (``liblgs_hip.so``): every coordinate
draw, the back-substitution, ``basis @ x`` and the log-density.  There is no CPU
sampling path; without a HIP device the constructor raises ``LgsError``.

Randomness: NumPy's global MT19937 stream is replaced by a Philox counter
stream keyed by ``seed``.  When ``seed`` is None it is drawn once from
``np.random`` at construction, so ``np.random.seed(k)`` still makes runs
reproducible, as in the reference's tests.  Sample ``s`` of a sampler always
uses counters (chain = s mod 2^32, step = s >> 32), so results do not depend
on how calls are batched.
"""
from __future__ import annotations

import logging
from typing import Any, Dict, Optional

import numpy as np

from .. import _capi
from .base import DiscreteGaussianSampler

logger = logging.getLogger(__name__)


def _default_seed() -> int:
    return int(np.random.randint(0, 2 ** 63 - 1, dtype=np.int64))


class RefinedKleinSampler(DiscreteGaussianSampler):
    """Klein's randomized nearest-plane sampler on MI355X (klein.py:21-54)."""

    def __init__(self, lattice, sigma: float, center: Optional[np.ndarray] = None,
                 precision: int = 10, use_log_space: bool = True, *, seed: Optional[int] = None,
                 device: int = 0, exact_order: bool = False, context: Optional[_capi.Context] = None):
        super().__init__(lattice, sigma, center)
        self.precision = precision
        self.use_log_space = use_log_space
        self.exact_order = exact_order
        self.seed = _default_seed() if seed is None else int(seed)
        self._next_sample = 0
        self._precompute_qr_stable()
        # the reference's approximate table cache does not exist here: every
        # draw uses the exact table of its own mean
        self._sample_cache: Dict = {}
        self._max_cache_size = 10000
        self._validate_klein_parameters()
        self._log_2pi = np.log(2 * np.pi)
        self._log_sigma = np.log(self.sigma)
        self._ctx = context if context is not None else _capi.Context(device)
        self._upload(self.precision)

    # ------------------------------------------------------------ set-up
    def _precompute_qr_stable(self):
        """klein.py:56-79: full QR, sign fix (R_ii > 0), c' = Q^T c."""
        self.Q, self.R = np.linalg.qr(self.lattice.basis, mode="full")
        self.P = np.arange(self.dimension)
        condition_number = np.linalg.cond(self.R)
        if condition_number > 1e10:
            logger.warning(f"Poorly conditioned basis: condition number = {condition_number:.2e}")
        for i in range(self.dimension):
            if self.R[i, i] < 0:
                self.R[i, :] *= -1
                self.Q[:, i] *= -1
        self.center_transformed = self.Q.T @ self.center
        self.R_diag = np.diag(self.R)
        self.log_R_diag = np.log(np.abs(self.R_diag) + 1e-300)

    def _validate_klein_parameters(self):
        """klein.py:81-99 (warnings only)."""
        min_gs_norm = self.lattice.min_gram_schmidt_norm
        klein_lower = min_gs_norm / np.sqrt(2 * np.log(self.dimension + 1))
        theoretical_optimal = min_gs_norm / (2 * np.sqrt(np.pi))
        if self.sigma < klein_lower * 0.9:
            logger.warning(f"σ={self.sigma:.4f} is below Klein's requirement "
                           f"(minimum ≈ {klein_lower:.4f}). Sampling may fail.")
        if theoretical_optimal * 0.8 <= self.sigma <= theoretical_optimal * 1.2:
            logger.info("σ is near optimal for BDD applications")

    def _upload(self, precision):
        self._ctx.set_basis(self.R, self.center_transformed, self.lattice.basis, self.sigma,
                            precision, linear_probs=not self.use_log_space)
        self._uploaded_precision = precision

    @property
    def context(self) -> _capi.Context:
        return self._ctx

    def _flags(self):
        return _capi.LGS_EXACT_ORDER if self.exact_order else 0

    # ------------------------------------------------------------ sampling
    def _draw(self, n: int, want_z=False, want_v=True, want_logw=False, flags=0):
        if self._uploaded_precision != self.precision:
            self._upload(self.precision)
        first = self._next_sample
        self._next_sample += n
        return self._ctx.klein_host(self.seed, first, n, want_z=want_z, want_v=want_v,
                                    want_logw=want_logw, flags=self._flags() | flags)

    def sample_single(self) -> np.ndarray:
        """One lattice point (klein.py:181-220)."""
        return self._draw(1)["v"][0]

    def sample_coefficients(self, num_samples: int = 1) -> np.ndarray:
        """Integer coefficient vectors, straight from the device (no lstsq needed)."""
        return self._draw(num_samples, want_z=True, want_v=False)["z"].astype(int)

    def sample_with_coefficients(self, num_samples: int = 1):
        """(lattice points, coefficients) of the same draws."""
        r = self._draw(num_samples, want_z=True, want_v=True)
        return r["v"], r["z"].astype(int)

    def parallel_sample_batch(self, num_samples: int, batch_size: int = 100) -> np.ndarray:
        """klein.py:304-322; the whole batch is one device launch (batch_size is moot)."""
        return self._draw(num_samples)["v"]

    def sample(self, num_samples: int = 1) -> np.ndarray:
        """(num_samples, dimension) lattice points (klein.py:324-337)."""
        if num_samples == 1:
            return self.sample_single().reshape(1, -1)
        return self.parallel_sample_batch(num_samples)

    def adaptive_precision_sample(self, target_distance: Optional[float] = None) -> np.ndarray:
        """klein.py:273-302."""
        if target_distance is None:
            return self.sample_single()
        old_precision = self.precision
        relative_distance = target_distance / self.sigma
        if relative_distance < 1:
            self.precision = max(20, 2 * old_precision)
        elif relative_distance > 5:
            self.precision = max(5, old_precision // 2)
        try:
            sample = self.sample_single()
        finally:
            self.precision = old_precision
        return sample

    # ------------------------------------------------------------ densities
    def _coefficients_of(self, lattice_point):
        try:
            coeffs = np.linalg.solve(self.lattice.basis, lattice_point)
            coeffs_int = np.round(coeffs).astype(np.int64)
            err = np.linalg.norm(self.lattice.basis @ coeffs_int - lattice_point)
            if err > 1e-10:
                return None
        except np.linalg.LinAlgError:
            return None
        return coeffs_int

    def compute_log_density(self, lattice_point: np.ndarray) -> float:
        """log q(v) of Klein's proposal (klein.py:222-271), evaluated on the device."""
        z = self._coefficients_of(np.asarray(lattice_point, dtype=np.float64))
        if z is None:
            return -np.inf
        if self._uploaded_precision != self.precision:
            self._upload(self.precision)
        return float(self._ctx.log_density(z[None, :])[0])

    def diagnostic_info(self) -> Dict[str, Any]:
        """klein.py:339-354."""
        return {
            "algorithm": "Refined Klein",
            "sigma": self.sigma,
            "precision": self.precision,
            "use_log_space": self.use_log_space,
            "cache_size": len(self._sample_cache),
            "condition_number": np.linalg.cond(self.R),
            "min_R_diag": np.min(np.abs(self.R_diag)),
            "max_R_diag": np.max(np.abs(self.R_diag)),
            "min_conditional_sigma": self.sigma / np.max(np.abs(self.R_diag)),
            "max_conditional_sigma": self.sigma / np.min(np.abs(self.R_diag)),
            "device": self._ctx.device_info()["name"],
            "seed": self.seed,
        }


KleinSampler = RefinedKleinSampler
