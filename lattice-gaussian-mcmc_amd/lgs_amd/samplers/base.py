"""Sampler base class -- contract of the reference's ``src/samplers/base.py``.

Mirrors ``DiscreteGaussianSampler`` (base.py:31-175) and ``SamplingStats``
(base.py:18-28): center handling, sigma validation, smoothing warning and the
moment helpers, with the same names, argument meaning and exceptions
(ValueError for sigma <= 0 and for a center of the wrong length).
"""
from __future__ import annotations

import logging
from abc import ABC, abstractmethod
from dataclasses import dataclass, field
from typing import Any, Dict, Optional

import numpy as np

logger = logging.getLogger(__name__)


@dataclass
class SamplingStats:
    """Statistics collected during sampling (base.py:18-28)."""
    samples_generated: int = 0
    time_elapsed: float = 0.0
    acceptance_rate: Optional[float] = None
    extra_stats: Dict[str, Any] = field(default_factory=dict)


class DiscreteGaussianSampler(ABC):
    """D_{L,sigma,c}(x) = rho_{sigma,c}(x) / rho_{sigma,c}(L) over a lattice L (base.py:31-42)."""

    def __init__(self, lattice, sigma: float, center: Optional[np.ndarray] = None):
        self.lattice = lattice
        self.sigma = sigma
        self.dimension = lattice.dimension
        if center is None:
            self.center = np.zeros(self.dimension)
        else:
            self.center = np.array(center, dtype=np.float64)
        if len(self.center) != self.dimension:
            raise ValueError(f"Center dimension {len(self.center)} != lattice dimension {self.dimension}")
        self.stats = SamplingStats()
        self._validate_parameters()
        logger.info(f"Initialized {self.__class__.__name__} with σ={sigma:.4f}")

    def _validate_parameters(self):
        if self.sigma <= 0:
            raise ValueError(f"Standard deviation must be positive, got {self.sigma}")
        smoothing = getattr(self.lattice, "smoothing_parameter", None)
        if callable(smoothing):
            eta = smoothing()
            if self.sigma < eta:
                logger.warning(f"σ={self.sigma:.4f} is below smoothing parameter "
                               f"η={float(eta):.4f}. Sampling may be biased.")

    @abstractmethod
    def sample(self, num_samples: int = 1) -> np.ndarray:
        """(num_samples, dimension) lattice points."""

    def sample_coefficients(self, num_samples: int = 1) -> np.ndarray:
        """Integer coefficients x with B x = sample (base.py:98-118)."""
        points = self.sample(num_samples)
        coeffs = np.zeros((num_samples, self.dimension), dtype=int)
        for i, point in enumerate(points):
            c = np.linalg.lstsq(self.lattice.basis, point, rcond=None)[0]
            coeffs[i] = np.round(c).astype(int)
        return coeffs

    def gaussian_weight(self, point: np.ndarray) -> float:
        diff = point - self.center
        return np.exp(-np.dot(diff, diff) / (2 * self.sigma ** 2))

    def log_gaussian_weight(self, point: np.ndarray) -> float:
        diff = point - self.center
        return -np.dot(diff, diff) / (2 * self.sigma ** 2)

    def reset_stats(self):
        self.stats = SamplingStats()

    def get_stats(self) -> SamplingStats:
        return self.stats

    def empirical_mean(self, samples: np.ndarray) -> np.ndarray:
        """np.mean(samples, axis=0) on the GPU (base.py:154-156)."""
        from ..diagnostics import moments
        return moments.empirical_mean(samples)

    def empirical_covariance(self, samples: np.ndarray) -> np.ndarray:
        """np.cov(samples.T) on the GPU (base.py:158-160): exact int64 second moments
        for integer-valued samples (lgs_gram, int8 MFMA)."""
        from ..diagnostics import moments
        return moments.empirical_covariance(samples)

    def theoretical_covariance(self) -> np.ndarray:
        return self.sigma ** 2 * np.eye(self.dimension)

    def __repr__(self) -> str:
        name = getattr(self.lattice, "name", type(self.lattice).__name__)
        return f"{self.__class__.__name__}(lattice={name}, σ={self.sigma:.4f}, center={self.center})"
