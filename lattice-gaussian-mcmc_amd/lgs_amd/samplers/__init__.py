"""Samplers for lattice Gaussian distributions -- same exports as the reference's
``src/samplers/__init__.py:3-5``."""
from .base import DiscreteGaussianSampler, SamplingStats
from .klein import RefinedKleinSampler as KleinSampler
from .klein import RefinedKleinSampler
from .imhk import IMHKSampler

__all__ = ["DiscreteGaussianSampler", "KleinSampler", "IMHKSampler", "RefinedKleinSampler",
           "SamplingStats"]
