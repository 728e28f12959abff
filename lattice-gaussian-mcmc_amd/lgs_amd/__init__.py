"""lgs_amd -- MI355X-native Klein / IMHK discrete-Gaussian lattice sampler.

Drop-in for the reference's sampler API (``src/samplers/__init__.py:3-5`` of
NickQrumpton/lattice-gaussian-mcmc)::

    from lgs_amd.samplers import KleinSampler, IMHKSampler

The compute path is the HIP C-ABI library ``liblgs_hip.so`` (``include/lgs.h``),
loaded through ctypes on first use; there is no CPU fallback.
"""
from .lattices import SimpleLattice, build_config  # noqa: F401

__all__ = ["SimpleLattice", "build_config", "samplers"]
__version__ = "0.1.0"


def __getattr__(name):
    if name in ("KleinSampler", "IMHKSampler", "DiscreteGaussianSampler"):
        from . import samplers
        return getattr(samplers, name)
    raise AttributeError(name)
