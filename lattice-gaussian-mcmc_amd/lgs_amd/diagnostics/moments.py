"""Empirical moments on the GPU: ``empirical_mean`` / ``empirical_covariance`` of
the reference's sampler base (``src/samplers/base.py:154-160``: np.mean(axis=0),
np.cov(samples.T)) and the exact integer sufficient statistics sum z, sum z z^T
 through ``lgs_gram``.

Integer-valued samples (the lattice points of integer bases, coefficient vectors)
are reduced EXACTLY in int64 on int8 MFMA after subtracting the rounded mean;
the covariance is then (G - S S^T / n) / (n - 1) with the small shifted sums
S, G -- as accurate as or better than NumPy's centred fp64 product.  Real-valued
samples use the fp64 VALU path centred on the device-computed mean.
"""
from __future__ import annotations

import numpy as np

from . import _gpu
from .. import _capi


def empirical_mean(samples) -> np.ndarray:
    """np.mean(samples, axis=0) (base.py:154-156)."""
    x = _gpu.as_input(samples)
    if x.ndim == 1:
        return _gpu.series_stats(x, **_gpu.columns(x), want=("mean",))["mean"][0]
    return _gpu.series_stats(x, **_gpu.columns(x), want=("mean",))["mean"]


def _integral(x) -> bool:
    if _gpu.is_device(x):
        import torch
        if x.dtype != torch.float64:
            return True
        return bool(torch.all(x == torch.round(x)).item()) and bool((x.abs() < 2 ** 62).all().item())
    if x.dtype != np.float64:
        return True
    return bool(np.all(x == np.round(x))) and bool(np.all(np.abs(x) < 2.0 ** 62))


def gram(x, shift=None):
    """(sum y, sum y y^T) of the rows of x (n x d), y = x - shift; int64 for integer
    x (exact), fp64 otherwise.  Host numpy results."""
    x = _gpu.as_input(x)
    n, d = x.shape
    dev = _gpu.is_device(x)
    integer = str(x.dtype).replace("torch.", "") in ("int32", "int64")
    odt = np.int64 if integer else np.float64
    ctx = _gpu.context(x.device.index if dev else None)
    if dev:
        import torch
        tdt = torch.int64 if integer else torch.float64
        s = torch.zeros(d, dtype=tdt, device=x.device)
        g = torch.zeros((d, d), dtype=tdt, device=x.device)
        sh = None if shift is None else torch.as_tensor(np.asarray(shift, dtype=odt), device=x.device)
        ctx.gram(x, shift=sh, sum_out=s, gram_out=g, flags=_capi.LGS_DEVICE_PTRS)
        return s.cpu().numpy(), g.cpu().numpy()
    s = np.zeros(d, dtype=odt)
    g = np.zeros((d, d), dtype=odt)
    sh = None if shift is None else np.ascontiguousarray(shift, dtype=odt)
    ctx.gram(x, shift=sh, sum_out=s, gram_out=g)
    return s, g


def empirical_covariance(samples) -> np.ndarray:
    """np.cov(samples.T): unbiased covariance of the rows (base.py:158-160)."""
    x = _gpu.as_input(samples)
    if x.ndim != 2:
        raise ValueError("empirical_covariance expects (num_samples, dimension) samples")
    n = x.shape[0]
    mean = empirical_mean(x)
    if _integral(x):
        if str(x.dtype).replace("torch.", "") == "float64":
            x = x.to(__import__("torch").int64) if _gpu.is_device(x) else x.astype(np.int64)
        shift = np.round(mean).astype(np.int64)
        s, g = gram(x, shift)
        sf = s.astype(np.float64)
        return (g.astype(np.float64) - np.outer(sf, sf) / n) / (n - 1)
    s, g = gram(x, np.asarray(mean, dtype=np.float64))
    return (g - np.outer(s, s) / n) / (n - 1)


def empirical_std(samples) -> np.ndarray:
    """np.std(samples, axis=0) (ddof 0), as in IMHKSampler.diagnose_convergence
    (imhk.py:303)."""
    x = _gpu.as_input(samples)
    n = x.shape[0]
    r = _gpu.series_stats(x, **_gpu.columns(x), max_lag=0, want=("c0",))
    return np.sqrt(r["c0"] / n)
