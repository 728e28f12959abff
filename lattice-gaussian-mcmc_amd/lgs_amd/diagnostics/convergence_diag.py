"""Convergence diagnostics on the GPU -- drop-in for the reference's
``src/diagnostics/convergence_diag.py`` (same names, arguments and defaults).

Sample-stream reductions run in ``csrc/lgs_diag.hip``: the discrete marginal
TVD (``lgs_marginal_tvd``; bit-identical to the reference's Counter loop), the
autocorrelation / windowed tau_int and the per-chain means / variances of
Gelman-Rubin and the batch means (``lgs_series_stats``).  The reference's FFT
autocovariance and its direct np.correlate one are the same quantity up to
rounding; the device computes it directly (fp64, blocked order).

Not provided: the histogram-binned TVD branch (``bins`` given) and the
sliced Wasserstein distance (``convergence_diag.py:232-292``), which are not
consumers of the Klein/IMHK stream in the reference's experiments;
``spectral_gap_estimate`` of an explicit transition matrix is a host LAPACK
call as in the reference.
"""
from __future__ import annotations

from typing import List, Optional

import numpy as np

from . import _gpu
from . import mcmc_diag as _md


def compute_tvd(samples1, samples2, bins: Optional[int] = None) -> float:
    """TVD(P, Q) = 0.5 sum |P(x) - Q(x)| of the empirical distributions; for
    multivariate samples the mean of the marginal TVDs (convergence_diag.py:15-72)."""
    if bins is not None:
        raise NotImplementedError("binned TVD (convergence_diag.py:50-64) is not part of the GPU "
                                  "diagnostics; use bins=None (discrete samples)")
    a = _gpu.as_input(samples1)
    b = _gpu.as_input(samples2)
    if a.shape[0] == 0 or b.shape[0] == 0:  # the reference's loop: 0.0 for two empty sets,
        if a.shape[0] == b.shape[0]:         # ZeroDivisionError (count / 0) for one
            return 0.0 if a.ndim == 1 else float(np.mean([0.0] * a.shape[1]))
        raise ZeroDivisionError("division by zero")
    if str(a.dtype) != str(b.dtype):
        a = _gpu.as_input(a.astype(np.float64) if not _gpu.is_device(a) else a.double())
        b = _gpu.as_input(b.astype(np.float64) if not _gpu.is_device(b) else b.double())
    a2 = a.reshape(-1, 1) if a.ndim == 1 else a
    b2 = b.reshape(-1, 1) if b.ndim == 1 else b
    d = a2.shape[1]
    ctx = _gpu.context(a.device.index if _gpu.is_device(a) else None)
    if _gpu.is_device(a):
        import torch
        out_d = torch.empty(d, dtype=torch.float64, device=a.device)
        ctx.marginal_tvd(a2, b2, out_d, flags=_gpu._capi.LGS_DEVICE_PTRS)
        tvds = out_d.cpu().numpy()
    else:
        tvds = np.empty(d)
        ctx.marginal_tvd(a2, b2, tvds)
    if a.ndim == 1 and b.ndim == 1:
        return float(tvds[0])
    return np.mean(list(tvds))


def compute_autocorrelation(x, max_lag: int = None) -> np.ndarray:
    """ACF for lags 0..max_lag, default len(x)//4 (convergence_diag.py:75-113)."""
    n = len(x)
    if max_lag is None:
        max_lag = n // 4
    return _md.compute_autocorrelation(x, max_lag=max_lag)


def integrated_autocorrelation_time(x, c: float = 5.0) -> float:
    """tau_int over lags 1..len(x)//4 with the window rule (convergence_diag.py:115-145)."""
    x = _gpu.as_input(x).reshape(-1)
    n = x.shape[0]
    r = _gpu.series_stats(x, **_gpu.columns(x), max_lag=n // 4, window_c=c, want=("tau",))
    return float(r["tau"][0])


def spectral_gap_estimate(transition_probs: np.ndarray) -> float:
    """1 - |lambda_2| of an explicit transition matrix (convergence_diag.py:148-173)."""
    ev = sorted(np.linalg.eigvals(transition_probs), key=abs, reverse=True)
    return float(1 - abs(ev[1])) if len(ev) > 1 else 1.0


def gelman_rubin_statistic(chains: List) -> float:
    """R-hat of m chains truncated to the shortest (convergence_diag.py:176-213)."""
    m = len(chains)
    n = min(len(ch) for ch in chains)
    dev = _gpu.is_device(chains[0])
    if dev:
        import torch
        X = torch.stack([ch[:n].to(torch.float64) for ch in chains]).contiguous()
    else:
        X = np.ascontiguousarray(np.stack([np.asarray(ch[:n], dtype=np.float64) for ch in chains]))
    r = _gpu.series_stats(X, n_series=m, n=n, group_size=1, group_stride=n, series_stride=0,
                          time_stride=1, max_lag=0, want=("mean", "c0"))
    chain_means = list(r["mean"])
    overall = np.mean(chain_means)
    B = n / (m - 1) * sum((mu - overall) ** 2 for mu in chain_means)
    W = np.mean([c0 / (n - 1) for c0 in r["c0"]])
    var_pooled = ((n - 1) / n) * W + (1 / n) * B
    return float(np.sqrt(var_pooled / W))


def compute_ess_per_second(samples, elapsed_time: float) -> float:
    """ESS / wall time (convergence_diag.py:216-229)."""
    return _md.effective_sample_size(samples) / elapsed_time


def mixing_time_estimate(tvd_values: List[float], threshold: float = 0.25) -> int:
    """First index with TVD below the threshold (convergence_diag.py:295-313)."""
    for i, tvd in enumerate(tvd_values):
        if tvd < threshold:
            return i
    return len(tvd_values)


def batch_means_variance(x, batch_size: Optional[int] = None) -> float:
    """batch_size * var(batch means, ddof=1) (convergence_diag.py:316-345)."""
    x = _gpu.as_input(x).reshape(-1)
    n = x.shape[0]
    if batch_size is None:
        batch_size = int(np.sqrt(n))
    bm = _gpu.series_stats(x, **_gpu.columns(x), batch_size=batch_size, want=("bmeans",))["bmeans"][0]
    return batch_size * np.var(bm, ddof=1)
