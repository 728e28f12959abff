"""Convergence diagnostics on the GPU -- drop-in for the reference's
``src/diagnostics/convergence_diag.py`` (same names, arguments and defaults).

Sample-stream reductions run in ``csrc/lgs_diag.hip``: the discrete marginal
TVD (``lgs_marginal_tvd``; bit-identical to the reference's Counter loop), the
histogram TVD (``lgs_column_range`` + ``lgs_histogram``: numpy's equal-width
bin counts on the device, the few per-bin normalisations on the host with the
reference's own NumPy expression), the autocorrelation / windowed tau_int and
the per-chain means / variances of Gelman-Rubin and the batch means
(``lgs_series_stats``).  The reference's FFT autocovariance and its direct
np.correlate one are the same quantity up to rounding; the device computes it
directly (fp64, blocked order).

Not provided: the sliced Wasserstein distance (``convergence_diag.py:232-292``),
not a consumer of the Klein/IMHK stream in the reference's experiments;
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
    a = _gpu.as_input(samples1)
    b = _gpu.as_input(samples2)
    if bins is not None:
        return _tvd_binned(a, b, bins)
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


def _outer_edges(lo, hi):
    """np.histogram's _get_outer_edges for range=(lo, hi) (numpy scalars)."""
    if lo > hi:
        raise ValueError("max must be larger than min in range parameter.")
    if not (np.isfinite(lo) and np.isfinite(hi)):
        raise ValueError(f"supplied range of [{lo}, {hi}] is not finite")
    if lo == hi:
        lo, hi = lo - 0.5, hi + 0.5
    return lo, hi


def _bin_setup(lo, hi, bins):
    """Edges and (first, denom) of numpy's uniform-bin path for one column
    (numpy/lib/_histograms_impl.py: np.linspace edges in the result type, float64
    for the int32 / int64 / float64 inputs taken here; the integer range width
    subtracted exactly before its conversion, as _unsigned_subtract does)."""
    first, last = _outer_edges(lo, hi)
    edges = np.linspace(first, last, bins + 1, endpoint=True, dtype=np.float64)
    if np.any(edges[:-1] >= edges[1:]):
        raise ValueError(f"Too many bins for data range. Cannot create {bins} finite-sized bins.")
    if isinstance(first, np.integer) and isinstance(last, np.integer):
        denom = float(int(last) - int(first))
    else:
        denom = float(np.float64(last) - np.float64(first))
    return edges, (float(first), denom)


def _tvd_binned(a, b, bins):
    """compute_tvd's histogram branch (convergence_diag.py:51-63, per column and
    averaged for 2-D input, :64-72): shared range over both sets, np.histogram
    counts on the device, then the reference's normalise / abs / sum in NumPy."""
    import operator
    bins = operator.index(bins)
    if bins < 1:
        raise ValueError("`bins` must be positive, when an integer")
    if a.shape[0] == 0 or b.shape[0] == 0:
        raise ValueError("zero-size array to reduction operation minimum which has no identity")
    if str(a.dtype) != str(b.dtype):
        a = _gpu.as_input(a.astype(np.float64) if not _gpu.is_device(a) else a.double())
        b = _gpu.as_input(b.astype(np.float64) if not _gpu.is_device(b) else b.double())
    a2 = a.reshape(-1, 1) if a.ndim == 1 else a
    b2 = b.reshape(-1, 1) if b.ndim == 1 else b
    d = a2.shape[1]
    dev = _gpu.is_device(a)
    ctx = _gpu.context(a.device.index if dev else None)
    flags = _gpu._capi.LGS_DEVICE_PTRS if dev else 0
    scal = np.dtype(str(a.dtype).replace("torch.", "")).type  # the samples' scalar type
    rng = []
    for x in (a2, b2):
        lo, hi = _gpu._empty(x, (d,)), _gpu._empty(x, (d,))
        try:
            ctx.column_range(x, lo, hi, flags=flags)
        except _gpu._capi.LgsError as e:
            if e.code == _gpu._capi.LGS_ERR_NONFINITE:
                raise ValueError("supplied range of the samples is not finite") from None
            raise
        rng.append((_gpu._host(lo), _gpu._host(hi)))
    edges = np.empty((d, bins + 1))
    fd = np.empty((d, 2))
    for i in range(d):
        lo = min(scal(rng[0][0][i]), scal(rng[1][0][i]))
        hi = max(scal(rng[0][1][i]), scal(rng[1][1][i]))
        edges[i], fd[i] = _bin_setup(lo, hi, bins)
    counts = []
    for x in (a2, b2):
        if dev:
            import torch
            e_d = torch.from_numpy(edges).to(x.device)
            f_d = torch.from_numpy(fd).to(x.device)
            c_d = torch.empty((d, bins), dtype=torch.int64, device=x.device)
            ctx.histogram(x, e_d, f_d, c_d, flags=flags)
            counts.append(c_d.cpu().numpy())
        else:
            c = np.empty((d, bins), dtype=np.int64)
            ctx.histogram(x, edges, fd, c)
            counts.append(c)
    tvds = []
    for i in range(d):
        hist1 = counts[0][i].astype(np.intp)
        hist2 = counts[1][i].astype(np.intp)
        hist1 = hist1 / hist1.sum()
        hist2 = hist2 / hist2.sum()
        tvds.append(0.5 * np.abs(hist1 - hist2).sum())
    if a.ndim == 1 and b.ndim == 1:
        return tvds[0]
    return np.mean(tvds)


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
