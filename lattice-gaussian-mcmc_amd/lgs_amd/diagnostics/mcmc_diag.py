"""MCMC diagnostics on the GPU -- drop-in for the reference's
``src/diagnostics/mcmc_diag.py`` (same function names, arguments, defaults and
return types).

Every O(n) / O(n * lags) reduction over the samples (means, autocovariances,
the windowed integrated autocorrelation time, batch means, jump distances) runs
in the HIP kernels of ``csrc/lgs_diag.hip`` through ``lgs_series_stats`` /
``lgs_jump_distance``; the host only combines the per-series scalars exactly as
the reference's Python does.  Inputs may be NumPy arrays or torch device
tensors (then nothing but the scalars leaves HBM).

Numerics: integer-valued data gives exact sums; autocovariances are fp64 sums in
blocked order (the reference's np.correlate / FFT orders differ by rounding,
~n * 1e-16 relative).
"""
from __future__ import annotations

from typing import Any, Dict, Optional

import numpy as np

from . import _gpu


def compute_autocorrelation(x, max_lag: int = None) -> np.ndarray:
    """ACF for lags 0..max_lag (mcmc_diag.py:12-33); default max_lag =
    min(len(x)//4, 1000)."""
    x = _gpu.as_input(x).reshape(-1)
    n = x.shape[0]
    if max_lag is None:
        max_lag = min(n // 4, 1000)
    r = _gpu.series_stats(x, **_gpu.columns(x), max_lag=max_lag, want=("acf",))
    return r["acf"][0]


def integrated_autocorrelation_time(x, c: float = 5.0) -> float:
    """1 + 2 sum acf[k] with the reference's window rule (mcmc_diag.py:36-56), over
    lags 1..min(len(x)//4, 1000); the device scan stops once the window closes."""
    x = _gpu.as_input(x).reshape(-1)
    n = x.shape[0]
    r = _gpu.series_stats(x, **_gpu.columns(x), max_lag=min(n // 4, 1000), window_c=c,
                          want=("tau",))
    return float(r["tau"][0])


def _ess_1d_from(n, tau=None, c0=None, bmeans=None, method="autocorr"):
    if method == "autocorr":
        return n / tau
    var_batch = np.var(bmeans)
    var_sample = (c0 / n) / n
    if var_batch > 0:
        return var_sample / var_batch * n
    return n


def effective_sample_size(x, method: str = "autocorr") -> float:
    """ESS = n / tau_int, or the batch-means estimate (mcmc_diag.py:59-104);
    multivariate input: the minimum over dimensions (Python min semantics, as
    the reference's list)."""
    x = _gpu.as_input(x)
    n = x.shape[0]
    lay = _gpu.columns(x)
    if method == "autocorr":
        r = _gpu.series_stats(x, **lay, max_lag=min(n // 4, 1000), want=("tau",))
        vals = [_ess_1d_from(n, tau=t) for t in r["tau"]]
    else:
        b = int(np.sqrt(n))
        r = _gpu.series_stats(x, **lay, max_lag=0, batch_size=b, want=("c0", "bmeans"))
        vals = [_ess_1d_from(n, c0=r["c0"][i], bmeans=r["bmeans"][i], method=method)
                for i in range(lay["n_series"])]
    if x.ndim == 1:
        return vals[0]
    return min(vals)


def compute_acceptance_rate(accepted) -> float:
    """Mean of the accept flags (mcmc_diag.py:107-117)."""
    if _gpu.is_device(accepted):
        import torch
        a = accepted.reshape(-1).to(torch.int32).contiguous()
    else:
        a = np.ascontiguousarray(np.asarray(accepted).reshape(-1), dtype=np.int32)
    r = _gpu.series_stats(a, **_gpu.columns(a), want=("mean",))
    return r["mean"][0]


def compute_jump_distance(samples) -> np.ndarray:
    """|x_{t+1} - x_t| (1-D) or Euclidean jump lengths (mcmc_diag.py:120-136)."""
    x = _gpu.as_input(samples)
    x2 = x.reshape(-1, 1) if x.ndim == 1 else x
    n = x2.shape[0]
    out = np.empty(max(n - 1, 0))
    if n >= 2:
        ctx = _gpu.context(x.device.index if _gpu.is_device(x) else None)
        if _gpu.is_device(x):
            import torch
            dev_out = torch.empty(n - 1, dtype=torch.float64, device=x.device)
            ctx.jump_distance(x2, dev_out, flags=_gpu._capi.LGS_DEVICE_PTRS)
            out = dev_out.cpu().numpy()
        else:
            ctx.jump_distance(x2, out)
    return out


def diagnose_chain(samples, burn_in: Optional[int] = None, thin: int = 1) -> Dict[str, Any]:
    """Summary diagnostics of one chain (mcmc_diag.py:139-211)."""
    if burn_in is not None:
        samples = samples[burn_in:]
    if thin > 1:
        samples = samples[::thin]
    x = _gpu.as_input(samples)
    n = x.shape[0]
    lay = _gpu.columns(x)
    r = _gpu.series_stats(x, **lay, max_lag=min(n // 4, 1000), want=("mean", "c0", "tau"))
    if x.ndim == 1:
        mean = float(r["mean"][0])
        std = float(np.sqrt(r["c0"][0] / n))
        xs = x.cpu().numpy() if _gpu.is_device(x) else x
        quantiles = np.percentile(xs, [2.5, 25, 50, 75, 97.5])  # order statistics of a 1-D chain
    else:
        mean = r["mean"]
        std = np.sqrt(r["c0"] / n)
        quantiles = None
    vals = [n / t for t in r["tau"]]
    ess = vals[0] if x.ndim == 1 else min(vals)
    # ACF of the first dimension to min(100, n//4) lags; tau_int of the first dimension
    lay0 = dict(lay, n_series=1)  # series 0 = the first dimension
    a0 = _gpu.series_stats(x, **lay0, max_lag=min(100, n // 4), want=("acf",))["acf"][0]
    tau0 = float(r["tau"][0])
    jumps = compute_jump_distance(x)
    out = {
        "n_samples": n,
        "mean": mean,
        "std": std,
        "ess": float(ess),
        "ess_per_sample": float(ess / n),
        "tau_int": tau0,
        "mean_jump_distance": float(np.mean(jumps)),
        "acf_lag_1": float(a0[1]) if len(a0) > 1 else None,
        "acf_lag_10": float(a0[10]) if len(a0) > 10 else None,
    }
    if quantiles is not None:
        out["quantiles"] = {"2.5%": float(quantiles[0]), "25%": float(quantiles[1]),
                            "50%": float(quantiles[2]), "75%": float(quantiles[3]),
                            "97.5%": float(quantiles[4])}
    return out


def compute_mcse(x, method: str = "batch") -> float:
    """Monte Carlo standard error of the mean (mcmc_diag.py:214-246)."""
    x = _gpu.as_input(x).reshape(-1)
    n = x.shape[0]
    lay = _gpu.columns(x)
    if method == "batch":
        b = int(np.sqrt(n))
        bm = _gpu.series_stats(x, **lay, batch_size=b, want=("bmeans",))["bmeans"][0]
        return np.std(bm, ddof=1) / np.sqrt(len(bm))
    r = _gpu.series_stats(x, **lay, max_lag=min(n // 4, 1000), want=("c0", "tau"))
    var_x = r["c0"][0] / (n - 1)
    return np.sqrt(var_x * r["tau"][0] / n)
