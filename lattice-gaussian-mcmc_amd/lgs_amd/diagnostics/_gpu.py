"""Device plumbing shared by the diagnostics mirrors: one lazily created HIP
context, host/device buffer handling and the per-series statistics call
(``lgs_series_stats``, ``include/lgs.h``).  Every statistic over the sample
stream is computed by the HIP kernels of ``csrc/lgs_diag.hip``; the host only
combines per-series scalars (as the reference's Python does around NumPy)."""
from __future__ import annotations

import numpy as np

from .. import _capi

_CTX = {}


def context(device=None):
    """The diagnostics context of `device` (default: torch's current device, else 0)."""
    if device is None:
        try:
            import torch
            device = torch.cuda.current_device() if torch.cuda.is_available() else 0
        except ImportError:
            device = 0
    ctx = _CTX.get(device)
    if ctx is None:
        ctx = _CTX[device] = _capi.Context(device)
    return ctx


def is_device(a) -> bool:
    return hasattr(a, "data_ptr") and getattr(getattr(a, "device", None), "type", "cpu") == "cuda"


def as_input(x):
    """Host arrays become C-contiguous float64 / int32 / int64 numpy arrays (other
    dtypes are converted to float64, as NumPy promotes them in the reference's
    arithmetic); device tensors are passed through (made contiguous)."""
    if is_device(x):
        import torch
        if x.dtype not in (torch.float64, torch.int32, torch.int64):
            x = x.to(torch.float64)
        return x.contiguous()
    x = np.asarray(x)
    if x.dtype not in (np.float64, np.int32, np.int64):
        x = x.astype(np.float64)
    return np.ascontiguousarray(x)


def _empty(like, shape):
    if is_device(like):
        import torch
        return torch.empty(shape, dtype=torch.float64, device=like.device)
    return np.empty(shape, dtype=np.float64)


def _host(a):
    return a.cpu().numpy() if is_device(a) else a


def series_stats(x, *, n_series, n, group_size, group_stride, series_stride, time_stride,
                 max_lag=-1, window_c=5.0, batch_size=0, want=("mean",)):
    """Run lgs_series_stats over a strided family of series; returns host arrays
    for the requested outputs: mean, c0, acf (n_series x (L+1)), tau, bmeans."""
    ctx = context(x.device.index if is_device(x) else None)
    L = min(max_lag, n - 1) if max_lag >= 0 else -1
    out = {k: None for k in ("mean", "c0", "acf", "tau", "bmeans")}
    if "mean" in want:
        out["mean"] = _empty(x, (n_series,))
    if "c0" in want:
        out["c0"] = _empty(x, (n_series,))
    if "tau" in want:
        out["tau"] = _empty(x, (n_series,))
    if "acf" in want:
        out["acf"] = _empty(x, (n_series, L + 1))
    if "bmeans" in want:
        out["bmeans"] = _empty(x, (n_series, n // batch_size))
    flags = _capi.LGS_DEVICE_PTRS if is_device(x) else 0
    ctx.series_stats(x, n_series, n, group_size, group_stride, series_stride, time_stride,
                     max_lag=max_lag, window_c=window_c, batch_size=batch_size, mean=out["mean"],
                     c0=out["c0"], acf=out["acf"], tau=out["tau"], batch_means=out["bmeans"],
                     flags=flags)
    return {k: _host(v) for k, v in out.items() if v is not None}


def columns(x):
    """series_stats layout of x: 1-D -> one series; (n, d) row-major -> d series."""
    if x.ndim == 1:
        return dict(n_series=1, n=x.shape[0], group_size=1, group_stride=0, series_stride=0,
                    time_stride=1)
    n, d = x.shape
    return dict(n_series=d, n=n, group_size=d, group_stride=0, series_stride=1, time_stride=d)


def column(x, i):
    """Layout of column i of a row-major (n, d) array (as a 1-series family)."""
    n, d = x.shape
    return dict(n_series=1, n=n, group_size=1, group_stride=0, series_stride=0, time_stride=d), i


def offset_view(x, off):
    """x shifted by `off` elements (series_stats addresses relative to the pointer)."""
    if off == 0:
        return x
    if is_device(x):
        return x.reshape(-1)[off:]
    return x.reshape(-1)[off:]
