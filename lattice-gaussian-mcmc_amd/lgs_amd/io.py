"""Sample dumps and result records in the reference's formats.

* ``save_samples_npz`` / ``load_samples_npz`` -- the compressed sample dumps of
  ``experiments/run_core_experiments.sage:69-73`` (arrays ``samples`` and
  ``norms``); loading never unpickles (``allow_pickle=False``).
* ``basis_properties`` -- ``klein_scaling_analysis.py:136-165`` (determinant,
  condition number, row Gram-Schmidt norms), host LAPACK set-up like the QR.
* ``sample_quality_metrics`` -- ``klein_scaling_analysis.py:191-242`` computed from
  the integer coefficient vectors the device already returns (no B^{-1} solve):
  per-coordinate means / standard deviations on the GPU (``lgs_series_stats``,
  exact sums), ranges and the distinct-sample count on the host.
* ``klein_scaling_record`` / ``save_results_json`` -- the per-dimension JSON
  record of ``klein_scaling_analysis.py:322-340``.
"""
from __future__ import annotations

import json
from typing import Any, Dict, Optional

import numpy as np


def save_samples_npz(path: str, samples, norms: Optional[np.ndarray] = None) -> None:
    """np.savez_compressed(path, samples=..., norms=...) as the reference's drivers."""
    s = np.asarray(samples.cpu().numpy() if hasattr(samples, "cpu") else samples)
    if norms is None:
        norms = np.linalg.norm(s.astype(np.float64), axis=1)
    np.savez_compressed(path, samples=s, norms=np.asarray(norms))


def load_samples_npz(path: str) -> Dict[str, np.ndarray]:
    with np.load(path, allow_pickle=False) as f:
        return {k: f[k] for k in f.files}


def basis_properties(B) -> Dict[str, Any]:
    """Determinant, condition number and row Gram-Schmidt norms of B."""
    Bf = np.asarray(B, dtype=np.float64)
    r = np.linalg.qr(Bf.T, mode="r")             # |R_ii| of B^T = norms of the row GS vectors
    gs = [float(x) for x in np.abs(np.diag(r))]
    mx, mn = max(gs), min(gs)
    return {"determinant": float(np.linalg.det(Bf)), "condition_number": float(np.linalg.cond(Bf)),
            "gs_norms": gs, "max_gs_norm": mx, "min_gs_norm": mn,
            "gs_norm_ratio": mx / mn if mn > 0 else float("inf")}


def sample_quality_metrics(coefficients) -> Dict[str, Any]:
    """Quality metrics of klein_scaling_analysis.py:191-242 from integer coefficients (n x d)."""
    from .diagnostics import _gpu
    z = _gpu.as_input(coefficients)
    n = z.shape[0]
    r = _gpu.series_stats(z, **_gpu.columns(z), max_lag=0, want=("mean", "c0"))
    means, stds = r["mean"], np.sqrt(r["c0"] / n)
    zh = z.cpu().numpy() if _gpu.is_device(z) else z
    lo, hi = zh.min(axis=0), zh.max(axis=0)
    unique = len(np.unique(np.ascontiguousarray(zh).view(np.void), axis=0))
    mean_std = np.mean(stds)
    return {
        "x1_mean": float(means[0]),
        "x1_std": float(stds[0]),
        "x1_range": [int(lo[0]), int(hi[0])],
        "mean_magnitude": float(np.mean(np.abs(means))),
        "std_uniformity": float(np.std(stds) / mean_std) if mean_std > 0 else float("inf"),
        "sample_diversity": float(unique / n),
        "all_means": [float(x) for x in means],
        "all_stds": [float(x) for x in stds],
        "all_ranges": [int(x) for x in hi - lo],
    }


def klein_scaling_record(n: int, B, sigma: float, time_per_sample_ms: float, sampling_time: float,
                         quality_metrics: Dict[str, Any], seed: int,
                         sigma_multiplier: float) -> Dict[str, Any]:
    """The JSON record of klein_scaling_analysis.py:322-336."""
    p = basis_properties(B)
    return {
        "n": n,
        "determinant": p["determinant"],
        "condition_number": p["condition_number"],
        "max_GS_norm": p["max_gs_norm"],
        "sigma": sigma,
        "time_per_sample_ms": time_per_sample_ms,
        "quality_metrics": quality_metrics,
        "seed": seed,
        "additional_info": {
            "sampling_time_total": sampling_time,
            "gs_norms": p["gs_norms"],
            "sigma_multiplier": sigma_multiplier,
        },
    }


def save_results_json(path: str, record) -> None:
    with open(path, "w") as f:
        json.dump(record, f, indent=2)
