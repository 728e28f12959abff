"""GPU: diagnostics kernels (csrc/lgs_diag.hip) through the C-ABI and the
drop-in modules lgs_amd.diagnostics, against the reference-generated fixtures
(tests/golden/diag_*.npz) and the oracle (oracle/lgs_diag_oracle.py).

Tolerances: autocovariances are fp64 sums in a different (blocked) order than
np.correlate / FFT -> relative 1e-10 on ACF values and derived scalars; integer
moments, TVD and the window position of tau_int are exact.
"""
import glob
import os

import numpy as np
import pytest

from conftest import GOLDEN, load_golden

import lgs_diag_oracle as O

pytestmark = pytest.mark.gpu
SERIES = sorted(os.path.basename(p) for p in glob.glob(os.path.join(GOLDEN, "diag_series_*.npz")))
RT = 1e-10


@pytest.fixture(scope="module")
def D():
    from lgs_amd import diagnostics
    return diagnostics


@pytest.mark.parametrize("name", SERIES)
def test_series_diagnostics_match_reference(D, name):
    g = load_golden(name)
    x = g["x"]
    np.testing.assert_allclose(D.compute_autocorrelation(x), g["acf_direct"], rtol=RT, atol=1e-13)
    np.testing.assert_allclose(D.mcmc_diag.compute_autocorrelation(x, 100), g["acf_direct_100"], rtol=RT,
                               atol=1e-13)
    np.testing.assert_allclose(D.convergence_diag.compute_autocorrelation(x), g["acf_fft"], rtol=RT,
                               atol=1e-12)
    np.testing.assert_allclose(D.integrated_autocorrelation_time(x), g["tau_direct"], rtol=RT)
    np.testing.assert_allclose(D.convergence_diag.integrated_autocorrelation_time(x), g["tau_fft"], rtol=RT)
    np.testing.assert_allclose(D.effective_sample_size(x), g["ess_autocorr"], rtol=RT)
    np.testing.assert_allclose(D.effective_sample_size(x, "batch_means"), g["ess_batch"], rtol=RT)
    np.testing.assert_allclose(D.compute_mcse(x, "batch"), g["mcse_batch"], rtol=RT)
    np.testing.assert_allclose(D.compute_mcse(x, "spectral"), g["mcse_spectral"], rtol=RT)
    np.testing.assert_allclose(D.batch_means_variance(x), g["bm_var"], rtol=RT)
    dg = D.diagnose_chain(x)
    for k in ("mean", "std", "ess", "ess_per_sample", "tau_int", "mean_jump_distance", "acf_lag_1",
              "acf_lag_10"):
        val = np.nan if dg[k] is None else dg[k]  # the fixture stores None as NaN
        np.testing.assert_allclose(val, g["diag_" + k], rtol=RT, atol=1e-13, err_msg=k)
    np.testing.assert_array_equal([dg["quantiles"][q] for q in ("2.5%", "25%", "50%", "75%", "97.5%")],
                                  g["diag_quantiles"])


def test_multivariate_trace_diagnostics(D):
    g = load_golden("diag_trace_ntru32.npz")
    z = g["z"]
    for tag, x in (("z", z.astype(np.float64)), ("v", g["v"]), ("zh", z[:, 16:].astype(np.float64)),
                   ("zh", np.ascontiguousarray(z[:, 16:]))):  # int64 input: exact sums
        dg = D.diagnose_chain(x)
        for k in ("ess", "ess_per_sample", "tau_int", "mean_jump_distance", "acf_lag_1", "acf_lag_10"):
            np.testing.assert_allclose(dg[k], g[f"{tag}_{k}"], rtol=RT, atol=1e-13, err_msg=f"{tag} {k}")
        np.testing.assert_array_equal(dg["mean"], g[f"{tag}_mean"])
        np.testing.assert_allclose(dg["std"], g[f"{tag}_std"], rtol=1e-12)
    np.testing.assert_allclose(D.effective_sample_size(z[:, 16:].astype(np.float64), "batch_means"),
                               g["zh_ess_batch"], rtol=RT)
    np.testing.assert_allclose(D.compute_jump_distance(z.astype(np.int32)), g["z_jumps"], rtol=1e-15)
    np.testing.assert_allclose(D.empirical_covariance(g["v"]), g["v_cov"], rtol=1e-12, atol=1e-9)
    np.testing.assert_allclose(D.empirical_covariance(z), g["z_cov"], rtol=1e-12, atol=1e-9)


def test_gelman_rubin_tvd_mixing(D):
    g = load_golden("diag_gelman_rubin.npz")
    chains = [g[f"chain{i}"] for i in range(5)]
    np.testing.assert_allclose(D.gelman_rubin_statistic(chains), g["rhat"], rtol=RT)
    t = load_golden("diag_tvd.npz")
    assert D.compute_tvd(t["a"], t["b"]) == t["tvd"]                    # bit-identical
    assert D.compute_tvd(t["a"][:, 4], t["b"][:, 4]) == t["tvd_1d"]
    assert D.compute_tvd(t["a"].astype(np.int32), t["b"].astype(np.int32)) == t["tvd"]
    assert D.mixing_time_estimate([0.9, 0.5, 0.3, 0.2, 0.1]) == t["mixing"]
    with pytest.raises(Exception):
        D.compute_tvd(t["a"] + 0.5, t["b"])                             # not integer-valued


@pytest.mark.parametrize("name", ["f2d", "intval", "i64", "i32", "const"])
def test_binned_tvd_matches_reference(D, name):
    """compute_tvd(..., bins=k) (convergence_diag.py:51-63): the device's
    np.histogram counts equal numpy's, the TVD the reference's (bit-identical)."""
    import torch
    from lgs_amd.diagnostics import _gpu
    t = load_golden("diag_tvd_binned.npz")
    a, b = t[f"{name}_a"], t[f"{name}_b"]
    for bins in (1, 7, 10, 64):
        assert D.compute_tvd(a, b, bins=bins) == t[f"{name}_tvd_{bins}"], bins
        ad = torch.from_numpy(np.ascontiguousarray(a)).cuda()
        bd = torch.from_numpy(np.ascontiguousarray(b)).cuda()
        assert D.compute_tvd(ad, bd, bins=bins) == t[f"{name}_tvd_{bins}"], bins
        # the counts themselves, through the C-ABI
        a2 = np.ascontiguousarray(a.reshape(len(a), -1))
        ctx = _gpu.context()
        d = a2.shape[1]
        lo, hi = np.empty(d), np.empty(d)
        ctx.column_range(a2, lo, hi)
        np.testing.assert_array_equal(lo, a2.min(axis=0))
        np.testing.assert_array_equal(hi, a2.max(axis=0))
        b2 = b.reshape(len(b), -1)
        edges = np.empty((d, bins + 1))
        fd = np.empty((d, 2))
        for i in range(d):
            mn = min(a2[:, i].min(), b2[:, i].min())
            mx = max(a2[:, i].max(), b2[:, i].max())
            edges[i], fd[i] = D.convergence_diag._bin_setup(mn, mx, bins)
        c = np.empty((d, bins), dtype=np.int64)
        ctx.histogram(a2, edges, fd, c)
        np.testing.assert_array_equal(c, t[f"{name}_counts_a_{bins}"])


def test_binned_tvd_edges(D):
    """Histogram branch edge cases: values on every bin edge (the +-1 index
    corrections), a NaN (the reference's range check raises ValueError), empty input."""
    x = np.linspace(-3.0, 5.0, 81)      # many values exactly on the edges of 8 / 16 / 80 bins
    y = np.concatenate([x, x[::3]])
    for bins in (8, 16, 80, 81, 3):
        assert D.compute_tvd(x, y, bins=bins) == O.tvd_binned(x, y, bins)
    big = np.array([2 ** 52, 2 ** 52 + 1, -(2 ** 52), 5], dtype=np.int64)
    assert D.compute_tvd(big, big[::-1].copy(), bins=5) == O.tvd_binned(big, big[::-1], 5)
    with pytest.raises(ValueError):
        D.compute_tvd(np.array([1.0, np.nan]), np.array([1.0, 2.0]), bins=4)
    with pytest.raises(ValueError):
        D.compute_tvd(np.array([]), np.array([1.0]), bins=4)


@pytest.mark.parametrize("n,d,lo,hi", [(1, 5, -3, 3), (63, 130, -32639, 32640), (1000, 128, -200, 200),
                                       (4099, 257, -3000, 3000), (777, 33, -40000, 40000)])
def test_gram_exact(D, n, d, lo, hi):
    rng = np.random.default_rng(n * 7 + d)
    z = rng.integers(lo, hi, size=(n, d)).astype(np.int32)
    s_ref, G_ref = O.gram_exact(z)
    s, G = D.gram(z)
    np.testing.assert_array_equal(s, s_ref.astype(np.int64))
    np.testing.assert_array_equal(G, G_ref.astype(np.int64))
    s64, G64 = D.gram(z.astype(np.int64))
    np.testing.assert_array_equal(G64, G)
    sh = rng.integers(-50, 50, size=d)
    s2, G2 = D.gram(z, shift=sh)
    _, G2_ref = O.gram_exact(z.astype(np.int64) - sh)
    np.testing.assert_array_equal(G2, G2_ref.astype(np.int64))


def test_gram_accumulates_and_coordinate_major():
    from lgs_amd import _capi
    from lgs_amd.diagnostics import _gpu
    ctx = _gpu.context()
    rng = np.random.default_rng(5)
    z = rng.integers(-900, 900, size=(300, 40)).astype(np.int32)
    s = np.full(40, 7, dtype=np.int64)
    G = np.ones((40, 40), dtype=np.int64)
    ctx.gram(np.ascontiguousarray(z.T), sum_out=s, gram_out=G, coord_major=True)
    _, G_ref = O.gram_exact(z)
    np.testing.assert_array_equal(G, G_ref.astype(np.int64) + 1)
    np.testing.assert_array_equal(s, z.sum(0) + 7)


def test_covariance_real_and_device_tensors(D):
    import torch
    rng = np.random.default_rng(9)
    x = rng.standard_normal((5000, 24)) * np.linspace(0.5, 3, 24) + 10.0
    np.testing.assert_allclose(D.empirical_covariance(x), np.cov(x.T), rtol=1e-10, atol=1e-12)
    np.testing.assert_allclose(D.empirical_mean(x), np.mean(x, axis=0), rtol=1e-13)
    xt = torch.as_tensor(x, device="cuda")
    np.testing.assert_allclose(D.empirical_covariance(xt), np.cov(x.T), rtol=1e-10, atol=1e-12)
    zi = np.round(x * 100).astype(np.int64)
    zt = torch.as_tensor(zi, device="cuda")
    np.testing.assert_allclose(D.empirical_covariance(zt), np.cov(zi.T.astype(np.float64)), rtol=1e-12)
    np.testing.assert_allclose(D.effective_sample_size(xt), O.effective_sample_size(x), rtol=RT)
    np.testing.assert_allclose(D.compute_jump_distance(xt), O.jump_distance(x), rtol=1e-14)
    a = rng.integers(0, 2, size=1000).astype(bool)
    assert D.compute_acceptance_rate(a) == np.mean(a)


def test_series_long_and_strided_layouts():
    """Chunked time axis (n > 4096), many lag blocks, IMHK-trace layout (chains x
    steps x d) read in place, early-exit tau equals the full-scan tau."""
    from lgs_amd.diagnostics import _gpu
    rng = np.random.default_rng(11)
    nc, T, d = 3, 9000, 5
    e = rng.standard_normal((nc, T, d))
    x = np.empty_like(e)
    x[:, 0] = e[:, 0]
    for t in range(1, T):
        x[:, t] = 0.995 * x[:, t - 1] + 0.1 * e[:, t]
    x = np.ascontiguousarray(x)
    L = 700
    r = _gpu.series_stats(x, n_series=nc * d, n=T, group_size=d, group_stride=T * d, series_stride=1,
                          time_stride=d, max_lag=L, want=("mean", "c0", "acf", "tau"))
    r2 = _gpu.series_stats(x, n_series=nc * d, n=T, group_size=d, group_stride=T * d, series_stride=1,
                           time_stride=d, max_lag=L, want=("tau",))
    for c in range(nc):
        for i in range(d):
            s = c * d + i
            ref = O.autocorrelation_direct(x[c, :, i], L)
            np.testing.assert_allclose(r["acf"][s], ref, rtol=1e-9, atol=1e-12)
            np.testing.assert_allclose(r["tau"][s], O.tau_window(ref), rtol=1e-9)
            assert r2["tau"][s] == r["tau"][s]
            np.testing.assert_allclose(r["mean"][s], np.mean(x[c, :, i]), rtol=1e-12)


def test_series_edge_cases(D):
    # constant series: 0/0 -> NaN exactly like the reference (mcmc_diag.py:31)
    acf = D.compute_autocorrelation(np.full(40, 3.0))
    assert np.isnan(acf).all() and len(acf) == 11
    assert np.isnan(D.integrated_autocorrelation_time(np.full(40, 3.0)))
    # single sample
    assert len(D.compute_autocorrelation(np.array([2.0]))) == 1
    # max_lag beyond the series: numpy slicing keeps n lags
    x = np.arange(6, dtype=np.float64)
    np.testing.assert_allclose(D.compute_autocorrelation(x, 50), O.autocorrelation_direct(x, 50), rtol=1e-12)


def test_reference_style_statistical_properties(D):
    """The assertion styles of the reference's tests/unit/test_diagnostics.py on the
    GPU drop-ins: ESS of independent draws > n/2 and above that of an AR(1) chain,
    R-hat ~ 1 for converged chains and > 1.1 for shifted ones, TVD of a set with
    itself exactly 0, mixing time monotone in the threshold."""
    rng = np.random.default_rng(7)
    n = 4000
    iid = rng.standard_normal(n)
    ar = np.zeros(n)
    for i in range(1, n):
        ar[i] = 0.9 * ar[i - 1] + np.sqrt(1 - 0.81) * rng.standard_normal()
    ess_iid, ess_ar = D.effective_sample_size(iid), D.effective_sample_size(ar)
    assert n * 0.5 < ess_iid <= n * 1.5 and 1 < ess_ar < ess_iid
    conv = [rng.standard_normal(1000) for _ in range(4)]
    shifted = [rng.standard_normal(1000) + i for i in range(4)]
    r1, r2 = D.gelman_rubin_statistic(conv), D.gelman_rubin_statistic(shifted)
    assert 1.0 <= r1 < 1.2 and r2 > 1.1 and r2 > r1
    s = np.array([1, 2, 3, 1, 2, 3], dtype=np.float64)
    assert D.compute_tvd(s, s) == 0.0
    assert D.compute_tvd(np.ones(100), np.ones(100)) == 0.0
    assert D.compute_tvd(np.array([]), np.array([])) == 0.0
    with pytest.raises(ZeroDivisionError):
        D.compute_tvd(np.array([]), np.array([1.0]))
    tv = [0.9, 0.6, 0.4, 0.2, 0.05]
    assert D.mixing_time_estimate(tv, 0.1) >= D.mixing_time_estimate(tv, 0.5)


def test_sample_quality_metrics_on_gpu():
    """klein_scaling_analysis.py:191-242 metrics from device-computed moments."""
    from lgs_amd import io
    rng = np.random.default_rng(12)
    z = rng.integers(-40, 40, size=(3000, 9)).astype(np.int64)
    z[5] = z[6]
    m = io.sample_quality_metrics(z)
    means, stds = np.mean(z, axis=0), np.std(z, axis=0)
    np.testing.assert_array_equal(m["all_means"], means)
    np.testing.assert_allclose(m["all_stds"], stds, rtol=1e-13)
    assert m["all_ranges"] == [int(x) for x in np.ptp(z, axis=0)]
    assert m["sample_diversity"] == len(np.unique(z.view(np.void), axis=0)) / 3000
    assert m["x1_range"] == [int(z[:, 0].min()), int(z[:, 0].max())]
