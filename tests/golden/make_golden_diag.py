"""Generate the diagnostics golden fixtures by running the REFERENCE's own
diagnostics modules (``src/diagnostics/mcmc_diag.py``,
``src/diagnostics/convergence_diag.py``), imported read-only from
/root/reference with bytecode writing disabled.  Inputs are synthetic and
seeded here (AR(1) series with short and long memory, an integer IMHK trace
from the build's C oracle, integer sample sets); only inputs and outputs are
stored.

Usage:  python3 -B tests/golden/make_golden_diag.py          (writes tests/golden/diag_*.npz)
        python3 -B tests/golden/make_golden_diag.py binned   (only diag_tvd_binned.npz)
"""
from __future__ import annotations

import os
import sys

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "lattice-gaussian-mcmc_amd"))
sys.path.insert(0, os.path.join(REPO, "oracle"))
sys.path.insert(0, "/root/reference")

import numpy as np  # noqa: E402

from src.diagnostics import convergence_diag as cd  # noqa: E402
from src.diagnostics import mcmc_diag as md  # noqa: E402


def ar1(rng, n, rho, scale=1.0):
    x = np.zeros(n)
    e = rng.standard_normal(n)
    x[0] = e[0]
    for i in range(1, n):
        x[i] = rho * x[i - 1] + np.sqrt(1 - rho ** 2) * e[i]
    return x * scale


def series_case(name, x):
    out = {"x": x}
    out["acf_direct"] = md.compute_autocorrelation(x)
    out["acf_direct_100"] = md.compute_autocorrelation(x, max_lag=100)
    out["tau_direct"] = np.float64(md.integrated_autocorrelation_time(x))
    out["acf_fft"] = cd.compute_autocorrelation(x)
    out["tau_fft"] = np.float64(cd.integrated_autocorrelation_time(x))
    out["ess_autocorr"] = np.float64(md.effective_sample_size(x, "autocorr"))
    out["ess_batch"] = np.float64(md.effective_sample_size(x, "batch_means"))
    out["mcse_batch"] = np.float64(md.compute_mcse(x, "batch"))
    out["mcse_spectral"] = np.float64(md.compute_mcse(x, "spectral"))
    out["bm_var"] = np.float64(cd.batch_means_variance(x))
    dg = md.diagnose_chain(x)
    for k in ("mean", "std", "ess", "ess_per_sample", "tau_int", "mean_jump_distance", "acf_lag_1",
              "acf_lag_10"):
        out["diag_" + k] = np.float64(dg[k])
    out["diag_quantiles"] = np.array([dg["quantiles"][q] for q in ("2.5%", "25%", "50%", "75%", "97.5%")])
    np.savez_compressed(os.path.join(HERE, f"diag_series_{name}.npz"), **out)


def main():
    rng = np.random.default_rng(20261016)
    series_case("ar09", ar1(rng, 2000, 0.9))          # window closes within the first lag block
    series_case("ar099", ar1(rng, 9000, 0.99, 3.0))   # long memory: several lag blocks, chunked time axis
    series_case("iid_int", np.round(rng.standard_normal(3001) * 40.0))  # integer-valued, odd length
    series_case("short", ar1(rng, 9, 0.5))            # max_lag = n // 4 = 2

    # multivariate integer trace: IMHK chain of the C oracle on the NTRU d=32 basis (chain 0)
    import lgs_oracle
    from lgs_amd import lattices
    B = lattices.ntru_basis(16, 12289, 3)
    R, cp = lgs_oracle.qr_prepare(B)
    st = lgs_oracle.imhk(R, cp, B, 165.7, 2, 400, seed=11, first_step=1, trace=True,
                         mode=lgs_oracle.IMHK_WANG_LING)
    z = st["trace"][0].astype(np.int64)               # 400 x 32 coefficients
    v = (z.astype(np.float64) @ B.T)                  # lattice points B z (integer-valued)
    dgz = md.diagnose_chain(z.astype(np.float64))
    dgv = md.diagnose_chain(v)
    dgh = md.diagnose_chain(z[:, 16:].astype(np.float64))  # the coordinates that move
    out = {"z": z, "v": v, "B": B}
    for tag, dg in (("z", dgz), ("v", dgv), ("zh", dgh)):
        for k in ("ess", "ess_per_sample", "tau_int", "mean_jump_distance", "acf_lag_1", "acf_lag_10"):
            out[f"{tag}_{k}"] = np.float64(dg[k])
        out[f"{tag}_mean"] = np.asarray(dg["mean"])
        out[f"{tag}_std"] = np.asarray(dg["std"])
    out["z_ess_batch"] = np.float64(md.effective_sample_size(z.astype(np.float64), "batch_means"))
    out["zh_ess_batch"] = np.float64(md.effective_sample_size(z[:, 16:].astype(np.float64), "batch_means"))
    out["z_jumps"] = md.compute_jump_distance(z.astype(np.float64))
    out["v_cov"] = np.cov(v.T)
    out["z_cov"] = np.cov(z.astype(np.float64).T)
    np.savez_compressed(os.path.join(HERE, "diag_trace_ntru32.npz"), **out)

    # Gelman-Rubin over chains of unequal length (truncated to the shortest)
    chains = [ar1(rng, 1500 + 17 * i, 0.8, 1.0 + 0.1 * i) + 0.05 * i for i in range(5)]
    np.savez_compressed(os.path.join(HERE, "diag_gelman_rubin.npz"),
                        **{f"chain{i}": c for i, c in enumerate(chains)},
                        rhat=np.float64(cd.gelman_rubin_statistic(chains)))

    # discrete TVD: integer-valued sample sets (float arrays, as the samplers return)
    a = np.round(rng.standard_normal((3000, 6)) * np.array([1, 2, 5, 0.3, 40, 3]))
    b = np.round(rng.standard_normal((2000, 6)) * np.array([1.1, 2, 5.5, 0.3, 35, 3]) + 0.2)
    a1 = a[:, 4].copy()
    b1 = b[:, 4].copy()
    np.savez_compressed(os.path.join(HERE, "diag_tvd.npz"), a=a, b=b,
                        tvd=np.float64(cd.compute_tvd(a, b)),
                        tvd_marg=np.array([cd.compute_tvd(a[:, i], b[:, i]) for i in range(6)]),
                        tvd_1d=np.float64(cd.compute_tvd(a1, b1)),
                        mixing=np.int64(cd.mixing_time_estimate([0.9, 0.5, 0.3, 0.2, 0.1])))
    binned()
    print("wrote diag fixtures to", HERE)


def binned():
    """compute_tvd's histogram branch (convergence_diag.py:51-63, 64-72): float,
    integer-valued and int32 / int64 sample sets, a constant column (the +-0.5
    range expansion), bins = 1 .. 64; the per-column np.histogram counts the
    reference forms are stored beside its TVDs."""
    rng = np.random.default_rng(20261017)
    cases = {
        "f2d": (rng.standard_normal((2500, 5)) * [1, 3, 0.01, 50, 2] + [0, 1, 0, -7, 1e3],
                rng.standard_normal((1700, 5)) * [1.2, 3, 0.01, 45, 2] + [0.1, 1, 0, -7, 1e3 + 0.3]),
        "intval": (np.round(rng.standard_normal((3000, 4)) * [2, 40, 165.7, 0.4]),
                   np.round(rng.standard_normal((2000, 4)) * [2.2, 38, 170, 0.4])),
        "i64": (np.round(rng.standard_normal(4001) * 700).astype(np.int64),
                np.round(rng.standard_normal(3000) * 650 + 3).astype(np.int64)),
        "i32": (np.round(rng.standard_normal((1024, 3)) * [5, 5000, 1]).astype(np.int32),
                np.round(rng.standard_normal((999, 3)) * [5, 5100, 1]).astype(np.int32)),
        "const": (np.full((300, 2), 7.0), np.full((200, 2), 7.0)),
    }
    out = {}
    for name, (a, b) in cases.items():
        out[f"{name}_a"] = a
        out[f"{name}_b"] = b
        for bins in (1, 7, 10, 64):
            out[f"{name}_tvd_{bins}"] = np.float64(cd.compute_tvd(a, b, bins=bins))
            a2 = a.reshape(len(a), -1)
            b2 = b.reshape(len(b), -1)
            c1, c2 = [], []
            for i in range(a2.shape[1]):
                lo = min(a2[:, i].min(), b2[:, i].min())
                hi = max(a2[:, i].max(), b2[:, i].max())
                c1.append(np.histogram(a2[:, i], bins=bins, range=(lo, hi))[0])
                c2.append(np.histogram(b2[:, i], bins=bins, range=(lo, hi))[0])
            out[f"{name}_counts_a_{bins}"] = np.array(c1, dtype=np.int64)
            out[f"{name}_counts_b_{bins}"] = np.array(c2, dtype=np.int64)
    np.savez_compressed(os.path.join(HERE, "diag_tvd_binned.npz"), **out)


if __name__ == "__main__":
    if sys.argv[1:] == ["binned"]:
        binned()
    else:
        main()
