"""HIP path vs the oracle and the reference's golden vectors (needs an MI355X).

Integer outputs (coefficients z, accept decisions, moments) must be bit-exact;
lattice points v = B z are exact for integer bases (all partial sums are
integers < 2^53) and within rtol 1e-12 otherwise.  Both device samplers are
checked: LGS_EXACT_ORDER (the reference's sequential fp64 order) and the
default blocked panel kernel.
"""
import os

import numpy as np
import pytest

from conftest import golden_R, klein_goldens, load_golden

pytestmark = pytest.mark.gpu

MODES = {"exact": 2, "panel": 0}  # LGS_EXACT_ORDER = 0x2


@pytest.fixture(scope="module")
def capi():
    from lgs_amd import _capi
    return _capi


@pytest.fixture(scope="module")
def ctx(capi):
    return capi.Context(0)


def _is_int(B):
    return B is not None and np.array_equal(B, np.round(B))


@pytest.mark.parametrize("mode", list(MODES))
@pytest.mark.parametrize("name", klein_goldens())
def test_klein_matches_reference_goldens(ctx, name, mode):
    g = load_golden(name)
    R, cp, B = golden_R(g)
    ctx.set_basis(R, cp, B, float(g["sigma"]))
    r = ctx.klein_host(int(g["seed"]), int(g["first_sample"]), int(g["n"]), want_z=True,
                       want_v=True, flags=MODES[mode])
    mism = ~(r["z"] == g["z"]).all(1)
    assert mism.sum() == 0, f"{mism.sum()} of {len(mism)} samples differ"
    if "v" in g:
        if _is_int(B):
            assert np.array_equal(r["v"], g["v"])
        else:
            np.testing.assert_allclose(r["v"], g["v"], rtol=1e-12, atol=1e-9)


@pytest.mark.parametrize("mode", list(MODES))
@pytest.mark.parametrize("case", ["ntru128", "qary128", "gauss16", "Z64", "B2_center"])
def test_klein_matches_oracle_seeded(ctx, oracle, case, mode):
    g = load_golden(f"klein_{case}.npz")
    R, cp, B = golden_R(g)
    sigma = float(g["sigma"])
    seed, first, n = 0xC0FFEE + len(case), 12345, 1536
    ctx.set_basis(R, cp, B, sigma)
    r = ctx.klein_host(seed, first, n, want_z=True, want_v=True, flags=MODES[mode])
    o = oracle.klein(R, cp, sigma, n, seed=seed, first_sample=first, B=B)
    assert np.array_equal(r["z"], o["z"])
    if _is_int(B):
        assert np.array_equal(r["v"], o["v"])
    else:
        np.testing.assert_allclose(r["v"], o["v"], rtol=1e-12, atol=1e-9)


@pytest.fixture(scope="module")
def ctx_libm(capi):
    """A context on the generic SampleZ path (ocml erf/exp/erfinv, no per-coordinate constants)."""
    return capi.Context(0, samplez_libm=True)


def _wide_sigma_basis(d, seed):
    """Upper-triangular basis whose sigma_i = sigma/R_ii span every SampleZ kind:
    tiny (< 0.1), small (< 4), uncapped wide (4..50), capped (> 50), clamped (> 1e10)."""
    rng = np.random.default_rng(seed)
    sig_i = np.exp(rng.uniform(np.log(1e-3), np.log(3e3), d))
    sig_i[::7] = rng.uniform(45, 55, len(sig_i[::7]))  # around the cap threshold
    sig_i[3] = 1e11
    diag = 10.0 / sig_i
    R = np.diag(diag)
    R[np.arange(d - 1), np.arange(1, d)] = diag[:-1] * rng.uniform(-0.5, 0.5, d - 1)
    R[np.arange(d - 2), np.arange(2, d)] = diag[:-2] * rng.uniform(-0.2, 0.2, d - 2)
    return R, rng.normal(size=d) * diag * 300.0


@pytest.mark.parametrize("precision", [3, 8, 10, 20])
@pytest.mark.parametrize("wl", [False, True])
def test_klein_coord_constants_vs_generic_samplez(ctx, ctx_libm, oracle, capi, precision, wl):
    """Per-coordinate SampleZ constants (closed-form / fitted window normalisers)
    give the generic path's decisions and log-weights, and the oracle's z."""
    R, cp = _wide_sigma_basis(96, precision)
    out = []
    flags = capi.LGS_WANG_LING if wl else 0
    for c in (ctx, ctx_libm):
        c.set_basis(R, cp, None, 10.0, precision=precision)
        out.append(c.klein_host(99, 5, 3000, want_z=True, want_v=False, want_logw=True, flags=flags))
    assert np.array_equal(out[0]["z"], out[1]["z"])
    np.testing.assert_allclose(out[0]["logw"], out[1]["logw"], rtol=1e-12, atol=1e-9)
    o = oracle.klein(R, cp, 10.0, 200, seed=99, first_sample=5, precision=precision)
    assert np.array_equal(out[0]["z"][:200], o["z"])


@pytest.fixture(scope="module")
def ctx_far64(capi):
    """A context whose 32-row-panel kernel uses the fp64 MFMA far field."""
    return capi.Context(0, far="fp64")


def test_int8_digit_far_field_matches_fp64_far_field(ctx, ctx_far64, oracle):
    """The exact int8-digit far field and the fp64 MFMA far field give the same
    coefficients on the full-size NTRU basis, and both match the oracle."""
    from lgs_amd.lattices import build_config
    lat, sigma = build_config("C3_ntru512")
    B = lat.basis
    R = np.linalg.qr(B)[1]
    R = np.ascontiguousarray(R * np.where(np.diag(R) < 0, -1.0, 1.0)[:, None])
    cp = np.zeros(B.shape[0])
    out = []
    for c in (ctx, ctx_far64):
        c.set_basis(R, cp, B, sigma)
        out.append(c.klein_host(7, 1 << 20, 4096, want_z=True, want_v=False)["z"])
    assert np.array_equal(out[0], out[1])
    o = oracle.klein(R, cp, sigma, 64, seed=7, first_sample=1 << 20)
    assert np.array_equal(out[0][:64], o["z"])


def test_int8_digit_far_field_zero_panel_skip(ctx, oracle):
    """Far-field chunks whose panels are zero in every sample of a block are
    skipped.  Panels 1, 2 and 5 (rows d-32(q+1) .. d-32q-1) are pinned to z = 0
    (sigma_i ~ 3e-4); one row of panel 6 is a centred sigma_i = 0.25 coordinate, so
    it is nonzero in only a few samples of a few 256-sample blocks: those blocks
    must keep the chunk, the others skip it.  Bit-exact against the oracle."""
    rng = np.random.default_rng(17)
    d, sigma, n = 320, 3.0, 4096
    R = np.triu(rng.normal(size=(d, d)) * 0.3, 1)
    R[np.diag_indices(d)] = rng.uniform(0.5, 2.0, d)
    cp = rng.normal(size=d)
    for q in (1, 2, 5):
        rows = np.arange(d - 32 * (q + 1), d - 32 * q)
        R[rows, rows] = 1e4
        cp[rows] = 0.0
    rare = d - 32 * 7 + 5  # in panel 6
    q6 = np.arange(d - 32 * 7, d - 32 * 6)
    R[q6, q6] = 1e4
    cp[q6] = 0.0
    R[rare, rare + 1:] = 0.0
    R[rare, rare] = sigma / 0.25
    ctx.set_basis(R, cp, None, sigma)
    r = ctx.klein_host(23, 0, n, want_z=True, want_v=False)["z"]
    o = oracle.klein(R, cp, sigma, n, seed=23, first_sample=0)["z"]
    for q in (1, 2, 5):
        assert not o[:, d - 32 * (q + 1):d - 32 * q].any()
    hits = np.flatnonzero(o[:, rare])
    blocks = np.unique(hits // 256)
    assert 0 < len(blocks) < n // 256, (hits, blocks)
    assert not np.delete(o[:, q6], rare - q6[0], axis=1).any()
    assert np.array_equal(r, o)


def test_int8_digit_far_field_overflow_falls_back(capi, oracle):
    """|z| > 32639 cannot use the int16 history (it holds z + 128): the launch is
    redone with the fp64 far field (same counters) and the context keeps it."""
    rng = np.random.default_rng(5)
    d = 96
    R = np.triu(rng.normal(size=(d, d)) * 0.01, 1)
    R[np.diag_indices(d)] = rng.uniform(0.5, 2.0, d)
    cp = rng.normal(size=d) * 4e4
    c = capi.Context(0)
    c.set_basis(R, cp, None, 3.0)
    r = c.klein_host(11, 0, 256, want_z=True, want_v=False)
    o = oracle.klein(R, cp, 3.0, 256, seed=11, first_sample=0)
    assert np.abs(o["z"]).max() > 32767
    assert np.array_equal(r["z"], o["z"])


def test_klein_full_size_ntru1024_vs_oracle(ctx, oracle):
    """BASELINE config C3 basis (d = 1024): device vs oracle on 64 samples, both kernels."""
    from lgs_amd.lattices import build_config
    lat, sigma = build_config("C3_ntru512")
    R, cp = oracle.qr_prepare(lat.basis)
    ctx.set_basis(R, cp, lat.basis, sigma)
    o = oracle.klein(R, cp, sigma, 64, seed=99, first_sample=7, B=lat.basis)
    for f in MODES.values():
        r = ctx.klein_host(99, 7, 64, want_z=True, want_v=True, flags=f)
        assert np.array_equal(r["z"], o["z"])
        assert np.array_equal(r["v"], o["v"])


def test_klein_batch_and_offset_invariance(ctx):
    g = load_golden("klein_ntru128.npz")
    R, cp, B = golden_R(g)
    ctx.set_basis(R, cp, B, float(g["sigma"]))
    a = ctx.klein_host(5, 0, 3000, want_z=True, want_v=False)["z"]
    b1 = ctx.klein_host(5, 0, 1234, want_z=True, want_v=False)["z"]
    b2 = ctx.klein_host(5, 1234, 3000 - 1234, want_z=True, want_v=False)["z"]
    assert np.array_equal(a, np.vstack([b1, b2]))
    c = ctx.klein_host(5, 1000, 10, want_z=True, want_v=False)["z"]
    assert np.array_equal(c, a[1000:1010])
    d = ctx.klein_host(6, 0, 10, want_z=True, want_v=False)["z"]
    assert not np.array_equal(d, a[:10])


def test_small_launch_chunks_and_panel16(capi, oracle):
    """Chunked launches (max_proposals) and the 16-row panel give identical z."""
    g = load_golden("klein_qary128.npz")
    R, cp, B = golden_R(g)
    c2 = capi.Context(0, max_proposals=100, panel=16)
    c2.set_basis(R, cp, B, float(g["sigma"]))
    r = c2.klein_host(int(g["seed"]), 0, int(g["n"]), want_z=True, want_v=True)
    assert np.array_equal(r["z"], g["z"])
    assert np.array_equal(r["v"], g["v"])


def test_overflow_falls_back_to_int64(ctx, capi):
    g = load_golden("klein_edge6.npz")
    R, cp, B = golden_R(g)
    ctx.set_basis(R, cp, B, float(g["sigma"]))
    z32 = np.empty((4, 6), dtype=np.int32)
    with pytest.raises(capi.LgsError) as e:
        ctx.klein(int(g["seed"]), 0, 4, z32, None, None, 0)
    assert e.value.code == capi.LGS_ERR_OVERFLOW
    r = ctx.klein_host(int(g["seed"]), 0, int(g["n"]), want_z=True, want_v=True)
    assert np.array_equal(r["z"], g["z"])


def test_device_pointers_coordinate_major(ctx, capi):
    import torch
    g = load_golden("klein_ntru32.npz")
    R, cp, B = golden_R(g)
    ctx.set_basis(R, cp, B, float(g["sigma"]))
    n, d = int(g["n"]), R.shape[0]
    z = torch.empty((d, n), dtype=torch.int32, device="cuda:0")
    v = torch.empty((n, d), dtype=torch.float64, device="cuda:0")
    lw = torch.empty((n,), dtype=torch.float64, device="cuda:0")
    torch.cuda.synchronize()
    ctx.klein(int(g["seed"]), 0, n, z, v, lw, capi.LGS_DEVICE_PTRS | capi.LGS_COORD_MAJOR)
    assert np.array_equal(z.cpu().numpy().T, g["z"])
    assert np.array_equal(v.cpu().numpy(), g["v"])
    zr = torch.empty((n, d), dtype=torch.int32, device="cuda:0")
    ctx.klein(int(g["seed"]), 0, n, zr, None, None, capi.LGS_DEVICE_PTRS)
    assert np.array_equal(zr.cpu().numpy(), g["z"])


def test_lattice_points_and_log_density(ctx, oracle):
    g = load_golden("klein_gauss16.npz")
    R, cp, B = golden_R(g)
    sigma = float(g["sigma"])
    ctx.set_basis(R, cp, B, sigma)
    v = ctx.lattice_points(g["z"].astype(np.int64))
    np.testing.assert_allclose(v, g["v"], rtol=1e-12, atol=1e-9)
    lq = ctx.log_density(g["z"][:32])
    for k in range(32):
        z = g["z"][k]
        lw = oracle.log_weight(R, cp, B, sigma, z, center=g["center"])
        vv = B @ z
        log_target = -np.dot(vv - g["center"], vv - g["center"]) / (2 * sigma ** 2)
        assert lq[k] == pytest.approx(log_target - lw, rel=1e-11, abs=1e-9)


# ------------------------------------------------------------------ IMHK
def _imhk_dev(ctx, R, cp, B, sigma, nc, steps, seed, thin=1, flags=0, split=None, moments=False):
    d = R.shape[0]
    ctx.set_basis(R, cp, B, sigma)
    st = dict(z=np.zeros((nc, d), dtype=np.int32), lw=np.zeros(nc), init=np.zeros(nc, dtype=np.int32),
              acc=np.zeros(nc, dtype=np.int64))
    mom = np.zeros(2 * d, dtype=np.int64) if moments else None
    parts = [steps] if split is None else split
    outs, t = [], 1
    for s in parts:
        zs = np.zeros((nc, s // thin, d), dtype=np.int32)
        ctx.imhk(seed, 0, nc, t, s, thin, st["z"], st["lw"], st["init"], st["acc"], z_samples=zs,
                 moments=mom, flags=flags)
        outs.append(zs)
        t += s
    return st, np.concatenate(outs, axis=1), mom


@pytest.mark.parametrize("mode", list(MODES))
@pytest.mark.parametrize("name", ["imhk_ntru32.npz", "imhk_B2.npz"])
def test_imhk_matches_reference_goldens(ctx, name, mode):
    g = load_golden(name)
    nc, ns, d = g["z"].shape
    st, trace, _ = _imhk_dev(ctx, g["R"], g["cprime"], g["B"], float(g["sigma"]), nc, ns,
                             int(g["seed"]), flags=MODES[mode])
    assert np.array_equal(trace, g["z"])
    assert np.array_equal(st["acc"], g["accepted"].sum(1))
    np.testing.assert_allclose(st["lw"], g["log_weight"][:, -1], rtol=1e-10)


@pytest.mark.parametrize("wl", [False, True])
def test_imhk_matches_oracle(ctx, oracle, capi, wl):
    g = load_golden("klein_ntru32.npz")
    R, cp, B = golden_R(g)
    sigma = float(g["sigma"])
    nc, steps, thin = 8, 48, 3
    flags = capi.LGS_WANG_LING if wl else 0
    st, zs, mom = _imhk_dev(ctx, R, cp, B, sigma, nc, steps, 777, thin=thin, flags=flags,
                            split=[24, 24], moments=True)
    o = oracle.imhk(R, cp, B, sigma, nc, steps, seed=777, first_step=1,
                    mode=oracle.IMHK_WANG_LING if wl else oracle.IMHK_REFERENCE, trace=True)
    kept = o["trace"][:, thin - 1::thin]
    assert np.array_equal(zs, kept)
    assert np.array_equal(st["acc"], o["accepts"])
    assert np.array_equal(st["z"], o["z"])
    np.testing.assert_allclose(st["lw"], o["lw"], rtol=1e-9)
    flat = kept.reshape(-1, R.shape[0]).astype(np.int64)
    assert np.array_equal(mom[: R.shape[0]], flat.sum(0))
    assert np.array_equal(mom[R.shape[0]:], (flat * flat).sum(0))
    if not wl:
        assert st["acc"].sum() == nc * steps  # reference-mode acceptance is exactly 1


def test_imhk_block_split_invariance(capi):
    g = load_golden("klein_ntru128.npz")
    R, cp, B = golden_R(g)
    c2 = capi.Context(0, max_proposals=200)
    st_a, zs_a, mom_a = _imhk_dev(c2, R, cp, B, float(g["sigma"]), 16, 40, 31, thin=2,
                                  flags=capi.LGS_WANG_LING, moments=True)
    c3 = capi.Context(0)
    st_b, zs_b, mom_b = _imhk_dev(c3, R, cp, B, float(g["sigma"]), 16, 40, 31, thin=2,
                                  flags=capi.LGS_WANG_LING, split=[10, 30], moments=True)
    assert np.array_equal(zs_a, zs_b)
    assert np.array_equal(st_a["acc"], st_b["acc"])
    assert np.array_equal(mom_a, mom_b)


# ------------------------------------------------------------------ drop-in API
def test_drop_in_klein_sampler(oracle):
    from lgs_amd.lattices import SimpleLattice
    from lgs_amd.samplers import KleinSampler
    B = np.array([[4.0, 1.0], [1.0, 3.0]])
    s = KleinSampler(SimpleLattice(B), 2.0, seed=11)
    v = s.sample(2000)
    assert v.shape == (2000, 2) and s.sample(1).shape == (1, 2) and s.sample_single().shape == (2,)
    R, cp = oracle.qr_prepare(B)
    o = oracle.klein(R, cp, 2.0, 2000, seed=11, B=B)
    assert np.array_equal(v, o["v"])
    np.random.seed(3)
    a = KleinSampler(SimpleLattice(B), 2.0).sample(50)
    np.random.seed(3)
    b = KleinSampler(SimpleLattice(B), 2.0).sample(50)
    assert np.array_equal(a, b)
    # empirical moments (reference test style: mean within 3 sigma / sqrt(N))
    big = KleinSampler(SimpleLattice(np.eye(8)), 5.0, seed=4).sample(20000)
    assert np.all(np.abs(big.mean(0)) < 3 * 5 / np.sqrt(20000) * 1.5)
    np.testing.assert_allclose(np.cov(big.T), 25 * np.eye(8), atol=0.1 * 25)
    assert np.isfinite(s.compute_log_density(v[0]))
    assert s.compute_log_density(v[0] + 0.5) == -np.inf
    info = s.diagnostic_info()
    assert info["algorithm"] == "Refined Klein"


def test_drop_in_imhk_sampler(oracle):
    from lgs_amd.lattices import SimpleLattice
    from lgs_amd.samplers import IMHKSampler
    g = load_golden("imhk_B2.npz")
    s = IMHKSampler(SimpleLattice(g["B"]), float(g["sigma"]), burn_in=0, seed=int(g["seed"]),
                    chain_id=0)
    states = [s.step()[0] for _ in range(5)]
    rest = s.sample(195)
    V = np.vstack([np.array(states), rest])
    ref = (g["B"] @ g["z"][0].T).T
    assert np.array_equal(V, ref)
    assert s.accepted_proposals == s.total_proposals == 200
    assert s.stats.acceptance_rate == 1.0
    chain = s.run_chain(10, save_every=3)
    assert len(chain) == 4


# ------------------------------------------------------------------ SampleZ unit tests
@pytest.mark.parametrize("table", [False, True])
def test_samplez_reference_decision_table(ctx, table):
    """Device SampleZ (Euler-Maclaurin path and table walk) vs the reference's own
    decisions over 13 sigma regimes (tests/golden/samplez_table.npz)."""
    g = load_golden("samplez_table.npz")
    z, ln = ctx.sample_z(g["mu"], g["sigma"], g["u"], table=table)
    assert np.array_equal(z, g["z"])


def test_samplez_log_normalisers_vs_reference(ctx):
    """Device 1-D normalisers (the Wang-Ling weight's factors) vs
    the reference's own window logsumexp (tests/golden/samplez_lognorm.npz), on the
    Euler-Maclaurin path and the table walk."""
    g = load_golden("samplez_lognorm.npz")
    u = np.full(g["mu"].size, 0.5)
    for table in (False, True):
        _, ln = ctx.sample_z(g["mu"], g["sigma"], u, table=table)
        np.testing.assert_allclose(ln, g["log_norm"], rtol=1e-12, atol=1e-12)


def _window(mu, sig, precision=10):
    rf = np.where(sig < 0.1, max(precision, 3), precision).astype(np.float64)
    lo = np.floor(mu - rf * sig).astype(np.int64)
    hi = np.ceil(mu + rf * sig).astype(np.int64)
    cap = hi - lo > 1000
    c = np.rint(mu).astype(np.int64)
    return np.where(cap, c - 500, lo), np.where(cap, c + 500, hi)


def test_samplez_decision_golden(ctx):
    """Decision-only mode (fp32 certificate for wide windows) on the reference's decisions."""
    g = load_golden("samplez_table.npz")
    z, _ = ctx.sample_z(g["mu"], g["sigma"], g["u"], mode="decision")
    assert np.array_equal(z, g["z"])


def test_samplez_near_boundaries(ctx):
    """u placed at +-eps around exact CDF boundaries (long-double table sums):
    the tabulated Euler-Maclaurin path, the libm path and the table walk agree
    (draws inside the 1e-12 S margin go to the table walk in both EM paths)."""
    rng = np.random.default_rng(77)
    mus, sigs, us = [], [], []
    for _ in range(300):
        sig = float(np.exp(rng.uniform(np.log(4.0), np.log(1e6))))
        mu = float(rng.uniform(-1, 1) * rng.choice([1.0, 50.0, 1e5]))
        lo, hi = _window(np.array([mu]), np.array([sig]))
        k = np.arange(lo[0], hi[0] + 1, dtype=np.longdouble)
        w = np.exp(-0.5 * ((k - np.longdouble(mu)) / np.longdouble(sig)) ** 2)
        F = np.cumsum(w) / np.sum(w)
        for j in rng.choice(len(F) - 1, 3):
            for eps in (-1e-6, -1e-9, -1e-11, -1e-13, 1e-13, 1e-11, 1e-9, 1e-6):
                u = float(F[j]) + eps
                if 0.0 <= u < 1.0:
                    mus.append(mu), sigs.append(sig), us.append(u)
    mu, sig, u = np.array(mus), np.array(sigs), np.array(us)
    z_t, ln_t = ctx.sample_z(mu, sig, u, table=True)
    for mode in (None, "decision", "libm", "libm_decision"):
        z, ln = ctx.sample_z(mu, sig, u, mode=mode)
        assert np.array_equal(z, z_t), mode
        if mode in (None, "libm"):
            np.testing.assert_allclose(ln, ln_t, rtol=1e-13, atol=1e-13)


def test_samplez_capped_quantile_near_boundaries(ctx):
    """The capped kind (sigma >= 360, window rint(mu) +- 500) decides most draws from
    the quantile alone (lgs_device.h sample_z_capped): u placed just around exact
    CDF boundaries (long-double sums) over sigma in [360, 1e10] and m over
    [-1/2, 1/2], including the window's first and last points, equals the table walk."""
    rng = np.random.default_rng(79)
    mus, sigs, us = [], [], []
    for _ in range(200):
        sig = float(np.exp(rng.uniform(np.log(360.0), np.log(1e10))))
        mu = float(rng.uniform(-0.5, 0.5) + rng.choice([0.0, 7.0, -1e6]))
        c = np.rint(mu)
        k = np.arange(c - 500, c + 501, dtype=np.longdouble)
        w = np.exp(-0.5 * ((k - np.longdouble(mu)) / np.longdouble(sig)) ** 2)
        F = np.cumsum(w) / np.sum(w)
        for j in np.concatenate([[0, 1, 998, 999], rng.choice(len(F) - 1, 6)]):
            for eps in (-1e-7, -1e-9, -3e-12, 3e-12, 1e-9, 1e-7):
                u = float(F[j]) + eps
                if 0.0 <= u < 1.0:
                    mus.append(mu), sigs.append(sig), us.append(u)
    mu, sig, u = np.array(mus), np.array(sigs), np.array(us)
    z_t, ln_t = ctx.sample_z(mu, sig, u, table=True)
    z, ln = ctx.sample_z(mu, sig, u)
    assert np.array_equal(z, z_t)
    np.testing.assert_allclose(ln, ln_t, rtol=1e-13, atol=1e-13)


def test_samplez_tab_vs_libm_random(ctx):
    """Tabulated erf/exp path vs ocml libm path vs table walk on 400k random draws
    over sigma in [4, 1e6] (wide windows, capped and uncapped)."""
    rng = np.random.default_rng(78)
    n = 400000
    sig = np.exp(rng.uniform(np.log(4.0), np.log(1e6), n))
    mu = rng.uniform(-1, 1, n) * rng.choice([1.0, 30.0, 1e4, 1e9], n)
    u = rng.random(n)
    z_t, _ = ctx.sample_z(mu, sig, u, table=True)
    z_d, _ = ctx.sample_z(mu, sig, u, mode="decision")
    z_l, _ = ctx.sample_z(mu, sig, u, mode="libm_decision")
    assert np.array_equal(z_d, z_t)
    assert np.array_equal(z_l, z_t)


def test_samplez_em_vs_table_vs_oracle_stress(ctx, oracle):
    rng = np.random.default_rng(123)
    n = 20000
    sig = np.exp(rng.uniform(np.log(0.005), np.log(3e3), n))
    sig[:500] = 1e6
    mu = rng.uniform(-1, 1, n) * np.maximum(sig, 1) * rng.choice([1, 10, 1000], n)
    u = rng.random(n)
    u[:50] = 0.0
    u[50:100] = 1.0 - 2.0 ** -53
    z_em, ln_em = ctx.sample_z(mu, sig, u)
    z_tb, ln_tb = ctx.sample_z(mu, sig, u, table=True)
    assert np.array_equal(z_em, z_tb)
    np.testing.assert_allclose(ln_em, ln_tb, rtol=1e-13, atol=1e-13)
    idx = rng.choice(n, 3000, replace=False)
    z_or = np.array([oracle.sample_z(mu[i], sig[i], u[i])[0] for i in idx])
    assert np.array_equal(z_em[idx], z_or)


# ------------------------------------------------------------------ B z kernels
@pytest.mark.parametrize("zmax", [1500, 32639, 40000, 10 ** 7])
def test_lattice_points_integer_basis_exact(ctx, zmax):
    """Int8-digit MFMA path (|z| <= 32639) and its fp64 replay (larger |z|) are exact."""
    from lgs_amd.lattices import ntru_basis
    B = ntru_basis(64, 12289, 3)
    R, cp = np.linalg.qr(B)[1], np.zeros(128)
    R = R * np.where(np.diag(R) < 0, -1.0, 1.0)[:, None]
    ctx.set_basis(R, cp, B, 165.7)
    rng = np.random.default_rng(zmax)
    z = rng.integers(-zmax, zmax + 1, size=(777, 128)).astype(np.int64)
    z[0, :] = zmax
    z[1, :] = -zmax
    v = ctx.lattice_points(z)
    assert np.array_equal(v, (B @ z.T).T)


def test_imhk_device_v_samples(ctx, capi):
    import torch
    g = load_golden("klein_qary128.npz")
    R, cp, B = golden_R(g)
    ctx.set_basis(R, cp, B, float(g["sigma"]))
    d, nc, steps, thin = R.shape[0], 64, 12, 2
    dev = "cuda:0"
    z = torch.zeros((d, nc), dtype=torch.int32, device=dev)
    lw = torch.zeros(nc, dtype=torch.float64, device=dev)
    init = torch.zeros(nc, dtype=torch.int32, device=dev)
    acc = torch.zeros(nc, dtype=torch.int64, device=dev)
    zs = torch.zeros((nc, steps // thin, d), dtype=torch.int32, device=dev)
    vs = torch.zeros((nc, steps // thin, d), dtype=torch.float64, device=dev)
    torch.cuda.synchronize()
    f = capi.LGS_DEVICE_PTRS | capi.LGS_COORD_MAJOR
    # z_samples is row-major only; pass a row-major z_state for that call
    ctx.imhk(9, 0, nc, 1, steps, thin, z, lw, init, acc, v_samples=vs, flags=f)
    zr = torch.zeros((nc, d), dtype=torch.int32, device=dev)
    lw2 = torch.zeros(nc, dtype=torch.float64, device=dev)
    init2 = torch.zeros(nc, dtype=torch.int32, device=dev)
    acc2 = torch.zeros(nc, dtype=torch.int64, device=dev)
    ctx.imhk(9, 0, nc, 1, steps, thin, zr, lw2, init2, acc2, z_samples=zs, flags=capi.LGS_DEVICE_PTRS)
    zsn = zs.cpu().numpy().astype(np.int64)
    assert np.array_equal(vs.cpu().numpy(), np.einsum("rc,nkc->nkr", B, zsn))
    assert np.array_equal(z.cpu().numpy().T, zr.cpu().numpy())
    assert torch.equal(acc, acc2)


@pytest.mark.parametrize("nc,steps,cm", [(64, 12, True), (37, 7, True), (40, 9, False)])
def test_imhk_fused_final_state_with_moments(ctx, capi, oracle, nc, steps, cm):
    """Moments + lattice points (carry columns) take the fused moments/final-state
    pass (vectorised when the store is 8-aligned -- 16-bit store, 8 proposals per lane, chain boundaries inside a vector -- scalar otherwise); Wang-Ling
    weights make chains reject, so some chains keep their carried-in state.
    Final states, moments and acceptances equal the oracle's."""
    import torch
    g = load_golden("klein_ntru32.npz")
    R, cp, B = golden_R(g)
    sigma = float(g["sigma"])
    ctx.set_basis(R, cp, B, sigma)
    d = R.shape[0]
    dev = "cuda:0"
    z = torch.zeros((d, nc) if cm else (nc, d), dtype=torch.int32, device=dev)
    lw = torch.zeros(nc, dtype=torch.float64, device=dev)
    init = torch.zeros(nc, dtype=torch.int32, device=dev)
    acc = torch.zeros(nc, dtype=torch.int64, device=dev)
    mom = torch.zeros(2 * d, dtype=torch.int64, device=dev)
    vs = torch.zeros((nc, steps, d), dtype=torch.float64, device=dev)
    f = capi.LGS_DEVICE_PTRS | capi.LGS_WANG_LING | (capi.LGS_COORD_MAJOR if cm else 0)
    half = steps // 2
    ctx.imhk(31, 0, nc, 1, half, 1, z, lw, init, acc, v_samples=vs[:, :half].contiguous(), moments=mom, flags=f)
    ctx.imhk(31, 0, nc, 1 + half, steps - half, 1, z, lw, init, acc,
             v_samples=vs[:, half:].contiguous(), moments=mom, flags=f)
    o = oracle.imhk(R, cp, B, sigma, nc, steps, seed=31, first_step=1, mode=oracle.IMHK_WANG_LING, trace=True)
    zf = z.cpu().numpy()
    assert np.array_equal(zf.T if cm else zf, o["z"])
    assert np.array_equal(acc.cpu().numpy(), o["accepts"])
    assert 0 < o["accepts"].sum() < nc * steps
    flat = o["trace"].reshape(-1, d).astype(np.int64)
    m = mom.cpu().numpy()
    assert np.array_equal(m[:d], flat.sum(0))
    assert np.array_equal(m[d:], (flat * flat).sum(0))
