"""Generate the golden fixtures by running the REFERENCE implementation itself.

Runs only in the build container, where the reference is mounted read-only at
/root/reference (it never travels to the GPU box).  The reference's own
``RefinedKleinSampler`` / ``IMHKSampler`` (src/samplers/klein.py,
src/samplers/imhk.py) are imported with bytecode writing disabled and driven
unmodified, except that the module attributes ``numpy.random.choice``
(klein.py:175) and ``numpy.random.rand`` (imhk.py:167) are swapped for shims
that draw their uniform from this build's Philox counter layout
 instead of the global MT19937 stream.  The choice shim is
NumPy's legacy algorithm verbatim (NaN check, cdf = cumsum(p); cdf /= cdf[-1];
searchsorted(u, side='right')), so every table, normalisation and decision is
the reference's own arithmetic.

Per draw the generator also records
  * ``cache``  -- the reference's approximate ``_sample_cache`` (klein.py:148-162)
                  served a table built for a different mean, and
  * ``margin`` -- |u - nearest CDF boundary|,
so tests can tell a legitimate near-tie apart from a real mismatch.

Usage:  python3 -B tests/golden/make_golden.py [--out DIR] [--only NAME ...]
        (writes DIR/*.npz, default tests/golden; --only klein_ntru128 etc.)
"""
from __future__ import annotations

import argparse
import os
import sys

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "lattice-gaussian-mcmc_amd"))
sys.path.insert(0, "/root/reference")

import numpy as np  # noqa: E402

from lgs_amd import _philox, lattices  # noqa: E402
from src.samplers.imhk import IMHKSampler  # noqa: E402
from src.samplers.klein import RefinedKleinSampler  # noqa: E402

_np_choice = np.random.choice
_np_rand = np.random.rand


class DuckLattice:
    """The attributes the reference samplers read (simple.py:74-82)."""

    def __init__(self, B, name):
        self.basis = np.asarray(B, dtype=np.float64)
        self.dimension = self.basis.shape[0]
        self.name = name
        r = np.linalg.qr(self.basis.T, mode="r")
        self.min_gram_schmidt_norm = float(np.min(np.abs(np.diag(r))))

    def smoothing_parameter(self):
        return 0.0


class Cursor:
    """Maps each reference draw to its Philox counter."""

    def __init__(self, seed):
        self.seed = seed
        self.slots = []
        self.step = 0
        self.chain = 0
        self.log = []          # (u, margin, cache_flag)
        self.cache_flag = False

    def start_sample(self, sigma_i, chain, step):
        d = len(sigma_i)
        self.slots = [d - 1 - i for i in range(d - 1, -1, -1) if sigma_i[i] >= 1e-10]
        self.chain, self.step = chain, step

    def next_coord_u(self):
        slot = self.slots.pop(0)
        return float(_philox.coord_uniform(self.seed, slot, self.step, self.chain))

    def accept_u(self):
        return float(_philox.accept_uniform(self.seed, self.step, self.chain))


CUR = None
OUT = HERE


def choice_shim(a, size=None, replace=True, p=None):
    """numpy legacy RandomState.choice (replace=True, size=None, p given) with Philox u."""
    assert size is None and replace and p is not None
    p = np.asarray(p, dtype=np.float64)
    if np.isnan(p).any():
        raise ValueError("probabilities contain NaN")
    if np.logical_or.reduce(p < 0):
        raise ValueError("probabilities are not non-negative")
    cdf = p.cumsum()
    cdf /= cdf[-1]
    u = CUR.next_coord_u()
    idx = int(cdf.searchsorted(u, side="right"))
    hi = cdf[idx] - u if idx < len(cdf) else 1.0
    lo = u - cdf[idx - 1] if idx > 0 else u
    CUR.log.append((u, float(min(hi, lo)), CUR.cache_flag))
    CUR.cache_flag = False
    return np.asarray(a)[idx]


def rand_shim(*args):
    assert not args
    return CUR.accept_u()


def instrument(sampler):
    """Flag draws whose table came from the approximate cache with a different mean."""
    orig = sampler._sample_1d_discrete_gaussian

    def wrapped(mean, sigma):
        key = (round(mean, 6), round(sigma, 6), sampler.precision)
        if key in sampler._sample_cache:
            sup, lp = sampler._sample_cache[key]
            sup2, lp2 = sampler._compute_1d_probabilities(mean, sigma, sampler.precision)
            CUR.cache_flag = not (np.array_equal(sup, sup2) and np.array_equal(lp, lp2))
        return orig(mean, sigma)

    sampler._sample_1d_discrete_gaussian = wrapped


def klein_fixture(name, B, sigma, n, seed, center=None, first=0, store_basis=True, extra=None):
    global CUR
    lat = DuckLattice(B, name)
    s = RefinedKleinSampler(lat, sigma, center=center)
    instrument(s)
    sig_i = sigma / np.abs(s.R_diag)
    CUR = Cursor(seed)
    orig_single = s.sample_single
    counter = {"k": first}

    def single():
        chain, step = _philox.sample_counter(counter["k"])
        counter["k"] += 1
        CUR.start_sample(sig_i, chain, step)
        out = orig_single()
        assert not CUR.slots, "draw count mismatch"
        return out

    s.sample_single = single
    np.random.choice, np.random.rand = choice_shim, rand_shim
    try:
        V = s.sample(n)
    finally:
        np.random.choice, np.random.rand = _np_choice, _np_rand
    Z = np.rint(np.linalg.solve(lat.basis, V.T).T).astype(np.int64)
    tri = np.array_equal(lat.basis, np.triu(lat.basis))
    if tri and not np.array_equal(lat.basis @ Z.T, V.T):  # ill-conditioned triangular basis
        import scipy.linalg
        Z = np.rint(scipy.linalg.solve_triangular(lat.basis, V.T).T).astype(np.int64)
    assert np.allclose(lat.basis @ Z.T, V.T, atol=1e-6 * max(1.0, np.abs(V).max()))
    log = np.array([(u, m) for u, m, _ in CUR.log]).reshape(-1, 2)
    flags = np.array([f for _, _, f in CUR.log], dtype=bool)
    out = dict(name=name, sigma=sigma, seed=np.uint64(seed), first_sample=first, n=n,
               R=s.R, cprime=s.center_transformed, center=s.center, z=Z,
               u=log[:, 0], margin=log[:, 1], cache_flag=flags)
    if store_basis:
        out["B"] = lat.basis
        out["v"] = V
    else:  # large case: tests rebuild B; the reference's R is stored as its upper
        # triangle (LAPACK builds differ by ulps between hosts) plus, per row, whether
        # the sign fix (klein.py:69-73) left -0.0 below the diagonal, and its digest
        import hashlib
        Rr = np.ascontiguousarray(s.R)
        d = Rr.shape[0]
        out["R_sha256"] = hashlib.sha256(Rr.tobytes()).hexdigest()
        out["R_upper"] = Rr[np.triu_indices(d)]
        out["R_lower_negzero_rows"] = np.array([i > 0 and bool(np.signbit(Rr[i, 0])) for i in range(d)])
        del out["R"]
    if extra:
        out.update(extra)
    np.savez_compressed(os.path.join(OUT, f"klein_{name}.npz"), **out)
    print(f"klein_{name}: n={n} d={lat.dimension} draws={len(log)} "
          f"min_margin={log[:, 1].min() if len(log) else 0:.3g} cache_flags={flags.sum()}")


def imhk_fixture(name, B, sigma, n_chains, n_steps, seed, center=None):
    global CUR
    lat = DuckLattice(B, name)
    CUR = Cursor(seed)
    Zs, acc, lws = [], [], []
    np.random.choice, np.random.rand = choice_shim, rand_shim
    try:
        for c in range(n_chains):
            s = IMHKSampler(lat, sigma, center=center, burn_in=0)
            ps = s.proposal_sampler
            instrument(ps)
            sig_i = sigma / np.abs(ps.R_diag)
            orig_single = ps.sample_single
            calls = {"k": 0}

            def single(orig_single=orig_single, sig_i=sig_i, c=c, calls=calls):
                CUR.start_sample(sig_i, c, calls["k"])
                calls["k"] += 1
                out = orig_single()
                assert not CUR.slots
                return out

            ps.sample_single = single
            zc, ac, lc = [], [], []
            for _ in range(n_steps):
                state, a = s.step()
                zc.append(np.rint(np.linalg.solve(lat.basis, state)).astype(np.int64))
                ac.append(a)
                lc.append(s.current_log_weight)
            Zs.append(zc)
            acc.append(ac)
            lws.append(lc)
            R, cp = ps.R, ps.center_transformed
    finally:
        np.random.choice, np.random.rand = _np_choice, _np_rand
    np.savez_compressed(os.path.join(OUT, f"imhk_{name}.npz"), name=name, sigma=sigma,
                        seed=np.uint64(seed), B=lat.basis, R=R, cprime=cp,
                        center=np.zeros(lat.dimension) if center is None else np.asarray(center),
                        z=np.array(Zs, dtype=np.int64), accepted=np.array(acc, dtype=bool),
                        log_weight=np.array(lws))
    print(f"imhk_{name}: chains={n_chains} steps={n_steps} acceptance={np.mean(acc):.4f}")


def samplez_fixture(seed=7):
    """Reference SampleZ decisions (klein.py:101-179) over sigma regimes."""
    global CUR
    lat = DuckLattice(np.eye(1), "Z1")
    s = RefinedKleinSampler(lat, 1.0)
    CUR = Cursor(seed)
    sigmas = [0.0096, 0.05, 0.0999999, 0.1, 0.5, 1.0, 5.0, 49.9, 50.0, 50.1, 165.7, 781.5, 1e6]
    rows = []
    rng = np.random.default_rng(seed)
    for si, sig in enumerate(sigmas):
        mus = np.concatenate([rng.uniform(-3, 3, 300) * max(sig, 1.0),
                              np.round(rng.uniform(-50, 50, 50)) + 0.5,   # exact half-integers
                              np.round(rng.uniform(-50, 50, 50)),          # exact integers
                              rng.uniform(-1e4, 1e4, 100)])
        for k, mu in enumerate(mus):
            s._sample_cache.clear()
            CUR.slots = [si * 100000 + k]
            CUR.chain, CUR.step = 0, 0
            np.random.choice = choice_shim
            try:
                z = s._sample_1d_discrete_gaussian(float(mu), float(sig))
            finally:
                np.random.choice = _np_choice
            u, m, _ = CUR.log[-1]
            rows.append((mu, sig, u, int(z), m))
    a = np.array(rows)
    np.savez_compressed(os.path.join(OUT, "samplez_table.npz"), mu=a[:, 0], sigma=a[:, 1],
                        u=a[:, 2], z=a[:, 3].astype(np.int64), margin=a[:, 4])
    print(f"samplez_table: {len(rows)} decisions, min margin {a[:, 4].min():.3g}")


def fixtures():
    """name -> generator of every fixture this script writes (in its order)."""
    seed = 0x5EED_1234_ABCD
    rng = np.random.default_rng(11)
    G = rng.standard_normal((16, 16)) * 3 + np.eye(16) * 4
    cG = rng.standard_normal(16)
    # edge: sigma_i < 1e-10 (rounding, no draw) and sigma_i > 1e10 (clamped to 1e6)
    E = np.diag([1e12, 1e-11, 1.0, 3.0, 0.5, 7.0]) + np.triu(np.arange(36).reshape(6, 6) % 5, 1)
    B2 = np.array([[4.0, 1.0], [1.0, 3.0]])
    return {
        "samplez_table": lambda: samplez_fixture(),
        "klein_Z64": lambda: klein_fixture("Z64", np.eye(64), 5.0, 1024, seed),
        "klein_I2": lambda: klein_fixture("I2", np.eye(2), 2.0, 512, seed),
        "klein_B2": lambda: klein_fixture("B2", B2, 2.0, 512, seed),
        "klein_B2_center": lambda: klein_fixture("B2_center", B2, 2.0, 256, seed, center=[0.3, -1.7]),
        "klein_gauss16": lambda: klein_fixture("gauss16", G, 7.5, 256, seed, center=cG),
        "klein_edge6": lambda: klein_fixture("edge6", E, 5.0, 128, seed, center=[0.5, 0.25, -2.0, 1.5, 0.0, 3.3]),
        "klein_qary128": lambda: klein_fixture("qary128", lattices.qary_basis(64, 64, 3329, 1), 165.7, 256, seed),
        "klein_ntru32": lambda: klein_fixture("ntru32", lattices.ntru_basis(16, 12289, 1), 165.7, 128, seed),
        "klein_ntru128": lambda: klein_fixture("ntru128", lattices.ntru_basis(64, 12289, 1), 165.7, 128, seed),
        "klein_ntru1024": lambda: klein_fixture("ntru1024", lattices.ntru_basis(512, 12289, 1), 165.7, 4, seed,
                                                first=1 << 33, store_basis=False,
                                                extra={"ntru_n": 512, "ntru_q": 12289, "ntru_seed": 1}),
        "imhk_ntru32": lambda: imhk_fixture("ntru32", lattices.ntru_basis(16, 12289, 1), 165.7, 4, 64, seed),
        "imhk_B2": lambda: imhk_fixture("B2", B2, 2.0, 2, 200, seed),
    }


def main(argv=None):
    global OUT
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=HERE)
    ap.add_argument("--only", nargs="*")
    args = ap.parse_args(argv)
    OUT = args.out
    os.makedirs(OUT, exist_ok=True)
    fx = fixtures()
    for name in args.only or list(fx):
        fx[name]()


if __name__ == "__main__":
    main()
