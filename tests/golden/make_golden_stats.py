"""Statistical goldens: exact first and second moments of the
coefficient vectors drawn by the REFERENCE sampler itself, at sizes the device
tests also run.

Same harness as make_golden.py (the reference's RefinedKleinSampler driven
unmodified, numpy.random.choice swapped for NumPy's legacy inverse-CDF rule fed
with this build's Philox uniform), run over worker processes that each draw a
contiguous range of sample counters.  Stored per fixture: sum z (int64), sum z z^T
(int64, exact), n, the counters, and the number of draws served by the
reference's approximate _sample_cache with a table of another mean (klein.py:148-162),
the one reference behaviour that can legitimately change a decision.

Fixtures: Z^64, sigma = 5, 2^16 samples (C1 shape); q-ary d = 128, q = 3329,
sigma = 165.7, 2^16 samples (C2).  About 15 s and 20 min of CPU over 8 processes.

Usage:  python3 -B tests/golden/make_golden_stats.py   (writes tests/golden/stats_*.npz)
"""
import os
import sys
from multiprocessing import get_context

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)


def _worker(job):
    name, kind, sigma, first, n, seed = job
    import numpy as np
    import make_golden as mg
    from lgs_amd import _philox, lattices
    B = np.eye(64) if kind == "Z64" else lattices.qary_basis(64, 64, 3329, 1)
    lat = mg.DuckLattice(B, name)
    s = mg.RefinedKleinSampler(lat, sigma)
    mg.instrument(s)
    sig_i = sigma / np.abs(s.R_diag)
    mg.CUR = mg.Cursor(seed)
    orig = s.sample_single
    counter = {"k": first}

    def single():
        chain, step = _philox.sample_counter(counter["k"])
        counter["k"] += 1
        mg.CUR.start_sample(sig_i, chain, step)
        out = orig()
        assert not mg.CUR.slots
        return out

    s.sample_single = single
    np.random.choice, np.random.rand = mg.choice_shim, mg.rand_shim
    V = s.sample(n)
    Z = np.rint(np.linalg.solve(lat.basis, V.T).T).astype(np.int64)
    assert np.array_equal(lat.basis @ Z.T, V.T)
    flags = sum(1 for _, _, f in mg.CUR.log if f)
    return Z.sum(0), Z.T @ Z, flags


def make(name, kind, sigma, n, seed, procs=8):
    import numpy as np
    per = n // procs
    jobs = [(name, kind, sigma, k * per, per, seed) for k in range(procs)]
    with get_context("spawn").Pool(procs) as pool:
        res = pool.map(_worker, jobs)
    S = sum(r[0] for r in res)
    G = sum(r[1] for r in res)
    flags = sum(r[2] for r in res)
    np.savez_compressed(os.path.join(HERE, f"stats_{name}.npz"), name=name, sigma=sigma, n=n,
                        seed=np.uint64(seed), first_sample=0, sum_z=S, sum_zz=G, cache_flags=flags)
    mean = S / n
    cov = (G - np.outer(S, S) / n) / (n - 1)
    print(f"stats_{name}: n={n} d={len(S)} cache_flags={flags} mean[:3]={mean[:3]} var[:3]={np.diag(cov)[:3]}")


if __name__ == "__main__":
    seed = 0x5EED_57A7
    make("Z64", "Z64", 5.0, 1 << 16, seed)
    make("qary128", "qary128", 165.7, 1 << 16, seed)
