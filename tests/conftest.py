"""Test configuration: paths, the `gpu` marker, shared fixtures.

`-m "not gpu"` runs here (no GPU): oracle vs golden vectors, host logic, C-ABI
symbol checks.  `-m gpu` runs on an MI355X: HIP path vs oracle / goldens.
"""
import glob
import os
import sys

import numpy as np
import pytest

sys.dont_write_bytecode = True
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "lattice-gaussian-mcmc_amd")
for p in (PKG, os.path.join(REPO, "oracle"), REPO):
    if p not in sys.path:
        sys.path.insert(0, p)
GOLDEN = os.path.join(REPO, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device)")


def load_golden(name):
    return dict(np.load(os.path.join(GOLDEN, name), allow_pickle=False))


def klein_goldens():
    return sorted(os.path.basename(p) for p in glob.glob(os.path.join(GOLDEN, "klein_*.npz")))


def golden_R(g):
    """R / c' / B of a golden fixture (rebuilt for the large NTRU case)."""
    if "R" in g:
        return g["R"], g["cprime"], g.get("B")
    from lgs_amd import lattices
    import lgs_oracle
    B = lattices.ntru_basis(int(g["ntru_n"]), int(g["ntru_q"]), int(g["ntru_seed"]))
    if "R_upper" in g:
        # the reference's R, stored (upper triangle): LAPACK builds differ by ulps
        # between hosts (the GPU box's rebuild did not match R_sha256)
        d = B.shape[0]
        R = np.zeros((d, d))
        R[np.triu_indices(d)] = g["R_upper"]
        il = np.tril_indices(d, -1)  # the sign fix leaves -0.0 below the diagonal of flipped rows
        R[il] = np.where(g["R_lower_negzero_rows"][il[0]], -0.0, 0.0)
        R, cp = np.ascontiguousarray(R), g["cprime"]
    else:
        R, cp = lgs_oracle.qr_prepare(B)
    if "R_sha256" in g:  # the golden's input must be the reference's R bit for bit
        import hashlib
        got = hashlib.sha256(np.ascontiguousarray(R).tobytes()).hexdigest()
        assert got == str(g["R_sha256"]), "rebuilt R differs from the reference's (LAPACK build?)"
    return R, cp, B


@pytest.fixture(scope="session")
def oracle():
    import lgs_oracle
    lgs_oracle.lib()
    return lgs_oracle
