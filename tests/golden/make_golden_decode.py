"""Babai-rounding fixtures from the REFERENCE itself: runs
``DiscreteGaussianUtils.sample_discrete_gaussian_lattice`` (src/samplers/utils.py:558-579:
continuous Gaussian x, coefficients = round(solve(basis.T, x)), point = basis.T @ c)
imported read-only from /root/reference, seeding NumPy's global stream before each
call so the test can regenerate the same x (np.random.normal(0, sigma, n)).

Usage:  python3 -B tests/golden/make_golden_decode.py   (writes tests/golden/decode_round.npz)
"""
from __future__ import annotations

import os
import sys

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "lattice-gaussian-mcmc_amd"))
sys.path.insert(0, "/root/reference")

import numpy as np  # noqa: E402

from lgs_amd import lattices  # noqa: E402
from src.samplers.utils import DiscreteGaussianUtils  # noqa: E402


def main():
    u = DiscreteGaussianUtils()
    out = {}
    cases = {"qary32": (lattices.qary_basis(16, 16, 3329, 5), 900.0, 40),
             "ntru32": (lattices.ntru_basis(16, 12289, 2), 5000.0, 40),
             "gauss12": (np.random.default_rng(4).standard_normal((12, 12)) * 3.0, 7.5, 40)}
    for name, (basis, sigma, count) in cases.items():
        xs, pts = [], []
        for k in range(count):
            np.random.seed(1000 + k)
            xs.append(np.random.normal(0, sigma, basis.shape[0]))
            np.random.seed(1000 + k)
            pts.append(u.sample_discrete_gaussian_lattice(basis, sigma))
        out[f"{name}_basis"] = basis
        out[f"{name}_sigma"] = np.float64(sigma)
        out[f"{name}_x"] = np.array(xs)
        out[f"{name}_points"] = np.array(pts, dtype=np.float64)
    np.savez_compressed(os.path.join(HERE, "decode_round.npz"), **out)
    print("wrote", os.path.join(HERE, "decode_round.npz"))


if __name__ == "__main__":
    main()
