"""The golden generator reproduces the committed fixtures (CPU; needs the
reference at /root/reference, which only the build container has).

tests/golden/make_golden.py imports the reference's samplers read-only and
drives them with the Philox-shimmed draws; re-running it for the q-ary/NTRU
d = 128 case (about 5 s) must give every committed key back, array-equal, and
the d = 1024 case's stored R fields (R_upper, R_lower_negzero_rows, R_sha256)
must be what the generator writes."""
import os
import subprocess
import sys

import numpy as np
import pytest

from conftest import GOLDEN, REPO

REF = "/root/reference"
pytestmark = pytest.mark.skipif(not os.path.isdir(os.path.join(REF, "src", "samplers")),
                                reason="reference not present (GPU box)")


def _regen(tmp_path, names):
    env = dict(os.environ, PYTHONDONTWRITEBYTECODE="1")
    subprocess.run([sys.executable, "-B", os.path.join(REPO, "tests", "golden", "make_golden.py"),
                    "--out", str(tmp_path), "--only", *names], check=True, env=env, timeout=600,
                   stdout=subprocess.DEVNULL)


def _same(name, tmp_path):
    a = np.load(os.path.join(GOLDEN, name), allow_pickle=False)
    b = np.load(os.path.join(tmp_path, name), allow_pickle=False)
    assert sorted(a.files) == sorted(b.files), name
    for k in a.files:
        assert a[k].dtype == b[k].dtype and np.array_equal(a[k], b[k]), (name, k)
        if a[k].dtype.kind == "f":  # -0.0 vs 0.0 too
            assert np.array_equal(np.signbit(a[k]), np.signbit(b[k])), (name, k)


def test_regenerate_ntru128(tmp_path):
    _regen(tmp_path, ["klein_ntru128"])
    _same("klein_ntru128.npz", tmp_path)


def test_regenerate_ntru1024(tmp_path):
    _regen(tmp_path, ["klein_ntru1024"])
    _same("klein_ntru1024.npz", tmp_path)
