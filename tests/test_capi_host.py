"""CPU-side checks of the boundary: the C-ABI library loads and exports every
entry point include/lgs.h declares; host-side logic of the drop-in that needs
no device (validation, lattice builders, counters)."""
import ctypes
import os
import re

import numpy as np
import pytest

from conftest import REPO

HEADER = os.path.join(REPO, "include", "lgs.h")


def declared_symbols():
    txt = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:int|const char \*)\s*(lgs_\w+)\s*\(", txt, re.M)))


def test_header_declares_the_abi():
    syms = declared_symbols()
    for s in ("lgs_create", "lgs_set_basis", "lgs_klein", "lgs_imhk", "lgs_last_error"):
        assert s in syms


def test_library_exports_every_declared_symbol():
    from lgs_amd import _capi
    L = _capi.load_library()
    for s in declared_symbols():
        assert hasattr(L, s), f"{s} declared in lgs.h but not exported"
        assert s in _capi.EXPORTS, f"{s} not bound in _capi.EXPORTS"
    assert set(_capi.EXPORTS) == set(declared_symbols())
    assert L.lgs_version() == 100


def test_product_library_reads_no_environment():
    """Test and A/B switches exist only in the -DLGS_TEST_HOOKS build: the product
    library does not import getenv at all (nothing in a user's environment
    changes what it computes); the hooks library does, and exports the same ABI."""
    import subprocess
    from lgs_amd import _capi

    def undefined(path):
        out = subprocess.run(["nm", "-D", "--undefined-only", path], capture_output=True, text=True, check=True)
        return {ln.split()[-1].split("@")[0] for ln in out.stdout.splitlines() if ln.strip()}

    prod = os.path.join(os.path.dirname(_capi.__file__), "_lib", "liblgs_hip.so")
    assert "getenv" not in undefined(prod)
    assert "getenv" in undefined(_capi.HOOKS_LIB_PATH)
    H = ctypes.CDLL(_capi.HOOKS_LIB_PATH)
    for s in declared_symbols():
        assert hasattr(H, s), f"{s} missing from the hooks library"


def test_context_options_validated():
    from lgs_amd import _capi
    with pytest.raises(ValueError):
        _capi.Context(0, panel=24)
    with pytest.raises(ValueError):
        _capi.Context(0, far="fp32")


def test_library_is_gfx950_code_object():
    from lgs_amd import _capi
    blob = open(_capi.LIB_PATH, "rb").read()
    assert b"gfx950" in blob


def test_no_device_fails_loudly():
    import torch
    if torch.cuda.device_count() > 0:
        pytest.skip("a device is visible")
    from lgs_amd import _capi
    with pytest.raises(_capi.LgsError):
        _capi.Context(0)


def test_sampler_argument_validation_before_device():
    from lgs_amd.lattices import SimpleLattice
    from lgs_amd.samplers import IMHKSampler, KleinSampler
    lat = SimpleLattice(np.eye(3))
    with pytest.raises(ValueError):
        KleinSampler(lat, 0.0)
    with pytest.raises(ValueError):
        KleinSampler(lat, -1.0)
    with pytest.raises(ValueError):
        KleinSampler(lat, 1.0, center=[0.0, 1.0])
    with pytest.raises(ValueError):
        IMHKSampler(lat, -2.0)


def test_burn_in_overflow_like_reference():
    """imhk.py:82-88 raises OverflowError for large d; the drop-in keeps that."""
    from lgs_amd.lattices import build_config
    from lgs_amd.samplers.imhk import IMHKSampler

    class Fake:
        pass
    lat, sigma = build_config("C3_ntru512")
    f = Fake()
    f.dimension, f.sigma, f.lattice = lat.dimension, sigma, lat
    with pytest.raises(OverflowError):
        IMHKSampler._estimate_burn_in(f)
    g = Fake()
    small = np.eye(4) * 3
    from lgs_amd.lattices import SimpleLattice
    g.dimension, g.sigma, g.lattice = 4, 2.0, SimpleLattice(small)
    assert IMHKSampler._estimate_burn_in(g) == min(2 * int(np.ceil(-np.log(0.01) * 4 * (2 / 3) ** 4)), 10000)


def test_lattice_builders_match_reference_constructions():
    from lgs_amd import lattices
    B = lattices.ntru_basis(8, 97, seed=3)
    h = lattices.ntru_public(8, 97, seed=3)
    n = 8
    assert np.array_equal(B[:n, :n], 97 * np.eye(n)) and not B[:n, n:].any()
    assert np.array_equal(B[n:, n:], np.eye(n))
    for i in range(n):
        for j in range(n):
            assert B[n + i, j] == h[(j - i) % n]
    Q = lattices.qary_basis(4, 6, 31, seed=2)
    assert Q.shape == (10, 10) and np.array_equal(Q[:4, :4], 31 * np.eye(4))
    assert np.array_equal(Q[4:, 4:], np.eye(6)) and Q[4:, :4].max() < 31
    # deterministic across machines: Philox-generated integers
    assert np.array_equal(lattices.ntru_public(512, 12289, 1), lattices.ntru_public(512, 12289, 1))


def test_simple_lattice_duck_type():
    from lgs_amd.lattices import SimpleLattice
    B = np.array([[4.0, 1.0], [1.0, 3.0]])
    lat = SimpleLattice(B)
    assert lat.dimension == 2 and lat.basis is lat.get_basis()
    # row Gram-Schmidt: |b1| = sqrt(17), |b2*| = det / |b1|
    assert lat.min_gram_schmidt_norm == pytest.approx(min(np.sqrt(17), 11 / np.sqrt(17)))
    assert lat.smoothing_parameter() > 0


def test_io_formats_match_reference_schema(tmp_path):
    """Sample dumps (run_core_experiments.sage:69-73) and the scaling JSON record
    (klein_scaling_analysis.py:322-340): same keys, npz round trip, row GS norms equal
    to the reference's classical Gram-Schmidt loop (klein_scaling_analysis.py:113-135)."""
    from lgs_amd import io
    rng = np.random.default_rng(3)
    B = rng.integers(0, 51, size=(12, 12)).astype(np.float64)
    props = io.basis_properties(B)
    Bs = np.zeros_like(B)
    gs = []
    for i in range(12):                      # the reference's loop, restated
        Bs[i] = B[i]
        for j in range(i):
            Bs[i] -= np.dot(B[i], Bs[j]) / np.dot(Bs[j], Bs[j]) * Bs[j]
        gs.append(np.linalg.norm(Bs[i]))
    np.testing.assert_allclose(props["gs_norms"], gs, rtol=1e-9)
    assert props["determinant"] == pytest.approx(np.linalg.det(B))
    qm = {"x1_mean": 0.0, "x1_std": 1.0, "x1_range": [-3, 3], "mean_magnitude": 0.0,
          "std_uniformity": 0.0, "sample_diversity": 1.0, "all_means": [0.0], "all_stds": [1.0],
          "all_ranges": [6]}
    rec = io.klein_scaling_record(12, B, 3.5, 0.01, 2.0, qm, 42, 1.5)
    assert list(rec) == ["n", "determinant", "condition_number", "max_GS_norm", "sigma",
                         "time_per_sample_ms", "quality_metrics", "seed", "additional_info"]
    assert list(rec["additional_info"]) == ["sampling_time_total", "gs_norms", "sigma_multiplier"]
    io.save_results_json(str(tmp_path / "Klein_LLL_n=12.json"), rec)
    import json
    assert json.load(open(tmp_path / "Klein_LLL_n=12.json"))["max_GS_norm"] == rec["max_GS_norm"]
    s = rng.integers(-9, 9, size=(50, 12)).astype(np.float64)
    io.save_samples_npz(str(tmp_path / "s.npz"), s)
    back = io.load_samples_npz(str(tmp_path / "s.npz"))
    assert np.array_equal(back["samples"], s)
    np.testing.assert_allclose(back["norms"], np.linalg.norm(s, axis=1))


def test_buffer_checks_reject_mismatched_dtype_and_memory():
    """a buffer whose dtype or memory space disagrees with the call's
    flags is rejected before it reaches the C-ABI (it would be misread)."""
    import torch
    from lgs_amd import _capi
    ok32 = np.zeros((4, 3), dtype=np.int32)
    _capi._check_bufs(0, 0, ((ok32, "int32", "z"),))
    with pytest.raises(ValueError, match="expected int64"):
        _capi._check_bufs(_capi.LGS_Z64, 0, ((ok32, "int64", "z"),))
    with pytest.raises(ValueError, match="host buffer"):
        _capi._check_bufs(_capi.LGS_DEVICE_PTRS, 0, ((torch.zeros(3, dtype=torch.float64), "float64", "v"),))
    with pytest.raises(ValueError, match="contiguous"):
        _capi._ptr(torch.zeros((4, 4))[:, 1])


def test_imhk_outputs_struct_matches_header():
    """ctypes mirror of struct lgs_imhk_outputs: same field names, order and size."""
    import ctypes
    import re
    from lgs_amd import _capi
    hdr = open(os.path.join(REPO, "include", "lgs.h")).read()
    body = re.search(r"typedef struct lgs_imhk_outputs \{(.*?)\} lgs_imhk_outputs;", hdr, re.S).group(1)
    names = re.findall(r"\*?(\w+);", body)
    assert names == [f[0] for f in _capi.ImhkOutputs._fields_]
    assert ctypes.sizeof(_capi.ImhkOutputs) == 8 * len(names)
