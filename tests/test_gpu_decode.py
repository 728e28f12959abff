"""GPU: Babai decoding (nearest_plane_kernel, round_kernel, fp64 MFMA frame GEMM)
through the C-ABI and the SimpleLattice drop-in, against the reference-generated
rounding fixtures (tests/golden/decode_round.npz) and the nearest-plane
restatements (oracle/lgs_decode_oracle.py).  Coefficients are compared exactly;
targets are continuous so no half-integer ties occur."""
import numpy as np
import pytest

from conftest import load_golden

import lgs_decode_oracle as DO

pytestmark = pytest.mark.gpu


def test_round_decode_matches_reference():
    """SimpleLattice(basis).decode is the reference's row-lattice rounding
    (simple.py:126-128: solve_left, basis.T round(c)); the fixtures come from
    utils.py's generator, whose basis generates its rows too."""
    from lgs_amd.lattices import SimpleLattice
    g = load_golden("decode_round.npz")
    for name in ("qary32", "ntru32", "gauss12"):
        basis, xs, pts = g[f"{name}_basis"], g[f"{name}_x"], g[f"{name}_points"]
        lat = SimpleLattice(basis)
        z = lat._decoder().round_decode(xs, coefficients=True)
        np.testing.assert_array_equal(z, np.array([DO.round_decode_rows(basis, x)[0] for x in xs]))
        if name == "gauss12":   # real basis: B z summed in another order than basis.T @ c
            np.testing.assert_allclose(lat.decode(xs), pts, rtol=1e-13, atol=1e-12)
        else:                   # integer bases: lattice points exact
            np.testing.assert_array_equal(lat.decode(xs), pts)
            np.testing.assert_array_equal(lat.decode(xs[3]), pts[3])
            np.testing.assert_array_equal(lat.decode(xs), z.astype(np.float64) @ basis)


@pytest.mark.parametrize("kind", ["qary", "ntru", "gauss"])
def test_nearest_plane_matches_restatements(oracle, kind):
    """SimpleLattice(B).nearest_plane / decode_cvp walk the ROWS of B, as base.py:124-135
    does (t -= c[i] * basis[i]; sum c[i] * basis[i]); every basis here is non-symmetric."""
    from lgs_amd import lattices
    from lgs_amd.lattices import SimpleLattice
    rng = np.random.default_rng(21)
    B = {"qary": lattices.qary_basis(40, 40, 3329, 5), "ntru": lattices.ntru_basis(40, 12289, 2),
         "gauss": rng.standard_normal((37, 37)) * 4.0}[kind]
    assert not np.array_equal(B, B.T)
    T = rng.standard_normal((300, B.shape[0])) * 2500.0
    lat = SimpleLattice(B)
    z, v = lat._decoder().ctx.decode_host(T, "plane")
    for k in range(0, 300, 7):
        c_gs, v_gs = DO.nearest_plane_rows(B, T[k])
        np.testing.assert_array_equal(z[k], c_gs)
        np.testing.assert_array_equal(DO.nearest_plane_qr(B.T, T[k], oracle), c_gs)
    np.testing.assert_array_equal(lat.nearest_plane(T), v)
    if kind != "gauss":
        np.testing.assert_array_equal(v, z.astype(np.float64) @ B)     # sum_i c_i B[i]
    np.testing.assert_array_equal(lat.decode_cvp(T[5]), v[5])
    np.testing.assert_array_equal(lat.nearest_plane(T[7]), v[7])
    # idempotence: lattice points decode to themselves
    np.testing.assert_array_equal(lat._decoder().nearest_plane(v[:50], coefficients=True), z[:50])
    # the row lattice is not the column lattice: the samplers' column Decoder(B) decodes
    # the same targets to other points
    from lgs_amd.decode import Decoder
    assert not np.array_equal(Decoder(B).nearest_plane(T[:20]), v[:20])


def test_nearest_plane_full_size_ntru1024(oracle):
    """d = 1024 (C3 basis): bit-exact against the QR-frame oracle on a few targets,
    and Babai's parallelepiped property over a large batch."""
    from lgs_amd import lattices
    from lgs_amd.decode import Decoder
    B = lattices.ntru_basis(512, 12289, 1)
    dec = Decoder(B)
    rng = np.random.default_rng(3)
    T = rng.standard_normal((2048, 1024)) * 4000.0
    z = dec.nearest_plane(T, coefficients=True)
    for k in (0, 777, 2047):
        np.testing.assert_array_equal(DO.nearest_plane_qr(B, T[k], oracle), z[k])
    Q, R = DO.qr_frame(B)
    W = (Q.T @ (T - z.astype(np.float64) @ B.T).T) / np.diag(R)[:, None]
    assert np.all(np.abs(W) <= 0.5 + 1e-6)
    zr = dec.round_decode(T[:64], coefficients=True)
    np.testing.assert_array_equal(zr, np.round(np.linalg.solve(B, T[:64].T)).T.astype(np.int64))


def test_decode_device_pointers_coordinate_major():
    import torch
    from lgs_amd import _capi, lattices
    from lgs_amd.decode import Decoder
    B = lattices.qary_basis(32, 32, 3329, 9)
    dec = Decoder(B)
    rng = np.random.default_rng(4)
    T = rng.standard_normal((333, 64)) * 1000.0
    z_ref, v_ref = dec.ctx.decode_host(T, "plane")
    Tt = torch.as_tensor(np.ascontiguousarray(T.T), device="cuda")
    z = torch.empty((64, 333), dtype=torch.int64, device="cuda")
    v = torch.empty((333, 64), dtype=torch.float64, device="cuda")
    dec.ctx.decode(Tt, "plane", z, v, _capi.LGS_DEVICE_PTRS | _capi.LGS_COORD_MAJOR | _capi.LGS_Z64)
    np.testing.assert_array_equal(z.cpu().numpy().T, z_ref)
    np.testing.assert_array_equal(v.cpu().numpy(), v_ref)


def test_decode_errors():
    from lgs_amd import _capi, lattices
    ctx = _capi.Context(0)
    B = lattices.qary_basis(8, 8, 17, 1)
    Q, R = DO.qr_frame(B)
    ctx.set_basis(R, np.zeros(16), B, 1.0)
    with pytest.raises(_capi.LgsError):           # no decoder frame uploaded
        ctx.decode_host(np.zeros((2, 16)), "plane")
    ctx.set_decoder(Q, None)
    with pytest.raises(_capi.LgsError):
        ctx.decode_host(np.zeros((2, 16)), "round")
    z, v = ctx.decode_host(np.zeros((2, 16)), "plane")
    assert not z.any() and not v.any()
    with pytest.raises(_capi.LgsError):
        ctx.decode_host(np.full((1, 16), np.nan), "plane")
