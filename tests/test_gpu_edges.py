"""GPU edge cases of the Klein / IMHK path (empty and ragged inputs).

* Ragged shapes: lattice dimensions that are not multiples of the 16/32-row
  panels or the 64/128-wide B z tiles (d = 1, 2, 31, 33, 65, 100) and sample
  counts that are not multiples of the 64-lane wave; z and the integer lattice
  points v are bit-exact against the oracle in both kernel orders.
* Empty inputs: n = 0 Klein calls, IMHK with zero chains or zero steps, and
  zero-vector moments / decodes are no-ops that leave the outputs untouched.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

MODES = {"exact": 2, "panel": 0}  # LGS_EXACT_ORDER = 0x2


@pytest.fixture(scope="module")
def capi():
    from lgs_amd import _capi
    return _capi


@pytest.fixture(scope="module")
def ctx(capi):
    return capi.Context(0)


def _int_basis(d, seed):
    """Well-conditioned integer basis: 6 I plus three +-1 entries per row."""
    rng = np.random.default_rng(seed)
    B = 6 * np.eye(d)
    for i in range(d):
        B[i, rng.integers(0, d, 3)] += rng.choice([-1.0, 1.0], 3)
    return B


def _ill_basis(d, seed):
    """Integer basis L U with unit-ish triangles: condition number ~1e15, so the
    coefficients grow to ~2^50 and ulp(mu) approaches the integer spacing."""
    rng = np.random.default_rng(seed)
    L = np.tril(rng.integers(-2, 3, (d, d)), -1) + np.diag(rng.integers(1, 4, d))
    U = np.triu(rng.integers(-2, 3, (d, d)), 1) + np.eye(d, dtype=np.int64)
    return (L @ U).astype(np.float64)


@pytest.mark.parametrize("mode", list(MODES))
@pytest.mark.parametrize("d,n", [(1, 1), (2, 65), (31, 130), (33, 63), (65, 129), (100, 200)])
def test_klein_ragged_shapes_vs_oracle(ctx, oracle, d, n, mode):
    B = _int_basis(d, d)
    R, cp = oracle.qr_prepare(B)
    sigma = 8.0
    ctx.set_basis(R, cp, B, sigma)
    r = ctx.klein_host(777 + d, 31, n, want_z=True, want_v=True, flags=MODES[mode])
    o = oracle.klein(R, cp, sigma, n, seed=777 + d, first_sample=31, B=B)
    assert r["z"].shape == (n, d)
    assert np.array_equal(r["z"], o["z"])
    assert np.array_equal(r["v"], o["v"])


def test_exact_order_on_ill_conditioned_basis(ctx, oracle):
    """LGS_EXACT_ORDER keeps the reference's sequential fp64 order, so it stays
    bit-exact even where |mu| ~ 2^50 and the blocked default order's ulp-level
    differences in mu change many decisions."""
    B = _ill_basis(64, 64)
    R, cp = oracle.qr_prepare(B)
    ctx.set_basis(R, cp, B, 3.5)
    r = ctx.klein_host(841, 31, 128, want_z=True, want_v=True, flags=MODES["exact"])
    o = oracle.klein(R, cp, 3.5, 128, seed=841, first_sample=31, B=B)
    assert np.abs(o["z"]).max() > 1 << 40
    assert np.array_equal(r["z"], o["z"])


@pytest.mark.parametrize("n", [256, 128, 130])
def test_certified_default_order_on_ill_conditioned_basis(capi, oracle, n):
    """The default blocked kernels certify every decision against a bound on
    |mu_blocked - mu_reference| and redo the uncovered ones at the reference-order
    mean (lgs_device.h, certified decisions), so they are bit-exact on the same
    basis where half the samples used to change.  n = 256: int8-digit
    far field (which hands over to the fp64 far field once |z| > 32639), 128: fp64
    MFMA far field, 130: VALU panel kernel (ragged launch)."""
    ctx = capi.Context(0)  # fresh: the |z| > 32639 hand-over is sticky per context
    B = _ill_basis(64, 64)
    R, cp = oracle.qr_prepare(B)
    ctx.set_basis(R, cp, B, 3.5)
    ctx.resolved(reset=True)
    r = ctx.klein_host(841, 31, n, want_z=True, want_v=False)
    o = oracle.klein(R, cp, 3.5, n, seed=841, first_sample=31, B=B)
    assert np.abs(o["z"]).max() > 1 << 40
    assert np.array_equal(r["z"], o["z"])
    assert ctx.resolved() > 0  # the certificate declined some decisions here


def test_klein_empty(ctx, oracle, capi):
    B = _int_basis(33, 1)
    R, cp = oracle.qr_prepare(B)
    ctx.set_basis(R, cp, B, 2.0)
    r = ctx.klein_host(5, 0, 0, want_z=True, want_v=True, want_logw=True)
    assert r["z"].shape == (0, 33) and r["v"].shape == (0, 33) and r["logw"].shape == (0,)
    ctx.klein(5, 0, 0, None, None, None, 0)  # nothing requested, nothing done


def test_imhk_zero_steps_and_zero_chains(ctx, oracle, capi):
    B = _int_basis(33, 2)
    R, cp = oracle.qr_prepare(B)
    ctx.set_basis(R, cp, B, 2.0)
    nc, d = 70, 33
    z = np.zeros((nc, d), dtype=np.int32)
    lw = np.zeros(nc)
    init = np.zeros(nc, dtype=np.int32)
    acc = np.zeros(nc, dtype=np.int64)
    ctx.imhk(9, 0, nc, 1, 3, 1, z, lw, init, acc, flags=capi.LGS_WANG_LING)
    assert init.all()
    z0, lw0, acc0 = z.copy(), lw.copy(), acc.copy()
    mom = np.zeros(2 * d, dtype=np.int64)
    ctx.imhk(9, 0, nc, 4, 0, 1, z, lw, init, acc, moments=mom, flags=capi.LGS_WANG_LING)
    assert np.array_equal(z, z0) and np.array_equal(lw, lw0) and np.array_equal(acc, acc0)
    assert not mom.any()
    e = np.zeros((0, d), dtype=np.int32)
    ctx.imhk(9, 0, 0, 1, 5, 1, e, np.zeros(0), np.zeros(0, dtype=np.int32), np.zeros(0, dtype=np.int64),
             moments=mom, flags=capi.LGS_WANG_LING)
    assert not mom.any()


def test_zero_vector_reductions_and_decodes(ctx, oracle):
    from lgs_amd import diagnostics
    B = _int_basis(17, 3)
    R, cp = oracle.qr_prepare(B)
    ctx.set_basis(R, cp, B, 2.0)
    s = np.full(17, 7, dtype=np.int64)
    G = np.full((17, 17), 3, dtype=np.int64)
    ctx.gram(np.zeros((0, 17), dtype=np.int32), sum_out=s, gram_out=G)
    assert (s == 7).all() and (G == 3).all()
    s2, G2 = diagnostics.gram(np.zeros((0, 17), dtype=np.int32))
    assert not s2.any() and not G2.any()


def test_imhk_16bit_store_with_wide_carried_states(capi, oracle):
    """The default 16-bit proposal store receives the chain states through the carry
    columns; caller-supplied states beyond int16 switch it to 32 bits, so lattice
    points, moments and final states are those of a 32-bit store (LGS_CTX_STORE32)."""
    import torch
    d, nc, T = 40, 64, 6
    B = _int_basis(d, 5)
    R, cp = oracle.qr_prepare(B)
    z0 = np.random.default_rng(1).integers(-5, 6, (nc, d)).astype(np.int32)
    z0[:, 0] = 50000
    z0[3, 5] = -70000
    for zint in ("2", "4"):
        c = capi.Context(0, store32=zint == "4")
        c.set_basis(R, cp, B, 3.0)
        dev = "cuda:0"
        z = torch.from_numpy(z0.copy()).to(dev)
        lw = torch.full((nc,), 1e6, dtype=torch.float64, device=dev)  # no proposal reaches it
        init = torch.ones(nc, dtype=torch.int32, device=dev)
        acc = torch.zeros(nc, dtype=torch.int64, device=dev)
        vs = torch.zeros((nc, T, d), dtype=torch.float64, device=dev)
        mom = torch.zeros(2 * d, dtype=torch.int64, device=dev)
        c.imhk(3, 0, nc, 1, T, 1, z, lw, init, acc, v_samples=vs, moments=mom,
               flags=capi.LGS_DEVICE_PTRS | capi.LGS_WANG_LING)
        assert not acc.cpu().numpy().any()
        assert np.array_equal(z.cpu().numpy(), z0)
        v0 = z0.astype(np.float64) @ B.T
        assert np.array_equal(vs.cpu().numpy(), np.repeat(v0[:, None, :], T, axis=1))
        zz = z0.astype(np.int64)
        m = mom.cpu().numpy()
        assert np.array_equal(m[:d], T * zz.sum(0))
        assert np.array_equal(m[d:], T * (zz * zz).sum(0))


@pytest.mark.parametrize("wl", [False, True])
def test_imhk_lattice_points_from_klein_history(capi, oracle, wl):
    """With the int8-digit far field (NTRU d = 1024, whole 256-proposal blocks) B z
    reads each proposal's digits from the Klein launch's int16 history and the
    carried-in states from the store; over two calls with Wang-Ling rejections the
    kept states mix both sources.  v must equal B z of the kept coefficients."""
    import torch
    from lgs_amd.lattices import build_config
    lat, sigma = build_config("C3_ntru512")
    B = lat.basis
    R, cp = oracle.qr_prepare(B)
    ctx = capi.Context(0)
    ctx.set_basis(R, cp, B, sigma)
    d, nc, T = B.shape[0], 256, 4
    dev = "cuda:0"
    z = torch.zeros((nc, d), dtype=torch.int32, device=dev)
    lw = torch.zeros(nc, dtype=torch.float64, device=dev)
    init = torch.zeros(nc, dtype=torch.int32, device=dev)
    acc = torch.zeros(nc, dtype=torch.int64, device=dev)
    f = capi.LGS_DEVICE_PTRS | (capi.LGS_WANG_LING if wl else 0)
    for call in range(2):
        zs = torch.zeros((nc, T, d), dtype=torch.int32, device=dev)
        vs = torch.zeros((nc, T, d), dtype=torch.float64, device=dev)
        ctx.imhk(7, 0, nc, 1 + call * T, T, 1, z, lw, init, acc, z_samples=zs, v_samples=vs, flags=f)
        zsn = zs.cpu().numpy().reshape(-1, d).astype(np.float64)
        assert np.array_equal(vs.cpu().numpy().reshape(-1, d), zsn @ B.T)
    a = acc.cpu().numpy()
    assert a.sum() == (2 * T * nc if not wl else a.sum())
    if wl:
        assert 0 < a.sum() < 2 * T * nc  # some chains kept a carried-in state


def test_lattice_points_into_8_byte_aligned_output(capi, oracle):
    """B z writes 16 bytes per lane (two coordinates of a row) when d, the row pitch and
    the output pointer allow it, 8 bytes otherwise: an output that starts one double into
    its allocation (8-byte aligned only) gets the same lattice points as an aligned one."""
    import torch
    from lgs_amd.lattices import build_config
    lat, sigma = build_config("C2_qary128")
    B = lat.basis
    R, cp = oracle.qr_prepare(B)
    ctx = capi.Context(0)
    ctx.set_basis(R, cp, B, sigma)
    d, n = B.shape[0], 1024
    f = capi.LGS_DEVICE_PTRS | capi.LGS_COORD_MAJOR
    out = []
    for off in (0, 1):
        z = torch.zeros((d, n), dtype=torch.int32, device="cuda:0")
        lw = torch.zeros(n, dtype=torch.float64, device="cuda:0")
        buf = torch.full((n * d + 2,), -1.0, dtype=torch.float64, device="cuda:0")
        v = buf[off:off + n * d].view(n, d)
        assert (v.data_ptr() % 16 == 0) == (off == 0)
        ctx.klein(5, 0, n, z, v, lw, f)
        torch.cuda.synchronize()
        zn = z.cpu().numpy().T.astype(np.float64)
        assert np.array_equal(v.cpu().numpy(), zn @ B.T)
        b = buf.cpu().numpy()
        assert np.all(b[:off] == -1.0) and np.all(b[off + n * d:] == -1.0)  # nothing outside
        out.append(v.cpu().numpy())
    assert np.array_equal(out[0], out[1])


def test_klein_lattice_points_from_klein_history(capi, oracle):
    """lgs_klein with lattice points (NTRU d = 1024, 512 samples: int8-digit far
    field): B z from the launch's history equals B z of the returned coefficients,
    and the coefficients are the oracle's."""
    from lgs_amd.lattices import build_config
    lat, sigma = build_config("C3_ntru512")
    B = lat.basis
    R, cp = oracle.qr_prepare(B)
    ctx = capi.Context(0)
    ctx.set_basis(R, cp, B, sigma)
    r = ctx.klein_host(4321, 77, 512, want_z=True, want_v=True)
    assert np.array_equal(r["v"], r["z"].astype(np.float64) @ B.T)
    o = oracle.klein(R, cp, sigma, 16, seed=4321, first_sample=77)
    assert np.array_equal(r["z"][:16], o["z"])


def test_imhk_halves_its_block_when_allocation_fails(capi, monkeypatch):
    """an allocation failure of a block-sized buffer halves lgs_imhk's
    block (the smaller cap stays with the context) instead of returning LGS_ERR_NOMEM.
    With every device allocation above 6 MiB refused (hooks build), a 256-chain, 64-step
    call whose default block (64 steps: a 16 MiB proposal store) does not fit runs in
    smaller blocks -- pipelined on a caller's stream, and host-checked -- and gives the
    same chains as an unconstrained context (counter-addressed proposals)."""
    import torch
    from conftest import golden_R, load_golden
    g = load_golden("klein_qary128.npz")
    R, cp, B = golden_R(g)
    d, nc, T = R.shape[0], 256, 64
    dev = "cuda:0"

    def run(ctx, stream):
        st = dict(z=torch.zeros((d, nc), dtype=torch.int32, device=dev),
                  lw=torch.zeros(nc, dtype=torch.float64, device=dev),
                  init=torch.zeros(nc, dtype=torch.int32, device=dev),
                  acc=torch.zeros(nc, dtype=torch.int64, device=dev),
                  mom=torch.zeros(2 * d, dtype=torch.int64, device=dev))
        v = torch.zeros((nc, T, d), dtype=torch.float64, device=dev)
        s = torch.cuda.Stream(device=dev)
        torch.cuda.synchronize()
        if stream:
            ctx.set_stream(s.cuda_stream)
        with torch.cuda.stream(s):
            ctx.imhk(21, 0, nc, 1, T, 1, st["z"], st["lw"], st["init"], st["acc"], v_samples=v, moments=st["mom"],
                     flags=capi.LGS_DEVICE_PTRS | capi.LGS_COORD_MAJOR)
        torch.cuda.synchronize()
        return [v.cpu().numpy(), st["z"].cpu().numpy(), st["acc"].cpu().numpy(), st["mom"].cpu().numpy(),
                st["lw"].cpu().numpy()]

    ref = capi.Context(0, max_proposals=nc * T)
    ref.set_basis(R, cp, B, float(g["sigma"]))
    want = run(ref, False)
    ref.close()
    for stream in (True, False):
        ctx = capi.Context(0, max_proposals=nc * T, hooks=True)
        ctx.set_basis(R, cp, B, float(g["sigma"]))
        monkeypatch.setenv("LGS_TEST_NOMEM_ABOVE", str(6 << 20))
        try:
            got = run(ctx, stream)
        finally:
            monkeypatch.delenv("LGS_TEST_NOMEM_ABOVE")
        ctx.close()
        for a, b in zip(got, want):
            assert np.array_equal(a, b)
