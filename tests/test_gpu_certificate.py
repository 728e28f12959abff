"""Certified decisions of the default (blocked-order) Klein kernels at BASELINE scale.

The default kernels form each conditional mean in blocked order (int8-digit /
fp64 MFMA far field, FMA near field, reciprocal of R_ii); every SampleZ decision is
certified against a rigorous bound on its distance to the reference-order mean
(klein.py:191-195) or replayed in that order (lgs_device.h, certified decisions).
Their coefficients must therefore equal LGS_EXACT_ORDER's -- which follows the
reference's arithmetic order and is bit-exact against the oracle
(test_gpu_parity.py) -- on every sample, at the sizes the bench runs.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def capi():
    from lgs_amd import _capi
    return _capi


@pytest.mark.parametrize("cfg,n", [("C3_ntru512", 1 << 16), ("C2_qary128", 1 << 18),
                                   ("C4_qary1024", 1 << 15)])
def test_default_order_equals_exact_order_at_scale(capi, oracle, cfg, n):
    import torch
    from lgs_amd.lattices import build_config
    lat, sigma = build_config(cfg)
    B = lat.basis
    R, cp = oracle.qr_prepare(B)
    ctx = capi.Context(0)
    ctx.set_basis(R, cp, B, sigma)
    d = B.shape[0]
    za = torch.empty((d, n), dtype=torch.int32, device="cuda")
    zb = torch.empty_like(za)
    f = capi.LGS_DEVICE_PTRS | capi.LGS_COORD_MAJOR
    ctx.resolved(reset=True)
    ctx.klein(77, 0, n, za, None, None, f)
    redos = ctx.resolved()
    assert ctx.fallbacks() == 0  # the int8-digit far field / 16-bit store path itself was checked
    ctx.klein(77, 0, n, zb, None, None, f | capi.LGS_EXACT_ORDER)
    torch.cuda.synchronize()
    bad = int((za != zb).any(dim=0).sum())
    print(f"{cfg}: {n} samples, {redos} certificate replays, {bad} samples differ")
    assert bad == 0


@pytest.mark.parametrize("cfg,center_scale,wl", [("C3_ntru512", 0.0, False), ("C3_ntru512", 3e4, False),
                                                 ("C4_qary1024", 0.0, False), ("C4_qary1024", 3e4, False),
                                                 ("C3_ntru512", 0.0, True), ("C3_ntru512", 3e4, True)])
def test_speculative_small_kind_subpanels(capi, oracle, cfg, center_scale, wl):
    """Sub-panels of tiny-sigma coordinates (the q-coordinates) are decided all at
    once on the speculation that every z of the sub-panel is 0 (kRecSpec): kept
    when it holds in the whole wave, else redone in order.  Center 0: the
    speculation holds (z = 0 there); a center of scale ~q moves those means off 0,
    so the redo path runs.  Both must equal the reference-order kernel: z exactly,
    the log weights to rounding (their terms use the blocked-order means), in
    reference mode and with Wang-Ling weights.  That the
    kept speculation reproduces the sequential default kernel bit for bit (z and log
    weights) is checked across builds (LGS_NO_SPEC) with tools/kbench.py --hash
    (profiles/r03v_*)."""
    import torch
    from lgs_amd.lattices import build_config
    lat, sigma = build_config(cfg)
    B = lat.basis
    d = B.shape[0]
    rng = np.random.default_rng(5)
    center = rng.uniform(-center_scale, center_scale, d) if center_scale else None
    R, cp = oracle.qr_prepare(B, center)
    ctx = capi.Context(0)
    ctx.set_basis(R, cp, B, sigma)
    n = 1 << 14
    za = torch.empty((d, n), dtype=torch.int32, device="cuda")
    zb = torch.empty_like(za)
    la2 = torch.empty(2 * n, dtype=torch.float64, device="cuda")  # weights, then their bounds
    la, ea = la2[:n], la2[n:]
    lb2 = torch.empty_like(la2)
    lb, eb = lb2[:n], lb2[n:]
    f = capi.LGS_DEVICE_PTRS | capi.LGS_COORD_MAJOR | (capi.LGS_WANG_LING | capi.LGS_LOGW_BOUND if wl else 0)
    ctx.klein(91, 0, n, za, None, la2 if wl else la, f)
    ctx.klein(91, 0, n, zb, None, lb2 if wl else lb, f | capi.LGS_EXACT_ORDER)
    torch.cuda.synchronize()
    small = torch.as_tensor(np.flatnonzero(sigma / np.diag(R) < 4.0), device="cuda")  # the q-coordinates
    assert small.numel() >= d // 4
    nz_q = int((za[small] != 0).any(dim=0).sum())
    print(f"{cfg} center {center_scale}: samples with a nonzero q-coordinate: {nz_q} of {n}")
    if center_scale == 0.0:
        assert nz_q == 0
    else:
        assert nz_q > n // 2
    assert int((za != zb).any(dim=0).sum()) == 0
    dif = (la - lb).abs()
    rel = float((dif / lb.abs().clamp_min(1.0)).max())
    print(f"  log weights: max difference {float(dif.max()):.2e}, relative {rel:.2e}")
    # Reference mode: the weight terms cancel to rounding.  Wang-Ling: the normaliser
    # of a sigma_i ~ 1e-2 coordinate moves by |mu - rint(mu)| / sigma_i^2 per unit of
    # mean, and the default kernels' means are within the certificate's dmu of the
    # reference-order ones: every sample's weight must lie within the bound the kernel
    # derives from those dmu (lgs_kernels.hip wl_bound_*, LGS_LOGW_BOUND); the
    # reference-order kernel reports bound 0.  The accept decisions are certified
    # against these bounds (test_gpu_wl_accept.py).
    if wl:
        assert float(eb.abs().max()) == 0.0
        assert bool((dif <= ea).all()), float((dif - ea).max())
        print(f"  bounds: median {float(ea.median()):.2e}, max {float(ea.max()):.2e}; "
              f"max |dlw| / bound {float((dif / ea.clamp_min(1e-300)).max()):.3f}")
    else:
        assert rel < 1e-10


@pytest.mark.parametrize("scale", [1.0, 0.02])
def test_low_z1_cap_forces_verification_not_speculation(capi, oracle, scale, monkeypatch):
    """The certificate's bound dmu = Ca + Cb * cap holds only while the sample's
    sum |z_j| stays below the context's cap (twice the largest sum of recent
    launches).  A 64-sample launch first sets a cap from few samples; a cap scaled
    far below every sum (LGS_TEST_Z1CAP_SCALE) makes every sub-panel exceed it: the
    sequential sub-panels verify / replay in the reference's order and the
    speculative (all-small-kind) sub-panels must not be kept on a bound that no
    longer holds.  NTRU n = 128 (d = 256): half the coordinates are speculative
    q-coordinates.  Output must equal the reference-order kernel's."""
    import torch
    from lgs_amd import lattices
    if scale != 1.0:  # (a test hook: liblgs_hip_hooks.so reads it, the product library has none)
        monkeypatch.setenv("LGS_TEST_Z1CAP_SCALE", str(scale))
    B = lattices.ntru_basis(128, 12289, 3)
    R, cp = oracle.qr_prepare(B)
    ctx = capi.Context(0, hooks=scale != 1.0)
    ctx.set_basis(R, cp, B, 165.7)
    d = B.shape[0]
    f = capi.LGS_DEVICE_PTRS | capi.LGS_COORD_MAJOR
    z0 = torch.empty((d, 64), dtype=torch.int32, device="cuda")
    ctx.klein(5, 0, 64, z0, None, None, f)  # the cap now comes from these 64 samples
    n = 1 << 14
    za = torch.empty((d, n), dtype=torch.int32, device="cuda")
    zb = torch.empty_like(za)
    la = torch.empty(n, dtype=torch.float64, device="cuda")
    lb = torch.empty_like(la)
    ctx.resolved(reset=True)
    ctx.klein(6, 1 << 20, n, za, None, la, f)
    redos = ctx.resolved()
    ctx.klein(6, 1 << 20, n, zb, None, lb, f | capi.LGS_EXACT_ORDER)
    torch.cuda.synchronize()
    print(f"cap scale {scale}: {redos} verified sub-panels")
    if scale != 1.0:
        assert redos >= n // 64  # every wave verified (cap below every sum)
    assert int((za != zb).any(dim=0).sum()) == 0
    assert float(((la - lb).abs() / lb.abs().clamp_min(1.0)).max()) < 1e-10


@pytest.mark.parametrize("cfg,center_scale", [("C3_ntru512", 0.0), ("C3_ntru512", 3e4), ("C5_ntru2048", 0.0)])
def test_q_panel_skip_equals_full_computation(capi, oracle, cfg, center_scale, monkeypatch):
    """Reference mode skips a panel of speculative (tiny-sigma) rows when the host's
    Cauchy-Schwarz bound on every row's mean, from ||z_W|| of the sample, certifies
    z = 0 there (lgs_set_basis, klein_mfma_kernel).  z must equal the launch that
    computes those panels (LGS_CTX_NO_QSKIP) and the reference-order kernel; the weights
    differ by the rows' mean-dependent rounding only (the terms are lterm at mu = 0).
    A center of scale ~q moves the means off 0: the bound fails and nothing is skipped."""
    import torch
    from lgs_amd.lattices import build_config
    lat, sigma = build_config(cfg)
    B = lat.basis
    d = B.shape[0]
    center = np.random.default_rng(5).uniform(-center_scale, center_scale, d) if center_scale else None
    R, cp = oracle.qr_prepare(B, center)
    n = 1 << 14 if d <= 1024 else 1 << 12
    out = {}
    for skip in ("0", "1"):
        ctx = capi.Context(0, qskip=skip == "0")
        ctx.set_basis(R, cp, B, sigma)
        z = torch.empty((d, n), dtype=torch.int32, device="cuda")
        lw = torch.empty(n, dtype=torch.float64, device="cuda")
        ctx.timing_enable(True)
        ctx.counter(capi.LGS_COUNTER_QSKIP, reset=True)
        ctx.klein(17, 3 << 20, n, z, None, lw, capi.LGS_DEVICE_PTRS | capi.LGS_COORD_MAJOR)
        ms, _ = ctx.timing_get(capi.KERNEL_KLEIN)
        out[skip] = (z, lw, ms, ctx.counter(capi.LGS_COUNTER_QSKIP))
    ctx.klein(17, 3 << 20, n, out["1"][0], None, None, capi.LGS_DEVICE_PTRS | capi.LGS_COORD_MAJOR | capi.LGS_EXACT_ORDER)
    torch.cuda.synchronize()
    qs = out["0"][3]
    print(f"{cfg} center {center_scale}: skip {out['0'][2]:.3f} ms ({qs} wave-panels skipped), "
          f"no skip {out['1'][2]:.3f} ms")
    assert out["1"][3] == 0
    nq = (sigma / np.diag(R) < 4.0).sum() // 32  # the q-panels
    if center_scale == 0.0:
        # (nearly) every q-panel of every wave: a block votes as one, and a block with a
        # sample whose ||z_W|| exceeds a panel's bound computes that panel
        assert 0.95 * (nq * n // 64) <= qs <= nq * n // 64
    else:
        assert qs == 0
    assert torch.equal(out["0"][0], out["1"][0])  # skipped panels: the same z as computed ones
    rel = float(((out["0"][1] - out["1"][1]).abs() / out["1"][1].abs().clamp_min(1.0)).max())
    assert rel < 1e-12, rel
