"""StreamingShard's per-block lag-sum update replayed as a captured HIP graph (the
bench's timed path) equals the eager update, block by block, on the same inputs."""
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(__file__)), "lattice-gaussian-mcmc_amd"))

pytestmark = pytest.mark.gpu


def _run(graph: bool, blocks: int = 5):
    import torch
    from lgs_amd import distributed as D
    old = os.environ.get("LGS_NO_GRAPH")
    os.environ["LGS_NO_GRAPH"] = "0" if graph else "1"
    try:
        nc, T, d = 96, 8, 24
        buf = torch.empty((nc, T, d), dtype=torch.float64, device="cuda:0")
        rng = np.random.default_rng(5)
        data = [rng.integers(-300, 300, size=(nc, T, d)).astype(np.float64) for _ in range(blocks)]
        it = iter(data)

        def advance(first_step, n_steps, acc, mom):
            buf.copy_(torch.from_numpy(next(it)))  # same buffer every block, as gpu_advance
            acc += 1
            return buf

        binv = rng.standard_normal(d) * 0.01
        sh = D.StreamingShard(advance, nc, d, binv_row=binv, device="cuda:0", lag_chains=64, lags=5)
        for _ in range(blocks):
            sh.step(T)
        torch.cuda.synchronize()
        return ([x.cpu().numpy().copy() for x in sh.lag_z.parts()], [x.cpu().numpy().copy() for x in sh.lag_v.parts()],
                sh._graph is not None)
    finally:
        if old is None:
            os.environ.pop("LGS_NO_GRAPH", None)
        else:
            os.environ["LGS_NO_GRAPH"] = old


def test_lag_sums_graph_replay_equals_eager():
    z_g, v_g, captured = _run(True)
    z_e, v_e, eager_captured = _run(False)
    assert captured and not eager_captured
    for a, b in zip(z_g, z_e):
        assert np.array_equal(a, b)
    for a, b in zip(v_g, v_e):
        assert np.array_equal(a, b)


def _gpu_shard(sync_each: bool, blocks: int = 4, flags=None, work_stream: bool = False):
    """StreamingShard driven through gpu_advance (lgs_imhk on the library's stream,
    the lag-sum graph and the thinned Gram on the caller's), C2 q-ary d = 128;
    work_stream: everything on one non-default current stream (as bench.py)."""
    import torch
    from lgs_amd import _capi
    from lgs_amd import distributed as D
    from lgs_amd.lattices import build_config
    import lgs_oracle
    lat, sigma = build_config("C2_qary128")
    B = lat.basis
    R, cp = lgs_oracle.qr_prepare(B)
    d = B.shape[0]
    ctx = _capi.Context(0)
    ctx.set_basis(R, cp, B, sigma)
    dev = torch.device("cuda", 0)
    nc, T = 2048, 16
    prev = torch.cuda.current_stream(dev)
    if work_stream:
        torch.cuda.synchronize()
        torch.cuda.set_stream(torch.cuda.Stream(device=dev))
    try:
        return _gpu_shard_run(ctx, D, B, d, dev, nc, T, sync_each, blocks,
                              _capi.LGS_WANG_LING if flags is None else flags)
    finally:
        torch.cuda.synchronize()
        torch.cuda.set_stream(prev)


def _gpu_shard_run(ctx, D, B, d, dev, nc, T, sync_each, blocks, flags):
    import torch
    adv = D.gpu_advance(ctx, 31, 0, nc, d, dev, flags=flags, block_steps=T)
    sh = D.StreamingShard(adv, nc, d, binv_row=np.linalg.inv(B)[d - 1], device=dev, lag_chains=512, lags=6,
                          gram_every=2)
    for _ in range(blocks):
        sh.step(T)
        if sync_each:
            torch.cuda.synchronize()
    st = sh.reduce()
    torch.cuda.synchronize()
    return {k: ([x.cpu().numpy().copy() for x in v] if isinstance(v, list) else v.cpu().numpy().copy())
            for k, v in st.items()}


def test_gpu_advance_streams_match_synchronized_run():
    """The library's stream waits for the caller's stream before each call (the lag
    update still reading the reused v buffer): results equal a run synchronised
    after every block."""
    a = _gpu_shard(False)
    b = _gpu_shard(True)
    assert set(a) == set(b) and "gram" in a
    for k in a:
        xa, xb = (a[k], b[k]) if isinstance(a[k], list) else ([a[k]], [b[k]])
        for x, y in zip(xa, xb):
            assert np.array_equal(x, y), k
    assert 0 < int(a["accepts"][0]) < 2048 * 64


def test_gpu_advance_on_the_callers_work_stream():
    """Reference weights (the early check) with the library on the caller's own
    non-default stream (bench.py's layout: no cross-stream waits) equal the run on
    the default stream synchronised after every block."""
    a = _gpu_shard(False, flags=0, work_stream=True)
    b = _gpu_shard(True, flags=0)
    assert set(a) == set(b) and "gram" in a
    for k in a:
        xa, xb = (a[k], b[k]) if isinstance(a[k], list) else ([a[k]], [b[k]])
        for x, y in zip(xa, xb):
            assert np.array_equal(x, y), k
    assert int(a["accepts"][0]) > 0


@pytest.mark.parametrize("cfg", ["C3_ntru512", "C2_qary128"])
def test_imhk_ex_functionals_equal_recomputation(cfg):
    """lgs_imhk_ex's per-kept-state functionals -- ||v||^2 summed in the B z epilogue
    and coefficient d-1 gathered from the proposal store -- equal the same quantities
    recomputed from the kept lattice points / coefficients it also returns."""
    import torch
    from lgs_amd import _capi
    from lgs_amd.lattices import build_config
    import lgs_oracle
    lat, sigma = build_config(cfg)
    B = lat.basis
    R, cp = lgs_oracle.qr_prepare(B)
    d = B.shape[0]
    ctx = _capi.Context(0)
    ctx.set_basis(R, cp, B, sigma)
    nc, T = 512, 8
    dev = "cuda:0"
    z = torch.zeros((nc, d), dtype=torch.int32, device=dev)
    lw = torch.zeros(nc, dtype=torch.float64, device=dev)
    init = torch.zeros(nc, dtype=torch.int32, device=dev)
    acc = torch.zeros(nc, dtype=torch.int64, device=dev)
    for wl in (0, _capi.LGS_WANG_LING):  # (Wang-Ling: rejections keep carried-in states)
        zs = torch.empty((nc, T, d), dtype=torch.int32, device=dev)
        vs = torch.empty((nc, T, d), dtype=torch.float64, device=dev)
        vn2 = torch.full((nc, T), -1.0, dtype=torch.float64, device=dev)
        zk = torch.full((nc, T), -7, dtype=torch.int64, device=dev)
        ctx.imhk(3, 0, nc, 1 + 2 * T * (wl != 0), T, 1, z, lw, init, acc, z_samples=zs, v_samples=vs,
                 flags=_capi.LGS_DEVICE_PTRS | wl, vnorm2_samples=vn2, zk_samples=zk, zk_index=d - 1)
        torch.cuda.synchronize()
        assert torch.equal(vn2, (vs * vs).sum(-1))
        assert torch.equal(zk, zs[:, :, d - 1].long())
        assert torch.equal(vs, zs.double() @ torch.as_tensor(B, device=dev).T)


@pytest.mark.parametrize("fn", [1, 100, 511])
def test_imhk_ex_functionals_of_leading_chains(fn):
    """fn_chains: the functionals of the leading fn chains only (fn x n_keep arrays),
    equal to the all-chains run's first rows; nothing written past them."""
    import torch
    from lgs_amd import _capi
    from lgs_amd.lattices import build_config
    import lgs_oracle
    lat, sigma = build_config("C3_ntru512")
    B = lat.basis
    R, cp = lgs_oracle.qr_prepare(B)
    d = B.shape[0]
    ctx = _capi.Context(0)
    ctx.set_basis(R, cp, B, sigma)
    nc, T = 512, 8
    dev = "cuda:0"
    res = []
    for f in (0, fn):
        z = torch.zeros((nc, d), dtype=torch.int32, device=dev)
        lw = torch.zeros(nc, dtype=torch.float64, device=dev)
        init = torch.zeros(nc, dtype=torch.int32, device=dev)
        acc = torch.zeros(nc, dtype=torch.int64, device=dev)
        rows = nc if f == 0 else f + 1  # (one guard row)
        vs = torch.empty((nc, T, d), dtype=torch.float64, device=dev)
        vn2 = torch.full((rows, T), -1.0, dtype=torch.float64, device=dev)
        zk = torch.full((rows, T), -7, dtype=torch.int64, device=dev)
        ctx.imhk(9, 0, nc, 1, T, 1, z, lw, init, acc, v_samples=vs, flags=_capi.LGS_DEVICE_PTRS,
                 vnorm2_samples=vn2, zk_samples=zk, zk_index=d - 1, fn_chains=f)
        torch.cuda.synchronize()
        res.append((vs, vn2, zk))
    (va, na, ka), (vb, nb, kb) = res
    assert torch.equal(va, vb)
    assert torch.equal(nb[:fn], na[:fn]) and torch.equal(kb[:fn], ka[:fn])
    assert torch.equal(na, (va * va).sum(-1))
    assert bool((nb[fn] == -1.0).all()) and bool((kb[fn] == -7).all())


def _lag_shard(fused: bool):
    import torch
    from lgs_amd import _capi
    from lgs_amd import distributed as D
    from lgs_amd.lattices import build_config
    import lgs_oracle
    lat, sigma = build_config("C3_ntru512")
    B = lat.basis
    R, cp = lgs_oracle.qr_prepare(B)
    d = B.shape[0]
    ctx = _capi.Context(0)
    ctx.set_basis(R, cp, B, sigma)
    dev = torch.device("cuda", 0)
    nc, T = 1024, 8
    adv = D.gpu_advance(ctx, 12, 0, nc, d, dev, block_steps=T, fn_chains=300)
    sh = D.StreamingShard(adv, nc, d, binv_row=np.linalg.inv(B)[d - 1], device=dev, lag_chains=300, lags=11,
                          fused_lag=fused)
    assert sh._fused_lag == fused
    for _ in range(3):  # T = 8 < L = 11: the ring carries values across blocks
        sh.step(T)
    st = sh.reduce()
    torch.cuda.synchronize()
    return {k: ([x.cpu().numpy().copy() for x in v] if isinstance(v, list) else v.cpu().numpy().copy())
            for k, v in st.items()}


def test_fused_lag_sums_equal_torch_update():
    """lgs_imhk_ex's lag sums (lag_L, inside the call) equal LagSums' torch update on
    the returned series: int64 z series exactly, the fp64 ||v||^2 series to 1e-12."""
    a, b = _lag_shard(True), _lag_shard(False)
    for k in ("accepts", "moments"):
        assert np.array_equal(a[k], b[k])
    for x, y in zip(a["lag_z"], b["lag_z"]):
        assert np.array_equal(x, y)
    for x, y in zip(a["lag_v"], b["lag_v"]):
        np.testing.assert_allclose(x, y, rtol=1e-12, atol=0)
    assert a["lag_z"][0][0] > 0


def test_imhk_ex_lag_sums_with_thinning_across_calls():
    """lgs_imhk_ex lag_L on its own (no StreamingShard): thin = 2, two calls whose
    series continue through the caller's ring; the sums equal numpy's over the
    concatenated kept-state series (int64 exactly, the scaled ||v||^2 to 1e-12)."""
    import torch
    from lgs_amd import _capi
    from lgs_amd.lattices import build_config
    import lgs_oracle
    lat, sigma = build_config("C2_qary128")
    B = lat.basis
    R, cp = lgs_oracle.qr_prepare(B)
    d = B.shape[0]
    ctx = _capi.Context(0)
    ctx.set_basis(R, cp, B, sigma)
    nc, steps, thin, L, fn = 300, 12, 2, 5, 200
    dev = "cuda:0"
    z = torch.zeros((d, nc), dtype=torch.int32, device=dev)
    lw = torch.zeros(nc, dtype=torch.float64, device=dev)
    init = torch.zeros(nc, dtype=torch.int32, device=dev)
    acc = torch.zeros(nc, dtype=torch.int64, device=dev)
    zr = torch.zeros((fn, L), dtype=torch.int64, device=dev)
    zsum = torch.zeros(L + 2, dtype=torch.int64, device=dev)
    vr = torch.zeros((fn, L), dtype=torch.float64, device=dev)
    vsum = torch.zeros(L + 2, dtype=torch.float64, device=dev)
    xs_z, xs_v = [], []
    for call in range(2):
        nk = steps // thin
        vs = torch.empty((nc, nk, d), dtype=torch.float64, device=dev)
        vn2 = torch.empty((fn, nk), dtype=torch.float64, device=dev)
        zk = torch.empty((fn, nk), dtype=torch.int64, device=dev)
        ctx.imhk(5, 0, nc, 1 + call * steps, steps, thin, z, lw, init, acc, v_samples=vs,
                 flags=_capi.LGS_DEVICE_PTRS | _capi.LGS_COORD_MAJOR | _capi.LGS_WANG_LING,
                 vnorm2_samples=vn2, zk_samples=zk, zk_index=d - 1, fn_chains=fn,
                 lag=(L, zr, zsum, vr, vsum, 1e-6))
        torch.cuda.synchronize()
        xs_z.append(zk.cpu().numpy())
        xs_v.append(vn2.cpu().numpy() * 1e-6)
    for xs, got, exact in ((np.concatenate(xs_z, 1), zsum.cpu().numpy(), True),
                           (np.concatenate(xs_v, 1), vsum.cpu().numpy(), False)):
        n = xs.shape[1]
        want = [sum((xs[:, t] * xs[:, t - k]).sum() for t in range(k, n)) for k in range(L + 1)]
        want.append(xs.sum())
        want = np.array(want, dtype=xs.dtype)
        if exact:
            assert np.array_equal(got, want)
        else:
            np.testing.assert_allclose(got, want, rtol=1e-12, atol=0)
    assert np.array_equal(zr.cpu().numpy(), np.concatenate(xs_z, 1)[:, -L:])


@pytest.fixture(scope="module")
def capi():
    from lgs_amd import _capi
    _capi.load_library()
    return _capi


def _imhk_carried(capi, on_caller_stream: bool, zmax: int):
    """lgs_imhk_ex with device pointers: chain states carried in with |z| up to zmax
    and a log weight no proposal beats, so every kept state is the carried one."""
    import torch
    from conftest import golden_R, load_golden
    g = load_golden("klein_qary128.npz")
    R, cp, B = golden_R(g)
    ctx = capi.Context(0)  # fresh: the wider store after a 16-bit overflow is sticky
    ctx.set_basis(R, cp, B, float(g["sigma"]))
    d, nc, steps = R.shape[0], 256, 6
    dev = "cuda:0"
    rng = np.random.default_rng(zmax)
    z0 = rng.integers(-zmax, zmax + 1, size=(d, nc)).astype(np.int32)
    z0[:, 0] = zmax
    z = torch.from_numpy(z0).to(dev)
    lw = torch.full((nc,), 1e300, dtype=torch.float64, device=dev)
    init = torch.ones(nc, dtype=torch.int32, device=dev)
    acc = torch.zeros(nc, dtype=torch.int64, device=dev)
    mom = torch.zeros(2 * d, dtype=torch.int64, device=dev)
    vs = torch.zeros((nc, steps, d), dtype=torch.float64, device=dev)
    vn2 = torch.zeros((nc, steps), dtype=torch.float64, device=dev)
    zk = torch.zeros((nc, steps), dtype=torch.int64, device=dev)
    # lag sums continued inside the call: they read ||v||^2 before the call returns, so
    # a digit-range replay of B z must reach them (on the library's own
    # stream it used to be a host replay after them)
    L = 3
    zr = torch.zeros((nc, L), dtype=torch.int64, device=dev)
    zsum = torch.zeros(L + 2, dtype=torch.int64, device=dev)
    vr = torch.zeros((nc, L), dtype=torch.float64, device=dev)
    vsum = torch.zeros(L + 2, dtype=torch.float64, device=dev)
    torch.cuda.synchronize()
    s = torch.cuda.Stream(device=dev)
    if on_caller_stream:  # lgs_set_stream: the call's early check applies
        ctx.set_stream(s.cuda_stream)
    ctx.imhk(5, 0, nc, 1, steps, 1, z, lw, init, acc, v_samples=vs, moments=mom, vnorm2_samples=vn2,
             zk_samples=zk, zk_index=3, flags=capi.LGS_DEVICE_PTRS | capi.LGS_COORD_MAJOR,
             lag=(L, zr, zsum, vr, vsum, 1e-6))
    torch.cuda.synchronize()
    out = {k: t.cpu().numpy() for k, t in dict(z=z, acc=acc, mom=mom, v=vs, vn2=vn2, zk=zk, zsum=zsum,
                                                 vsum=vsum, zr=zr, vr=vr).items()}
    ctx.close()
    return z0, B, out


@pytest.mark.parametrize("zmax", [200, 32639, 32700, 40000])
def test_early_check_equals_synchronised_call(capi, zmax):
    """lgs_imhk on a caller's stream checks each block's flags right after its abort
    producers and leaves B z's digit-range replay to the device (gated fp64 launch);
    the results equal the same call on the library's own stream (host-checked), and
    v is exactly B z of the carried states -- including |z| beyond the int8 digits
    (32640..32767: the replay alone; > 32767: also the 16-bit store's redo)."""
    z0, B, a = _imhk_carried(capi, True, zmax)
    _, _, b = _imhk_carried(capi, False, zmax)
    for k in a:
        assert np.array_equal(a[k], b[k]), k
    assert not a["acc"].any()
    # moments of the 6 kept states per chain (all the carried one): on the caller's stream
    # from B z's digit tiles, or (|z| beyond two digits) from the gated moments pass
    z64 = z0.astype(np.int64)
    assert np.array_equal(a["mom"], np.concatenate([6 * z64.sum(1), 6 * (z64 ** 2).sum(1)]))
    want = (B.astype(np.int64) @ z0.astype(np.int64)).T  # nc x d
    # ||v||^2 reaches ~1e20 at |z| ~ 32639 (beyond 2^53: fp64 sums in another order than
    # numpy's), so against numpy to rounding; the early-checked and host-checked calls
    # above are equal bit for bit
    n2 = (want.astype(np.float64) ** 2).sum(1)
    for t in range(a["v"].shape[1]):
        assert np.array_equal(a["v"][:, t, :], want.astype(np.float64)), t
        assert np.array_equal(a["zk"][:, t], z0[3, :].astype(np.int64)), t
        np.testing.assert_allclose(a["vn2"][:, t], n2, rtol=1e-13, atol=0)
    # the lag sums of the constant series x_t = 1e-6 ||v||^2 (and z_3) over the 6 steps
    L, n = len(a["vsum"]) - 2, a["v"].shape[1]
    for xs, got, exact in ((np.repeat(z0[3, :].astype(np.int64)[:, None], n, 1), a["zsum"], True),
                           (np.repeat((n2 * 1e-6)[:, None], n, 1), a["vsum"], False)):
        w = [sum((xs[:, t] * xs[:, t - k]).sum() for t in range(k, n)) for k in range(L + 1)] + [xs.sum()]
        w = np.array(w, dtype=xs.dtype)
        if exact:
            assert np.array_equal(got, w)
        else:
            np.testing.assert_allclose(got, w, rtol=1e-12, atol=0)


def _imhk_calls(capi, on_caller_stream: bool, flags_extra: int, calls: int = 3, blocks: int = 3, plan=None,
                thin: int = 1, z64: bool = False, cu_split: bool = True, gauge=None, hooks: bool = False):
    """Several lgs_imhk_ex calls of several blocks each (max_proposals: T = 4 steps
    per block), chain state, accept counts, moments, lattice points, functionals and
    lag sums carried across them -- on a caller's stream the blocks are pipelined
    (each block's Klein launch on the context's Klein stream into alternating buffer
    sets, beside the previous block's dependants)."""
    import torch
    from conftest import golden_R, load_golden
    g = load_golden("klein_qary128.npz")
    R, cp, B = golden_R(g)
    d, nc, T = R.shape[0], 256, 4
    ctx = capi.Context(0, max_proposals=nc * T, cu_split=cu_split, hooks=hooks)
    ctx.set_basis(R, cp, B, float(g["sigma"]))
    dev = "cuda:0"
    plan = plan or [T * blocks] * calls  # steps per call (a changed count discards the look-ahead launch)
    z = torch.zeros((d, nc), dtype=torch.int64 if z64 else torch.int32, device=dev)
    lw = torch.zeros(nc, dtype=torch.float64, device=dev)
    init = torch.zeros(nc, dtype=torch.int32, device=dev)
    acc = torch.zeros(nc, dtype=torch.int64, device=dev)
    mom = torch.zeros(2 * d, dtype=torch.int64, device=dev)
    if z64:
        flags_extra |= capi.LGS_Z64
    L = 5
    zr = torch.zeros((nc, L), dtype=torch.int64, device=dev)
    zsum = torch.zeros(L + 2, dtype=torch.int64, device=dev)
    vr = torch.zeros((nc, L), dtype=torch.float64, device=dev)
    vsum = torch.zeros(L + 2, dtype=torch.float64, device=dev)
    torch.cuda.synchronize()
    s = torch.cuda.Stream(device=dev)
    if on_caller_stream:
        ctx.set_stream(s.cuda_stream)
    vs_all, vn_all, zk_all = [], [], []
    with torch.cuda.stream(s):
        first = 1
        for steps in plan:
            kept = steps // thin
            vs = torch.zeros((nc, kept, d), dtype=torch.float64, device=dev)
            vn2 = torch.zeros((nc, kept), dtype=torch.float64, device=dev)
            zk = torch.zeros((nc, kept), dtype=torch.int64, device=dev)
            ctx.imhk(11, 0, nc, first, steps, thin, z, lw, init, acc, v_samples=vs, moments=mom,
                     vnorm2_samples=vn2, zk_samples=zk, zk_index=5,
                     flags=capi.LGS_DEVICE_PTRS | capi.LGS_COORD_MAJOR | flags_extra,
                     lag=(L, zr, zsum, vr, vsum, 1e-6))
            first += steps
            vs_all.append(vs)
            vn_all.append(vn2)
            zk_all.append(zk)
    torch.cuda.synchronize()
    out = {k: t.cpu().numpy() for k, t in dict(z=z, lw=lw, init=init, acc=acc, mom=mom, zsum=zsum, vsum=vsum,
                                                 zr=zr, vr=vr).items()}
    out["v"] = torch.cat(vs_all, 1).cpu().numpy()
    out["vn2"] = torch.cat(vn_all, 1).cpu().numpy()
    out["zk"] = torch.cat(zk_all, 1).cpu().numpy()
    if gauge is not None:
        gauge.append((ctx.counter(capi.LGS_COUNTER_KLEIN_CUS), ctx.device_info()["n_cu"]))
    ctx.close()
    return B, out


@pytest.mark.parametrize("mode,plan,thin,z64", [("reference", None, 1, False), ("wang_ling_exact", None, 1, False),
                                               ("reference", [12, 4, 4, 8], 1, False), ("reference", None, 2, False),
                                               ("reference", None, 1, True)])
def test_pipelined_blocks_equal_synchronised_calls(capi, mode, plan, thin, z64):
    """Pipelined blocks (caller's stream) give every output of the host-checked calls
    on the library's own stream, bit for bit, over 3 calls x 3 blocks (each call's
    first block from the previous call's look-ahead launch), or calls of 3, 1, 1 and 2
    blocks (a look-ahead discarded on the changed step count, used on the repeated
    one); v is B z of the kept states (z_k recovered from v through the basis' inverse
    is checked against zk)."""
    fx = 0 if mode == "reference" else capi.LGS_WANG_LING | capi.LGS_EXACT_ORDER
    B, a = _imhk_calls(capi, True, fx, plan=plan, thin=thin, z64=z64)
    _, b = _imhk_calls(capi, False, fx, plan=plan, thin=thin, z64=z64)
    for k in a:
        assert np.array_equal(a[k], b[k]), k
    steps = a["v"].shape[1] * thin  # (thin 2: the moments and v count the kept states only)
    assert a["acc"].sum() > 0 and (mode == "reference") == bool((a["acc"] == steps).all())
    # v = B z: z = B^-1 v is integral and its coordinate 5 is the zk series
    zrec = np.rint(np.linalg.solve(B.astype(np.float64), a["v"].reshape(-1, B.shape[0]).T)).T
    assert np.array_equal(zrec[:, 5].astype(np.int64), a["zk"].reshape(-1))
    np.testing.assert_allclose(a["vn2"].reshape(-1), (a["v"].reshape(-1, B.shape[0]) ** 2).sum(1), rtol=1e-13)
    # moments: sum over every kept state of z and z^2 (exact integers)
    assert np.array_equal(a["mom"][:B.shape[0]], zrec.astype(np.int64).sum(0))
    assert np.array_equal(a["mom"][B.shape[0]:], (zrec.astype(np.int64) ** 2).sum(0))


def test_cu_split_klein_stream_equals_unmasked(capi, monkeypatch):
    """The pipelined Klein launches on a stream whose queue is masked off 1/8 of the CUs
    (forced here through the hooks build's LGS_PIPE_CU_RESERVE; by default the library
    takes it when the B z stores outweigh 1/7 of the timed Klein launch) give every
    output of the launches on every CU (LGS_CTX_NO_CU_SPLIT); LGS_COUNTER_KLEIN_CUS
    reports the mask.  Without the hook, this small lattice (d = 128: B z is a tenth of
    the Klein time) keeps every CU."""
    import torch
    ncu = torch.cuda.get_device_properties(0).multi_processor_count
    res = ncu // 8 if ncu % 32 == 0 else 0
    g1, g2, g3 = [], [], []
    monkeypatch.setenv("LGS_PIPE_CU_RESERVE", str(res))
    _, a = _imhk_calls(capi, True, 0, gauge=g1, hooks=True)
    monkeypatch.delenv("LGS_PIPE_CU_RESERVE")
    _, b = _imhk_calls(capi, True, 0, cu_split=False, gauge=g2)
    _, c = _imhk_calls(capi, True, 0, gauge=g3)
    for k in a:
        assert np.array_equal(a[k], b[k]), k
        assert np.array_equal(a[k], c[k]), k
    assert g1[0] == ((ncu - res) if res else 0, ncu)
    assert g2[0][0] == 0 and g3[0][0] in (0, ncu - res)


def test_lookahead_discarded_on_new_basis_and_changed_call(capi):
    """A pipelined call leaves the next call's first Klein launch enqueued; lgs_set_basis
    (another lattice) and a call with other arguments (another seed) must discard it:
    the later calls equal the same calls on a fresh context."""
    import torch
    from conftest import golden_R, load_golden
    ga, gb = load_golden("klein_qary128.npz"), load_golden("klein_ntru128.npz")
    Ra, cpa, Ba = golden_R(ga)
    Rb, cpb, Bb = golden_R(gb)
    assert Ra.shape == Rb.shape
    d, nc, steps = Ra.shape[0], 256, 8
    dev = "cuda:0"

    def state():
        return dict(z=torch.zeros((d, nc), dtype=torch.int32, device=dev),
                    lw=torch.zeros(nc, dtype=torch.float64, device=dev),
                    init=torch.zeros(nc, dtype=torch.int32, device=dev),
                    acc=torch.zeros(nc, dtype=torch.int64, device=dev),
                    mom=torch.zeros(2 * d, dtype=torch.int64, device=dev))

    def call(ctx, st, seed, first, B):
        v = torch.zeros((nc, steps, d), dtype=torch.float64, device=dev)
        ctx.imhk(seed, 0, nc, first, steps, 1, st["z"], st["lw"], st["init"], st["acc"], v_samples=v,
                 moments=st["mom"], flags=capi.LGS_DEVICE_PTRS | capi.LGS_COORD_MAJOR)
        return v

    s = torch.cuda.Stream(device=dev)
    torch.cuda.synchronize()
    ctx = capi.Context(0)
    ctx.set_stream(s.cuda_stream)
    with torch.cuda.stream(s):
        ctx.set_basis(Ra, cpa, Ba, float(ga["sigma"]))
        call(ctx, state(), 3, 1, Ba)  # leaves a look-ahead for (seed 3, step 9) on basis a
        ctx.set_basis(Rb, cpb, Bb, float(gb["sigma"]))
        st1 = state()
        v1 = call(ctx, st1, 3, 9, Bb)  # the look-ahead's arguments, but another basis
        v2 = call(ctx, st1, 4, 17, Bb)  # another seed than this call's look-ahead
    torch.cuda.synchronize()
    got = [v1.cpu().numpy(), v2.cpu().numpy(), st1["z"].cpu().numpy(), st1["mom"].cpu().numpy()]
    ctx.close()
    ref = capi.Context(0)  # fresh, on its own stream (host-checked calls)
    ref.set_basis(Rb, cpb, Bb, float(gb["sigma"]))
    st2 = state()
    w1 = call(ref, st2, 3, 9, Bb)
    w2 = call(ref, st2, 4, 17, Bb)
    torch.cuda.synchronize()
    want = [w1.cpu().numpy(), w2.cpu().numpy(), st2["z"].cpu().numpy(), st2["mom"].cpu().numpy()]
    ref.close()
    for g_, w_ in zip(got, want):
        assert np.array_equal(g_, w_)
    # v = B z for the fresh basis (not the look-ahead's)
    zrec = np.rint(np.linalg.solve(Bb.astype(np.float64), got[0].reshape(-1, d).T)).T
    assert np.array_equal(Bb.astype(np.float64) @ zrec.T, got[0].reshape(-1, d).T)


def test_pipelined_call_error_then_next_call(capi):
    """a pipelined call that ends in an error (here LGS_ERR_OVERFLOW:
    |z| beyond the int32 state: a center of 3e9 on Z^16) leaves its block's readers enqueued on
    the caller's stream; the set's free event is recorded on that exit too, so the next
    call's Klein launch into the same buffer set waits for them.  The next call (int64
    state) equals the same call on a fresh context."""
    import torch
    d, nc, T = 16, 256, 4
    B = np.eye(d)
    R, cp = np.eye(d), np.full(d, 3.0e9)
    dev = "cuda:0"
    ctx, ref = capi.Context(0, max_proposals=nc * T), capi.Context(0, max_proposals=nc * T)

    def state(dt):
        return dict(z=torch.zeros((d, nc), dtype=dt, device=dev), lw=torch.zeros(nc, dtype=torch.float64, device=dev),
                    init=torch.zeros(nc, dtype=torch.int32, device=dev),
                    acc=torch.zeros(nc, dtype=torch.int64, device=dev),
                    mom=torch.zeros(2 * d, dtype=torch.int64, device=dev))

    def call(c, st, flags):
        v = torch.zeros((nc, 3 * T, d), dtype=torch.float64, device=dev)
        c.imhk(5, 0, nc, 1, 3 * T, 1, st["z"], st["lw"], st["init"], st["acc"], v_samples=v, moments=st["mom"],
               flags=capi.LGS_DEVICE_PTRS | capi.LGS_COORD_MAJOR | flags)
        return v

    out = []
    for c, pipelined in ((ctx, True), (ref, False)):
        c.set_basis(R, cp, B, 3.0)
        s = torch.cuda.Stream(device=dev)
        torch.cuda.synchronize()
        if pipelined:
            c.set_stream(s.cuda_stream)
        with torch.cuda.stream(s):
            if pipelined:
                with pytest.raises(capi.LgsError):
                    call(c, state(torch.int32), 0)
            st = state(torch.int64)
            v = call(c, st, capi.LGS_Z64)
        torch.cuda.synchronize()
        out.append([v.cpu().numpy(), st["z"].cpu().numpy(), st["acc"].cpu().numpy(), st["lw"].cpu().numpy()])
        c.close()
    for a, b in zip(*out):
        assert np.array_equal(a, b)
    assert np.abs(out[0][1]).max() > 2 ** 31  # the int64 states hold what the int32 call could not
