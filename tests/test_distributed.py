"""Multi-process path on CPU (gloo, world size 2): sharding + the single all-reduce.

The per-rank compute is the oracle (test infrastructure); the GPU path uses the
same `imhk_sharded` with `gpu_compute`.  The all-reduced statistics must equal a
single-process run over all chains (counter-addressed draws make them
bit-identical for any world size)."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from conftest import golden_R, load_golden


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    repo = os.path.dirname(here)
    for p in (os.path.join(repo, "lattice-gaussian-mcmc_amd"), os.path.join(repo, "oracle"), here):
        sys.path.insert(0, p)
    import torch.distributed as dist
    import lgs_oracle
    from lgs_amd.distributed import imhk_sharded
    from _oracle_shard import oracle_compute_factory
    from conftest import golden_R, load_golden
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    g = load_golden("klein_ntru32.npz")
    R, cp, B = golden_R(g)
    comp = oracle_compute_factory(lgs_oracle, R, cp, B, float(g["sigma"]), 4242, thin=2,
                                  mode=lgs_oracle.IMHK_WANG_LING, want_gram=True, gr_coord=31)
    js = imhk_sharded(comp, 7, 10, rank=rank, world=world)
    out[rank] = (js.accepts, js.moments.tolist(), js.kept, js.gram.tolist(), js.chain_stats.tolist())
    dist.barrier()
    dist.destroy_process_group()


def test_shard_range_partitions():
    from lgs_amd.distributed import shard_range
    for n in (1, 7, 16, 1000):
        for w in (1, 2, 3, 8):
            parts = [shard_range(n, r, w) for r in range(w)]
            assert sum(c for _, c in parts) == n
            assert all(parts[i][0] + parts[i][1] == parts[i + 1][0] for i in range(w - 1))


@pytest.mark.timeout(300)
def test_gloo_world2_matches_single_process(oracle):
    from _oracle_shard import oracle_compute_factory
    mgr = mp.Manager()
    out = mgr.dict()
    port = _free_port()
    mp.start_processes(_worker, args=(2, port, out), nprocs=2, join=True, start_method="spawn")
    g = load_golden("klein_ntru32.npz")
    R, cp, B = golden_R(g)
    single = oracle_compute_factory(oracle, R, cp, B, float(g["sigma"]), 4242, thin=2,
                                    mode=oracle.IMHK_WANG_LING, want_gram=True, gr_coord=31)(0, 7, 1, 10)
    from lgs_amd.distributed import JobStats
    for rank in (0, 1):
        acc, mom, kept, gram, cs = out[rank]
        assert acc == single.accepts
        assert kept == single.kept == 7 * 5
        assert np.array_equal(np.array(mom), single.moments)
        assert np.array_equal(np.array(gram), single.gram)                 # all-reduced sum z z^T
        np.testing.assert_array_equal(np.array(cs), single.chain_stats)    # gathered, global order
        js = JobStats(acc, np.array(mom), kept, np.array(gram), np.array(cs))
        flat = oracle.imhk(R, cp, B, float(g["sigma"]), 7, 10, seed=4242, first_step=1,
                           mode=oracle.IMHK_WANG_LING, trace=True)["trace"][:, 1::2]
        np.testing.assert_allclose(js.covariance(), np.cov(flat.reshape(-1, R.shape[0]).T.astype(float)),
                                   rtol=1e-12, atol=1e-12)
        import lgs_diag_oracle as O
        np.testing.assert_allclose(js.gelman_rubin(5), O.gelman_rubin([c for c in flat[:, :, 31].astype(float)]),
                                   rtol=1e-12)


def _stream_worker(rank, world, port, out):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    repo = os.path.dirname(here)
    for p in (os.path.join(repo, "lattice-gaussian-mcmc_amd"), os.path.join(repo, "oracle"), here):
        sys.path.insert(0, p)
    import torch
    import torch.distributed as dist
    import lgs_oracle
    from lgs_amd import distributed as D
    from _oracle_shard import oracle_advance_factory
    from conftest import golden_R, load_golden
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    D.init_process_group("gloo", 0, world, rank=rank)
    out[rank] = _stream_stats(D, lgs_oracle, oracle_advance_factory, golden_R(load_golden("klein_ntru32.npz")),
                              rank, world, torch)
    dist.barrier()
    dist.destroy_process_group()


def _stream_stats(D, oracle, factory, RcpB, rank, world, torch):
    """bench.py's timed path (StreamingShard: blocks of IMHK steps, lag sums, one
    all-reduce) over this rank's contiguous shard of 6 chains, Wang-Ling weights."""
    R, cp, B = RcpB
    first, count = D.shard_range(6, rank, world)
    adv = factory(oracle, R, cp, B, 165.7, 99, first, count, mode=oracle.IMHK_WANG_LING)
    binv = np.linalg.inv(B)[B.shape[0] - 1]
    sh = D.StreamingShard(adv, count, B.shape[0], binv_row=binv, device="cpu", lag_chains=6, lags=5,
                          gram_every=2)
    sh.step(3)  # warm-up block, then fresh statistics as the bench does
    sh.reduce()
    sh.reset_stats()
    for _ in range(4):
        sh.step(4)
    st = sh.reduce()
    return {"accepts": st["accepts"].tolist(), "moments": st["moments"].tolist(),
            "lag_z": [x.tolist() for x in st["lag_z"]], "lag_v": [x.tolist() for x in st["lag_v"]],
            "gram": [x.tolist() for x in st["gram"]], "cov": D.StreamingShard.covariance(st["gram"]).tolist()}


@pytest.mark.timeout(300)
def test_streaming_shard_gloo_world2_matches_single_process(oracle):
    """The bench's aggregation (StreamingShard + allreduce_parts) over gloo, world 2,
    equals the single-process run over all chains.  The lag sums are over each
    rank's first `lag_chains` chains, so the single-process reference sums the
    same chains (lag_chains = 6: every chain of every shard)."""
    import torch
    from lgs_amd import distributed as D
    from _oracle_shard import oracle_advance_factory
    mgr = mp.Manager()
    out = mgr.dict()
    mp.start_processes(_stream_worker, args=(2, _free_port(), out), nprocs=2, join=True, start_method="spawn")
    g = golden_R(load_golden("klein_ntru32.npz"))
    single = _stream_stats(D, oracle, oracle_advance_factory, g, 0, 1, torch)
    for r in (0, 1):
        assert out[r]["accepts"] == single["accepts"]
        assert out[r]["moments"] == single["moments"]
        assert out[r]["lag_z"] == single["lag_z"]          # int64: exact
        np.testing.assert_allclose(np.array(out[r]["lag_v"][0]), np.array(single["lag_v"][0]), rtol=1e-13)
        assert out[r]["lag_v"][1] == single["lag_v"][1]
        assert out[r]["gram"] == single["gram"]            # int64 sum z z^T, sum z, count: exact
    assert 0 < single["accepts"][0] < 6 * 16  # Wang-Ling: some rejections
    # the thinned Gram = the chains' states after blocks 2 and 4 of the timed stretch
    # (steps 11 and 19: a 3-step warm-up block, then blocks of 4), base.py:154-160
    R, cp, B = g
    tr = oracle.imhk(R, cp, B, 165.7, 6, 19, seed=99, first_step=1, mode=oracle.IMHK_WANG_LING,
                     trace=True)["trace"]
    kept = np.concatenate([tr[:, 10], tr[:, 18]]).astype(np.int64)
    assert single["gram"][2] == [12]
    assert single["gram"][0] == (kept.T @ kept).tolist()
    np.testing.assert_allclose(np.array(single["cov"]), np.cov(kept.T.astype(float)), rtol=1e-12, atol=1e-12)


def test_init_process_group_needs_launcher_env_for_several_ranks(monkeypatch):
    """A random per-process port only serves a one-rank group; several ranks without
    MASTER_ADDR / MASTER_PORT would each wait at their own rendezvous."""
    from lgs_amd import distributed as D
    for k in ("MASTER_ADDR", "MASTER_PORT", "RANK", "WORLD_SIZE"):
        monkeypatch.delenv(k, raising=False)
    with pytest.raises(RuntimeError, match="MASTER_ADDR"):
        D.init_process_group("gloo", 0, 2, rank=0)


def test_imhk_sharded_rejects_world_mismatch(monkeypatch):
    """world must be the active group's size: a world=2 shard inside a one-rank group
    (or the reverse) would all-reduce / gather over the wrong set of ranks."""
    import torch.distributed as dist
    from lgs_amd import distributed as D
    for k in ("MASTER_ADDR", "MASTER_PORT", "RANK", "WORLD_SIZE"):
        monkeypatch.delenv(k, raising=False)
    D.init_process_group("gloo", 0, 1)
    try:
        def compute(**kw):
            raise AssertionError("must not run")
        with pytest.raises(ValueError, match="process group"):
            D.imhk_sharded(compute, 4, 2, rank=0, world=2)
    finally:
        dist.destroy_process_group()
