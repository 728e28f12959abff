"""Host logic of bench.py (CPU): the lag-L autocovariance sums carried across bench
steps, the exact int64-in-fp64 packing of the single all-reduce, and a
gloo world-2 reduction that equals the single-process statistics."""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402


def _direct(x, L):
    """sum_t x_t x_{t-k} and pair counts over whole series (n_chains x T)."""
    S = [float((x[:, k:] * x[:, :x.shape[1] - k]).sum()) for k in range(L + 1)]
    N = [x.shape[0] * (x.shape[1] - k) for k in range(L + 1)]
    return np.array(S), np.array(N)


@pytest.mark.parametrize("T,L", [(64, 16), (5, 16), (16, 16), (1, 3)])
def test_lag_sums_across_blocks_equal_whole_series(T, L):
    rng = np.random.default_rng(T + L)
    x = rng.integers(-50, 50, (7, 6 * T)).astype(np.int64)
    acc = bench.LagSums(torch, 7, L, torch.int64, "cpu")
    for b in range(6):
        acc.update(torch.from_numpy(x[:, b * T:(b + 1) * T]))
    S, N = _direct(x, L)
    np.testing.assert_array_equal(acc.S.numpy(), S)
    np.testing.assert_array_equal(acc.N, N)
    assert int(acc.S1) == x.sum() and int(acc.n) == x.size
    a = bench.LagSums.acf(S, N, float(x.sum()), float(x.size))
    assert a[0] == pytest.approx(1.0)


def test_pack_unpack_exact_int64():
    ints = torch.tensor([0, 1, -1, 2**62 - 5, -(2**61) + 3], dtype=torch.int64)
    f = torch.tensor([1.5, -2.25])
    flat, layout = bench.pack_f64(torch, [ints, f])
    a, b = bench.unpack_f64(torch, flat, layout)
    assert torch.equal(a, ints) and torch.equal(b, f)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, x, out):
    sys.path.insert(0, REPO)
    import torch.distributed as dist
    import bench as bm
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    half = x.shape[0] // world
    mine = x[rank * half:(rank + 1) * half]
    acc = bm.LagSums(torch, half, 8, torch.int64, "cpu")
    for b in range(4):
        acc.update(torch.from_numpy(mine[:, b * 10:(b + 1) * 10]))
    flat, layout = bm.pack_f64(torch, acc.parts())
    dist.all_reduce(flat)
    out[rank] = [t.numpy().tolist() for t in bm.unpack_f64(torch, flat, layout)]
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_gloo_world2_lag_sums_match_single_process():
    x = np.random.default_rng(3).integers(-9, 9, (8, 40)).astype(np.int64)
    mgr = mp.Manager()
    out = mgr.dict()
    mp.start_processes(_worker, args=(2, _free_port(), x, out), nprocs=2, join=True, start_method="spawn")
    single = bench.LagSums(torch, 8, 8, torch.int64, "cpu")
    for b in range(4):
        single.update(torch.from_numpy(x[:, b * 10:(b + 1) * 10]))
    for r in (0, 1):
        S, N, S1, n = out[r]
        assert S == single.S.tolist() and N == single.N.tolist()
        assert S1 == single.S1.tolist() and n == [single.n]
