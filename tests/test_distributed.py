"""Multi-rank path on CPU (gloo, world_size 2): the row-block/triangle-tile work split of the
implicit matrix and the per-iteration all-reduce exchange, with the library's own partition
function (plssvm_mi_partition, host-only) and a numpy restatement of the tile contributions.

On the GPU the same split drives kp_tile_kernel / kp_reduce_kernel and the all-reduce is RCCL
(engine.hip: kp_device); tests/test_gpu_parity.py checks the split on one GPU with simulated ranks.
"""
import os
import socket

import numpy as np
import pytest

TILE, SUPER = 128, 8


def tri_tile(t):
    i = int((np.sqrt(8.0 * t + 1.0) - 1.0) * 0.5)
    while i * (i + 1) // 2 > t:
        i -= 1
    while (i + 1) * (i + 2) // 2 <= t:
        i += 1
    return i, t - i * (i + 1) // 2


def rank_share(K, p, s0, s1):
    """sum over the owned super-blocks' tiles of K_IJ p_J (rows I) and K_IJ^T p_I (rows J, I != J)."""
    m = K.shape[0]
    nb = -(-m // TILE)
    out = np.zeros(m)
    for s in range(s0, s1):
        SI, SJ = tri_tile(s)
        for a in range(SUPER):
            for b in range(SUPER):
                I, J = SI * SUPER + a, SJ * SUPER + b
                if I >= nb or J > I:
                    continue
                ri = slice(I * TILE, min(m, (I + 1) * TILE))
                rj = slice(J * TILE, min(m, (J + 1) * TILE))
                out[ri] += K[ri, rj] @ p[rj]
                if I != J:
                    out[rj] += K[ri, rj].T @ p[ri]
    return out


def qtilde_rank1(K_full_last, QA, cost, p, q):
    return (QA - q) * p.sum() - q @ p + p / cost


def _worker(rank, world, port, m, result):
    import torch
    import torch.distributed as dist

    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import plssvm_sparse_fp22_amd as pm

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    rng = np.random.default_rng(3)
    X = rng.uniform(-1, 1, size=(m + 1, 8))
    gamma = 1.0 / 8
    D = ((X[:, None, :] - X[None, :, :]) ** 2).sum(-1)
    Kfull = np.exp(-gamma * D)
    K, q, QA, cost = Kfull[:m, :m], Kfull[:m, m], Kfull[m, m] + 1.0, 1.0
    s0, s1, tt, tl = pm.partition(m, rank, world)

    def kp(p):  # one K·p: local share + all-reduce (RCCL on the GPU) + replicated rank-1 terms
        share = torch.from_numpy(rank_share(K, p, s0, s1))
        dist.all_reduce(share)
        return share.numpy() + qtilde_rank1(None, QA, cost, p, q)

    p = rng.uniform(1, 2, m)
    full = K @ p + qtilde_rank1(None, QA, cost, p, q)
    kp_err = float(np.abs(kp(p) - full).max() / np.abs(full).max())
    counts = torch.tensor([tl], dtype=torch.int64)
    dist.all_reduce(counts)
    # replicated CG (OpenMP/csvm.cpp:82-170) driven by the distributed K·p
    b = np.where(rng.random(m) < 0.5, 2.0, 0.0) - 1.0
    x = np.ones(m)
    r = b - kp(x)
    delta = r @ r
    d = r.copy()
    for it in range(12):
        Ad = kp(d)
        a = delta / (d @ Ad)
        x = x + a * d
        r = b - kp(x) if it % 50 == 49 else r - a * Ad
        delta_old, delta = delta, r @ r
        d = (delta / delta_old) * d + r
    xs = [torch.zeros(m, dtype=torch.float64) for _ in range(world)]
    dist.all_gather(xs, torch.from_numpy(x))
    result[rank] = dict(kp_err=kp_err, tiles=int(counts.item()), tt=tt, tl=tl,
                        x_same=bool(all(torch.equal(xs[0], xx) for xx in xs)),
                        x=x)
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


@pytest.mark.parametrize("m", [700, 1300])
def test_two_rank_split_and_exchange(m):
    import torch.multiprocessing as mp

    manager = mp.Manager()
    result = manager.dict()
    port = _free_port()
    mp.spawn(_worker, args=(2, port, m, result), nprocs=2, join=True)
    r0, r1 = result[0], result[1]
    nb = -(-m // TILE)
    assert r0["tt"] == nb * (nb + 1) // 2
    assert r0["tiles"] == r0["tt"]  # every tile owned by exactly one rank
    assert abs(r0["tl"] - r1["tl"]) <= 64  # balanced to a super-block
    assert r0["kp_err"] < 1e-13 and r1["kp_err"] < 1e-13
    assert r0["x_same"] and r1["x_same"]  # replicated CG stays identical on every rank


@pytest.mark.parametrize("world", [1, 2, 3, 8])
@pytest.mark.parametrize("m", [1, 127, 128, 1025, 99_999])
def test_partition_covers_triangle(world, m):
    import plssvm_sparse_fp22_amd as pm

    parts = [pm.partition(m, r, world) for r in range(world)]
    nb = -(-m // TILE)
    assert sum(p[3] for p in parts) == nb * (nb + 1) // 2
    for a, b in zip(parts, parts[1:]):
        assert a[1] == b[0]  # contiguous
    ns = -(-nb // SUPER)
    assert parts[0][0] == 0 and parts[-1][1] == ns * (ns + 1) // 2
    if nb > 64 * world:
        loads = [p[3] for p in parts]
        assert max(loads) - min(loads) <= 2 * 64  # each boundary within one super-block


def _xchg_worker(rank, world, port, result):
    import torch.distributed as dist

    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import plssvm_sparse_fp22_amd as pm
    from plssvm_sparse_fp22_amd import _abi

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    fn = pm.torch_exchange(dist)
    rng = np.random.default_rng(100 + rank)
    a = rng.standard_normal(1001)
    parts = [np.random.default_rng(100 + r).standard_normal(1001) for r in range(world)]
    want = parts[0].copy()
    for r in range(1, world):
        want += parts[r]
    fn(a, _abi.XCHG_ALLREDUCE)
    g = np.zeros(world * 7, dtype=np.float32)
    g[rank * 7:(rank + 1) * 7] = rank + 1
    fn(g, _abi.XCHG_ALLGATHER)
    result[rank] = dict(sum_ok=bool(np.array_equal(a, want)), gather=g)
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_host_exchange_over_gloo(world):
    """plssvm_mi_comm_init_host's exchange over torch.distributed (torch_exchange): the all-reduce is the
    rank-order sum (the reference's device_reduction order, gpu_csvm.cpp:366-386) with identical bits on
    every rank; the all-gather fills every rank's chunk."""
    import torch.multiprocessing as mp

    manager = mp.Manager()
    result = manager.dict()
    mp.spawn(_xchg_worker, args=(world, _free_port(), result), nprocs=world, join=True)
    for r in range(world):
        assert result[r]["sum_ok"]
        np.testing.assert_array_equal(result[r]["gather"], np.repeat(np.arange(1, world + 1), 7).astype(np.float32))


def _xchg_fail_worker(rank, world, port, result):
    import torch.distributed as dist

    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import plssvm_sparse_fp22_amd as pm
    from plssvm_sparse_fp22_amd import _abi

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    fn = pm.torch_exchange(dist)
    a = np.ones(64)
    try:
        # the last rank's local step fails before its collective; it must still join, and every rank raises
        fn(a, _abi.XCHG_ALLREDUCE, local_error=ValueError("local failure") if rank == world - 1 else None)
        result[rank] = "no error"
    except RuntimeError as e:
        result[rank] = str(e)
    b = np.full(8, float(rank))  # the group is still usable afterwards
    fn(b, _abi.XCHG_ALLREDUCE)
    result[(rank, "after")] = float(b[0])
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_host_exchange_failure_reaches_every_rank(world):
    """a rank whose exchange fails locally still takes part in the collective (status
    element), so every rank raises — the library then returns PLSSVM_MI_ERR_RCCL on all of them — and
    nobody hangs in the collective."""
    import torch.multiprocessing as mp

    manager = mp.Manager()
    result = manager.dict()
    mp.spawn(_xchg_fail_worker, args=(world, _free_port(), result), nprocs=world, join=True)
    for r in range(world):
        assert f"rank(s) [{world - 1}]" in result[r], result[r]
        assert result[(r, "after")] == float(sum(range(world)))
