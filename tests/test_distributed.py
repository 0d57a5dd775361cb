"""The multi-GPU path of bench.py on CPU: scenario sharding and the rank-combination step, run over a
world-size-2 gloo group (the GPU run uses the same functions over RCCL/xGMI, one process per GPU)."""

import os
import socket

import numpy as np
import pytest

torch = pytest.importorskip("torch")
import torch.distributed as dist  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402

import bench  # noqa: E402


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, B, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        # counters: solves, ipm iters, hl ms, elapsed, row iters
        tot = np.array([100.0 * (rank + 1), 600.0 * (rank + 1), 5.0 + rank, 1.0 + 0.5 * rank, 1800.0 * (rank + 1)])
        sf, seed = bench.shard(rank, B, 64)
        metrics = np.stack([np.full(B, float(rank)), sf.astype(np.float64), np.zeros(B)], 1)
        sums, maxs, gathered = bench.combine_ranks(dist, world, tot, metrics, "cpu")
        if rank == 0:
            np.save(out, np.concatenate([sums, maxs, gathered.reshape(-1), [seed]]))
    finally:
        dist.destroy_process_group()


def test_shard_is_a_partition():
    B, F, world = 96, 64, 4
    ids = np.concatenate([np.arange(B) + r * B for r in range(world)])
    assert len(np.unique(ids)) == B * world
    for r in range(world):
        sf, seed = bench.shard(r, B, F)
        assert np.array_equal(sf, (np.arange(B) + r * B) % F)
        assert seed == 1000 + r


def test_combine_ranks_gloo_world2(tmp_path):
    B, world = 8, 2
    out = str(tmp_path / "r0.npy")
    mp.spawn(_worker, args=(world, _free_port(), B, out), nprocs=world, join=True)
    v = np.load(out)
    sums, maxs, g = v[:5], v[5:10], v[10:-1].reshape(world * B, 3)
    np.testing.assert_allclose(sums, [300.0, 1800.0, 11.0, 2.5, 5400.0])
    assert maxs[3] == 1.5  # elapsed: max over ranks
    # all-gather keeps rank order, each rank's shard of scenarios contiguous
    assert np.array_equal(g[:B, 0], np.zeros(B)) and np.array_equal(g[B:, 0], np.ones(B))
    assert np.array_equal(g[:, 1], np.arange(world * B) % 64)
