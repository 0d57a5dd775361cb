"""The multi-GPU path of bench.py on CPU: scenario sharding and the rank-combination step, run over a
world-size-2 gloo group through the test harness's GlooComm (tests/_gloo_comm.py; the GPU run uses the same
functions over sharding.Comm, RCCL over xGMI through libdat.so, one process per GPU)."""

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
        from tests._gloo_comm import GlooComm

        sums, maxs, gathered = bench.combine_ranks(GlooComm(), tot, metrics)
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


def test_bench_spawns_ranks_selftest():
    """`python bench.py --gpus 2` without a launcher spawns two rank processes (gloo here, --selftest:
    no solver work) that shard, combine over the process group and print ONE line from rank 0."""
    import json
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--selftest", "--steps", "2",
                        "--warmup", "1", "--batch", "16"], capture_output=True, text=True, timeout=240,
                       env=dict(os.environ, MASTER_ADDR="127.0.0.1"))
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["config"]["parallelism"] == "scenario-sharded x2"
    assert out["stats"]["agent_qp_solves"] == 2 * 2 * 16 * 6  # ranks x steps x scenarios x agents
    assert out["stats"]["mean_admm_iters"] == 1.5             # gathered from both ranks (1 and 2)
    assert out["data"].startswith("selftest")


def test_strong_shard_partitions_the_total():
    for total, world in ((65536, 8), (65536, 1), (32, 2), (35, 4)):
        parts = [bench.strong_shard(r, world, total) for r in range(world)]
        ids = np.concatenate([np.arange(lo, lo + c) for lo, c in parts])
        assert np.array_equal(ids, np.arange(total))
        assert max(c for _, c in parts) - min(c for _, c in parts) <= 1
    assert bench.strong_shard(3, 8, 65536) == (3 * 8192, 8192)  # BASELINE configs[3]: 8,192 per GPU


def test_bench_strong_scaling_selftest():
    """`bench.py --gpus 2 --selftest --total-batch 32`: strong scaling, 16 scenarios per rank, 32 in total."""
    import json
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--selftest", "--steps", "2",
                        "--warmup", "1", "--total-batch", "32"], capture_output=True, text=True, timeout=240,
                       env=dict(os.environ, MASTER_ADDR="127.0.0.1"))
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["scaling"] == "strong"
    assert out["config"]["scenarios_per_gpu"] == 16 and out["config"]["total_scenarios"] == 32
    assert out["stats"]["agent_qp_solves"] == 2 * 2 * 16 * 6  # ranks x steps x scenarios per rank x agents


def test_bench_default_is_baseline_config_strong():
    """With no --batch / --total-batch, C4 measures BASELINE configs[3] at every N: 65,536 scenarios split
    over the ranks (strong scaling; a driver SCALE run at 8 GPUs runs 8,192 per GPU)."""
    import sys

    argv = sys.argv
    try:
        for extra, per, scaling_total in (([], 65536, 65536), (["--batch", "1024"], 1024, None)):
            sys.argv = ["bench.py", "--gpus", "8"] + extra
            a = bench.parse()
            assert a.total_batch == scaling_total
            B = a.batch if a.total_batch is None else bench.strong_shard(7, 8, a.total_batch)[1]
            assert B == (8192 if scaling_total else per)
        sys.argv = ["bench.py", "--config", "C2"]
        a = bench.parse()
        assert a.total_batch is None and a.batch == 1024
    finally:
        sys.argv = argv


def _uneven_worker(rank, world, port, total, out):
    from distributed_aerial_transportation_amd.sharding import gather_rows, reduce_values, shard_range

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from tests._gloo_comm import GlooComm

        comm = GlooComm()
        lo, cnt = shard_range(rank, world, total)
        ids = np.arange(lo, lo + cnt, dtype=np.float64)
        rows = gather_rows(np.stack([ids, np.full(cnt, float(rank))], 1), comm)
        s = reduce_values([cnt, 1.0], "sum", comm)
        m = reduce_values([cnt, rank], "max", comm)
        if rank == 0:
            np.save(out, np.concatenate([rows.reshape(-1), s, m]))
    finally:
        dist.destroy_process_group()


def test_sharding_gather_uneven_gloo_world3(tmp_path):
    """The package's sharding collectives (sharding.py): 10 scenarios over 3 ranks (4 / 3 / 3) gather
    back in global scenario order; sums and maxima over ranks."""
    from distributed_aerial_transportation_amd.sharding import shard_range

    total, world = 10, 3
    assert [shard_range(r, world, total) for r in range(world)] == [(0, 4), (4, 3), (7, 3)]
    out = str(tmp_path / "u.npy")
    mp.spawn(_uneven_worker, args=(world, _free_port(), total, out), nprocs=world, join=True)
    v = np.load(out)
    rows = v[: 2 * total].reshape(total, 2)
    assert np.array_equal(rows[:, 0], np.arange(total))
    assert np.array_equal(rows[:, 1], [0, 0, 0, 0, 1, 1, 1, 2, 2, 2])
    np.testing.assert_array_equal(v[2 * total: 2 * total + 2], [10.0, 3.0])
    np.testing.assert_array_equal(v[2 * total + 2:], [4.0, 2.0])


def test_auto_sub_batches_policy():
    """C4 stream count per GPU: one stream for the full 65,536-scenario batch (the N = 1 headline), four for
    the per-GPU batches of the 2-, 4- and 8-GPU strong splits of BASELINE configs[3]."""
    from distributed_aerial_transportation_amd.sharding import shard_range

    assert bench.auto_sub_batches(65536) == 1
    for world in (2, 4, 8):
        assert bench.auto_sub_batches(shard_range(0, world, 65536)[1]) == 4
