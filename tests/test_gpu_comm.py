"""K8's metric collectives through libdat.so's RCCL C-ABI (sharding.Comm, dat_comm_*), world size 1 on the
one-GPU box: the id exchange, the uneven-row gather, sum / max reductions and the barrier, without PyTorch.
(The multi-rank paths of the same functions run over the gloo test harness in tests/test_distributed.py; an
8-GPU node runs them over RCCL in the driver's scaling bench.)"""

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_gpu_rccl_comm_world1(monkeypatch):
    from distributed_aerial_transportation_amd.sharding import Comm, gather_rows, reduce_values

    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.delenv("RANK", raising=False)
    comm = Comm.from_env(device=0)
    assert (comm.world, comm.rank) == (1, 0)
    rows = np.random.default_rng(0).normal(size=(7, 4))
    np.testing.assert_array_equal(gather_rows(rows, comm), rows)
    np.testing.assert_array_equal(gather_rows(np.zeros((0, 4)), comm), np.zeros((0, 4)))
    v = np.array([1.5, -2.0, 3.25])
    np.testing.assert_array_equal(reduce_values(v, "sum", comm), v)
    np.testing.assert_array_equal(reduce_values(v, "max", comm), v)
    comm.barrier()
    g = comm.allgather(np.arange(5.0))
    assert g.shape == (1, 5) and np.array_equal(g[0], np.arange(5.0))
    comm.close()
